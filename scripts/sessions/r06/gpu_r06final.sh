# Round 6, final tree: the whole -m gpu suite, smoke() and the driver's
# default bench command on the shipped library (6f21f47a).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r06final.log 2>&1
rc=$?; tail -3 $O/pytest_r06final.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_r06final.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r06final.log 2>&1
rc=$?; tail -1 $O/smoke_r06final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_r06final.json 2> $O/bench_r06final.err
rc=$?; tail -c 600 $O/bench_r06final.json; exit $rc
