# Round 6 session w (flakiness check on another box): the whole -m gpu suite and smoke() on the current build.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r06w.log 2>&1
rc=$?; tail -3 $O/pytest_r06w.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_r06w.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r06w.log 2>&1
rc=$?; tail -1 $O/smoke_r06w.log; exit $rc
