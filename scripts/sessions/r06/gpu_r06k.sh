# Round 6 session k: the sorted kernel's tail pool (tree) -- pool tests, the
# ragged / parity / golden suites, then cfg3 A/B against the previous build.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_tiny.py tests/test_gpu_parity.py \
  tests/test_gpu_golden.py tests/test_gpu_recv.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r06k.log 2>&1
rc=$?; tail -3 $O/pytest_r06k.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_r06k.log | head -20; exit $rc; }
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/head.so \
  scratch/libs/pool3.so > $O/ab_r06k.log 2>&1
rc=$?; cat $O/ab_r06k.log; exit $rc
