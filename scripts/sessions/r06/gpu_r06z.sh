# Round 6 session z: the compact kernel's output-ring edge cases.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r06z.log 2>&1
rc=$?; tail -3 $O/pytest_r06z.log; [ $rc -eq 0 ] || grep -E "FAILED|Error|assert" $O/pytest_r06z.log | head -20; exit $rc
