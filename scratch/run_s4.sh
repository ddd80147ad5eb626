set -u
mkdir -p gpurun_out
make -C oracle -s || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s4.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_s4.log; [ $rc -eq 0 ] || exit $rc
echo "== staged"; timeout -k 10 120 python scripts/latency.py 2>&1 | grep call || exit 1
echo "== prev"; ROCE_ICRC_LIB=$PWD/scratch/libs/prev.so timeout -k 10 120 python scripts/latency.py 2>&1 | grep call || exit 1
