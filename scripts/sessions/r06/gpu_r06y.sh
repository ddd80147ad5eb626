# Round 6 session y: the compact kernel's first three descriptor loads issued
# with the table words (pre1) against the same code without (pre0) and the
# tree's build (cur); tiny-frame tests on pre1.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/pre1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r06y.log 2>&1
rc=$?; tail -2 $O/pytest_r06y.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 4 scratch/libs/cur.so \
  scratch/libs/pre0.so scratch/libs/pre1.so > $O/ab_r06y.log 2>&1
rc=$?; cat $O/ab_r06y.log; exit $rc
