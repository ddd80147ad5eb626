# Round 6 session v: the sorted kernel's endgame -- once fewer than T packets
# of the window are left, claims of half the size (8 long packets -> 4, 16
# short -> 8), so the waves' last sets end closer together (T = 128 / 256 /
# 512, A/B on cfg3); sorted / tiny / parity tests on eg256.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/eg256.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sorted.py \
  tests/test_gpu_tiny.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r06v.log 2>&1
rc=$?; tail -2 $O/pytest_r06v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/cur.so \
  scratch/libs/eg128.so scratch/libs/eg256.so scratch/libs/eg512.so > $O/ab_r06v.log 2>&1
rc=$?; cat $O/ab_r06v.log; exit $rc
