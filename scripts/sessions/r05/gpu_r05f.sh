# Round 5 session f: segmentation kernel at 12 waves x 3 loads in flight per
# lane (s12u3) against 8 waves x 4 (h05 = HEAD): segment tests, then A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/s12u3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_segment.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05f.log 2>&1
rc=$?; tail -2 $O/pytest_r05f.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads seg --rounds 4 scratch/libs/h05.so \
  scratch/libs/s12u3.so > $O/ab_r05f.log 2>&1
rc=$?; cat $O/ab_r05f.log; exit $rc
