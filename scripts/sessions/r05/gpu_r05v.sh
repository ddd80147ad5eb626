# Round 5 session v: cache policy of the small-frame kernel's ring flushes
# with the 28 register rounds: default (op0), nt (op2), nt sc1 (op18) against
# sc1 (h10 = 4c5b4f77): cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/op2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05v.log 2>&1
rc=$?; tail -1 $O/pytest_r05v.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/h10.so \
  scratch/libs/op0.so scratch/libs/op2.so scratch/libs/op18.so > $O/ab_r05v.log 2>&1
rc=$?; cat $O/ab_r05v.log; exit $rc
