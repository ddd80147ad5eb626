# Round 6 session p: cfg5 with the last batch (read straight from global
# memory by one wave) folded at the start instead of after the tail claims
# (lf): the small-frame tests on lf, then the cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/lf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r06p.log 2>&1
rc=$?; tail -2 $O/pytest_r06p.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/head.so \
  scratch/libs/lf.so > $O/ab_r06p.log 2>&1
rc=$?; cat $O/ab_r06p.log; exit $rc
