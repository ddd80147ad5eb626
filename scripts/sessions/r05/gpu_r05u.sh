# Round 5 session u: the small-frame kernel's tail stealing -- no victims
# (sv0), 2 (sv2), the last 1/32 claimable (st32) -- against 4 victims over the
# last 1/16 (h10 = 4c5b4f77): small-frame tests on each, cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
for v in sv0 sv2 st32; do
  ROCE_ICRC_LIB=$PWD/scratch/libs/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05u_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_r05u_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/h10.so \
  scratch/libs/sv0.so scratch/libs/sv2.so scratch/libs/st32.so > $O/ab_r05u.log 2>&1
rc=$?; cat $O/ab_r05u.log; exit $rc
