# Round 5 session k: small-frame kernel with the first 8 / 16 / 32 rounds of
# each output-ring window held in registers (rr8, rr16, rr32) against the LDS
# ring alone (h06 = HEAD): small-frame tests on each, cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
for v in rr16 rr8 rr32; do
  ROCE_ICRC_LIB=$PWD/scratch/libs/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05k_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_r05k_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 700 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/h06.so \
  scratch/libs/rr8.so scratch/libs/rr16.so scratch/libs/rr32.so > $O/ab_r05k.log 2>&1
rc=$?; cat $O/ab_r05k.log; exit $rc
