# Round 5 session m: small-frame kernel with the unmasked DMA / slot reads at
# register-ring depths 24 and 28 (nm24, nm28), and with the first batch's DMA
# issued before the tables are staged (ne24, ne28), against h07 (session l's
# baseline): small-frame and ring tests on each variant and the in-tree
# library, then a cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
for v in tree nm28 ne24 ne28; do
  if [ $v = tree ]; then unset ROCE_ICRC_LIB; else export ROCE_ICRC_LIB=$PWD/scratch/libs/$v.so; fi
  timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_parity.py -k "small or Small" -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05m_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_r05m_$v.log; [ $rc -eq 0 ] || exit $rc
done
unset ROCE_ICRC_LIB
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/h07.so \
  scratch/libs/nm24.so scratch/libs/nm28.so scratch/libs/ne24.so scratch/libs/ne28.so > $O/ab_r05m.log 2>&1
rc=$?; cat $O/ab_r05m.log; exit $rc
