# Round 5 session l: the full -m gpu suite and smoke() on HEAD's library, then
# the small-frame kernel's register-ring depth (16 = HEAD, 24) and the unmasked DMA / slot reads (nm, nm24) in a cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r05l.log 2>&1
rc=$?; tail -3 $O/pytest_r05l.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r05l.log 2>&1
rc=$?; tail -2 $O/smoke_r05l.log; [ $rc -eq 0 ] || exit $rc
for v in rr24 nm nm24; do
  ROCE_ICRC_LIB=$PWD/scratch/libs/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py -m gpu -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05l_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_r05l_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 700 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/h07.so \
  scratch/libs/rr24.so scratch/libs/nm.so scratch/libs/nm24.so > $O/ab_r05l.log 2>&1
rc=$?; cat $O/ab_r05l.log; exit $rc
