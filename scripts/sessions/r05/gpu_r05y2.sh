# Round 5 session y2: the compact kernel's last 1/16 of groups claimed in runs
# of 16 through one counter (ctail = the tree) against static ranges only
# (h10 = 4c5b4f77): tiny-frame, golden, ragged parity and C-ABI tests on the
# tree, ACK A/B, workgroup end times of the diagnostic build.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_golden.py tests/test_gpu_parity.py \
  tests/test_gpu_recv.py tests/test_gpu_capi.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_r05y2.log 2>&1
rc=$?; tail -2 $O/pytest_r05y2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 5 scratch/libs/h10.so \
  scratch/libs/ctail.so > $O/ab_r05y2.log 2>&1
rc=$?; cat $O/ab_r05y2.log; [ $rc -eq 0 ] || exit $rc
ROCE_ICRC_LIB=$PWD/scratch/libs/diag.so timeout -k 10 400 python scratch/tail_times.py > $O/tail_times_ctail.log 2>&1
rc=$?; grep ack $O/tail_times_ctail.log; exit $rc
