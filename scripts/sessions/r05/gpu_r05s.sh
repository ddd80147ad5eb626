# Round 5 session s: the compact kernel writes every span chunk to its own
# slot address (cst = the tree) instead of clamping past-span chunks onto the
# span's last one (h10 = 4c5b4f77): small-frame (incl. the under-44-B
# strides) and tiny-frame tests, ACK / cfg3 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_tiny.py tests/test_gpu_golden.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05s.log 2>&1
rc=$?; tail -2 $O/pytest_r05s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads ack,cfg3 --rounds 4 scratch/libs/h10.so \
  scratch/libs/cst.so > $O/ab_r05s.log 2>&1
rc=$?; cat $O/ab_r05s.log; exit $rc
