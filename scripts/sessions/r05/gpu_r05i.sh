# Round 5 session i: compact groups of one frame length apply masks and seed
# in registers (rp) against the in-place LDS patch (ch2 = HEAD): tiny-frame
# and parity tests, ACK A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/rp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_golden.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05i.log 2>&1
rc=$?; tail -2 $O/pytest_r05i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads ack --rounds 4 scratch/libs/ch2.so \
  scratch/libs/rp.so > $O/ab_r05i.log 2>&1
rc=$?; cat $O/ab_r05i.log; exit $rc
