# Round 5 session j: uniform 16-byte-aligned compact groups read their frames
# with ds_read_b128 into registers (rq) against b32 reads from the slot (h06 =
# HEAD): tiny-frame and golden tests, ACK A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/rq.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_golden.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05j.log 2>&1
rc=$?; tail -2 $O/pytest_r05j.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads ack --rounds 4 scratch/libs/h06.so \
  scratch/libs/rq.so > $O/ab_r05j.log 2>&1
rc=$?; cat $O/ab_r05j.log; exit $rc
