# Round 5 session h: the compact kernel folding two chains over Mul(64)
# (ch2) against four over Mul(128) (h05 = HEAD): tiny-frame tests, ACK A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/ch2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05h.log 2>&1
rc=$?; tail -2 $O/pytest_r05h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads ack --rounds 4 scratch/libs/h05.so \
  scratch/libs/ch2.so > $O/ab_r05h.log 2>&1
rc=$?; cat $O/ab_r05h.log; exit $rc
