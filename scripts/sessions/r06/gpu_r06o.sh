# Round 6 session o: waves kept together by bare barriers (A/B).  cfg5: an
# extra barrier every 4 / 8 / 16 rounds (ss4 / ss8 / ss16; the ring flush
# already meets every ~42).  ACK: a barrier after every full 8-group turn
# (as1) or every second (as2).  The tiny-frame tests run on as1 first.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/as1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r06o.log 2>&1
rc=$?; tail -2 $O/pytest_r06o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg5 --rounds 3 scratch/libs/head.so \
  scratch/libs/ss4.so scratch/libs/ss8.so scratch/libs/ss16.so > $O/ab_r06o_cfg5.log 2>&1
rc=$?; cat $O/ab_r06o_cfg5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 3 scratch/libs/head.so \
  scratch/libs/as1.so scratch/libs/as2.so > $O/ab_r06o_ack.log 2>&1
rc=$?; cat $O/ab_r06o_ack.log; exit $rc
