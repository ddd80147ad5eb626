# Round 6 session b: ACK compact-kernel ablations (diagnostic builds, not
# kept): 1 no output stores, 2 no fold, 3 span loads from the L2-hot table
# image, 4 no fold and no stores -- against round 5's library.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 3 scratch/libs/r05.so \
  scratch/libs/diag1.so scratch/libs/diag2.so scratch/libs/diag3.so scratch/libs/diag4.so > $O/ab_r06b.log 2>&1
rc=$?; cat $O/ab_r06b.log; exit $rc
