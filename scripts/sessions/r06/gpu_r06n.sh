# Round 6 session n: what cfg5's output words cost now (diagnostic builds):
# s1 = the ring flushes without their stores (barriers kept), s2 = no flush
# at all (no barriers, no stores).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg5 --rounds 3 scratch/libs/head.so \
  scratch/libs/s1.so scratch/libs/s2.so > $O/ab_r06n.log 2>&1
rc=$?; cat $O/ab_r06n.log; exit $rc
