# Round 6 session l: the tail pool's cost split -- the pool build with no pool
# (p0: pool_packets() = 0, every other change in) and with a 1/32 pool, against
# the pre-pool build and the 1/8 pool (cfg3); pool4 = counters on their own lines.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/head.so \
  scratch/libs/p0.so scratch/libs/p32.so scratch/libs/pool3.so scratch/libs/pool4.so > $O/ab_r06l.log 2>&1
rc=$?; cat $O/ab_r06l.log; exit $rc
