# Round 6 session d: the compact kernel's register ring (16 rounds, 16
# consecutive groups per wave per turn) under store policies (s = sc1, ns =
# nt sc1, p0 = default, plain = nt) and an 8-round ring / 8-group turns.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 3 scratch/libs/r05.so \
  scratch/libs/r16c.so scratch/libs/r16cs.so scratch/libs/r16cns.so scratch/libs/r16cp0.so \
  scratch/libs/r8cs.so scratch/libs/r16c8s.so > $O/ab_r06d.log 2>&1
rc=$?; cat $O/ab_r06d.log; exit $rc
