# Round 6 session c: the compact kernel's output words.  d5 = words to an
# L2-resident 16-KiB window (diagnostic); r16 / r32 = 16 / 32 rounds of words
# held in registers and flushed back to back; c16 / c32 = each wave takes 16 /
# 32 consecutive groups per turn (its flush one contiguous run); s = sc1 stores.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 3 scratch/libs/r05.so \
  scratch/libs/d5.so scratch/libs/r16.so scratch/libs/r16c.so scratch/libs/r16s.so scratch/libs/c16.so \
  scratch/libs/r32c.so > $O/ab_r06c.log 2>&1
rc=$?; cat $O/ab_r06c.log; exit $rc
