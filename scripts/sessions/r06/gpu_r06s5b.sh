# Round 6: cfg5 A/B, more rounds (the box's runs are bimodal): shipped,
# nt flushes, 1/8 tail.
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 1100 python -u scratch/bench_ab.py --workloads cfg5 --rounds 7 scratch/libs/cur.so scratch/libs/s5pol2.so scratch/libs/s5tail8.so > $O/ab_r06s5b.txt 2>&1
rc=$?; cat $O/ab_r06s5b.txt; exit $rc
