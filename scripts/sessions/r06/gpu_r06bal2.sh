# Round 6: cfg3 A/B, byte-balanced ranges: shipped build, the new prologue
# order alone, balanced by bytes, by bytes + 1 KiB / 4 KiB per packet.
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 1000 python -u scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/cur.so scratch/libs/balord.so scratch/libs/bal0.so scratch/libs/bal1k.so scratch/libs/bal4k.so > $O/ab_r06bal2.txt 2>&1
rc=$?; cat $O/ab_r06bal2.txt; exit $rc
