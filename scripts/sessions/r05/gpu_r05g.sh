# Round 5 session g: segmentation kernel lanes per packet (G = 4 / 8 / 16).
set -u
O=gpurun_out
mkdir -p $O
: > $O/ab_r05g.log
for G in 8 16 4; do
  echo "lanes $G" >> $O/ab_r05g.log
  timeout -k 10 300 python scratch/bench_ab.py --workloads seg --rounds 2 --bench-args "--lanes $G" \
    scratch/libs/h05.so >> $O/ab_r05g.log 2>&1 || { cat $O/ab_r05g.log; exit 1; }
done
cat $O/ab_r05g.log
