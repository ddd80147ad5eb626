# Round 6 session r: the segmentation kernel's frame-store cache policy (A/B):
# nt (the tree), default (sp0), sc1 (sp16), nt sc1 (sp18).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads seg --rounds 3 scratch/libs/cur.so \
  scratch/libs/sp0.so scratch/libs/sp16.so scratch/libs/sp18.so > $O/ab_r06r.log 2>&1
rc=$?; cat $O/ab_r06r.log; exit $rc
