# Round 6 session s: seg and cfg2 on round 5's library against the current
# one (is the slower seg of session r the box or the build?).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python scratch/bench_ab.py --workloads seg,cfg2 --rounds 2 scratch/libs/r05.so \
  scratch/libs/cur.so > $O/ab_r06s.log 2>&1
rc=$?; cat $O/ab_r06s.log; exit $rc
