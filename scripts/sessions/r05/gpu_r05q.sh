# Round 5 session q: one round trip for every kernel's prologue (table words
# loaded together; the sorted and compact kernels' first descriptors issued
# before them) -- `pro` = the tree -- against h09 (fd8190f6, the r05y
# evidence): the full -m gpu suite on the tree, then an A/B of every workload.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r05q.log 2>&1
rc=$?; tail -2 $O/pytest_r05q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scratch/bench_ab.py --workloads cfg3,ack,cfg2,cfg5 --rounds 3 scratch/libs/h09.so \
  scratch/libs/pro.so > $O/ab_r05q.log 2>&1
rc=$?; cat $O/ab_r05q.log; exit $rc
