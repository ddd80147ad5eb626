# Round 5 session r: tail stealing from the fullest tail left (richest_tail;
# `steal` = the tree) against a fixed list of 4 victims (pro = 2ade14b, h09 =
# fd8190f6): the full -m gpu suite, A/B of cfg2 / cfg5 / seg / cfg3, and the
# workgroup end times of the diagnostic build.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r05r.log 2>&1
rc=$?; tail -2 $O/pytest_r05r.log; [ $rc -eq 0 ] || exit $rc
ROCE_ICRC_LIB=$PWD/scratch/libs/diag_steal.so timeout -k 10 400 python scratch/tail_times.py > $O/tail_times_steal.log 2>&1
rc=$?; cat $O/tail_times_steal.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python scratch/bench_ab.py --workloads cfg2,cfg5,seg,cfg3 --rounds 3 scratch/libs/pro.so \
  scratch/libs/steal.so > $O/ab_r05r.log 2>&1
rc=$?; cat $O/ab_r05r.log; exit $rc
