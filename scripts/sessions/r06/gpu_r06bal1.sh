# Round 6: byte-balanced ranges for the sorted ragged kernel (variant
# scratch/libs/bal.so): its tests, then cfg3 A/B against the shipped build.
set -u
O=gpurun_out
mkdir -p $O
ROCE_ICRC_LIB=scratch/libs/bal.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_sorted.py tests/test_gpu_parity.py -k "sorted or balanced or cfg3 or ragged" > $O/pytest_bal_r06a.log 2>&1
rc=$?; tail -30 $O/pytest_bal_r06a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/cur.so scratch/libs/bal.so > $O/ab_r06bal1.txt 2>&1
rc=$?; cat $O/ab_r06bal1.txt; exit $rc
