# Round 5 session t: tail stealing with 8 / 16 fixed victims (v8, v16) and 16
# victims over the last quarter (v16t4) against 4 over the last eighth (h10 =
# 4c5b4f77): strided / small-frame parity tests on each, cfg2 / cfg5 A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
for v in v8 v16 v16t4; do
  ROCE_ICRC_LIB=$PWD/scratch/libs/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_parity.py \
    -k "strided or small or full_size" -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05t_$v.log 2>&1
  rc=$?; tail -1 $O/pytest_r05t_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 1000 python scratch/bench_ab.py --workloads cfg2,cfg5 --rounds 4 scratch/libs/h10.so \
  scratch/libs/v8.so scratch/libs/v16.so scratch/libs/v16t4.so > $O/ab_r05t.log 2>&1
rc=$?; cat $O/ab_r05t.log; exit $rc
