# Round 5 session e: the compact kernel with a bank-skewed span slot and a
# replicated Mul(-32) combine (c10) -- tiny-frame tests, A/B against c07 on
# ACK and cfg3, SQ counters of the ACK launch.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py -m gpu -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $O/pytest_r05e.log 2>&1
rc=$?; tail -2 $O/pytest_r05e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads ack,cfg3 --rounds 3 scratch/libs/c07.so \
  scratch/libs/c10.so > $O/ab_r05e.log 2>&1
rc=$?; cat $O/ab_r05e.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_sq.sh r05e ack
