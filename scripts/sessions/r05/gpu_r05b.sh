# Round 5 session b: small / tiny GPU tests on the in-tree library, then A/B
# of the cfg5 and ACK workloads across library builds in scratch/libs/.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_tiny.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05b.log 2>&1
rc=$?; tail -3 $O/pytest_r05b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads cfg5 --rounds 3 scratch/libs/base.so \
  scratch/libs/regpatch.so scratch/libs/exact.so scratch/libs/compact12.so > $O/ab_r05b_cfg5.log 2>&1
rc=$?; cat $O/ab_r05b_cfg5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads ack,cfg3 --rounds 3 scratch/libs/base.so \
  scratch/libs/compact12.so > $O/ab_r05b_ack.log 2>&1
rc=$?; cat $O/ab_r05b_ack.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads seg --rounds 3 scratch/libs/base.so \
  scratch/libs/seg_nt.so > $O/ab_r05b_seg.log 2>&1
rc=$?; cat $O/ab_r05b_seg.log; exit $rc
