# Round 5 session d: the compact kernel's variants -- 12 / 16 waves, two or
# three span buffers -- bit-exact through the tiny-frame tests, then A/B on
# the ACK workload.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
for v in c08 c09; do
  ROCE_ICRC_LIB=$PWD/scratch/libs/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py \
    -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05d_$v.log 2>&1
  rc=$?; tail -2 $O/pytest_r05d_$v.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 3 scratch/libs/c05.so \
  scratch/libs/c06.so scratch/libs/c07.so scratch/libs/c08.so scratch/libs/c09.so > $O/ab_r05d.log 2>&1
rc=$?; cat $O/ab_r05d.log; exit $rc
