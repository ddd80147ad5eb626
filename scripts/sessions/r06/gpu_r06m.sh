# Round 6 session m: compact-kernel micro-options (RICRC_ACK_OPT bits: 1 skip
# the zero pad step, 2 unclamped slot writes, 4 16-byte slot reads of aligned
# 48/64-B frames): the tiny-frame tests on o7 (all three), then the ACK A/B.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
ROCE_ICRC_LIB=$PWD/scratch/libs/o7.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py \
  -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r06m.log 2>&1
rc=$?; tail -2 $O/pytest_r06m.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest_r06m.log | head; exit $rc; }
timeout -k 10 900 python scratch/bench_ab.py --workloads ack --rounds 3 scratch/libs/head.so \
  scratch/libs/o1.so scratch/libs/o2.so scratch/libs/o4.so scratch/libs/o7.so > $O/ab_r06m.log 2>&1
rc=$?; cat $O/ab_r06m.log; exit $rc
