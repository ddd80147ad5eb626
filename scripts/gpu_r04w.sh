# Round 4 session w: the next window's descriptor lines touched into L2 during
# phase 0 (touch) against the final library (base): tiny / parity tests through touch, ragged A/B,
# the ACK workload through bench.py.
set -u
O=gpurun_out
mkdir -p $O
step() {  # step <name> <seconds> <command...>: output in $O/<name>.log
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -25 "$O/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
make -C oracle -s || exit 1
L=$PWD/scratch/libs
step pytest_touch_r04w 600 env ROCE_ICRC_LIB=$L/touch.so python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step ragged_ab_r04w 500 python scripts/ragged_ab.py --rounds 2 --cases u4,mix $L/base.so $L/touch.so
step bench_ab_r04w 600 python scratch/bench_ab.py --workloads ack --rounds 3 $L/base.so $L/touch.so
exit 0
