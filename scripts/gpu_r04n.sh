# Round 4 session n: k5 = k4 + contiguous compact batches take their lengths
# from LDS and their offsets from a prefix sum (compute), no second descriptor
# read: tiny / parity tests on the in-tree k5, ragged A/B k4 / k5, the ACK
# bench line and its FETCH_SIZE pass.
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
L=scratch/libs
step pytest_r04n 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step ragged_ab_r04n 500 python scripts/ragged_ab.py --rounds 2 --cases u4,mix,cfg3 $L/k4.so $L/k5.so
step bench_ack_r04n 300 python bench.py --workload ack
exit 0
