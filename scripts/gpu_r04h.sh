# Round 4 session h: cfg3 through bench.py (r03: round-3 library, m5:
# committed, nc: m5 without the compact test, to see what the test costs on
# windows without tiny frames); ACK frames with the phase-0 chain rotation
# (m6, in-tree) against m5; the tiny / parity tests and the ACK bench line on m6.
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
step pytest_r04h 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step ragged_ab_r04h 500 python scripts/ragged_ab.py --rounds 2 --cases u4,mix scratch/libs/m5.so scratch/libs/m6.so
step bench_ab_r04h 700 python scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/r03.so scratch/libs/m5.so scratch/libs/nc.so
step bench_ack_r04h 300 python bench.py --workload ack
exit 0
