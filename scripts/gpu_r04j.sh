# Round 4 session j: the ragged kernel with two window loops (phase 0 only
# where the workgroup's first packets hold a tiny frame; tl, in-tree) against
# the round-3 library and m5 on cfg3 (bench.py), and against m5 on the ACK
# frames; the tiny / parity / golden tests on the in-tree tl.
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
step pytest_r04j 600 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_ab_r04j 600 python scratch/bench_ab.py --workloads cfg3 --rounds 3 $L/r03.so $L/m5.so $L/tl.so
step ragged_ab_r04j 500 python scripts/ragged_ab.py --rounds 2 --cases u4,mix,cfg3 $L/m5.so $L/tl.so
exit 0
