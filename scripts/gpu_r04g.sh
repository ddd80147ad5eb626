# Round 4 session g: is cfg3 slower than round 3 through bench.py (r03: the
# round-3 library, m4: committed, m5: m4 + phase-0 stores specialised on the
# outputs present); ragged A/B of m4 / m5 on the ACK frames; SQ counters of
# the ACK and cfg5 kernels; tiny / parity / service tests on the in-tree m5.
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
step pytest_r04g 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_tiny.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_ab_r04g 700 python scratch/bench_ab.py --workloads cfg3 --rounds 3 scratch/libs/r03.so scratch/libs/m4.so scratch/libs/m5.so
step ragged_ab_r04g 500 python scripts/ragged_ab.py --rounds 2 --cases u4,mix scratch/libs/m4.so scratch/libs/m5.so
step sq_r04g 400 bash scripts/gpu_pmc_sq.sh r04g ack cfg5
exit 0
