# Round 4 session e: the phase-0 loop without the spilled slot register (its
# scratch reload waited for the next batch's loads too) -- the ragged A/B (base4: before the
# fix, m1: fixed, one batch ahead, m2: fixed, two ahead, m3: m1 with the wave
# index scalar, fewer spills, m4: m3 + the next window's descriptors loaded
# during a compact-only window's phase 0, compute), then the service / tiny /
# parity tests on the in-tree library (m4) and the ACK bench line.
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
step ragged_ab_r04e 800 python scripts/ragged_ab.py --rounds 2 --cases u4,mix,cfg3 scratch/libs/base4.so scratch/libs/m1.so scratch/libs/m2.so scratch/libs/m3.so scratch/libs/m4.so
step pytest_r04e 600 python -u -m pytest tests/test_gpu_service.py tests/test_gpu_tiny.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_ack_r04e 300 python bench.py --workload ack
exit 0
