# Round 4 session d: the -m gpu suite + smoke on the in-tree library (service
# relaunch held back while batches run, ACK-sized inline frames folded by the
# per-lane multiplies, phase 0 one ahead, LDS-DMA small staging), the
# cross-context stall, the service latency, then phase-0 diagnostics on the
# ACK frames (dc1: phase 0 skipped, dc2: no fold, dc3: no stores).
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
step pytest_r04d 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke_r04d 200 python -c "import __graft_entry__ as g; g.smoke()"
step svc_r04d 300 python scripts/svc_contention.py
gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lroce-sim_amd/roce_icrc -l:libroceicrc.so \
  -Wl,-rpath,$PWD/roce-sim_amd/roce_icrc -o $O/latency_c || exit 1
step latency_c_r04d 300 ./$O/latency_c
step latency_py_r04d 300 python scripts/latency.py
step bench_ack_r04d 300 python bench.py --workload ack
step ragged_ab_r04d 700 python scripts/ragged_ab.py --rounds 2 --cases u4,mix scratch/libs/base4.so scratch/libs/dc1.so scratch/libs/dc2.so scratch/libs/dc3.so
exit 0
