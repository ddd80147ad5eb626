# Round 4 final evidence, second call: the ACK / seg / cfg4 workloads (bench
# line, rocprof summary, PMC traffic passes), the cross-context stall, the
# multi-device host rates, SQ counters of the ACK and cfg5 kernels and the
# Python-binding latency, on the same library as the first call.
# usage: bash scripts/gpu_r04z2.sh [tag]  (the first call's tag, default r04z)
set -u
T=${1:-r04z}
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
SKIP_TESTS=1 bash scripts/gpu_r04b.sh $T ack seg cfg4 || exit $?
step() {  # step <name> <seconds> <command...>: output in $O/<name>.log
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -6 "$O/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
step svc_$T 300 python scripts/svc_contention.py
step multi_$T 300 python scripts/multi_host_rate.py --ks 1,2,8
step latency_py_$T 300 python scripts/latency.py
step sq_$T 400 bash scripts/gpu_pmc_sq.sh $T ack cfg5
exit 0
