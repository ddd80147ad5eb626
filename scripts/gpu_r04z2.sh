# Round 4 final evidence, second call: the ACK / seg / cfg4 workloads (bench
# line, rocprof summary, PMC traffic passes), the cross-context stall, the
# multi-device host rates, SQ counters of the ACK and cfg5 kernels and the
# Python-binding latency, on the same library as the first call.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
SKIP_TESTS=1 bash scripts/gpu_r04b.sh r04z ack seg cfg4 || exit $?
step() {  # step <name> <seconds> <command...>: output in $O/<name>.log
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -6 "$O/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
step svc_r04z 300 python scripts/svc_contention.py
step multi_r04z 300 python scripts/multi_host_rate.py --ks 1,2,8
step latency_py_r04z 300 python scripts/latency.py
step sq_r04z 400 bash scripts/gpu_pmc_sq.sh r04z ack cfg5
exit 0
