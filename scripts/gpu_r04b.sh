# Round 4 session b: the evidence for the final library -- the -m gpu suite and
# smoke, then for every workload a bench line, the rocprofv3 kernel-trace
# summary and the two PMC traffic passes (bound to this build's sha256), and
# the per-call latency from C.  usage: bash scripts/gpu_r04b.sh <tag> [workloads...]
# (SKIP_TESTS=1: the workloads only, for a second call of the same session)
set -u
TAG=${1:-r04b}
shift || true
WLS=${*:-cfg2 cfg3 cfg5 ack seg cfg4}
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_$TAG.log 2>&1
rc=$?; tail -4 $O/pytest_$TAG.log; echo "== pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1
rc=$?; tail -2 $O/smoke_$TAG.log; echo "== smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lroce-sim_amd/roce_icrc -l:libroceicrc.so \
  -Wl,-rpath,$PWD/roce-sim_amd/roce_icrc -o $O/latency_c || exit 1
timeout -k 10 300 ./$O/latency_c > $O/latency_c_$TAG.jsonl 2>&1
rc=$?; cat $O/latency_c_$TAG.jsonl; echo "== latency_c rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for WL in $WLS; do
  echo "==== $WL"
  SKIP_TESTS=1 bash scripts/gpu_profile.sh ${TAG}_$WL $WL || exit $?
done
exit 0
