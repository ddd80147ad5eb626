# One GPU session (round 5 on): the -m gpu suite and smoke(), then per workload
# the evidence set of scripts/gpu_profile.sh (bench line, rocprofv3 kernel-trace
# summary, PMC FETCH/WRITE passes bound to this build's sha256).
# usage: bash scripts/gpu_session.sh <tag> [workloads...]
#   SKIP_TESTS=1  workloads only          TESTS="<pytest args>"  a subset of the suite
#   QUICK=1       bench line + rocprof kernel trace only (no PMC passes)
set -u
TAG=${1:-r05}
shift || true
WLS=${*:-}
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
step() {  # step <name> <seconds> <command...>: output in $O/<name>.log, stop on failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -4 "$O/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_$TAG 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider
  step smoke_$TAG 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
for WL in $WLS; do
  echo "==== $WL"
  if [ -n "${QUICK:-}" ]; then
    step bench_${TAG}_$WL 300 python bench.py --workload $WL
    cat $O/bench_${TAG}_$WL.log | grep '^{' > $O/bench_${TAG}_$WL.json
    R=$PWD
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $R/$O/prof_${TAG}_$WL -o run -- python3 $R/bench.py --workload $WL \
      --no-cpu-baseline --no-e2e > $R/$O/prof_${TAG}_$WL.log 2>&1) || exit $?
    python3 scripts/prof_summary.py $O/prof_${TAG}_$WL $O/bench_${TAG}_$WL.json "::icrc_" \
      > $O/prof_summary_${TAG}_$WL.txt || exit 1
    cat $O/prof_summary_${TAG}_$WL.txt
  else
    SKIP_TESTS=1 bash scripts/gpu_profile.sh ${TAG}_$WL $WL || exit $?
  fi
done
exit 0
