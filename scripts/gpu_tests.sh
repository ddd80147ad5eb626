# GPU session: host probe, the -m gpu suite, smoke, then bench lines.
# usage: bash scripts/gpu_tests.sh <tag> [workloads...]   (from the repo root on the box)
set -u
TAG=${1:-r03}
shift || true
WLS=${*:-cfg2}
OUT=gpurun_out
mkdir -p $OUT
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  echo "cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}";
  rocm-smi --showuse --showmemuse 2>/dev/null | head -20; } > $OUT/host_$TAG.txt 2>&1
make -C oracle -s || exit 1
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread \
    -p no:cacheprovider > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -15 $OUT/pytest_$TAG.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
  rc=$?; tail -2 $OUT/smoke_$TAG.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for WL in $WLS; do
  timeout -k 10 400 python bench.py --workload $WL > $OUT/bench_${TAG}_$WL.json 2> $OUT/bench_${TAG}_$WL.err
  rc=$?; cat $OUT/bench_${TAG}_$WL.json; echo "bench $WL rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_${TAG}_$WL.err; exit $rc; }
done
exit 0
