# FETCH_SIZE calibration passes on each workload's own access pattern
# (scripts/fetch_calib.py): packed and spaced layouts, one rocprofv3 pass each.
# usage: bash scripts/gpu_calib.sh <tag> [workloads...]
set -u
TAG=${1:-r03}
shift || true
WLS=${*:-cfg3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/calib_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for WL in $WLS; do
  for LAY in packed spaced; do
    timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${WL}_$LAY -o run -- \
      python3 $R/scripts/fetch_calib.py --workload $WL --layout $LAY > $OUT/${WL}_$LAY.json 2> $OUT/${WL}_$LAY.err
    rc=$?; tail -1 $OUT/${WL}_$LAY.json; echo "$WL $LAY rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/${WL}_$LAY.err; exit $rc; }
  done
done
exit 0
