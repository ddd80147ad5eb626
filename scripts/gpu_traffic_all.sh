# GPU session: bench line, rocprofv3 kernel-trace summary and the two PMC
# traffic passes for every workload, on the library as built (its sha256 is
# recorded in each pmc_traffic json).  usage: bash scripts/gpu_traffic_all.sh <tag> [workloads...]
set -u
TAG=${1:-r03}
shift || true
WLS=${*:-cfg2 cfg3 cfg5 seg cfg4}
for WL in $WLS; do
  echo "==== $WL"
  SKIP_TESTS=1 bash scripts/gpu_profile.sh ${TAG}_$WL $WL || exit $?
done
exit 0
