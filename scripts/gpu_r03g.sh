set -u
bash scripts/gpu_tests.sh r03g cfg2 cfg3 cfg5 seg || exit $?
for W in cfg3 cfg2; do for L in packed spaced; do
  timeout -k 10 300 python scripts/fetch_calib.py --workload $W --layout $L --time 40 2>/dev/null | tail -1 || exit 1
done; done
SKIP_TESTS=1 bash scripts/gpu_profile.sh r03g cfg2
