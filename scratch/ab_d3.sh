set -u
ROCE_ICRC_LIB=$PWD/scratch/libs/d3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_small.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1 || exit 1
for L in d2 d3 d3_nofold d2 d3; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 30 --lanes 0 2>&1 | grep -v amdgpu.ids | grep -E "lanes" || exit 1
done
