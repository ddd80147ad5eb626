set -u
timeout -k 10 200 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit 1
for L in prev w8 w12 w16 prev w12 w16; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 30 --lanes 0 2>&1 | grep -v amdgpu.ids | grep lanes || exit 1
done
