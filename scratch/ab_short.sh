set -u
for L in short6 short4; do
ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_faults.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit 1
done
for L in base short0 short4 short6 base short6; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 3,u256,u512 --reps 9 --lanes 8 2>&1 | grep -v amdgpu.ids | grep lanes || exit 1
done
