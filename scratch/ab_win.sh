set -u
ROCE_ICRC_LIB=$PWD/scratch/libs/eqwin.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_faults.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1 || exit 1
for L in pre eqwin pre eqwin pre eqwin; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 3 --reps 30 --lanes 8 2>&1 | grep -v amdgpu.ids | grep -E "lanes" || exit 1
done
