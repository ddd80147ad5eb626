set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_faults.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1 || exit 1
for L in pretrl trl pretrl trl pretrl trl; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 3 --reps 15 --lanes 8 2>&1 | grep -v amdgpu.ids | grep -E "verify" || exit 1
done
