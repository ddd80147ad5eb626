set -u
timeout -k 10 200 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3 || exit 1
for L in scratch/libs/base.so roce-sim_amd/roce_icrc/libroceicrc.so scratch/libs/base.so roce-sim_amd/roce_icrc/libroceicrc.so; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/$L timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 9 --lanes 0 2>&1 | grep -v amdgpu.ids | grep lanes || exit 1
done
