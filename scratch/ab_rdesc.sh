set -u

for L in pre rdesc pre rdesc pre rdesc; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 3 --reps 40 --lanes 8 2>&1 | grep -v amdgpu.ids | grep -E "lanes" || exit 1
done
