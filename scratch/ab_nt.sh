set -u
for L in ns_ring262144 ns_ring2097152 ns_ring8388608 nostage; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 30 --lanes 0 2>&1 | grep -v amdgpu.ids | grep -E "lanes" || exit 1
done
