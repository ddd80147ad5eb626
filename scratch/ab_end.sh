set -u
for L in ns_nostore ns_end4 ns_end ns_end4 ns_end ns_end4 ns; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 30 --lanes 0 2>&1 | grep -v amdgpu.ids | grep -E "lanes" | sed 's/, "GiBps_best.*//' || exit 1
done
