set -u
for L in cur plain ns plain_ns cur plain; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 5 --reps 30 --lanes 0 2>&1 | grep -v amdgpu.ids | grep -E "lanes" | sed 's/, "GBps_alg.*//' || exit 1
done
