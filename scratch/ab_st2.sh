set -u
for L in cur obuf nost cur obuf nost; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 2 --reps 40 --lanes 8 2>&1 | grep -v amdgpu.ids | grep -E "lanes" | sed 's/, "GBps_alg.*//' || exit 1
done
