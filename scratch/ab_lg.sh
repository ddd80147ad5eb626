set -u
for L in lg_t1024u4 lg_t512u8 lg_t768u6 lg_t1024u4 lg_t512u8 lg_t768u6; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg 2,3 --reps 15 --lanes 8 2>&1 | grep -v amdgpu.ids | grep -E "lanes" | sed 's/, "GBps_alg.*//' || exit 1
done
