set -u
for L in cur seg_noout cur seg_noout cur seg_noout; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scratch/seg_explore.py --lanes 8 --shift 0 2>&1 | grep -v amdgpu.ids | grep -E "lanes" || exit 1
done
