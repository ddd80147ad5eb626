set -u
for L in seg_line_t512 seg_line_t512u6 seg_line_t512u5 seg_line_t512 seg_line_t512u6 seg_line_t512u5; do
  echo "== $L"
  ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scratch/seg_explore.py --lanes 8 --shift 0 2>&1 | grep -v amdgpu.ids | grep -E "lanes|copy" || exit 1
done
