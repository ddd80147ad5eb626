# Round 6: copy-only replica of the segmentation pattern, loads in flight per
# lane x waves per CU (scratch/seg_copy.hip).
set -u
O=gpurun_out
mkdir -p $O
timeout -k 10 300 ./scratch/seg_copy_bin > $O/seg_copy_r06c.jsonl 2>&1
rc=$?; cat $O/seg_copy_r06c.jsonl; exit $rc
