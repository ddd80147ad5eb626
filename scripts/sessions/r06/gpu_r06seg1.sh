# Round 6: segmentation access pattern, lanes per packet 8 / 16 / 32 / 64
# (64 / G packets per wave in flight), variant library with G = 32, 64.
set -u
O=gpurun_out
mkdir -p $O
ROCE_ICRC_LIB=scratch/libs/seg64.so timeout -k 10 300 python -u scratch/seg_lanes_ab.py --tag seg64 > $O/seg_lanes_r06a.txt 2>&1
rc=$?; cat $O/seg_lanes_r06a.txt; exit $rc
