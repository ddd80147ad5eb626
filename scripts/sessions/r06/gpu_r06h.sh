# Round 6 session h: where the sorted kernel's tail pool spends its time
# (diagnostic build, per-wave stamps and claim counts), cfg3.
set -u
O=gpurun_out
mkdir -p $O
ROCE_ICRC_LIB=$PWD/scratch/libs/pooldiag.so timeout -k 10 300 python scratch/pool_times.py > $O/pool_r06h.log 2>&1
rc=$?; grep -v amdgpu.ids $O/pool_r06h.log; exit $rc
