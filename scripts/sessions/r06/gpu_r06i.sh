# Round 6 session i: are the sorted kernel's slow workgroups the same from
# launch to launch?  Per-block window durations of 5 cfg3 launches (phase
# diagnostic build over the pre-pool source), their correlation and the
# per-XCD (block mod 8) means.
set -u
O=gpurun_out
mkdir -p $O
ROCE_ICRC_LIB=$PWD/scratch/libs/phase.so timeout -k 10 300 python scratch/phase_times.py > $O/phase_r06i.log 2>&1
rc=$?; grep -v amdgpu.ids $O/phase_r06i.log | tail -2; exit $rc
