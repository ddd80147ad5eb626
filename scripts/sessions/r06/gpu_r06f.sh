# Round 6 session f: per-wave phase clocks of the sorted ragged kernel on cfg3
# (diagnostic library, scratch/attic/sorted_phase_times_r06.diff).
set -u
O=gpurun_out
mkdir -p $O
ROCE_ICRC_LIB=$PWD/scratch/libs/phase.so timeout -k 10 300 python scratch/phase_times.py > $O/phase_r06f.log 2>&1
rc=$?; cat $O/phase_r06f.log | grep -v amdgpu.ids; exit $rc
