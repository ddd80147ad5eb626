# Round 6 session t: per-workgroup clocks of the compact (ACK) kernel.
set -u
O=gpurun_out
mkdir -p $O
ROCE_ICRC_LIB=$PWD/scratch/libs/ackt.so timeout -k 10 300 python scratch/ack_times.py > $O/ack_times_r06t.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ack_times_r06t.log; exit $rc
