# Round 6 session u: SQ counters (two passes each) of the final library on
# the ACK, cfg5 and cfg3 kernels.
set -u
bash scripts/gpu_pmc_sq.sh r06x ack cfg5 cfg3
