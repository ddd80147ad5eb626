set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; cd /tmp && export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmcsq_cfg2 -o run -- python3 $R/bench.py --workload cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmcsq_cfg2.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmcsq_cfg5 -o run -- python3 $R/bench.py --workload cfg5 --packets 4194304 --lanes 2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmcsq_cfg5.log 2>&1 || exit 1
C2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --pmc $C2 --output-format csv -d $OUT/pmcsq2_cfg2 -o run -- python3 $R/bench.py --workload cfg2 --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/pmcsq2_cfg2.log 2>&1 || exit 1
echo done
