# SQ counter passes (two per workload) of bench.py, summarised by scripts/pmc_sq.py.
# usage: bash scripts/gpu_pmc_sq.sh <tag> <workload> [<workload> ...]
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"
C2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
for WL in "$@"; do
  for P in 1 2; do
    eval C=\$C$P
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/sq${P}_${TAG}_$WL -o run -- python3 $R/bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/sq${P}_${TAG}_$WL.log 2>&1 || { tail -5 $OUT/sq${P}_${TAG}_$WL.log; exit 1; }
  done
  python3 $R/scripts/pmc_sq.py $OUT/sq1_${TAG}_$WL $OUT/sq2_${TAG}_$WL > $OUT/sq_${TAG}_$WL.txt || exit 1
  cat $OUT/sq_${TAG}_$WL.txt
done
