set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD"
C2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
for L in base short4; do
for P in 1 2; do
  eval C=\$C$P
  ROCE_ICRC_LIB=$R/scratch/libs/$L.so timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/u256_${L}_$P -o run -- python3 $R/scripts/explore.py --cfg u256 --reps 2 --lanes 8 > $OUT/u256_${L}_$P.log 2>&1 || { tail -5 $OUT/u256_${L}_$P.log; exit 1; }
done
echo "=== $L"
python3 $R/scripts/pmc_sq.py $OUT/u256_${L}_1 $OUT/u256_${L}_2 | grep -v "^  SQ_[A-Z_]* *[0-9.]*$" 
done
