set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python scratch/seg_explore.py --lanes 8,16 --shift 0 --tag clamp > $OUT/sx_v5.log 2>&1 || { tail $OUT/sx_v5.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/sx5_pmcf -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift 0 > $OUT/sx5_pmcf.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/sx5_pmcw -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift 0 > $OUT/sx5_pmcw.log 2>&1 || exit 1
cat $OUT/sx_v5.log | grep "{"
