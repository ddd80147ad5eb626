set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python scratch/seg_explore.py --lanes 4,8,16 --shift 0,8 --tag base > $OUT/sx_base.log 2>&1 || { tail $OUT/sx_base.log; exit 1; }
ROCE_ICRC_LIB=$R/scratch/libroceicrc_ablate.so timeout -k 10 200 python scratch/seg_explore.py --lanes 8,16 --shift 0,8 --tag ablate > $OUT/sx_abl.log 2>&1 || { tail $OUT/sx_abl.log; exit 1; }
timeout -k 10 200 python scratch/seg_explore.py --lanes 2,4,8 --shift 0 --pmtu 1024 --msg 65536 --tag p1024 > $OUT/sx_p1k.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/sx_pmcf -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift 0 > $OUT/sx_pmcf.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/sx_pmcw -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift 0 > $OUT/sx_pmcw.log 2>&1 || exit 1
cat $OUT/sx_base.log $OUT/sx_abl.log $OUT/sx_p1k.log | grep "{"
