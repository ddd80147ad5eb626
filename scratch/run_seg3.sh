set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python scratch/seg_explore.py --lanes 8,16 --shift 0,8 --tag plain > $OUT/sx_v3.log 2>&1 || { tail $OUT/sx_v3.log; exit 1; }
ROCE_ICRC_LIB=$R/scratch/libroceicrc_segnt.so timeout -k 10 200 python scratch/seg_explore.py --lanes 8,16 --shift 0,8 --tag nt >> $OUT/sx_v3.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for v in plain nt; do for sh in 0 8; do
 if [ $v = nt ]; then export ROCE_ICRC_LIB=$R/scratch/libroceicrc_segnt.so; else unset ROCE_ICRC_LIB; fi
 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/sx3_pmcf_${v}_$sh -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift $sh > $OUT/sx3_pmcf_${v}_$sh.log 2>&1 || exit 1
done; done
unset ROCE_ICRC_LIB
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/sx3_pmcw_plain_0 -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift 0 > $OUT/sx3_pmcw.log 2>&1 || exit 1
cat $OUT/sx_v3.log | grep "{"
