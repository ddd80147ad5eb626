set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 200 python scratch/seg_explore.py --lanes 8,16 --shift 0,40,104 --tag plain > $OUT/sx_v4.log 2>&1 || { tail $OUT/sx_v4.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for sh in 40; do
 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/sx4_pmcf_$sh -o run -- python3 $R/scratch/seg_explore.py --lanes 8 --shift $sh > $OUT/sx4_pmcf_$sh.log 2>&1 || exit 1
done
cat $OUT/sx_v4.log | grep "{"
