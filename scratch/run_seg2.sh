set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
make -C oracle -s || exit 1
timeout -k 10 300 python -m pytest tests/test_gpu_segment.py -q -x -p no:cacheprovider > $OUT/seg2_t.log 2>&1; rc=$?; tail -3 $OUT/seg2_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scratch/seg_explore.py --lanes 4,8,16 --shift 0,8 --tag v2 > $OUT/sx_v2.log 2>&1 || { tail $OUT/sx_v2.log; exit 1; }
timeout -k 10 200 python scratch/seg_explore.py --lanes 2,4,8 --shift 0 --pmtu 1024 --msg 65536 --tag v2p1k >> $OUT/sx_v2.log 2>&1 || exit 1
cat $OUT/sx_v2.log | grep "{"
