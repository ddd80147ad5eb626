timeout -k 10 900 python -u -m pytest tests/test_gpu_tiny.py tests/test_gpu_service.py tests/test_gpu_recv.py tests/test_gpu_golden.py tests/test_gpu_capi.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_r03d.log 2>&1; rc=$?; tail -25 gpurun_out/t_r03d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/latency.py --reps 300 > gpurun_out/latency_r03d.jsonl 2>&1; rc=$?; cat gpurun_out/latency_r03d.jsonl; [ $rc -eq 0 ] || exit $rc
for L in new tiny0; do echo "== $L"; ROCE_ICRC_LIB=$PWD/scratch/libs/$L.so timeout -k 10 200 python scripts/explore.py --cfg u4,u60 --reps 20 --lanes 0,1 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 500 python scratch/bench_ab.py --workloads cfg3 --rounds 2 scratch/libs/tiny0.so scratch/libs/new.so
