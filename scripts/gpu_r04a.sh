# Round 4 session a: tests + smoke + bench lines, the cross-context stall,
# the 2-rank bench launch, and the multi-device host path rate.
bash scripts/gpu_tests.sh r04a cfg2 cfg5 || exit $?
timeout -k 10 300 python scripts/svc_contention.py > gpurun_out/svc_r04a.json 2> gpurun_out/svc_r04a.err
rc=$?; cat gpurun_out/svc_r04a.json; echo "svc rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/svc_r04a.err; exit $rc; }
ROCE_ICRC_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --packets 40000 > gpurun_out/bench2_r04a.json 2> gpurun_out/bench2_r04a.err
rc=$?; cat gpurun_out/bench2_r04a.json; echo "bench2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench2_r04a.err; exit $rc; }
timeout -k 10 300 python scripts/multi_host_rate.py > gpurun_out/multi_r04a.jsonl 2> gpurun_out/multi_r04a.err
rc=$?; cat gpurun_out/multi_r04a.jsonl; echo "multi rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/multi_r04a.err; exit $rc; }
