# Round 4 session a: tests + smoke + bench lines, the cross-context stall,
# the 2-rank bench launch, and the multi-device host path rate.
bash scripts/gpu_tests.sh r04a cfg2 cfg5 || exit $?
timeout -k 10 300 python scripts/svc_contention.py > gpurun_out/svc_r04a.json 2> gpurun_out/svc_r04a.err
rc=$?; cat gpurun_out/svc_r04a.json; echo "svc rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/svc_r04a.err; exit $rc; }
ROCE_ICRC_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --packets 40000 > gpurun_out/bench2_r04a.json 2> gpurun_out/bench2_r04a.err
rc=$?; cat gpurun_out/bench2_r04a.json; echo "bench2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench2_r04a.err; exit $rc; }
timeout -k 10 300 python scripts/multi_host_rate.py > gpurun_out/multi_r04a.jsonl 2> gpurun_out/multi_r04a.err
rc=$?; cat gpurun_out/multi_r04a.jsonl; echo "multi rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/multi_r04a.err; exit $rc; }
timeout -k 10 600 python scripts/ragged_ab.py --rounds 2 scratch/libs/base.so scratch/libs/compact.so > gpurun_out/ragged_ab_r04a.jsonl 2> gpurun_out/ragged_ab_r04a.err
rc=$?; cat gpurun_out/ragged_ab_r04a.jsonl; echo "ragged_ab rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/ragged_ab_r04a.err; exit $rc; }
timeout -k 10 120 ./scratch/small_stage > gpurun_out/small_stage_r04a.jsonl 2>&1
rc=$?; cat gpurun_out/small_stage_r04a.jsonl; echo "small_stage rc=$rc"
gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lroce-sim_amd/roce_icrc -l:libroceicrc.so -Wl,-rpath,$PWD/roce-sim_amd/roce_icrc -o gpurun_out/latency_c && \
timeout -k 10 300 ./gpurun_out/latency_c > gpurun_out/latency_c_r04a.jsonl 2>&1
rc=$?; cat gpurun_out/latency_c_r04a.jsonl; echo "latency_c rc=$rc"
