set -u
make -C oracle -s
for wl in cfg2 cfg3; do
  timeout -k 10 300 python bench.py --workload $wl --steps 50 --warmup 20 2>gpurun_out/bench_$wl.err | tee gpurun_out/bench_$wl.json || { tail gpurun_out/bench_$wl.err; exit 1; }
done
timeout -k 10 300 python bench.py --workload cfg5 --steps 50 --warmup 20 --no-cpu-baseline 2>gpurun_out/bench_cfg5.err | tee gpurun_out/bench_cfg5.json || { tail gpurun_out/bench_cfg5.err; exit 1; }
ROCE_ICRC_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 30 --warmup 10 2>gpurun_out/bench_n2.err | tee gpurun_out/bench_n2.json || { tail gpurun_out/bench_n2.err; exit 1; }
