set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python bench.py --workload cfg5 > $OUT/bench_cfg5_s3.json 2> $OUT/bench_cfg5_s3.err || { tail -5 $OUT/bench_cfg5_s3.err; exit 1; }
cat $OUT/bench_cfg5_s3.json
ROCE_ICRC_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --packets 262144 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_n2_s3.json 2> $OUT/bench_n2_s3.err || { tail -5 $OUT/bench_n2_s3.err; exit 1; }
cat $OUT/bench_n2_s3.json
bash scripts/gpu_pmc_sq.sh s3 cfg5
