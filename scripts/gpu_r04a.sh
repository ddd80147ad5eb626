# Round 4 session a: the -m gpu suite + smoke on the in-tree library (phase-0
# compact tiny batches, inline service requests, pinned multi split), then
# A/B and latency measurements, the cross-context stall, the 2-rank bench
# launch, the multi-device host path rate and the default bench lines.
# Every GPU step has its own time limit; the session stops at the first
# failing step.
set -u
O=gpurun_out
mkdir -p $O
step() {  # step <name> <seconds> <command...>: output in $O/<name>.log
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -25 "$O/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
make -C oracle -s || exit 1
step pytest_r04a 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke_r04a 200 python -c "import __graft_entry__ as g; g.smoke()"
step ragged_ab_r04a 700 python scripts/ragged_ab.py --rounds 2 --cases u4,mix,cfg3 scratch/libs/base.so scratch/libs/compact_fast.so scratch/libs/compact_agg.so
gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lroce-sim_amd/roce_icrc -l:libroceicrc.so \
  -Wl,-rpath,$PWD/roce-sim_amd/roce_icrc -o $O/latency_c || exit 1
step latency_c_r04a 300 ./$O/latency_c
gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lscratch/libs/polls4 -l:libroceicrc.so \
  -Wl,-rpath,$PWD/scratch/libs/polls4 -o $O/latency_c_polls4 || exit 1
step latency_c_polls4_r04a 300 ./$O/latency_c_polls4
step small_stage_r04a 120 ./scratch/small_stage
step cfg5_ab_r04a 600 python scratch/bench_ab.py --workloads cfg5 --rounds 2 scratch/libs/base.so scratch/libs/small_dma.so scratch/libs/comb8.so scratch/libs/comb8w10.so
step svc_r04a 300 python scripts/svc_contention.py
step bench2_r04a 300 env ROCE_ICRC_BENCH_DEVICE=0 python bench.py --gpus 2 --packets 40000
step multi_r04a 300 python scripts/multi_host_rate.py
step bench_cfg2_r04a 300 python bench.py --workload cfg2
step bench_cfg5_r04a 300 python bench.py --workload cfg5
# last: a probe that writes device memory from the host (a segfault ends the call)
step pingpong_r04a 120 ./scratch/pingpong
exit 0
