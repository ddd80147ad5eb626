# Round 4 session c: the -m gpu suite + smoke on the in-tree library (global
# frame loads again, phase 0 two batches ahead, service leaves for batches),
# then A/B: ragged tiny frames and cfg3 (round 3 / phase 0 one / two ahead),
# cfg5 register vs LDS-DMA staging, the cross-context stall, the service
# latency, the multi-device host rate and the request-slot ping-pong.
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
step pytest_r04c 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke_r04c 200 python -c "import __graft_entry__ as g; g.smoke()"
step ragged_ab_r04c 700 python scripts/ragged_ab.py --rounds 2 --cases u4,mix,cfg3 scratch/libs/base.so scratch/libs/ca1.so scratch/libs/ca2.so
step cfg5_ab_r04c 600 python scratch/bench_ab.py --workloads cfg5 --rounds 3 scratch/libs/ca2.so scratch/libs/small_dma.so
step svc_r04c 300 python scripts/svc_contention.py
gcc -std=c99 -O2 -Iinclude scripts/latency_c.c -Lroce-sim_amd/roce_icrc -l:libroceicrc.so \
  -Wl,-rpath,$PWD/roce-sim_amd/roce_icrc -o $O/latency_c || exit 1
step latency_c_r04c 300 ./$O/latency_c
step latency_py_r04c 300 python scripts/latency.py
step multi_r04c 300 python scripts/multi_host_rate.py --ks 1,2,8
step bench_ack_r04c 300 python bench.py --workload ack
# last: a probe that writes device memory from the host (a segfault ends the call)
step pingpong_r04c 120 ./scratch/pingpong
exit 0
