# Round 4 session l: two ragged kernels chosen per context from the hint word,
# now one store per launch from the first workgroup (k3, in-tree; k2 stored
# once per wave: ACK 2.9x slower): the -m gpu suite and smoke; cfg3 through
# bench.py (r03, m5 = one kernel, k3); ragged A/B m5 / k3; the ACK bench line.
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
L=scratch/libs
step pytest_r04l 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke_r04l 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_ab_r04l 600 python scratch/bench_ab.py --workloads cfg3 --rounds 3 $L/r03.so $L/m5.so $L/k3.so
step ragged_ab_r04l 500 python scripts/ragged_ab.py --rounds 2 --cases u4,mix,cfg3 $L/m5.so $L/k3.so
step bench_ack_r04l 300 python bench.py --workload ack
exit 0
