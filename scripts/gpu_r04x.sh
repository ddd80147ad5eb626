# Round 4 session x: ACK frames through bench.py with the whole library built
# without wave-priority raises (prio0) and with non-temporal (nt) or sc1 stores
# of the per-packet words, against the final library (base).
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
L=$PWD/scratch/libs
step bench_ab_r04x 900 python scratch/bench_ab.py --workloads ack,cfg3 --rounds 3 $L/base.so $L/prio0.so $L/nt.so $L/sc1.so
exit 0
