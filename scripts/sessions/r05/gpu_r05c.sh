# Round 5 session c: the full -m gpu suite and smoke on the in-tree library,
# then A/B of cfg3 / ACK / cfg5 against the round-4 library (scratch/libs).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
step() {  # step <name> <seconds> <command...>: output in $O/<name>.log
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -4 "$O/$name.log"
  echo "== $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_r05c 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke_r05c 200 python -c "import __graft_entry__ as g; g.smoke()"
step ab_r05c 900 python scratch/bench_ab.py --workloads ack,cfg3,cfg5 --rounds 3 scratch/libs/base.so scratch/libs/compact12.so scratch/libs/c05.so scratch/libs/c06.so
cat $O/ab_r05c.log
