# Round 4 session p: the small-frame kernel's fold with two chains over Mul(64)
# (c2) against four over Mul(128) (c4, the same source; k4 = the evidence
# library): parity / golden tests through c2, then cfg5 through bench.py.
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
step pytest_c2_r04p 600 env ROCE_ICRC_LIB=$L/c2.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_ab_r04p 700 python scratch/bench_ab.py --workloads cfg5 --rounds 3 $L/k4.so $L/c4.so $L/c2.so
exit 0
