# Round 4 session q: the small-frame fold with one chain over Mul(32) (c1)
# against two over Mul(64) (c2): parity / golden / small-kernel tests through
# c1 and c2, then cfg5 through bench.py.
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
step pytest_c1_r04q 600 env ROCE_ICRC_LIB=$L/c1.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_small.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step pytest_c2_r04q 600 env ROCE_ICRC_LIB=$L/c2.so python -u -m pytest tests/test_gpu_small.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step bench_ab_r04q 700 python scratch/bench_ab.py --workloads cfg5 --rounds 3 $L/c2.so $L/c1.so
exit 0
