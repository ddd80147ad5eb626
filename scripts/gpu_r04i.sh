# Round 4 session i: which commit since round 3 slowed cfg3 (bench.py, the
# round-3 library and builds of the kernel-touching commits, oldest first,
# m5 = 164cc9d); then the ACK frames: m5 against the phase-0 variants
# (m7: chain rotation + replicated Mul(-32), m8: replicated Mul(-32),
# m9: two batches ahead, m10: two ahead + replicated Mul(-32)).
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
step bench_ab_r04i 600 python scratch/bench_ab.py --workloads cfg3 --rounds 2 $L/r03.so $L/b_bf9b9b0.so $L/b_1921259.so $L/b_3297227.so $L/b_fb7db8e.so $L/b_82333e6.so $L/m5.so
step ragged_ab_r04i 550 python scripts/ragged_ab.py --rounds 2 --cases u4,mix $L/m5.so $L/m7.so $L/m8.so $L/m9.so $L/m10.so
exit 0
