# Round 4 session r: the small-frame kernel with the two-chain fold -- staging
# (LDS-DMA default vs registers two ahead: dma0) and waves per workgroup (12
# default, 10, 8), cfg5 through bench.py; tests through each variant's small
# kernel first.
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
for v in dma0 w10 w8; do
  step pytest_${v}_r04r 300 env ROCE_ICRC_LIB=$L/$v.so python -u -m pytest tests/test_gpu_small.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
done
step bench_ab_r04r 900 python scratch/bench_ab.py --workloads cfg5 --rounds 3 $L/base.so $L/dma0.so $L/w10.so $L/w8.so
exit 0
