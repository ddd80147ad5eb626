# Round 5 session n: the full -m gpu suite on the tree (small-frame kernel of
# 75294b8), then kernel time against launch size (fixed cost per launch) for
# cfg2 / cfg3 / cfg5 / ack at 1/4, 1/2, 1 and 2 times their packet counts.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r05n.log 2>&1
rc=$?; tail -2 $O/pytest_r05n.log; [ $rc -eq 0 ] || exit $rc
: > $O/sweep_r05n.log
for wl in cfg5 cfg3 ack cfg2; do
  case $wl in cfg5|ack) base=16777216;; *) base=1048576;; esac
  for f in 4 2 1; do
    n=$((base / f))
    timeout -k 10 300 python bench.py --workload $wl --packets $n --no-cpu-baseline --no-e2e > $O/sweep_tmp.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/sweep_tmp.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open('$O/sweep_tmp.log').read().strip().splitlines()[-1]); print('$wl', $n, d['value'], d['kernel_ms_mean'], d['roofline']['frac'])" >> $O/sweep_r05n.log
  done
  n=$((base * 2))
  timeout -k 10 300 python bench.py --workload $wl --packets $n --no-cpu-baseline --no-e2e > $O/sweep_tmp.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $O/sweep_tmp.log; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/sweep_tmp.log').read().strip().splitlines()[-1]); print('$wl', $n, d['value'], d['kernel_ms_mean'], d['roofline']['frac'])" >> $O/sweep_r05n.log
done
cat $O/sweep_r05n.log
