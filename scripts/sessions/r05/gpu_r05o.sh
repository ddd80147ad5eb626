# Round 5 session o: the small-frame kernel's last batch folded from registers
# loaded in one round trip (lastg = the tree) against 75294b8 (h08): small-frame
# and parity tests, cfg5 A/B, and kernel time against launch size (down to a
# few packets per CU: the fixed cost of a launch).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_parity.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_r05o.log 2>&1
rc=$?; tail -1 $O/pytest_r05o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads cfg5 --rounds 4 scratch/libs/h08.so \
  scratch/libs/lastg.so > $O/ab_r05o.log 2>&1
rc=$?; cat $O/ab_r05o.log; [ $rc -eq 0 ] || exit $rc
: > $O/sweep_r05o.log
for wn in cfg5:65536 cfg5:1048576 cfg5:4194304 cfg5:8388608 cfg5:16777216 cfg2:4096 cfg2:65536 cfg3:16384 \
          cfg3:65536 ack:65536 ack:1048576; do
  wl=${wn%%:*}; n=${wn##*:}
  timeout -k 10 300 python bench.py --workload $wl --packets $n --no-cpu-baseline --no-e2e > $O/sweep_tmp.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 $O/sweep_tmp.log; exit $rc; }
  python -c "import json,sys; d=json.loads(open('$O/sweep_tmp.log').read().strip().splitlines()[-1]); print('$wl', $n, d['value'], d['kernel_ms_mean'], d['roofline']['frac'])" >> $O/sweep_r05o.log
done
cat $O/sweep_r05o.log
