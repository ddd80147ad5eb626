# Round 5 session p: bench lines of every workload with the timed launches
# between one pair of HIP events (bench.py of this session), 2 rounds.
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
: > $O/bench_r05p.log
for r in 0 1; do
  for wl in cfg2 cfg3 cfg5 ack seg; do
    timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline --no-e2e > $O/bench_tmp.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { tail -5 $O/bench_tmp.log; exit $rc; }
    python -c "import json; d=json.loads(open('$O/bench_tmp.log').read().strip().splitlines()[-1]); print('r$r', '$wl', d['value'], d['ms_per_step'], d['kernel_ms_mean'], d['roofline']['frac'], [v for k, v in d.items() if k.startswith('stream_')])" >> $O/bench_r05p.log
  done
done
cat $O/bench_r05p.log
