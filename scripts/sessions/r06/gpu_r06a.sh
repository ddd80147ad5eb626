# Round 6 session a: the -m gpu suite (new: IPv4-options API, cfg4 at its
# stated size in one process, the compact kernel's second chunk), smoke, the
# speed ratios moved out of the suite, then an A/B of the small-frame
# kernel's LDS-DMA table staging (tree) against round 5's library (cfg5, ack).
set -u
O=gpurun_out
mkdir -p $O
make -C oracle -s || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_r06a.log 2>&1
rc=$?; tail -3 $O/pytest_r06a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r06a.log 2>&1
rc=$?; tail -1 $O/smoke_r06a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/perf_ratios.py --out $O/perf_ratios_r06a.json > $O/perf_ratios_r06a.log 2>&1
rc=$?; tail -c 600 $O/perf_ratios_r06a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scratch/bench_ab.py --workloads cfg5,ack --rounds 3 scratch/libs/r05.so \
  roce-sim_amd/roce_icrc/libroceicrc.so > $O/ab_r06a.log 2>&1
rc=$?; cat $O/ab_r06a.log; exit $rc
