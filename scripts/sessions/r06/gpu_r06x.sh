# Round 6 evidence session (library 6f21f47a): per workload the bench line,
# the rocprofv3 kernel-trace summary and the PMC FETCH/WRITE passes bound to
# this build's sha256 (scripts/gpu_profile.sh), then the driver's own bench
# command and the speed ratios kept out of the test suite.
set -u
O=gpurun_out
SKIP_TESTS=1 bash scripts/gpu_session.sh r06x cfg2 cfg3 cfg5 ack seg cfg4 || exit $?
timeout -k 10 300 python bench.py > $O/driver_cmd_r06x.json 2> $O/driver_cmd_r06x.err
rc=$?; cat $O/driver_cmd_r06x.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/perf_ratios.py --out $O/perf_ratios_r06x.json > $O/perf_ratios_r06x.log 2>&1
rc=$?; tail -c 300 $O/perf_ratios_r06x.log; exit $rc
