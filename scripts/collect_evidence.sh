# Copy one session's evidence from gpurun_out/ into profiles/ (tracked).
# usage: bash scripts/collect_evidence.sh <tag> <workload> [<workload> ...]
set -eu
TAG=$1; shift
O=gpurun_out; P=profiles
for W in "$@"; do
  T=${TAG}_$W
  cp $O/bench_$T.json $P/${T}_bench.json
  cp $O/prof_$T/run_kernel_stats.csv $P/${T}_kernel_stats.csv
  cp $O/pmcf_$T/run_counter_collection.csv $P/${T}_pmc_fetch_size.csv
  cp $O/pmcw_$T/run_counter_collection.csv $P/${T}_pmc_write_size.csv
  cp $O/prof_summary_$T.txt $P/${T}_prof_summary.txt
  cp $O/pmc_traffic_${T}_$W.json $P/pmc_traffic_$W.json
done
