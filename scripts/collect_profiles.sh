# Copy one workload's gpu_profile.sh summaries from gpurun_out/ into profiles/.
# usage: bash scripts/collect_profiles.sh <session tag, e.g. r04z> <workload>
#   (gpu_r04b.sh ran gpu_profile.sh with the tag <session>_<workload>)
set -eu
TAG=$1
WL=$2
T=${TAG}_$WL
O=gpurun_out
P=profiles
cp $O/bench_$T.json $P/${T}_bench.json
cp $O/prof_$T/run_kernel_stats.csv $P/${T}_kernel_stats.csv
cp $O/prof_summary_$T.txt $P/${T}_prof_summary.txt
cp $O/pmcf_$T/run_counter_collection.csv $P/${T}_pmc_fetch_size.csv
cp $O/pmcw_$T/run_counter_collection.csv $P/${T}_pmc_write_size.csv
cp $O/pmc_traffic_${T}_$WL.json $P/pmc_traffic_$WL.json
ls -la $P/${T}_*
