# Copy one gpu_profile.sh session's summaries from gpurun_out/ into profiles/.
# usage: bash scripts/collect_profiles.sh <tag, e.g. r02a> <workload>
set -eu
TAG=$1
WL=$2
O=gpurun_out
P=profiles
cp $O/bench_$TAG.json $P/${TAG}_${WL}_bench.json
cp $O/prof_$TAG/run_kernel_stats.csv $P/${TAG}_${WL}_kernel_stats.csv
cp $O/prof_summary_$TAG.txt $P/${TAG}_${WL}_prof_summary.txt
cp $O/pmcf_$TAG/run_counter_collection.csv $P/${TAG}_${WL}_pmc_fetch_size.csv
cp $O/pmcw_$TAG/run_counter_collection.csv $P/${TAG}_${WL}_pmc_write_size.csv
cp $O/pmc_traffic_${TAG}_$WL.json $P/pmc_traffic_$WL.json
if [ -f $O/pytest_$TAG.log ]; then tail -3 $O/pytest_$TAG.log > $P/${TAG}_gpu_pytest_tail.txt; fi
ls -la $P/${TAG}_*
