#!/bin/bash
# Copy the judged summaries of a tools/gpu_profile_all.sh run from gpurun_out/ into profiles/r01/.
# usage: bash tools/collect_profiles.sh <tag>
TAG=$1
G=gpurun_out
P=profiles/r01
set -e
cp $G/${TAG}_bench.json $P/bench_diff_N40_B4096.json
cp $G/${TAG}_prof/run_kernel_stats.csv $P/bench_diff_N40_B4096_kernel_stats.csv
for c in diff1024 omni4 tric mixed; do cp $G/${TAG}_bench_$c.json $P/configs/bench_$c.json; done
cp $G/${TAG}_path_4096.json $P/path_discretize_B4096.json
cp $G/${TAG}_path_65536.json $P/path_discretize_B65536.json
cp $G/${TAG}_pathprof/run_kernel_stats.csv $P/path_discretize_B4096_kernel_stats.csv
for i in 1 2 3; do cp $(ls $G/${TAG}_pmc$i/*/*counter_collection.csv $G/${TAG}_pmc$i/*counter_collection.csv 2>/dev/null | head -1) $P/pmc/pmc${i}_counter_collection.csv; done
python tools/pmc_summary.py $G/$TAG diff_N40_B4096 > $P/pmc/summary.txt
echo "collected $TAG"
