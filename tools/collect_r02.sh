#!/bin/bash
# Copy the judged summaries of a tools/profile_round.sh run (and, if present, a tools/capsule_breakdown.sh run
# with TAG=<tag>c) from gpurun_out/ into profiles/r02/. usage: bash tools/collect_r02.sh <tag>
TAG=$1
G=gpurun_out
P=profiles/r02
set -e
for c in metric diff1024 omni4 tric mixed; do cp $G/${TAG}_bench_$c.json $P/configs/bench_$c.json; done
cp $G/${TAG}_bench_metric.json $P/bench_metric.json
cp $G/${TAG}_prof/run_kernel_stats.csv $P/bench_metric_kernel_stats.csv
cp $G/${TAG}_ubench.json $P/ubench_valu.json
cp $G/${TAG}_capsule_c.json $P/capsule_latency_c_diff_N80.json
python3 - "$G/${TAG}_prof/run_kernel_trace.csv" "$TAG" > $P/bench_metric_kernel_trace_timed.json <<'PY'
import csv, json, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_sqp_rti_team" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print(json.dumps({"source": f"rocprofv3 --kernel-trace of python3 bench.py --no-cpu-baseline (tools/profile_round.sh {sys.argv[2]})",
                  "launches": len(d), "mean_ms_all": sum(d) / len(d), "mean_ms_first_30_warmup": sum(d[:30]) / 30,
                  "mean_ms_last_100_timed": sum(d[-100:]) / 100,
                  "note": "the first 30 launches are the closed-loop and bench warm-up; the first ticks after create start the IPM cold (longer); bench.py's HIP-event kernel_ms_mean covers the last 100"}, indent=1))
PY
python3 tools/pmc_summary.py $G/${TAG}_metric diff_N40_B4096 --write
python3 tools/pmc_summary.py $G/${TAG}_diff1024 diff_N40_B1024 --write
python3 tools/pmc_summary.py $G/${TAG}_omni4 omni4_N40_B4096 --write
python3 tools/pmc_summary.py $G/${TAG}_tric tric_N60_B8192_g2 --write
python3 tools/pmc_summary.py $G/${TAG}_mixed "diff_N40_B2731+omni4_N40_B2731+tric_N40_B2730" --write
if [ -f $G/${TAG}c_prof/run_kernel_stats.csv ]; then cp $G/${TAG}c_prof/run_kernel_stats.csv $P/capsule_kernel_stats.csv; fi
echo "collected $TAG"
