#!/bin/bash
# Copy the judged summaries of tools/profile_r03.sh (part A, tag A) and tools/profile_r03b.sh (part B, tag B) runs from
# gpurun_out/ into profiles/r03/, stamping the commit both runs were made from.
# usage: bash tools/collect_r03.sh <tag A> <tag B> <commit of A> [commit of B, default: of A]
A=gpurun_out/$1; B=gpurun_out/$2; C=$3; CB=${4:-$3}
P=profiles/r03
set -e
mkdir -p $P/configs $P/pmc $P/stamps $P/windows
for c in metric diff1024 omni4 tric mixed; do cp $A/bench_$c.json $P/configs/bench_$c.json; done
cp $A/bench_metric.json $P/bench_metric.json
cp $A/ubench.json $P/ubench_valu.json
cp $A/capsule_c.json $P/capsule_latency_c_diff_N80.json
cp $A/capsule_c_team.json $P/capsule_latency_c_diff_N80_team_split.json
cp $A/capsule_py.json $P/capsule_diff_N80.json
cp $A/prof/run_kernel_stats.csv $P/bench_metric_kernel_stats.csv
cp $A/capprof/run_kernel_stats.csv $P/capsule_kernel_stats.csv
cp $A/stamps_team_B4096.txt $A/stamps_team_B1024.txt $A/stamps_rowpar_B4_N80.txt $P/stamps/
python3 - "$A/capprof" "$C" > $P/capsule_roctx_ranges.json <<'PY'
import csv, glob, json, sys
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*marker_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r.get("Function") or r.get("Operation") or "?"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {k: {"count": len(v), "median_us": sorted(v)[len(v) // 2], "mean_us": sum(v) / len(v), "min_us": min(v)}
       for k, v in sorted(d.items())}
print(json.dumps({"source": "rocprofv3 --marker-trace --kernel-trace of build/capsule_latency 300 (tools/profile_r03.sh)",
                  "source_commit": sys.argv[2], "ranges": out,
                  "note": "the first call's capsule.engine range includes the device and engine set-up (mean skewed)"}, indent=1))
PY
python3 - "$A/prof/run_kernel_trace.csv" "$C" > $P/bench_metric_kernel_trace_timed.json <<'PY'
import csv, json, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_sqp_rti_team" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
print(json.dumps({"source": "rocprofv3 --kernel-trace of python3 bench.py --no-cpu-baseline (tools/profile_r03.sh)",
                  "source_commit": sys.argv[2], "launches": len(d), "mean_ms_all": sum(d) / len(d),
                  "mean_ms_last_100_timed": sum(d[-100:]) / 100,
                  "note": "240 closed-loop warm-up ticks + 10 bench warm-up + 100 timed launches; bench.py's HIP-event "
                          "kernel_ms_mean covers the last 100"}, indent=1))
PY
for f in $B/win_*.json; do cp $f $P/windows/; done 2>/dev/null || true
for c in metric:diff_N40_B4096 diff1024:diff_N40_B1024 omni4:omni4_N40_B4096 tric:tric_N60_B8192_g2 \
         "mixed:diff_N40_B2731+omni4_N40_B2731+tric_N40_B2730"; do
  t=${c%%:*}; k=${c#*:}
  for d in $B ${B}2 ${B}c; do
    if ls -d $d/${t}_pmc1 >/dev/null 2>&1; then
      python3 tools/pmc_summary.py $d/$t "$k" --round r03 --last 10 --commit $CB --write > /dev/null; break
    fi
  done
done
echo "collected $1 $2 at $C"
