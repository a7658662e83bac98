"""Summarise rocprofv3 --pmc passes of tools/pmc.sh into per-dispatch averages per kernel, and write the
L2-fabric traffic of the solve kernel into profiles/pmc_traffic.json (read by bench.py's roofline.traffic).

usage: python tools/pmc_summary.py gpurun_out/<tag> <key e.g. diff_N40_B4096> [--write]

traffic = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes): MI355X_MICROARCH.md "HBM": on gfx950 FETCH_SIZE tallies
128-B requests at 64 B (x2 for wide reads); both counters sit at the L2 memory side, so Infinity-Cache (MALL)
hits are included -- this is L2-miss traffic, an upper bound on HBM bytes.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(prefix):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(prefix + "_pmc*/**/*counter_collection.csv", recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                m = re.search(r"\b(k_\w+)", row["Kernel_Name"])
                name = m.group(1) if m else row["Kernel_Name"][:60]
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main():
    prefix, key = sys.argv[1], sys.argv[2]
    summ = load(prefix)
    for k, d in sorted(summ.items()):
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:24s} {v:16.4g}")
    solve = [k for k in summ if "k_sqp_rti" in k]
    if not solve:
        sys.exit("no solve kernel in the counters")
    d = summ[solve[0]]
    traffic = 2 * d.get("FETCH_SIZE", 0.0) * 1024 + d.get("WRITE_SIZE", 0.0) * 1024
    rec = {"kernel": solve[0], "hbm_bytes_per_launch": traffic, "fetch_size_kb": d.get("FETCH_SIZE"),
           "write_size_kb": d.get("WRITE_SIZE"), "tcc_hit": d.get("TCC_HIT_sum"), "tcc_miss": d.get("TCC_MISS_sum"),
           "source": os.path.basename(prefix.rstrip("/")),
           "note": "2*FETCH_SIZE + WRITE_SIZE per dispatch (L2-miss traffic incl. MALL hits)"}
    print(json.dumps(rec, indent=1))
    if "--write" in sys.argv:
        out = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        data = json.load(open(out)) if os.path.exists(out) else {}
        data[key] = rec
        with open(out, "w") as fh:
            json.dump(data, fh, indent=1)


if __name__ == "__main__":
    main()
