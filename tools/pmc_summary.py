"""Summarise the rocprofv3 --pmc passes of tools/pmc.sh into per-dispatch averages per kernel and write the
solve kernel's record to profiles/<round>/pmc/pmc_<config>.json (read by bench.py's roofline: traffic and
issue figures).

usage: python tools/pmc_summary.py gpurun_out/<tag> <config key, e.g. diff_N40_B4096> [--round r03] [--last K]
                                   [--commit <sha>] [--write]
  --last K   average only the last K dispatches of each kernel (the stationary tail of the bench's closed loop;
             default: all dispatches)
  --commit   the commit the GPU run was made from (recorded as source_commit; default: this checkout's HEAD,
             else $NMPC_SOURCE_COMMIT)

Figures per launch of the solve kernel (for a mixed fleet: the sum over its per-model launches of one step):
  l2_fabric_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes). MI355X_MICROARCH.md "HBM": on gfx950
      FETCH_SIZE tallies 128-B requests at 64 B (x2 for wide reads); both counters sit at the L2's memory side,
      so Infinity-Cache (MALL) hits are included: L2-miss traffic, an upper bound on HBM bytes.
  valu_insts_per_wave = SQ_INSTS_VALU / SQ_WAVES.
  valu_issue_frac = SQ_INSTS_VALU / SQ_WAVE_CYCLES: SQ_WAVE_CYCLES counts quad-cycles (MI355X_MICROARCH.md
      "s_memtime tick vs SQ PMC units") and one wave issues at most one VALU instruction per quad-cycle
      (4 cycles, row "vector-instruction ISSUE cost"), so this is the share of the waves' lifetime spent
      issuing VALU at the one-wave minimum cost (fp64 FMAs measure 4.6 cycles, DPP forms 5.6: a lower bound).
  wait_frac / active_frac = SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint buckets).
"""
import csv
import glob
import json
import os
import re
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(prefix, last=None, runs="_pmc*"):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(prefix + runs + "/**/*counter_collection.csv", recursive=True):
        with open(path) as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r.get("Dispatch_Id") or 0))
            for row in rows:
                m = re.search(r"\b(k_\w+)", row["Kernel_Name"])
                name = m.group(1) if m else row["Kernel_Name"][:60]
                # one model's kernel template: keep the model in the name (mixed fleets launch three)
                t = re.search(r"k_sqp_rti_team<nmpc::(\w+)", row["Kernel_Name"])
                if t:
                    name = f"k_sqp_rti_team<{t.group(1)}>"
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if last:
        acc = {k: {c: v[-last:] for c, v in d.items()} for k, d in acc.items()}
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


C_F64 = 5.19  # cycles per v_fma_f64 wave instruction at one wave per SIMD (tools/ubench_valu.hip)
C_VALU = 4.0  # one quad-cycle: the wave64 issue cost of any other VALU instruction (a lower bound)


def per_wave(tot, c):
    return tot[c] / tot["SQ_WAVES"] if tot.get(c) is not None and tot.get("SQ_WAVES") else None


def issue_est(tot):
    """Estimated VALU issue cycles over the waves' lifetime (pass 4 counters)."""
    need = ("SQ_INSTS_VALU_FMA_F64", "SQ_WAVE_CYCLES")
    if not all(tot.get(c) for c in need) or not tot.get("SQ_INSTS_VALU"):
        return None
    f64 = tot["SQ_INSTS_VALU_FMA_F64"]
    cycles = f64 * C_F64 + (tot["SQ_INSTS_VALU"] - f64) * C_VALU
    return cycles / (4.0 * tot["SQ_WAVE_CYCLES"])


def mall(prefix):
    """--mall <prefix>: tools/mall_calibration.sh's two runs of tools/ubench_mall -> requests per KiB read and the
    verdict on TCC_EA0_RDREQ_DRAM (the last launch of each run; its JSON line is in the run's log)."""
    res = {}
    for mib in (64, 2048):
        d = load(f"{prefix}_{mib}", None, runs="")
        k = next((n for n in d if "k_stream" in n), None)
        line = next((ln for ln in open(f"{prefix}_{mib}.log") if ln.startswith("{")), None)
        bench = json.loads(line) if line else {}
        c = d.get(k, {}) if k else {}
        b = bench.get("bytes_read_per_launch")
        kib = b / 1024 if b else None
        res[f"table_{mib}MiB"] = {
            "bytes_read_per_launch": b, "GBs": bench.get("GBs"),
            "rdreq_per_kib": c.get("TCC_EA0_RDREQ_sum", 0) / kib if kib else None,
            "rdreq_dram_per_kib": c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / kib if kib else None,
            "rdreq_32b_per_kib": c.get("TCC_EA0_RDREQ_32B_sum", 0) / kib if kib else None,
            "dram_share": (c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / c["TCC_EA0_RDREQ_sum"]) if c.get("TCC_EA0_RDREQ_sum") else None}
    lo, hi = res["table_64MiB"], res["table_2048MiB"]
    if lo["dram_share"] is not None and hi["dram_share"] is not None:
        sep = lo["dram_share"] < 0.5 * hi["dram_share"]
        res["verdict"] = ("TCC_EA0_RDREQ_DRAM excludes Infinity-Cache hits: the resident table's re-reads are not "
                          "DRAM-destined" if sep else
                          "TCC_EA0_RDREQ_DRAM counts Infinity-Cache hits as DRAM-destined (same share for a resident "
                          "and a non-resident table): the L2 memory-side counters bound DRAM bytes from above only")
    res["source"] = "tools/mall_calibration.sh (tools/ubench_mall.hip: 64 MiB x 16 reps resident, 2 GiB x 2 reps not)"
    print(json.dumps(res, indent=1))


def main():
    if sys.argv[1] == "--mall":
        return mall(sys.argv[2])
    prefix, key = sys.argv[1], sys.argv[2]
    arg = lambda k, d=None: sys.argv[sys.argv.index(k) + 1] if k in sys.argv else d  # noqa: E731
    rnd = arg("--round", "r03")
    last = int(arg("--last", 0)) or None
    summ = load(prefix, last)
    for k, d in sorted(summ.items()):
        print(k)
        for c, v in sorted(d.items()):
            print(f"   {c:24s} {v:16.4g}")
    solve = sorted(k for k in summ if "k_sqp_rti" in k)
    if not solve:
        sys.exit("no solve kernel in the counters")
    tot = defaultdict(float)
    for k in solve:
        for c, v in summ[k].items():
            tot[c] += v
    fetch, write = tot.get("FETCH_SIZE", 0.0), tot.get("WRITE_SIZE", 0.0)
    cyc = tot.get("SQ_WAVE_CYCLES", 0.0)
    cyc4 = cyc
    hit, miss = tot.get("TCC_HIT_sum", 0.0), tot.get("TCC_MISS_sum", 0.0)
    commit = arg("--commit")
    if commit is None:
        try:
            commit = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True).stdout.strip()
        except OSError:
            commit = None
    # the GPU box's snapshot has no .git: tools/final_profile.sh passes the commit in NMPC_SOURCE_COMMIT
    commit = commit or os.environ.get("NMPC_SOURCE_COMMIT") or None
    rec = {"kernels": solve, "config": key, "l2_fabric_bytes_per_launch": 2 * fetch * 1024 + write * 1024,
           "fetch_size_kb": fetch, "write_size_kb": write,
           "tcc_hit_rate": hit / (hit + miss) if hit + miss > 0 else None,
           "valu_insts_per_wave": tot["SQ_INSTS_VALU"] / tot["SQ_WAVES"] if tot.get("SQ_WAVES") else None,
           "valu_issue_frac": tot["SQ_INSTS_VALU"] / cyc if cyc else None,
           "wait_frac": tot["SQ_WAIT_ANY"] / cyc if cyc else None,
           "active_frac": tot["SQ_ACTIVE_INST_ANY"] / cyc if cyc else None,
           "salu_insts_per_wave": tot["SQ_INSTS_SALU"] / tot["SQ_WAVES"] if tot.get("SQ_WAVES") else None,
           # pass 4: the VALU mix. fp64 FMAs issue at 5.19 cycles per wave instruction, any other VALU at >= 4
           # (one quad-cycle; profiles/<round>/ubench_valu.json, one wave per SIMD), so issue_cycles_est / (4 x
           # SQ_WAVE_CYCLES) is the share of the waves' lifetime the SIMD needs just to issue their VALU work.
           # The FLOPS counters count flops per wave instruction (2 per FMA; measured: FLOPS_FP64 ~= 2 x FMA_F64
           # x waves), so x 64 lanes gives the executed flops with idle team lanes and the lockstep max-of-4-teams
           # iterations included (exec masks ignored): executed_flops_per_launch against bench.py's algorithmic
           # flops.
           "valu_fma_f64_per_wave": per_wave(tot, "SQ_INSTS_VALU_FMA_F64"),
           "valu_fma_f32_per_wave": per_wave(tot, "SQ_INSTS_VALU_FMA_F32"),
           "valu_trans_f32_per_wave": per_wave(tot, "SQ_INSTS_VALU_TRANS_F32"),
           "valu_issue_est_frac": issue_est(tot),
           "valu_active_frac": (tot["SQ_ACTIVE_INST_VALU"] / cyc4 if tot.get("SQ_ACTIVE_INST_VALU") and cyc4 else None),
           "executed_flops_fp64_per_launch": (64 * tot["SQ_INSTS_VALU_FLOPS_FP64"]
                                              if tot.get("SQ_INSTS_VALU_FLOPS_FP64") else None),
           "executed_flops_fp32_per_launch": (64 * tot["SQ_INSTS_VALU_FLOPS_FP32"]
                                              if tot.get("SQ_INSTS_VALU_FLOPS_FP32") else None),
           # pass 5: L2 memory-side requests and the share destined for DRAM (TCC_EA0_*REQ_DRAM); whether that
           # share excludes Infinity-Cache hits is what tools/ubench_mall.hip calibrates (profiles/<round>/pmc/)
           "ea_rdreq": tot.get("TCC_EA0_RDREQ_sum"), "ea_rdreq_dram": tot.get("TCC_EA0_RDREQ_DRAM_sum"),
           "ea_wrreq": tot.get("TCC_EA0_WRREQ_sum"), "ea_wrreq_dram": tot.get("TCC_EA0_WRREQ_DRAM_sum"),
           "source": os.path.basename(prefix.rstrip("/")), "source_commit": commit,
           "dispatches_averaged": f"last {last} per kernel" if last else "all",
           "note": "per launch (mixed: summed over the per-model launches of one step); "
                   "traffic = 2*FETCH_SIZE + WRITE_SIZE (L2<->fabric incl. Infinity-Cache hits)"}
    print(json.dumps(rec, indent=1))
    if "--write" in sys.argv:
        out_dir = os.path.join(ROOT, "profiles", rnd, "pmc")
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, f"pmc_{key}.json"), "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
