"""The headline figures quoted in README.md, DESIGN.md and INTEGRATION.md match the round's committed profiles.

Each quoted figure carries a marker `<!-- fig:KEY -->` right before it; KEY names a source record under
profiles/<ROUND>/ and a format (the table below). The test formats the record's value and requires the text after
the marker to start with it, so a figure cannot go stale without this test failing. Every key
must be quoted at least once across the three documents, and every marker must name a known key.
"""
import csv
import json
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUND = "r06"
PROF = os.path.join(ROOT, "profiles", ROUND)
DOCS = ("README.md", "DESIGN.md", "INTEGRATION.md")
CONFIGS = ("metric", "diff1024", "omni4", "tric", "mixed")


def _bench(cfg):
    with open(os.path.join(PROF, "configs", f"bench_{cfg}.json")) as fh:
        return json.load(fh)


def _capsule(mode):
    with open(os.path.join(PROF, f"capsule_latency_c_diff_N80_{mode}.json")) as fh:
        return json.load(fh)


def _sources():
    """{key: formatted figure}"""
    out = {}
    for c in CONFIGS:
        b = _bench(c)
        out[f"{c}_its"] = f"{b['value'] / 1e6:.2f} M"
        out[f"{c}_ms"] = f"{b['ms_per_step']:.2f}"
        out[f"{c}_u0err"] = f"{b['u0_max_abs_err']:.1e}"
        out[f"{c}_frac"] = f"{100.0 * b['roofline']['frac']:.1f} %"
    for c in CONFIGS:
        b = _bench(c)
        out[f"{c}_iters"] = f"{b['qp_iter_mean']:.1f} / {b['qp_iter_max']}"
    out["metric_launch_ms"] = f"{_bench('metric')['roofline']['kernel_ms_mean']:.3f}"
    # the rocprofv3 record and the PMC counters the prose cites (figures citing
    # profiles/<round>/*trace* and pmc/ are checked like the bench figures)
    with open(os.path.join(PROF, "bench_metric_kernel_trace_timed.json")) as fh:
        tr = json.load(fh)
    out["metric_trace_ms"] = f"{tr['mean_ms']:.3f}"
    with open(os.path.join(PROF, "bench_metric_kernel_stats.csv")) as fh:
        row = next(r for r in csv.DictReader(fh) if "k_sqp_rti" in r["Name"])
    out["metric_stats_ms"] = f"{float(row['AverageNs']) * 1e-6:.3f}"
    out["metric_stats_calls"] = row["Calls"]
    for c, key in (("metric", "diff_N40_B4096"), ("diff1024", "diff_N40_B1024")):
        with open(os.path.join(PROF, "pmc", f"pmc_{key}.json")) as fh:
            pm = json.load(fh)
        out[f"{c}_pmc_traffic_gb"] = f"{pm['l2_fabric_bytes_per_launch'] / 1e9:.2f} GB"
        out[f"{c}_pmc_issue"] = f"{pm['valu_issue_frac']:.2f}"
        out[f"{c}_pmc_wait"] = f"{pm['wait_frac']:.2f}"
        out[f"{c}_pmc_active"] = f"{pm['active_frac']:.2f}"
        out[f"{c}_pmc_hit"] = f"{100 * pm['tcc_hit_rate']:.0f} %"
        out[f"{c}_pmc_write_gb"] = f"{pm['write_size_kb'] * 1024 / 1e9:.2f} GB"
    mr = _bench("metric")["roofline"]
    ex = mr["executed_flops"]
    out["metric_exec64_ratio"] = f"{ex['fp64_per_step'] / mr['fp64']['flop_per_step']:.2f}"
    out["metric_exec32_ratio"] = f"{ex['fp32_per_step'] / mr['fp32']['flop_per_step']:.2f}"
    out["metric_cpu_its"] = f"{_bench('metric')['cpu_baseline']['value'] / 1e3:.0f} k"
    for m in ("cold", "warm"):
        out[f"capsule_{m}_ms"] = f"{_capsule(m)['run_wall_ms_mean']:.3f}"
    with open(os.path.join(PROF, "capsule_diff_N80.json")) as fh:
        cap = json.load(fh)  # tools/bench_capsule.py
    out["oracle_1core_ms"] = f"{cap['oracle_fp64_1core_ms']:.3f}"
    out["batch512_ms"] = f"{cap['batch512_ms']:.2f}"
    out["batch512_us"] = f"{cap['batch512_us_per_robot']:.1f}"
    out["batch64_ms"] = f"{cap['batch64_ms']:.2f}"
    out["pymirror_ms"] = f"{cap['run_wall_ms_mean']:.2f}"
    return out


def _markers():
    found = []
    for doc in DOCS:
        with open(os.path.join(ROOT, doc)) as fh:
            text = fh.read()
        for m in re.finditer(r"<!-- fig:([a-z0-9_]+) -->\**([^|\n<]*)", text):
            found.append((doc, m.group(1), m.group(2)))
    return found


def test_headline_figures_match_profiles():
    src = _sources()
    found = _markers()
    assert found, "no <!-- fig:KEY --> markers in " + ", ".join(DOCS)
    for doc, key, text in found:
        assert key in src, (doc, key, "unknown figure key")
        assert text.startswith(src[key]), (doc, key, text[:40], "profiles say " + src[key])


@pytest.mark.parametrize("key", ["metric_its", "diff1024_its", "omni4_its", "tric_its", "mixed_its",
                                 "capsule_cold_ms", "capsule_warm_ms", "metric_u0err", "metric_frac"])
def test_headline_figure_is_quoted(key):
    assert key in {k for _, k, _ in _markers()}, f"{key} is not quoted in any of {DOCS}"
