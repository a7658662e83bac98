#!/usr/bin/env python3
"""Headline benchmark: batched SQP-RTI iterations/s (BASELINE.json metric), diff N=40 B=4096 per GPU.

One step = one control tick of a closed-loop robot fleet resident in HBM: the batched
NMPCNavControl::run() (x0 packing, reference unwrap/padding, terminal-weight hack, one SQP-RTI
iteration = RK4 linearisation + Riccati IPM QP + full step, post-solve command) followed by the
harness kernel that advances the plant one RK4 step and regenerates the path references.
value = (instances x steps, all ranks) / max-over-ranks wall time of the timed region.

Also reported: the u0 max-abs error against the fp64 CPU oracle on identical inputs,
the executed IPM iterations, the roofline of the dominant kernel (algorithmic FLOPs from the SURVEY
formula / HIP-event kernel time; FP32 peak 157.3 TF/s), and the CPU baseline (the oracle, OpenMP on
the host cores, on a bounded sample of the same workload, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from nmpc_nav_control_amd.fleet import FleetNode  # noqa: E402
from nmpc_nav_control_amd.scenario import DEFAULT_SEED  # noqa: E402
from nmpc_nav_control_amd.sharding import TimedRegion, mixed_counts, world_info  # noqa: E402

# BASELINE.json configs (index -> seed offset 20250824 + idx)
CONFIGS = {
    # groups: stream groups per model (FleetNode), decoupled closed loops on their own HIP streams; chosen per
    # config from same-box A/B runs with the single-direction IPM (profiles/r02/ab/ipm_single.txt): tric
    # 2.11 -> 2.37 M it/s with 2 groups; metric (3.52 -> 3.35 M) and diff1024 lose with 2; omni4 and mixed (one
    # stream per model already) lose with more (profiles/r02/ab/groups.txt)
    "metric": dict(idx=1, models=[("diff", 4096)], N=40, desc="diff2amr N=40 batch=4096 per GPU"),
    "diff1024": dict(idx=1, models=[("diff", 1024)], N=40, desc="diff2amr N=40 batch=1024"),
    "omni4": dict(idx=2, models=[("omni4", 4096)], N=40, desc="omni4amr (11x4) N=40 batch=4096"),
    "tric": dict(idx=3, models=[("tric", 8192)], N=60, groups=2, desc="tric3amr N=60 batch=8192, alpha bounds active"),
    # whole fleet: 65536 robots over 8 GPUs -> 8192 per GPU, a third of each model; the three models' streams run
    # decoupled (2.94 -> 3.71 M it/s against a fleet-wide tick boundary), also under the per-tick gather (staged
    # per stream, FleetNode)
    "mixed": dict(idx=4, models=[("diff", 2731), ("omni4", 2731), ("tric", 2730)], N=40,
                  desc="mixed fleet diff+omni4+tric, 8192 per GPU (65536 on 8 GPUs)"),
}
# SURVEY.md 8d algorithmic FLOPs per instance-iteration: F = N*F_lin + K*N*F_ipm
MODEL_FLOPS = {"diff": dict(nx=7, nu=2, nbx=2, nbu=2, nnz_jx=12, nnz_ju=2, c_f=20),
               "omni4": dict(nx=11, nu=4, nbx=4, nbu=4, nnz_jx=22, nnz_ju=4, c_f=40),
               "tric": dict(nx=7, nu=2, nbx=2, nbu=2, nnz_jx=12, nnz_ju=2, c_f=24)}
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector (and FP32-input MFMA) peak
FP64_PEAK_SPEC_TFLOPS = 78.6  # AMD spec FP64 vector (half the FP32 rate; the guide gives no FP64 figure)
PROFILE_ROUND = "r06"
HBM_PEAK_GBS = 8000.0


def flops_per_instance(model, N, K, split=False):
    """SURVEY 8d algorithmic flops per instance-iteration, F = N*F_lin + K*N*F_ipm. With split=True returns
    (fp32 flops, fp64 flops): the Riccati factorisation terms of F_ipm (P G, G'P G, the input-block Cholesky
    and its Schur complement) run in fp64 on the device, everything else in fp32."""
    m = MODEL_FLOPS[model]
    nx, nu, nv = m["nx"], m["nu"], m["nx"] + m["nu"]
    f_lin = 4 * (m["c_f"] + 2 * m["nnz_jx"] * nv + m["nnz_ju"]) + 16 * nx * (1 + nv)
    f_fact = 2 * nv * nx * nx + nv * (nv + 1) * nx + (nu ** 3) // 3 + nu * nu * nx + nx * nx * nu
    f_rest = (4 * nv * nx + 2 * nu * nx + nu * nu + 2 * nx * nv + 2 * nx * nx
              + 20 * (m["nbx"] + m["nbu"]) + 4 * nx * nv)
    total = N * f_lin + K * N * (f_fact + f_rest)
    if split:
        return N * f_lin + K * N * f_rest, K * N * f_fact
    return total


def _profile_json(name):
    path = os.path.join(ROOT, "profiles", PROFILE_ROUND, name)
    if os.path.exists(path):
        with open(path) as fh:
            return json.load(fh), os.path.relpath(path, ROOT)
    return None, None


def valu_peaks(basis="spec"):
    """(FP32, FP64) vector peaks in TFLOP/s on one stated basis:
    'spec'     -- FP32 157.3 (MI355X_MICROARCH.md) and FP64 78.6 (AMD spec; the guide gives none): the line's frac;
    'measured' -- both full-occupancy FMA rates of tools/ubench_valu.hip on this device (profiles/<round>/
                  ubench_valu.json: FP32 114.0, FP64 62.6), None when that record is absent."""
    if basis == "spec":
        return FP32_PEAK_TFLOPS, FP64_PEAK_SPEC_TFLOPS
    ub, _ = _profile_json("ubench_valu.json")
    if not ub:
        return None
    return float(ub["fp32_full"]["tflops"]), float(ub["fp64_full"]["tflops"])


def roofline(fleets, node, kernel_ms, steps, step_s=None):
    """Roofline record of the solve kernel(s) of one step: algorithmic flops, split into the fp32
    part and the fp64 Riccati factorisation, each priced at its own VALU peak; frac = the share of the VALU
    time budget of the timed launches that the algorithmic flops would need at peak. The PMC-side figures
    (L2<->fabric traffic, VALU issue share of the wave cycles) come from the rocprofv3 --pmc passes of the
    same config (tools/pmc.sh -> tools/pmc_summary.py -> profiles/<round>/pmc/pmc_<config>.json)."""
    t_launch = float(np.mean(kernel_ms)) * 1e-3
    # decoupled stream groups: the launches of a step overlap each other, so the rate is the step's flops over
    # the step's share of the timed region (conservative: it includes the plant steps and any idle gaps)
    t_k = step_s if node.decoupled else t_launch
    f32 = f64 = 0.0
    cbytes = 0
    for j, f in enumerate(fleets):
        sl = slice(node.offs[j], node.offs[j + 1])
        k_f = float(node.iters_sum[sl].sum().item()) / (f.B * steps)
        a, b = flops_per_instance(f.model, f.N, k_f, split=True)
        f32 += f.B * a
        f64 += f.B * b
        cbytes += f.B * bytes_per_instance(f.model, f.N)
    p32, p64 = valu_peaks("spec")
    a32, a64 = f32 / t_k / 1e12, f64 / t_k / 1e12
    frac = a32 / p32 + a64 / p64
    achieved = a32 + a64
    meas = valu_peaks("measured")
    frac_meas = (a32 / meas[0] + a64 / meas[1]) if meas else None
    per_model = {}
    for f in fleets:
        per_model[(f.model, f.N)] = per_model.get((f.model, f.N), 0) + f.B
    cfg = "+".join(f"{m}_N{n}_B{b}" for (m, n), b in per_model.items()) + (f"_g{node.groups}" if node.groups > 1 else "")
    pmc, src = _profile_json(f"pmc/pmc_{cfg}.json")
    traffic = pmc.get("l2_fabric_bytes_per_launch") if pmc else None
    if traffic is not None and node.groups > 1:
        traffic *= node.groups  # the PMC record averages one dispatch per kernel name; a step runs `groups` of each
    # per launch (the contract's figure, checkable against the rocprofv3 kernel-trace average): the flops of one
    # launch over the mean launch duration; with one launch per step this equals `achieved`
    n_launch = len(fleets)
    per_launch = None
    if n_launch > 1 and len({(f.model, f.N) for f in fleets}) == 1:
        per_launch = {"flop": (f32 + f64) / n_launch, "ms": round(t_launch * 1e3, 4),
                      "achieved_tflops": round((f32 + f64) / n_launch / t_launch / 1e12, 4),
                      "note": "one of the step's %d concurrent launches (%d robots)" % (n_launch, fleets[0].B)}
    return {"bound": "valu", "achieved": round(achieved, 4), "peak": round(achieved / frac, 2), "unit": "TFLOP/s",
            "frac": round(frac, 6), "traffic": traffic, "per_launch": per_launch,
            "peak_basis": "spec: FP32 157.3 TF (MI355X_MICROARCH.md), FP64 78.6 TF (AMD spec); each half of the flops "
                          "priced at its own peak, frac = fp32 / FP32 peak + fp64 / FP64 peak",
            "frac_measured_basis": (round(frac_meas, 6) if frac_meas is not None else None),
            "measured_peaks_tflops": ({"fp32": meas[0], "fp64": meas[1],
                                       "source": "tools/ubench_valu.hip full occupancy (profiles/%s/ubench_valu.json)"
                                       % PROFILE_ROUND} if meas else None),
            "fp32": {"flop_per_step": f32, "achieved_tflops": round(a32, 4), "peak_tflops": p32,
                     "frac": round(a32 / p32, 6)},
            "fp64": {"flop_per_step": f64, "achieved_tflops": round(a64, 4), "peak_tflops": p64,
                     "frac": round(a64 / p64, 6)},
            "issue": ({k: pmc.get(k) for k in ("valu_insts_per_wave", "valu_issue_frac", "valu_issue_est_frac",
                                               "valu_active_frac", "valu_fma_f64_per_wave", "wait_frac",
                                               "active_frac", "source_commit")} if pmc else None),
            "executed_flops": ({"fp64_per_step": _scaled(pmc.get("executed_flops_fp64_per_launch"), node.groups),
                                "fp32_per_step": _scaled(pmc.get("executed_flops_fp32_per_launch"), node.groups),
                                "note": "64 x SQ_INSTS_VALU_FLOPS_FP64/FP32 from the PMC record: every lane of "
                                        "every issued instruction, idle team lanes and the lockstep waves' extra "
                                        "iterations included"}
                               if pmc and pmc.get("executed_flops_fp64_per_launch") else None),
            "traffic_source": src, "kernel": _kernel_label(fleets[0]) +
            (f" x{len(fleets)} concurrent streams" if len(fleets) > 1 else ""),
            "kernel_ms_mean": round(t_launch * 1e3, 4),
            "timing": ("HIP events per launch on its stream; achieved = the step's flops / (timed region / steps), "
                       "the launches of %d decoupled streams overlapping" % len(fleets)) if node.decoupled else
                      "HIP events on the launch stream(s), timed region",
            "compulsory_bytes_per_launch": cbytes, "achieved_compulsory_GBs": round(cbytes / t_k / 1e9, 2),
            "hbm": hbm_block(pmc, src, traffic, cbytes, t_k, node.groups),
            "note": "VALU-bound, latency-limited: <=15x15 per-robot blocks, no GEMM-shaped work (no MFMA); "
                    "traffic = 2*FETCH_SIZE + WRITE_SIZE (L2<->fabric incl. Infinity-Cache hits) per step (the sum "
                    "over the step's launches: one per model and stream group)"}


def _kernel_label(fleet):
    """The solve kernel a fleet's run launches take (nmpc_batch_plan_ex, run mode): the team kernel with its record
    layout, or the row-parallel one with its waves per robot and horizon segments."""
    plan = getattr(fleet.solver, "plan_ex", None)
    if plan is None:
        return f"k_sqp_rti_{getattr(fleet.solver, 'kernel', 'team')}"
    p = plan(fleet.B, "run")
    if p["kernel"] == "team":
        return f"k_sqp_rti_team ({p['record_layout']} records)"
    segs = p["segments"]
    return (f"k_sqp_rti_rowpar ({p['waves_per_robot']} wave(s) per robot, " +
            (f"{segs} horizon segments)" if segs else "serial phases)"))


def hbm_block(pmc, src, traffic, cbytes, t_k, groups=1):
    """North-star HBM reporting: the memory-side bytes of the step's solve launches from the PMC record
    (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md "HBM"), their rate over the launch
    time and its fraction of the 8 TB/s HBM peak, beside the compulsory bytes and their fraction. The
    counters sit at the L2's memory side, so Infinity-Cache (MALL) hits are included: an upper bound on DRAM bytes.
    ea_*req_dram: the share of those requests gfx950 tags as destined for DRAM (TCC_EA0_*REQ_DRAM), whose
    meaning tools/ubench_mall.hip calibrates (profiles/<round>/pmc/mall_calibration.json)."""
    out = {"peak_GBs": HBM_PEAK_GBS, "compulsory_bytes_per_step": cbytes,
           "compulsory_GBs": round(cbytes / t_k / 1e9, 3), "compulsory_frac": round(cbytes / t_k / 1e9 / HBM_PEAK_GBS, 6)}
    if traffic is not None:
        gbs = traffic / t_k / 1e9
        out.update({"pmc_bytes_per_step": traffic, "pmc_GBs": round(gbs, 1), "pmc_frac": round(gbs / HBM_PEAK_GBS, 4),
                    "pmc_over_compulsory": round(traffic / cbytes, 1) if cbytes else None, "pmc_source": src,
                    "includes_mall_hits": True})
    if pmc and pmc.get("ea_rdreq"):
        # the L2's memory-side read requests, sized by tools/ubench_mall.hip (128 B each: 8.00 per KiB streamed,
        # profiles/<round>/pmc/mall_calibration.json): a second, independent count of the read bytes beside
        # 2 x FETCH_SIZE. Write requests are counted, not sized (partial-sector stores make them smaller than the
        # 64 B of the calibration's full-line fill). The _DRAM-tagged share is 1.0 for an Infinity-Cache-resident
        # table as well, so it cannot separate MALL hits from DRAM reads on gfx950
        g = groups if groups else 1
        rd, rdd = pmc["ea_rdreq"], pmc.get("ea_rdreq_dram")
        wr, wrd = pmc.get("ea_wrreq"), pmc.get("ea_wrreq_dram")
        out["ea_read_bytes_per_step"] = g * rd * 128
        out["ea_read_GBs"] = round(g * rd * 128 / t_k / 1e9, 1)
        out["ea_write_requests_per_step"] = g * wr if wr is not None else None
        out["dram_destined_share"] = {"read": round(rdd / rd, 4) if rdd is not None else None,
                                      "write": round(wrd / wr, 4) if wr and wrd is not None else None}
        cal, csrc = _profile_json("pmc/mall_calibration.json")
        if cal:
            out["dram_counter_calibration"] = {"source": csrc, "verdict": cal.get("verdict")}
    return out


def _scaled(v, g):
    return None if v is None else v * g


def bytes_per_instance(model, N):
    """Compulsory fp32 bytes per instance-iteration: x0, pose refs, iterate in+out, status."""
    m = MODEL_FLOPS[model]
    return 4 * (m["nx"] + 3 * (N + 1) + 2 * ((N + 1) * m["nx"] + N * m["nu"]) + 1)


def cpu_baseline(fleets, sample, ticks, nthreads):
    """Replay `ticks` closed-loop GPU ticks for the first `sample` robots (0: all) of each fleet through the
    fp64 oracle. Every tick the oracle starts from exactly the GPU's pre-tick state (iterate, carried refs,
    measurements, references), so the u0 error is the per-solve fp32-vs-fp64 error, not the divergence of
    two closed loops. The timed replay runs the oracle's "batched" exit rule (the batched API's); the same inputs
    go through its "acados" rule too (HPIPM: no infeasibility exit), untimed, for the second error figure. Returns
    (CPU instance-iterations/s, u0 max-abs err, failed, solves, 1-core rate, u0 max-abs err on the acados rule)."""
    from oracle.oracle import Oracle
    total_time, total_solves, err, fails = 0.0, 0, 0.0, 0
    time_1, solves_1, err_a = 0.0, 0, 0.0
    for f in fleets:
        S = f.B if sample <= 0 else min(sample, f.B)
        o = Oracle(f.model, f.N, rule="batched")
        oa = Oracle(f.model, f.N, rule="acados")
        for _ in range(ticks):
            torch.cuda.synchronize()
            sn = f.snapshot()
            sl = lambda a, n: None if a is None else np.ascontiguousarray(a[:n])  # noqa: E731
            args = [sl(sn[k], S) for k in ("pose", "vel", "steer", "traj", "tlen", "reset")]
            state = [sl(sn[k], S) for k in ("carried", "xbar", "ubar")]
            f.solve()
            # single-core rate on a slice of the same inputs (copies: batch_tick updates the iterate in place)
            S1 = min(S, 64)
            a1 = [sl(a, S1) for a in args]
            s1 = [np.array(a[:S1]) for a in state]
            t0 = time.perf_counter()
            o.batch_tick(*a1, *s1, nthreads=1)
            time_1 += time.perf_counter() - t0
            solves_1 += S1
            sa = [np.array(a) for a in state]  # batch_tick updates the iterate in place
            t0 = time.perf_counter()
            nf, cmd_o, u0_o, st_o, _ = o.batch_tick(*args, *state, nthreads=nthreads)
            total_time += time.perf_counter() - t0
            total_solves += S
            _, _, u0_a, st_a, _ = oa.batch_tick(*args, *sa, nthreads=nthreads)
            torch.cuda.synchronize()
            st_g = f.status[:S].cpu().numpy()
            u0_g = f.u0[:, :S].cpu().numpy().T
            ok = (st_o == 0) & (st_g == 0)
            fails += int((~ok).sum())
            if ok.any():
                err = max(err, float(np.abs(u0_g[ok] - u0_o[ok]).max()))
            ok_a = (st_a == 0) & (st_g == 0)
            if ok_a.any():
                err_a = max(err_a, float(np.abs(u0_g[ok_a] - u0_a[ok_a]).max()))
            f.advance()
    return total_solves / total_time, err, fails, total_solves, solves_1 / time_1, err_a


class LaunchTimer:
    """HIP events around each solve launch of a timed step, on the launch's own stream (FleetNode.step's timer)."""

    def __init__(self, n_fleets, steps):
        T = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
        self.ev = [([T() for _ in range(n_fleets)], [T() for _ in range(n_fleets)]) for _ in range(steps)]
        self.k = 0

    def start(self, j, stream):
        self.ev[self.k][0][max(j, 0)].record(stream)

    def end(self, j, stream):
        self.ev[self.k][1][j].record(stream)

    def kernel_ms(self, decoupled):
        """Per step: the mean launch duration (decoupled streams), or the latest end from the common start."""
        if decoupled:
            return [float(np.mean([a.elapsed_time(b) for a, b in zip(s, e)])) for s, e in self.ev]
        return [max(s[0].elapsed_time(b) for b in e) for s, e in self.ev]


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """`--gpus N` (N > 1) without torchrun's environment: start the N rank processes here, one per GPU, with
    torch.distributed.run as a child process (RCCL rendezvous on 127.0.0.1), and return its exit code. This
    process makes no HIP call before or after (it only parses arguments), so no GPU state is shared or inherited;
    rank 0 prints the one JSON line to the inherited stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, NMPC_BENCH_LAUNCHER="bench.py --gpus %d" % n)
    sys.stdout.flush()
    return subprocess.run(cmd, env=env).returncode


# --ipm-rules acados: HPIPM's defaults for the batched API (the reference's OCP sets none of
# them, scripts/diff/generate_c_code.py:68-74): no infeasibility exit, slack floor thr0 0.5 (the oracle's), every QP
# started cold. The product's own rules (nmpc_model_params_default) differ in exactly these three (DESIGN.md section
# 5); this line states what they are worth
ACADOS_RULES = dict(qp_infeas_lambda=0.0, qp_thr0=0.5, qp_warm_start=0)


def _factory(spec, ipm_rules="product", qp=None):
    """--test-solver MODULE:ATTR -> the solver class FleetNode builds its fleets with (default: BatchSolver);
    --ipm-rules acados -> BatchSolver with ACADOS_RULES; --qp k=v,... (A/B runs) -> nmpc_model_params overrides."""
    if spec:
        import importlib
        mod, attr = spec.split(":")
        return getattr(importlib.import_module(mod), attr)
    over = dict(ACADOS_RULES) if ipm_rules == "acados" else {}
    for kv in (qp.split(",") if qp else []):
        k, v = kv.split("=")
        over[k] = float(v)
    if over:
        from nmpc_nav_control_amd._lib import default_params
        from nmpc_nav_control_amd.batch import BatchSolver

        def make(model, N, B, device=None):
            prm = default_params(model, N)
            for k, v in over.items():
                setattr(prm, k, type(getattr(prm, k))(v))
            return BatchSolver(model, N, B, params=prm, device=device)
        return make
    return None


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU). Under torchrun it must equal WORLD_SIZE; without torchrun's "
                         "environment and N > 1, bench.py starts the N ranks itself")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--closed-loop-warmup", type=int, default=240,
                    help="ticks before timing (SURVEY 8d asks for >= 20; 240 = the longest goal / path ttl, so every "
                         "robot has been re-issued a goal or path once and the timed window is stationary)")
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="robots per model replayed on the CPU oracle (0: the whole batch)")
    ap.add_argument("--cpu-ticks", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true", help="all-gather u0+status to rank 0 every tick (RCCL)")
    ap.add_argument("--dist", action="store_true",
                    help="initialise the RCCL process group at world size 1 too (exercises the barrier, the MAX "
                         "all-reduce of the timed region and the command all-gather on a one-GPU box)")
    ap.add_argument("--groups", type=int, default=None,
                    help="stream groups per model (default: the config's); each is a Fleet on its own HIP stream")
    ap.add_argument("--joined", action="store_true",
                    help="fleet-wide tick boundary across streams (default: decoupled streams unless --gather)")
    ap.add_argument("--no-renew", action="store_true",
                    help="every robot keeps its first goal / path (the round-2 workload, which parks and drifts)")
    ap.add_argument("--batch-per-gpu", type=int, default=None,
                    help="robots per rank (default: the config's; mixed splits them over the three models)")
    # test hooks of the launch path (tests/test_bench_launch.py): CPU ranks over gloo with a CPU solver class
    ap.add_argument("--ipm-rules", default="product", choices=["product", "acados"],
                    help="acados: the batched solve with HPIPM's defaults (no infeasibility exit, thr0 0.5, cold QP "
                         "starts) instead of the product's IPM rules; not the headline")
    ap.add_argument("--qp", default=None, help=argparse.SUPPRESS)  # A/B: nmpc_model_params overrides k=v,...
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"], help=argparse.SUPPRESS)
    ap.add_argument("--test-solver", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:])

    # stdout carries exactly one JSON line: native libraries that print to fd 1 (RCCL's version banner at process
    # group start-up) are sent to stderr, the JSON line goes to the original stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    rank, world, local_rank = world_info()
    cpu = args.device == "cpu"
    dev = torch.device("cpu") if cpu else torch.device("cuda", local_rank)
    if not cpu:
        torch.cuda.set_device(dev)
    if world > 1 or args.dist:
        dist.init_process_group("gloo" if cpu else "nccl", **({} if cpu else {"device_id": dev}))
    ranks = dist.get_world_size() if dist.is_initialized() else 1
    backend = dist.get_backend() if dist.is_initialized() else None
    if ranks != args.gpus or ranks != world:
        print(f"bench.py: --gpus {args.gpus} but the process group has {ranks} rank(s) (WORLD_SIZE {world})",
              file=sys.stderr)
        if dist.is_initialized():
            dist.destroy_process_group()
        return 3

    cfg = CONFIGS[args.config]
    models = cfg["models"]
    if args.batch_per_gpu is not None:
        models = (mixed_counts(args.batch_per_gpu, [m for m, _ in models]) if len(models) > 1
                  else [(models[0][0], args.batch_per_gpu)])
    gather = args.gather or (args.config == "mixed" and world > 1)
    # weak scaling: the global fleet holds B x world robots of each model; this rank owns the contiguous
    # shard [rank*B, (rank+1)*B) of it (sharding.shard_range), no collective on the solve path
    if args.groups is None and os.environ.get("NMPC_BENCH_GROUPS"):  # A/B runs (tools/ab_env.py variants)
        args.groups = int(os.environ["NMPC_BENCH_GROUPS"])
    groups = cfg.get("groups", 1) if args.groups is None else args.groups
    node = FleetNode(models, cfg["N"], DEFAULT_SEED + cfg["idx"], dev, rank=rank, world=world, gather=gather,
                     groups=groups, decoupled=False if args.joined else None, renew=not args.no_renew,
                     solver_factory=_factory(args.test_solver, args.ipm_rules, args.qp))
    fleets = node.fleets
    if not cpu:
        torch.cuda.synchronize()

    # warmup runs every op of the timed loop (the first use of a torch kernel loads its code object)
    for _ in range(args.closed_loop_warmup + args.warmup):
        node.step()
    node.reset_stats()
    if not cpu:
        torch.cuda.synchronize()

    # per-launch timing of the solve kernels with HIP events on their launch streams (FleetNode.step calls the
    # timer around every solve launch). One stream: the solve's duration. Joined streams: from one start event
    # on the main stream to each stream's end-of-solve event (the region = the latest). Decoupled streams: each
    # launch from its own stream's start event.
    timer = None if cpu else LaunchTimer(len(fleets), args.steps)
    with TimedRegion(dev) as region:
        for k in range(args.steps):
            if timer is not None:
                timer.k = k
            node.step(timer)
    elapsed = region.elapsed

    kernel_ms = timer.kernel_ms(node.decoupled) if timer is not None else None
    its = node.iter_stats()
    B_rank = node.B
    k_mean = float(node.iters_sum.sum().item()) / (B_rank * args.steps)
    units = args.steps * B_rank * world
    value = units / elapsed

    result = None
    if rank == 0:
        roof = roofline(fleets, node, kernel_ms, args.steps, step_s=elapsed / args.steps) if not cpu else None
        cpu_base = None
        u0_err = None
        if not args.no_cpu_baseline and world == 1 and not cpu:
            nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
            cpu_rate, u0_err, nf, ns, rate_1, u0_err_acados = cpu_baseline(fleets, args.cpu_sample, args.cpu_ticks,
                                                                           nthreads)
            cpu_base = {"value": round(cpu_rate, 1), "unit": "SQP-RTI iterations/sec", "cores": nthreads,
                        "kind": "port", "oracle_rule": "batched (the batched API's IPM exit rule; oracle/oracle.py RULES)",
                        "u0_max_abs_err_acados_rule": u0_err_acados,
                        "sample": f"{ns} instance-iterations: {'all' if args.cpu_sample <= 0 else args.cpu_sample} robots of each model x "
                                  f"{args.cpu_ticks} closed-loop ticks after the timed region, fp64 oracle/nmpc_oracle.c, "
                                  f"OpenMP {nthreads} threads, identical inputs", "failed": nf,
                        "value_1core": round(rate_1, 1),
                        "note": "a reported baseline, not a target: timed after the timed region on the GPU box's shared "
                                "host cores, so it varies from run to run"}
        result = {
            "metric": "SQP-RTI iterations/sec (whole node), diff N=40 batch=4096; u0 max-abs err",
            "value": round(value, 1), "unit": "SQP-RTI iterations/sec", "n_gpus": ranks, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32+fp64",
            "data": ("synthetic seeded closed-loop fleet (SURVEY 8d), random-arc paths + goal poses" +
                     ("" if args.no_renew else ", stationary: new goal / path + reset_mpc on arrival or after a "
                                               "2-6 s ttl (NMPCNavControlROS.cpp:304-327)")),
            "config": {"workload": cfg["desc"], "config": args.config, "N": cfg["N"],
                       "batch_per_gpu": B_rank, "global_batch": B_rank * world,
                       "models": [m for m, _ in models], "parallelism": f"instance-sharded x{world}",
                       "ranks": ranks, "backend": backend,
                       "launcher": os.environ.get("NMPC_BENCH_LAUNCHER",
                                                  "torchrun" if "WORLD_SIZE" in os.environ else "single process"),
                       "closed_loop_warmup_ticks": args.closed_loop_warmup, "rccl_gather": gather,
                       "ipm_rules": args.ipm_rules + (f" + {args.qp}" if args.qp else "")},
            "u0_max_abs_err": u0_err, "qp_iter_mean": round(k_mean, 3), "qp_iter_max": int(node.iters_max.max().item()),
            "qp_iter": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in its.items()},
            "failed_solves": int(node.fail_cnt.sum().item()), "roofline": roof, "cpu_baseline": cpu_base,
        }
        print(json.dumps(result), file=json_out, flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
