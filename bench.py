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

from nmpc_nav_control_amd.batch import BatchSolver  # noqa: E402
from nmpc_nav_control_amd.scenario import DEFAULT_SEED, make_fleet  # noqa: E402
from nmpc_nav_control_amd.sharding import CommandGather, TimedRegion, shard_range, world_info  # noqa: E402

# BASELINE.json configs (index -> seed offset 20250824 + idx)
CONFIGS = {
    "metric": dict(idx=1, models=[("diff", 4096)], N=40, desc="diff2amr N=40 batch=4096 per GPU"),
    "diff1024": dict(idx=1, models=[("diff", 1024)], N=40, desc="diff2amr N=40 batch=1024"),
    "omni4": dict(idx=2, models=[("omni4", 4096)], N=40, desc="omni4amr (11x4) N=40 batch=4096"),
    "tric": dict(idx=3, models=[("tric", 8192)], N=60, desc="tric3amr N=60 batch=8192, alpha bounds active"),
    # whole fleet: 65536 robots over 8 GPUs -> 8192 per GPU, a third of each model
    "mixed": dict(idx=4, models=[("diff", 2731), ("omni4", 2731), ("tric", 2730)], N=40,
                  desc="mixed fleet diff+omni4+tric, 8192 per GPU (65536 on 8 GPUs)"),
}
# SURVEY.md 8d algorithmic FLOPs per instance-iteration: F = N*F_lin + K*N*F_ipm
MODEL_FLOPS = {"diff": dict(nx=7, nu=2, nbx=2, nbu=2, nnz_jx=12, nnz_ju=2, c_f=20),
               "omni4": dict(nx=11, nu=4, nbx=4, nbu=4, nnz_jx=22, nnz_ju=4, c_f=40),
               "tric": dict(nx=7, nu=2, nbx=2, nbu=2, nnz_jx=12, nnz_ju=2, c_f=24)}
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: FP32 vector (and FP32-input MFMA) peak
HBM_PEAK_GBS = 8000.0


def flops_per_instance(model, N, K):
    m = MODEL_FLOPS[model]
    nx, nu, nv = m["nx"], m["nu"], m["nx"] + m["nu"]
    f_lin = 4 * (m["c_f"] + 2 * m["nnz_jx"] * nv + m["nnz_ju"]) + 16 * nx * (1 + nv)
    f_ipm = (2 * nv * nx * nx + nv * (nv + 1) * nx + (nu ** 3) // 3 + nu * nu * nx + nx * nx * nu + 4 * nv * nx
             + 2 * nu * nx + nu * nu + 2 * nx * nv + 2 * nx * nx
             + 20 * (m["nbx"] + m["nbu"]) + 4 * nx * nv)
    return N * f_lin + K * N * f_ipm


def bytes_per_instance(model, N):
    """Compulsory fp32 bytes per instance-iteration: x0, pose refs, iterate in+out, status."""
    m = MODEL_FLOPS[model]
    return 4 * (m["nx"] + 3 * (N + 1) + 2 * ((N + 1) * m["nx"] + N * m["nu"]) + 1)


class Fleet:
    """One model's robots on this GPU: solver + closed-loop state, all device-resident."""

    def __init__(self, model, B, N, seed, dev, start=0, stream=None):
        self.model, self.B, self.N = model, B, N
        self.stream = stream  # None: the current stream; mixed fleets give each model its own HIP stream
        self.solver = BatchSolver(model, N, B, device=dev)
        if stream is not None and "NMPC_AMD_SCHED" not in os.environ:
            # concurrent launches of several models share the CUs: pair hard and easy blocks
            # (include/nmpc_amd/nmpc_batch.h NMPC_SCHED_INTERLEAVED)
            self.solver.set_schedule("interleaved")
        fl = make_fleet(model, B, seed=seed, start=start)
        t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
        self.pose, self.vel, self.path, self.s = t(fl["pose"]), t(fl["vel"]), t(fl["path"]), t(fl["s"])
        self.steer = t(fl["steer"]) if model == "tric" else None
        _, _, cr = self.solver.state()
        cr.copy_from(t(fl["carried"]))
        self.traj = torch.zeros(N + 1, 3, B, device=dev)
        self.tlen = torch.zeros(B, dtype=torch.int32, device=dev)
        self.cmd = torch.zeros(3, B, device=dev)
        self.u0 = torch.zeros(self.solver.nu, B, device=dev)
        self.status = torch.zeros(B, dtype=torch.int32, device=dev)
        self.qp_iter = torch.zeros(B, dtype=torch.int32, device=dev)
        self.solver.fleet_sim_step(self.path, self.s, self.pose, self.vel, self.steer, None, None, self.traj,
                                   self.tlen, advance=False)

    def solve(self):
        self.solver.run(self.pose, self.vel, self.traj, steer=self.steer, traj_len=self.tlen, cmd=self.cmd,
                        u0=self.u0, status=self.status, qp_iter=self.qp_iter, stream=self.stream)

    def advance(self):
        self.solver.fleet_sim_step(self.path, self.s, self.pose, self.vel, self.steer, self.u0, self.status,
                                   self.traj, self.tlen, advance=True, stream=self.stream)

    def tick(self):
        self.solve()
        self.advance()


def cpu_baseline(fleets, dev, sample, ticks, nthreads):
    """Replay `ticks` closed-loop GPU ticks for the first `sample` robots of each fleet through the fp64
    oracle. Every tick the oracle starts from exactly the GPU's pre-tick state (iterate, carried refs,
    measurements, references), so the u0 error is the per-solve fp32-vs-fp64 error, not the divergence of
    two closed loops. Returns (CPU instance-iterations/s, u0 max-abs err, failed, solves)."""
    from oracle.oracle import Oracle
    total_time, total_solves, err, fails = 0.0, 0, 0.0, 0
    time_1, solves_1 = 0.0, 0
    host = lambda a: np.ascontiguousarray(a.cpu().numpy(), np.float64)  # noqa: E731
    for f in fleets:
        S = min(sample, f.B)
        o = Oracle(f.model, f.N)
        xv, uv, cv = f.solver.state()
        for _ in range(ticks):
            torch.cuda.synchronize()
            X, U, Cr = xv.to_tensor(), uv.to_tensor(), cv.to_tensor()
            xbar = np.ascontiguousarray(host(X[:, :S]).T.reshape(S, f.N + 1, o.nx))
            ubar = np.ascontiguousarray(host(U[:, :S]).T.reshape(S, f.N, o.nu))
            carried = np.ascontiguousarray(host(Cr[:, :S]).T)
            pose = np.ascontiguousarray(host(f.pose[:, :S]).T)
            vel = np.ascontiguousarray(host(f.vel[:, :S]).T)
            steer = host(f.steer[:S]) if f.steer is not None else None
            traj = np.ascontiguousarray(host(f.traj[:, :, :S]).transpose(2, 0, 1))
            tlen = np.ascontiguousarray(f.tlen[:S].cpu().numpy(), np.int32)
            f.solve()
            # single-core rate on a slice of the same inputs (copies: batch_tick updates the iterate in place)
            S1 = min(S, 64)
            sl = lambda a: None if a is None else np.array(a[:S1])  # noqa: E731
            t0 = time.perf_counter()
            o.batch_tick(sl(pose), sl(vel), sl(steer), sl(traj), sl(tlen), None, sl(carried), sl(xbar), sl(ubar),
                         nthreads=1)
            time_1 += time.perf_counter() - t0
            solves_1 += S1
            t0 = time.perf_counter()
            nf, cmd_o, u0_o, st_o, _ = o.batch_tick(pose, vel, steer, traj, tlen, None, carried, xbar, ubar,
                                                    nthreads=nthreads)
            total_time += time.perf_counter() - t0
            total_solves += S
            torch.cuda.synchronize()
            ok = (st_o == 0) & (f.status[:S].cpu().numpy() == 0)
            fails += int((~ok).sum())
            if ok.any():
                err = max(err, float(np.abs(f.u0[:, :S].cpu().numpy().T[ok] - u0_o[ok]).max()))
            f.advance()
    return total_solves / total_time, err, fails, total_solves, solves_1 / time_1


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--closed-loop-warmup", type=int, default=20, help="ticks before timing (SURVEY 8d: T=20)")
    ap.add_argument("--cpu-sample", type=int, default=256, help="robots per model replayed on the CPU oracle")
    ap.add_argument("--cpu-ticks", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather", action="store_true", help="all-gather u0+status to rank 0 every tick (RCCL)")
    args = ap.parse_args()

    rank, world, local_rank = world_info()
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = CONFIGS[args.config]
    gather = args.gather or (args.config == "mixed" and world > 1)
    # weak scaling: the global fleet holds B x world robots of each model; this rank owns the contiguous
    # shard [rank*B, (rank+1)*B) of it (sharding.shard_range), no collective on the solve path
    fleets = []
    multi = len(cfg["models"]) > 1
    for j, (m, B) in enumerate(cfg["models"]):
        lo, hi = shard_range(B * world, rank, world)
        fleets.append(Fleet(m, hi - lo, cfg["N"], DEFAULT_SEED + cfg["idx"] + 100 * j, dev, start=lo,
                            stream=torch.cuda.Stream(dev) if multi else None))
    torch.cuda.synchronize()
    main_stream = torch.cuda.current_stream()

    def tick_all():
        """One tick of every model's fleet. A mixed fleet runs its models' kernels concurrently, one HIP stream
        each (every launch alone would leave SIMDs idle: ~2730 robots = 683 waves), joined on the main stream."""
        if not multi:
            fleets[0].tick()
            return
        start = torch.cuda.Event()
        start.record(main_stream)
        for f in fleets:
            f.stream.wait_event(start)
            f.tick()
            done = torch.cuda.Event()
            done.record(f.stream)
            main_stream.wait_event(done)
    B_rank = sum(f.B for f in fleets)
    cmd_gather = CommandGather(5, [B_rank] * world, dev) if gather else None

    def gather_commands():
        cmd_gather([torch.cat([f.u0, f.status.float()[None]]) for f in fleets])

    # executed IPM iterations and failures, accumulated on the device over the timed ticks
    iters_sum = torch.zeros(B_rank, dtype=torch.int64, device=dev)
    iters_max = torch.zeros(B_rank, dtype=torch.int32, device=dev)
    fail_cnt = torch.zeros(B_rank, dtype=torch.int64, device=dev)
    offs = [int(v) for v in np.cumsum([0] + [f.B for f in fleets])]

    def accumulate():
        for j, f in enumerate(fleets):
            sl = slice(offs[j], offs[j + 1])
            iters_sum[sl] += f.qp_iter
            torch.maximum(iters_max[sl], f.qp_iter, out=iters_max[sl])
            fail_cnt[sl] += f.status != 0

    # warmup runs every op of the timed loop (the first use of a torch kernel loads its code object)
    for _ in range(args.closed_loop_warmup + args.warmup):
        tick_all()
        accumulate()
        if gather:
            gather_commands()
    for t_ in (iters_sum, iters_max, fail_cnt):
        t_.zero_()
    torch.cuda.synchronize()

    # per-kernel timing of the solve launches with HIP events on the launch stream
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    with TimedRegion(dev) as region:
        for k in range(args.steps):
            if multi:
                tick_all()
            else:
                f = fleets[0]
                ev[k][0].record(stream)
                f.solve()
                ev[k][1].record(stream)
                f.advance()
            accumulate()
            if gather:
                gather_commands()
    elapsed = region.elapsed

    kernel_ms = [ev[k][0].elapsed_time(ev[k][1]) for k in range(args.steps)] if len(fleets) == 1 else None
    k_mean = float(iters_sum.sum().item()) / (B_rank * args.steps)
    units = args.steps * B_rank * world
    value = units / elapsed

    result = None
    if rank == 0:
        roof = None
        if kernel_ms:
            f = fleets[0]
            t_k = float(np.mean(kernel_ms)) * 1e-3
            flops = f.B * flops_per_instance(f.model, f.N, k_mean)
            achieved = flops / t_k / 1e12
            traffic = None
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                with open(pmc) as fh:
                    d = json.load(fh)
                key = f"{f.model}_N{f.N}_B{f.B}"
                traffic = d.get(key, {}).get("hbm_bytes_per_launch")
            roof = {"bound": "mfma", "achieved": round(achieved, 4), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(achieved / FP32_PEAK_TFLOPS, 6), "traffic": traffic,
                    "kernel": f"k_sqp_rti_{f.solver.kernel}", "kernel_ms_mean": round(t_k * 1e3, 4),
                    "algorithmic_flop_per_launch": flops, "qp_iter_mean": round(k_mean, 3),
                    "compulsory_bytes_per_launch": f.B * bytes_per_instance(f.model, f.N),
                    "achieved_compulsory_GBs": round(f.B * bytes_per_instance(f.model, f.N) / t_k / 1e9, 2),
                    "note": "FP32 VALU-bound (no GEMM-sized blocks); peak = MI355X FP32 vector = FP32 MFMA rate"}
        cpu = None
        u0_err = None
        if not args.no_cpu_baseline and world == 1:
            nthreads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
            cpu_rate, u0_err, nf, ns, rate_1 = cpu_baseline(fleets, dev, args.cpu_sample, args.cpu_ticks, nthreads)
            cpu = {"value": round(cpu_rate, 1), "unit": "SQP-RTI iterations/sec", "cores": nthreads, "kind": "port",
                   "sample": f"{ns} instance-iterations: first {args.cpu_sample} robots of each model x "
                             f"{args.cpu_ticks} closed-loop ticks after the timed region, fp64 oracle/nmpc_oracle.c, "
                             f"OpenMP {nthreads} threads, identical inputs", "failed": nf,
                   "value_1core": round(rate_1, 1)}
        result = {
            "metric": "SQP-RTI iterations/sec (whole node), diff N=40 batch=4096; u0 max-abs err",
            "value": round(value, 1), "unit": "SQP-RTI iterations/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32+fp64",
            "data": "synthetic seeded closed-loop fleet (SURVEY 8d), random-arc paths + goal poses",
            "config": {"workload": cfg["desc"], "config": args.config, "N": cfg["N"],
                       "batch_per_gpu": B_rank, "global_batch": B_rank * world,
                       "models": [m for m, _ in cfg["models"]], "parallelism": f"instance-sharded x{world}",
                       "closed_loop_warmup_ticks": args.closed_loop_warmup, "rccl_gather": gather},
            "u0_max_abs_err": u0_err, "qp_iter_mean": round(k_mean, 3), "qp_iter_max": int(iters_max.max().item()),
            "failed_solves": int(fail_cnt.sum().item()), "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
