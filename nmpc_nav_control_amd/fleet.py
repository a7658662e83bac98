"""A rank's closed-loop robot fleet: the driver loop bench.py times and the multi-GPU tests run.

One ``Fleet`` is one model's robots on this rank (solver handle + device-resident closed-loop state); a
``FleetNode`` is every model's fleet of one rank plus the per-tick bookkeeping of the whole-fleet config
(BASELINE config 5): concurrent per-model launches on their own HIP streams, device-side IPM statistics, and
the optional all-gather of u0 + status (RCCL over xGMI, sharding.CommandGather).

The reference runs one robot per ROS node (``NMPCNavControlROS::executeNMPC``, NMPCNavControlROS.cpp:700-719,
one ``run()`` per control tick); a ``Fleet`` tick is that call for B robots at once: the batched
``NMPCNavControl*::run`` followed by the harness plant / reference step (fleet_sim.hip).

The solver is pluggable (``solver_factory``): ``BatchSolver`` (libnmpc_amd.so) everywhere in the product and
the benches; the CPU multi-process tests plug an fp64 oracle-backed object with the same methods (state, run,
fleet_sim_step, set_schedule, nu) so that the code they exercise is this module, not a test-only copy.
"""
import os

import numpy as np
import torch

from .scenario import RENEW, SPEED, kappa_max_of, make_fleet
from .sharding import CommandGather, shard_range


class Fleet:
    """One model's robots on this rank: solver + closed-loop state, all resident on ``dev``.

    renew: the stationary loop (scenario.RENEW, nmpc_fleet_sim_step_renew): an arrived robot, or one whose goal /
    path has been active for its ttl, gets a new one and its next solve resets the controller (the reference's goal
    / path callbacks call reset_mpc, NMPCNavControlROS.cpp:304-327); a dict overrides RENEW's keys (the tests use
    short ttls). False: every robot keeps its first goal / path (the fleet parks), as round-2 benches ran."""

    def __init__(self, model, B, N, seed, dev, start=0, stream=None, solver_factory=None, schedule=None, renew=True,
                 record_layout=None):
        self.model, self.B, self.N = model, B, N
        self.seed, self.start = int(seed), int(start)
        self.dev = torch.device(dev)
        self.stream = stream  # None: the current stream; mixed fleets give each model its own HIP stream
        if solver_factory is None:
            from .batch import BatchSolver
            solver_factory = BatchSolver
        self.solver = solver_factory(model, N, B, device=self.dev)
        if schedule is not None and "NMPC_AMD_SCHED" not in os.environ:
            self.solver.set_schedule(schedule)
        if record_layout is not None and "NMPC_AMD_REC_SPLIT" not in os.environ:
            self.solver.set_record_layout(record_layout)
        fl = make_fleet(model, B, seed=seed, start=start)
        self.is_path = fl["is_path"]
        t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev, dt)  # noqa: E731
        self.pose, self.vel, self.path, self.s = t(fl["pose"]), t(fl["vel"]), t(fl["path"]), t(fl["s"])
        self.steer = t(fl["steer"]) if model == "tric" else None
        _, _, cr = self.solver.state()
        cr.copy_from(t(fl["carried"]))
        self.traj = torch.zeros(N + 1, 3, B, device=self.dev)
        self.tlen = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.cmd = torch.zeros(3, B, device=self.dev)
        self.u0 = torch.zeros(self.solver.nu, B, device=self.dev)
        self.status = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.qp_iter = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.renew = None
        if renew:
            self.renew = dict(RENEW, kappa_max=kappa_max_of(model), speed=SPEED.get(model, (0.2, 0.8)))
            if isinstance(renew, dict):
                self.renew.update(renew)
        self.ev = t(fl["ev"], torch.int32)
        self.ttl = t(np.minimum(fl["ttl"], self.renew["ttl_max"]) if self.renew else fl["ttl"], torch.int32)
        self.reset = torch.zeros(B, dtype=torch.uint8, device=self.dev)  # set by the renewal for the next solve
        self.solver.fleet_sim_step(self.path, self.s, self.pose, self.vel, self.steer, None, None, self.traj,
                                   self.tlen, advance=False, stream=self.stream)

    def solve(self):
        self.solver.run(self.pose, self.vel, self.traj, steer=self.steer, traj_len=self.tlen,
                        reset=self.reset if self.renew else None, cmd=self.cmd, u0=self.u0, status=self.status,
                        qp_iter=self.qp_iter, stream=self.stream)

    def advance(self, stats=None):
        """The plant / reference step after a solve; stats (renewal only): FleetNode's device statistics of this
        fleet, accumulated by the same launch (nmpc_fleet_stats)."""
        if self.renew:
            kw = {"stats": stats} if stats is not None else {}
            self.solver.fleet_sim_step_renew(self.path, self.s, self.pose, self.vel, self.steer, self.u0, self.status,
                                             self.traj, self.tlen, self.ev, self.ttl, self.reset, self.seed,
                                             self.start, self.renew, stream=self.stream, **kw)
        else:
            self.solver.fleet_sim_step(self.path, self.s, self.pose, self.vel, self.steer, self.u0, self.status,
                                       self.traj, self.tlen, advance=True, stream=self.stream)

    def tick(self):
        self.solve()
        self.advance()

    def snapshot(self):
        """Host copies (float64, robot-major) of everything a solve reads: the oracle replay inputs."""
        host = lambda a: np.ascontiguousarray(a.cpu().numpy(), np.float64)  # noqa: E731
        xv, uv, cv = self.solver.state()
        X, U, C = xv.to_tensor(), uv.to_tensor(), cv.to_tensor()
        B, N = self.B, self.N
        nx, nu = X.shape[0] // (N + 1), U.shape[0] // N
        return dict(xbar=np.ascontiguousarray(host(X[:, :B]).T.reshape(B, N + 1, nx)),
                    ubar=np.ascontiguousarray(host(U[:, :B]).T.reshape(B, N, nu)),
                    carried=np.ascontiguousarray(host(C[:, :B]).T),
                    pose=np.ascontiguousarray(host(self.pose).T), vel=np.ascontiguousarray(host(self.vel).T),
                    steer=host(self.steer) if self.steer is not None else None,
                    traj=np.ascontiguousarray(host(self.traj).transpose(2, 0, 1)),
                    tlen=np.ascontiguousarray(self.tlen.cpu().numpy(), np.int32),
                    reset=(np.ascontiguousarray(self.reset.cpu().numpy(), np.uint8) if self.renew else None))


class FleetNode:
    """Every model's fleet of one rank (weak scaling: rank r owns robots [r*B, (r+1)*B) of each model's
    seeded global fleet, sharding.shard_range), ticked together.

    models: [(model, B_per_rank), ...]. Each model's robots may be split further into ``groups`` contiguous
    stream groups (Fleet objects with their own HIP stream and handle; make_fleet(start=...) keeps every
    robot's data a function of its global index, so the robots are the same for any grouping).

    Launches on several streams (several models, or groups > 1) run concurrently. ``decoupled`` picks how the
    streams advance:
      * joined (False): every tick starts after the previous tick of every stream ended (one fleet-wide tick
        boundary per step);
      * decoupled (True, the default with several streams): each stream runs its own closed loop (solve ->
        plant/reference step -> statistics) with no cross-stream wait; the step boundary is only a count. A
        solve launch ends with its slowest wave (its hardest robot), and while it drains, the SIMDs its finished
        waves freed run the next launches of the other streams.
    With one stream (a single model, groups = 1) both are the same sequential loop.

    gather: the per-tick all-gather of [u0; status] of every robot to every rank (RCCL over xGMI). Joined ticks
    gather at the tick boundary; decoupled streams stage their commands into a double-buffered slot when their
    own tick is done, and a gather stream all-gathers the slot once every fleet's part of that tick has arrived
    (a fleet waits only before overwriting a slot whose gather, two ticks back, has not finished). On the CPU
    (gloo tests) the same code runs without streams."""

    def __init__(self, models, N, seed, dev, rank=0, world=1, gather=False, solver_factory=None, groups=1,
                 decoupled=None, schedule=None, renew=True):
        self.dev = torch.device(dev)
        self.rank, self.world = rank, world
        cuda = self.dev.type == "cuda"
        self.cuda = cuda
        self.groups = max(1, int(groups))
        self.multi = (len(models) > 1 or self.groups > 1) and cuda
        # CPU: decoupled=True runs the decoupled code path (staged gather) sequentially, for the gloo tests
        self.decoupled = self.multi if decoupled is None else (bool(decoupled) and (self.multi or not cuda))
        self.fleets = []
        for j, (m, B) in enumerate(models):
            lo, hi = shard_range(B * world, rank, world)
            for g in range(self.groups):
                glo, ghi = shard_range(hi - lo, g, self.groups)
                if ghi <= glo:
                    continue
                stream = torch.cuda.Stream(self.dev) if self.multi else None
                sched = schedule if schedule is not None else ("interleaved" if len(models) > 1 and stream is not None
                                                               else None)
                # diff's record layout: the handle's own choice alone (wide for the metric fleet), the split planes
                # beside other models' records on the same device (mixed: 5.25 -> 5.70 M it/s).
                # Decided here, once, from the node's configuration: no other handle can flip it
                layout = "split" if (m == "diff" and len(models) > 1 and cuda) else None
                self.fleets.append(Fleet(m, ghi - glo, N, seed + 100 * j, self.dev, start=lo + glo, stream=stream,
                                         solver_factory=solver_factory, schedule=sched, renew=renew,
                                         record_layout=layout))
        self.B = sum(f.B for f in self.fleets)
        self.offs = [int(v) for v in np.cumsum([0] + [f.B for f in self.fleets])]
        self.gather = CommandGather(5, [self.B] * world, self.dev) if gather else None
        self.gathered = None
        self.tick_no = 0
        if gather and self.decoupled and cuda:
            self.gstream = torch.cuda.Stream(self.dev)
            self.ev_staged = [[torch.cuda.Event() for _ in range(self.gather.slots)] for _ in self.fleets]
            self.ev_gdone = [torch.cuda.Event() for _ in range(self.gather.slots)]
        # executed IPM iterations and failures, accumulated on the device
        self.iters_sum = torch.zeros(self.B, dtype=torch.int64, device=self.dev)
        self.iters_max = torch.zeros(self.B, dtype=torch.int32, device=self.dev)
        self.fail_cnt = torch.zeros(self.B, dtype=torch.int64, device=self.dev)
        # per-fleet histograms of the executed IPM iterations (robot-ticks; the tail of the window) and the
        # count / iterations of the solves that followed a renewal (cold: reset iterate, cold IPM)
        self.iter_hist = [torch.zeros(64, dtype=torch.int64, device=self.dev) for _ in self.fleets]
        self._ones = torch.ones(max([f.B for f in self.fleets] + [1]), dtype=torch.int64, device=self.dev)
        self.cold_cnt = torch.zeros(self.B, dtype=torch.int64, device=self.dev)
        self.cold_iters = torch.zeros(self.B, dtype=torch.int64, device=self.dev)
        # the statistics of a renewing fleet on the device solver go into its plant / renewal launch (one launch per
        # tick instead of a dozen small torch ops on the fleet's stream); accumulate_one is the general form
        self.fused = []
        for j, f in enumerate(self.fleets):
            sl = slice(self.offs[j], self.offs[j + 1])
            ok = (cuda and f.renew is not None and getattr(f.solver, "fused_stats", False)
                  and os.environ.get("NMPC_FLEET_FUSED_STATS", "1") != "0")
            self.fused.append(dict(qp_iter=f.qp_iter, iters_sum=self.iters_sum[sl], iters_max=self.iters_max[sl],
                                   fail_cnt=self.fail_cnt[sl], hist=self.iter_hist[j], cold_cnt=self.cold_cnt[sl],
                                   cold_iters=self.cold_iters[sl]) if ok else None)

    def tick_all(self):
        """One control tick of every robot of this rank (joined: with the fleet-wide tick boundary)."""
        if not self.multi:
            for f in self.fleets:
                f.tick()
            return
        if self.decoupled:
            for f in self.fleets:
                f.tick()
            return
        main = torch.cuda.current_stream(self.dev)
        start = torch.cuda.Event()
        start.record(main)
        for f in self.fleets:
            f.stream.wait_event(start)
            f.tick()
            done = torch.cuda.Event()
            done.record(f.stream)
            main.wait_event(done)

    def accumulate_one(self, j):
        """Statistics of fleet j's last solve, on fleet j's stream (or the current one); called between the solve
        and the plant / renewal step, which rewrites the reset flags the solve ran with."""
        f = self.fleets[j]
        sl = slice(self.offs[j], self.offs[j + 1])
        ctx = torch.cuda.stream(f.stream) if f.stream is not None else _nullctx()
        with ctx:
            self.iters_sum[sl] += f.qp_iter
            torch.maximum(self.iters_max[sl], f.qp_iter, out=self.iters_max[sl])
            self.fail_cnt[sl] += f.status != 0
            # scatter_add, not bincount: torch.bincount sizes its output from the data (a device -> host sync)
            self.iter_hist[j].scatter_add_(0, f.qp_iter.clamp(0, 63).long(), self._ones[:f.B])
            if f.renew:
                cold = f.reset.to(torch.int64)  # the flags this solve ran with (advance() rewrites them)
                self.cold_cnt[sl] += cold
                self.cold_iters[sl] += cold * f.qp_iter

    def join(self):
        """Make the current stream wait for every fleet stream and the gather stream (end of a decoupled run)."""
        if self.multi:
            main = torch.cuda.current_stream(self.dev)
            for st in [f.stream for f in self.fleets] + ([self.gstream] if hasattr(self, "gstream") else []):
                done = torch.cuda.Event()
                done.record(st)
                main.wait_event(done)

    def reset_stats(self):
        self.join()
        for t_ in (self.iters_sum, self.iters_max, self.fail_cnt, self.cold_cnt, self.cold_iters, *self.iter_hist):
            t_.zero_()

    def iter_stats(self):
        """Executed IPM iterations over the robot-ticks since reset_stats: mean, p50, p99, p99.9, max (all fleets),
        and the solves after a renewal (count, mean iterations)."""
        h = torch.stack(self.iter_hist).sum(0).cpu().numpy().astype(np.float64)
        n = h.sum()
        if n == 0:
            return {}
        c = np.cumsum(h) / n
        q = lambda p: int(np.searchsorted(c, p))  # noqa: E731
        cold = int(self.cold_cnt.sum().item())
        return {"mean": float((np.arange(64) * h).sum() / n), "p50": q(0.5), "p99": q(0.99), "p999": q(0.999),
                "max": int(np.nonzero(h)[0].max()), "robot_ticks": int(n), "renewals": cold,
                "cold_mean": (float(self.cold_iters.sum().item()) / cold) if cold else None}

    def _stage(self, j, f, slot):
        """Fleet j's [u0 (rows nu..3 stay 0); status] of this tick into staging slot `slot`, on its stream, after
        the gather that last read the slot (two ticks back) has finished."""
        ctx = torch.cuda.stream(f.stream) if (self.cuda and f.stream is not None) else _nullctx()
        with ctx:
            if self.cuda and self.tick_no >= self.gather.slots:
                torch.cuda.current_stream(self.dev).wait_event(self.ev_gdone[slot])
            sb = self.gather.stage_bufs[slot]
            lo, hi = self.offs[j], self.offs[j + 1]
            sb[:f.u0.shape[0], lo:hi].copy_(f.u0)
            sb[4, lo:hi].copy_(f.status)
            if self.cuda:
                self.ev_staged[j][slot].record(torch.cuda.current_stream(self.dev))

    def _collect(self, slot):
        """All-gather staging slot `slot` on the gather stream once every fleet's part has been staged."""
        ctx = torch.cuda.stream(self.gstream) if self.cuda else _nullctx()
        with ctx:
            if self.cuda:
                for evs in self.ev_staged:
                    self.gstream.wait_event(evs[slot])
            self.gathered = self.gather.collect(slot)
            if self.cuda:
                self.ev_gdone[slot].record(self.gstream)

    def gather_commands(self):
        """All-gather [u0 (padded to 4 rows); status] of every robot to every rank: [5][B * world]."""
        if self.gather is not None:
            self.gathered = self.gather([torch.cat([f.u0, f.status.float()[None]]) if f.u0.shape[0] == 4 else
                                         torch.cat([f.u0, torch.zeros(4 - f.u0.shape[0], f.B, device=self.dev),
                                                    f.status.float()[None]]) for f in self.fleets])
        return self.gathered

    def step(self, timer=None):
        """One step of bench.py's timed region: every robot ticks once (solve -> plant / reference step), the
        statistics accumulate on the device, and (optional) the commands are all-gathered.

        timer: None, or an object with ``start(j, stream)`` / ``end(j, stream)`` called around fleet j's solve
        launch on the stream it runs on (bench.py records HIP events there). Joined streams start every fleet
        from one point of the current stream, so ``start`` is called once, with j = -1."""
        if self.decoupled:
            slot = self.tick_no % 2
            for j, f in enumerate(self.fleets):
                if timer is not None:
                    timer.start(j, f.stream)
                f.solve()
                if timer is not None:
                    timer.end(j, f.stream)
                if self.fused[j] is None:
                    self.accumulate_one(j)
                if self.gather is not None:
                    self._stage(j, f, slot)
                f.advance(self.fused[j])
            if self.gather is not None:
                self._collect(slot)
            self.tick_no += 1
            return
        cuda = self.dev.type == "cuda"
        main = torch.cuda.current_stream(self.dev) if cuda else None
        if timer is not None:
            timer.start(-1, main)
        if self.multi:
            start = torch.cuda.Event()
            start.record(main)
            for f in self.fleets:
                f.stream.wait_event(start)
        for j, f in enumerate(self.fleets):
            f.solve()
            if timer is not None:
                timer.end(j, f.stream if f.stream is not None else main)
            if self.fused[j] is None:
                self.accumulate_one(j)
            f.advance(self.fused[j])
            if self.multi:
                done = torch.cuda.Event()
                done.record(f.stream)
                main.wait_event(done)
        if self.gather is not None:
            self.gather_commands()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
