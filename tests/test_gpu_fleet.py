"""Bench-scale GPU parity: every robot of every BASELINE config replayed through the fp64 oracle, the mixed
fleet of BASELINE config 5 on concurrent streams, and per-robot failure isolation.

All three drive the shipping driver loop (nmpc_nav_control_amd/fleet.py: the code bench.py times). A replay
takes the GPU's pre-tick state of every robot (warm iterate, carried refs, measurements, references), runs the
oracle's batch_tick (prepare -> SQP-RTI -> post, NMPCNavControl*::run) on it, and compares with the GPU tick:
  |u0 - u0_oracle|_inf <= 1e-3 and the predicted state trajectory (the new iterate x_1..x_N) within 1e-3,
  SURVEY.md 8d; the GPU IPM stops by its fp32 rule, the oracle by its fp64 rule (DESIGN.md "Stopping rule").
"""
import os

import numpy as np
import pytest
import torch

from nmpc_nav_control_amd.batch import BatchSolver
from nmpc_nav_control_amd.fleet import Fleet, FleetNode
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_U = 1e-3
TOL_X = 1e-3
SEED = 20250824
NTHREADS = int(os.environ.get("OMP_NUM_THREADS", "16"))


def replay_and_compare(fleet, oracle, tick_fn):
    """Snapshot the fleet's pre-tick state, run `tick_fn` (the GPU solve), replay every robot through the
    oracle; returns (u0 err, x err, GPU statuses, oracle statuses, GPU iterate [B][N+1][NX])."""
    torch.cuda.synchronize()
    sn = fleet.snapshot()
    tick_fn()
    torch.cuda.synchronize()
    xb_o, ub_o, cr_o = sn["xbar"].copy(), sn["ubar"].copy(), sn["carried"].copy()
    nf, cmd_o, u0_o, st_o, _ = oracle.batch_tick(sn["pose"], sn["vel"], sn["steer"], sn["traj"], sn["tlen"], sn["reset"],
                                                 cr_o, xb_o, ub_o, nthreads=NTHREADS)
    after = fleet.snapshot()
    st = fleet.status.cpu().numpy()
    ok = (st == 0) & (st_o == 0)
    eu = float(np.abs(fleet.u0.cpu().numpy().T[ok] - u0_o[ok]).max()) if ok.any() else 0.0
    ex = float(np.abs(after["xbar"][ok] - xb_o[ok]).max()) if ok.any() else 0.0
    ec = float(np.abs(fleet.cmd.cpu().numpy().T[ok] - cmd_o[ok]).max()) if ok.any() else 0.0
    return eu, max(ex, 0.0), ec, st, st_o, after["xbar"]


@pytest.mark.parametrize("model,N,B,idx,layout,rules", [("diff", 40, 4096, 1, "wide", "product"),
                                                        ("diff", 40, 4096, 1, "split", "product"),
                                                        ("diff", 40, 4096, 1, "wide", "acados"),
                                                        ("diff", 40, 1024, 1, None, "product"),
                                                        ("omni4", 40, 4096, 2, "wide", "product"),
                                                        ("tric", 60, 8192, 3, "split", "product")])
def test_bench_config_full_batch_replay(built, model, N, B, idx, layout, rules):
    """BASELINE configs at full batch (the bench's own fleets): 20 closed-loop ticks with no failed solve, then
    two ticks on which EVERY robot is replayed through the fp64 oracle. The metric config runs once per record
    layout of diff's team kernel (wide: its own default alone on the device, what bench.py's metric line runs;
    split: the mixed fleet's), and the layout the launches took is asserted. tric: >= 10 % of
    the robots have their steering reference alpha_ref on its 45 deg bound somewhere on the horizon (SURVEY 8d
    config 4; NMPCNavControlTric.cpp:24-29, scripts/tric/generate_c_code.py:47-57). rules "acados": the metric
    fleet with HPIPM's defaults instead of the product's IPM rules (bench.py ACADOS_RULES: no infeasibility exit,
    thr0 0.5, cold QP starts), replayed through the oracle's acados rule."""
    import bench
    f = Fleet(model, B, N, SEED + idx, DEV, record_layout=layout if model == "diff" else None,
              solver_factory=bench._factory(None, rules))
    plan = f.solver.plan_ex(B, "run")
    if layout is None:
        assert plan["kernel"] == "rowpar", plan  # diff1024: the segmented row-parallel kernel
    else:
        assert plan["kernel"] == "team" and plan["record_layout"] == layout, plan
    if rules == "acados":
        prm = f.solver.params
        assert prm.qp_infeas_lambda == 0.0 and prm.qp_thr0 == 0.5 and prm.qp_warm_start == 0
    o = Oracle(model, N, rule="batched" if rules == "product" else "acados")
    for tick in range(20):
        f.tick()
        if tick % 5 == 4:
            st = f.status.cpu().numpy()
            assert (st == 0).all(), (tick, np.nonzero(st)[0][:8])
    worst_u = worst_x = worst_c = 0.0
    for _ in range(2):
        eu, ex, ec, st, st_o, xb = replay_and_compare(f, o, f.solve)
        assert (st == 0).all() and (st_o == 0).all(), (np.nonzero(st)[0][:8], np.nonzero(st_o)[0][:8])
        worst_u, worst_x, worst_c = max(worst_u, eu), max(worst_x, ex), max(worst_c, ec)
        if model == "tric":
            on_bound = (np.abs(xb[:, 1:, 6]) >= np.pi / 4 - 1e-3).any(axis=1)
            assert on_bound.mean() >= 0.10, on_bound.mean()
        f.advance()
    print(f"\n{model} N={N} B={B} {rules}: all robots, 2 ticks: u0 err {worst_u:.2e}, x err {worst_x:.2e}, "
          f"cmd {worst_c:.2e}")
    assert worst_u <= TOL_U, worst_u
    assert worst_x <= TOL_X, worst_x
    assert worst_c <= TOL_U, worst_c


MIXED = [("diff", 2731), ("omni4", 2731), ("tric", 2730)]  # bench.py "mixed": 8192 per GPU of 65536 on 8


def test_mixed_fleet_concurrent_streams_full_replay(built):
    """BASELINE config 5 on one GPU (this rank's 8192 robots of the 65536 fleet): the three models' solves run
    concurrently on their own HIP streams with interleaved team placement (FleetNode, as bench.py --config
    mixed). Every robot of every model is replayed through the oracle on two ticks; and a run of the same
    three fleets one after the other on the default stream gives bit-identical commands."""
    N = 40
    node = FleetNode(MIXED, N, SEED + 4, DEV)
    assert node.multi and all(f.stream is not None for f in node.fleets)
    seq = [Fleet(m, b, N, SEED + 4 + 100 * j, DEV) for j, (m, b) in enumerate(MIXED)]
    oracles = [Oracle(m, N, rule="batched") for m, _ in MIXED]
    for tick in range(20):
        node.step()
        for f in seq:
            f.tick()
        torch.cuda.synchronize()
        for fa, fb in zip(node.fleets, seq):
            assert torch.equal(fa.u0, fb.u0) and torch.equal(fa.cmd, fb.cmd), (tick, fa.model)
            assert torch.equal(fa.status, fb.status) and (fa.status == 0).all(), (tick, fa.model)
    assert int(node.fail_cnt.sum()) == 0
    for _ in range(2):
        snaps = [f.snapshot() for f in node.fleets]
        torch.cuda.synchronize()
        node.tick_all()
        torch.cuda.synchronize()
        for f, o, sn in zip(node.fleets, oracles, snaps):
            xb_o, ub_o, cr_o = sn["xbar"].copy(), sn["ubar"].copy(), sn["carried"].copy()
            _, cmd_o, u0_o, st_o, _ = o.batch_tick(sn["pose"], sn["vel"], sn["steer"], sn["traj"], sn["tlen"], sn["reset"],
                                                   cr_o, xb_o, ub_o, nthreads=NTHREADS)
            st = f.status.cpu().numpy()
            assert (st == 0).all() and (st_o == 0).all(), f.model
            eu = float(np.abs(f.u0.cpu().numpy().T - u0_o).max())
            ex = float(np.abs(f.snapshot()["xbar"] - xb_o).max())
            print(f"\nmixed/{f.model} B={f.B}: u0 err {eu:.2e}, x err {ex:.2e}")
            assert eu <= TOL_U and ex <= TOL_X, (f.model, eu, ex)


@pytest.mark.parametrize("model,N,B,idx", [("diff", 40, 4096, 1), ("tric", 60, 8192, 3)])
def test_stream_groups_decoupled_bit_identical(built, model, N, B, idx):
    """bench.py's metric and tric configs split each fleet into 2 stream groups whose closed loops run decoupled
    on their own HIP streams (FleetNode groups=2). The groups hold the same robots (make_fleet(start=...)), so
    after 15 ticks every robot's u0, command, status and IPM statistics equal the single-stream run bit for
    bit, and the decoupled node really did run on two streams without a fleet-wide tick boundary."""
    one = FleetNode([(model, B)], N, SEED + idx, DEV)
    two = FleetNode([(model, B)], N, SEED + idx, DEV, groups=2)
    assert not one.multi and two.multi and two.decoupled and len(two.fleets) == 2
    assert [f.B for f in two.fleets] == [B // 2, B // 2]
    for _ in range(15):
        one.step()
        two.step()
    torch.cuda.synchronize()
    f1 = one.fleets[0]
    for name in ("u0", "cmd", "status", "qp_iter"):
        cat = torch.cat([getattr(f, name) for f in two.fleets], dim=-1)
        assert torch.equal(getattr(f1, name), cat), name
    assert torch.equal(one.iters_sum, two.iters_sum) and torch.equal(one.fail_cnt, two.fail_cnt)
    assert int(two.fail_cnt.sum()) == 0


def _restore(f, st):
    f.solver.restore_state(st["handle"])  # iterate, carried refs and the IPM warm-start state
    for k in ("pose", "vel", "traj", "tlen"):
        getattr(f, k).copy_(st[k])


def _save(f):
    X, U, C = (v.to_tensor() for v in f.solver.state())
    return dict(handle=f.solver.save_state(), X=X, U=U, C=C, pose=f.pose.clone(), vel=f.vel.clone(),
                traj=f.traj.clone(), tlen=f.tlen.clone())


def _outputs(f):
    xv, uv, cv = f.solver.state()
    return dict(u0=f.u0.clone(), cmd=f.cmd.clone(), status=f.status.clone(), qp_iter=f.qp_iter.clone(),
                X=xv.to_tensor(), U=uv.to_tensor(), C=cv.to_tensor())


def _timed_solve(f, setup, reps=7):
    """Median kernel time of `reps` solves of the same tick (`setup` restores the pre-tick state each time)."""
    ms = []
    for _ in range(reps):
        setup()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f.solve()
        b.record()
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.median(ms))


def test_failure_stays_on_its_robot(built):
    """a NaN or a QP failure on one robot must not poison the others. In a B=4096 diff N=40 tick
    (the metric config) robot 7 gets a NaN pose (x0), robot 1001 NaN references (yref) and robot 2050 an
    infeasible QP (carried vel-ref 50 m/s against the 1 m/s bound at stage 1):
      - the NaN robots report status 1 after their first IPM iteration; the infeasible one reports status 4 (QP
        failure) from the IPM's infeasibility exit (diverging bound multipliers with an open bound residual,
        DESIGN.md "Stopping rule") well before qp_iter_max; a failed robot gets a zero (stop) command and keeps
        its carried refs and iterate: the reference throws (NMPCNavControl.cpp:14-23) and the node stops the robot
        (NMPCNavControlROS.cpp:716-719);
      - every other robot's u0, cmd, status, qp_iter, iterate and carried refs are bit-identical to the clean
        tick;
      - with all three injected the kernel time stays within 10 % of the clean tick: one hard robot does not
        hold the launch for 50 iterations."""
    N, B = 40, 4096
    f = Fleet("diff", B, N, SEED + 1, DEV)
    for _ in range(20):
        f.tick()
    torch.cuda.synchronize()
    st0 = _save(f)
    f.solve()
    clean = _outputs(f)
    assert (clean["status"] == 0).all()
    t_clean = _timed_solve(f, lambda: _restore(f, st0))

    bad_x0, bad_ref, bad_qp = 7, 1001, 2050

    def inject(with_qp):
        _restore(f, st0)
        f.pose[0, bad_x0] = float("nan")
        f.traj[:, :, bad_ref] = float("nan")
        if with_qp:
            xv, uv, cv = f.solver.state()
            C = st0["C"].clone()
            C[0, bad_qp] = 50.0
            cv.copy_from(C)

    inject(True)
    f.solve()
    dirty = _outputs(f)
    bad = [bad_x0, bad_ref, bad_qp]
    st, it = dirty["status"].cpu().numpy(), dirty["qp_iter"].cpu().numpy()
    assert st[bad_x0] == 1 and st[bad_ref] == 1 and it[bad_x0] == 0 and it[bad_ref] == 0, (st[bad], it[bad])
    assert st[bad_qp] == 4 and it[bad_qp] < 30, (st[bad_qp], it[bad_qp])
    good = np.ones(B, bool)
    good[bad] = False
    g = torch.from_numpy(good).to(DEV)
    for k in ("u0", "cmd", "X", "U", "C"):
        assert torch.equal(dirty[k][..., :B][..., g], clean[k][..., :B][..., g]), k
    for k in ("status", "qp_iter"):
        assert torch.equal(dirty[k][g], clean[k][g]), k
    for i in bad:
        if st[i] != 0:
            assert (dirty["cmd"][:, i] == 0).all(), i
            assert torch.equal(dirty["C"][:, i], st0["C"][:, i] if i != bad_qp else dirty["C"][:, i])
            assert torch.equal(dirty["X"][:, i], st0["X"][:, i]) and torch.equal(dirty["U"][:, i], st0["U"][:, i])

    t_bad = _timed_solve(f, lambda: inject(True))
    print(f"\nclean {t_clean:.3f} ms (max qp_iter {int(clean['qp_iter'].max())}), with 2 NaN robots and the "
          f"infeasible one {t_bad:.3f} ms; infeasible robot: status {st[bad_qp]}, qp_iter {it[bad_qp]}")
    assert t_bad <= 1.10 * t_clean, (t_bad, t_clean)


def test_layout_independent_of_other_handles(built):
    """a handle's record layout is its own, fixed at create. A metric fleet (4096 diff robots,
    107 MB of records: wide) ticks once undisturbed; then, from the same saved state, with a 214 MB diff handle
    (capacity 8192, split by its own size) created beside it and destroyed again, and once more with another large
    handle alive during the tick. Results, IPM counts, iterate and warm flags are bit-identical every time, and
    the fleet's plan never changes."""
    N, B = 40, 4096
    f = Fleet("diff", B, N, SEED + 1, DEV)
    for _ in range(20):
        f.tick()
    torch.cuda.synchronize()
    assert f.solver.plan_ex(B, "run")["record_layout"] == "wide"
    st0 = _save(f)

    def tick():
        f.solve()
        torch.cuda.synchronize()
        out = _outputs(f)
        out["warm"] = f.solver.warm_state()[0].to_tensor()
        return out

    ref = tick()
    assert int((ref["warm"][0, :B] == 1).sum()) > B // 2  # warm-started in the wide layout (NMPC_WARM_TAG_WIDE)
    big = BatchSolver("diff", N, 8192)
    p_big = big.plan_ex(8192, "run")
    assert p_big["record_layout"] == "split" and p_big["record_bytes"] > 200e6, p_big
    big.close()
    _restore(f, st0)
    got = tick()
    big2 = BatchSolver("diff", N, 8192)
    _restore(f, st0)
    got2 = tick()
    big2.close()
    for k in ref:
        assert torch.equal(got[k], ref[k]) and torch.equal(got2[k], ref[k]), k
    assert f.solver.plan_ex(B, "run")["record_layout"] == "wide"


def test_warm_tags_across_kernel_switch(built):
    """one tric handle alternates launches of 1025 robots (the team kernel, split record planes) and 1024
    robots (the segmented row-parallel kernel, wide records). Each robot's warm flag carries the tag of the layout
    its multipliers sit in (NMPC_WARM_TAG_SPLIT 2 / _WIDE 1), so a robot whose kernel changes starts cold on its own
    and no launch reads records another layout wrote; the robot outside the smaller launches keeps its flag. Every
    tick, every launched robot is replayed through the oracle from the GPU's pre-tick state."""
    N, BF = 40, 1025
    f = Fleet("tric", BF, N, SEED + 3, DEV)
    o = Oracle("tric", N, rule="batched")
    assert f.solver.plan_ex(BF, "run")["kernel"] == "team" and f.solver.plan_ex(BF - 1, "run")["kernel"] == "rowpar"
    for _ in range(6):
        f.tick()
    for tick in range(6):
        n = BF if tick % 2 == 0 else BF - 1
        torch.cuda.synchronize()
        warm_before = f.solver.warm_state()[0].to_tensor()[0, :BF].clone()
        sn = f.snapshot()
        sl = lambda a: None if a is None else np.ascontiguousarray(a[:n])  # noqa: E731
        cols = lambda t_: t_[..., :n].contiguous()  # noqa: E731
        u0 = torch.zeros(2, n, device=DEV)
        cmd = torch.zeros(3, n, device=DEV)
        status = torch.full((n,), -7, dtype=torch.int32, device=DEV)
        f.solver.run(cols(f.pose), cols(f.vel), cols(f.traj), steer=cols(f.steer), traj_len=cols(f.tlen),
                     reset=cols(f.reset), cmd=cmd, u0=u0, status=status)
        torch.cuda.synchronize()
        warm = f.solver.warm_state()[0].to_tensor()[0, :BF]
        tag = 2 if n == BF else 1
        assert set(warm[:n].unique().tolist()) <= {0, tag}, (tick, warm[:n].unique())
        assert int((warm[:n] == tag).sum()) > n // 2, tick
        if n < BF:
            assert int(warm[BF - 1]) == int(warm_before[BF - 1]), tick  # the robot outside the launch: untouched
        xb_o, ub_o, cr_o = sl(sn["xbar"]).copy(), sl(sn["ubar"]).copy(), sl(sn["carried"]).copy()
        _, cmd_o, u0_o, st_o, _ = o.batch_tick(sl(sn["pose"]), sl(sn["vel"]), sl(sn["steer"]), sl(sn["traj"]),
                                               sl(sn["tlen"]), sl(sn["reset"]), cr_o, xb_o, ub_o, nthreads=NTHREADS)
        st = status.cpu().numpy()
        assert (st == 0).all() and (st_o == 0).all(), tick
        eu = float(np.abs(u0.cpu().numpy().T - u0_o).max())
        assert eu <= TOL_U, (tick, n, eu)
        f.u0[:, :n] = u0
        f.cmd[:, :n] = cmd
        f.status[:n] = status
        f.advance()


def test_reset_mode_keeps_carried_refs(built):
    """nmpc_batch_init_iterate(mode=1) is {name}_acados_reset: the iterate is zeroed and the carried vel-ref
    states stay (as the per-robot reset mask does; NMPCNavControlDiff.cpp:177-181 resets only the capsule);
    mode 0 (create) also zeroes them."""
    s = BatchSolver("diff", 20, 64)
    xv, uv, cv = s.state()
    cv.copy_from(torch.full((2, 64), 0.3, device=DEV))
    uv.copy_from(torch.full((40, 64), 0.1, device=DEV))
    s.init_iterate(mode=1)
    torch.cuda.synchronize()
    assert (cv.to_tensor() == 0.3).all() and (uv.to_tensor() == 0).all() and (xv.to_tensor() == 0).all()
    s.init_iterate(mode=0)
    torch.cuda.synchronize()
    X = xv.to_tensor().reshape(21, 7, 64)
    assert (cv.to_tensor() == 0).all() and (X[:, 2] == np.float32(np.pi)).all()


def test_renewal_on_device(built):
    """The stationary loop on the device (nmpc_fleet_sim_step_renew): short ttls (2-6 ticks) make every robot renew
    its goal / path several times. Each renewal draws exactly the harness hash's values (ttl bit for bit; goal
    distance, heading, arc length and speed to fp32 rounding), sets the robot's reset flag for its next solve,
    and the reset solves match the fp64 oracle given the same flags (every robot replayed on the last tick)."""
    from nmpc_nav_control_amd.scenario import fleet_ttl, fleet_u
    lo, hi = 2, 6
    N, B, seed = 40, 1024, SEED + 1
    f = Fleet("diff", B, N, seed, DEV, renew=dict(ttl_min=lo, ttl_max=hi))
    o = Oracle("diff", N, rule="batched")
    gi = np.arange(B)
    total = 0
    for tick in range(12):
        f.solve()
        f.advance()
        torch.cuda.synchronize()
        st = f.status.cpu().numpy()
        assert (st == 0).all(), (tick, np.nonzero(st)[0][:8])
        r = f.reset.cpu().numpy().astype(bool)
        ev, ttl = f.ev.cpu().numpy(), f.ttl.cpu().numpy()
        path, pose, s = f.path.cpu().numpy(), f.pose.cpu().numpy(), f.s.cpu().numpy()
        total += int(r.sum())
        if not r.any():
            continue
        assert np.array_equal(ttl[r], fleet_ttl(seed, gi[r], ev[r], lo, hi))
        g = r & (path[5] < 0)
        p = r & (path[5] > 0)
        mx = lambda a: float(np.abs(a).max()) if a.size else 0.0  # noqa: E731
        u1 = fleet_u(seed, gi, ev, 1)
        u2 = fleet_u(seed, gi, ev, 2)
        dist = np.hypot(path[0] - pose[0], path[1] - pose[1])
        assert mx(dist[g] - (0.3 + 1.2 * u1[g])) < 1e-5
        assert mx(path[2, g] - np.pi * (2 * u2[g] - 1)) < 1e-5
        # progress restarts at 0 and is re-projected onto the new arc (its start lies within 0.2 m of the robot)
        assert ((s[p] >= 0) & (s[p] <= 0.2 + 1e-5)).all() and mx(dist[p] - 0.2 * u1[p]) < 1e-5
        assert mx(path[5, p] - (3.0 + 2.0 * fleet_u(seed, gi[p], ev[p], 5))) < 1e-5
        assert mx(path[4, p] - (0.2 + 0.6 * fleet_u(seed, gi[p], ev[p], 4))) < 1e-5
    assert total >= 2 * B, total
    eu, ex, ec, st, st_o, _ = replay_and_compare(f, o, f.solve)
    assert int(f.reset.sum()) > 0
    assert (st == 0).all() and (st_o == 0).all()
    print(f"\nrenewals {total} over 12 ticks; reset-tick replay: u0 err {eu:.2e}, x err {ex:.2e}")
    assert eu <= TOL_U and ex <= TOL_X and ec <= TOL_U


def test_decoupled_gather_on_device(built):
    """The whole-fleet command gather with decoupled streams (bench.py's mixed config at world > 1; here world 1,
    the same stream and event code): every tick's gathered [u0; status] equals the fleets' own outputs of that
    tick, while the three models' closed loops run on their own streams without a tick boundary."""
    node = FleetNode([("diff", 512), ("omni4", 256), ("tric", 300)], 40, SEED + 4, DEV, gather=True)
    assert node.decoupled and node.multi and node.gather is not None
    for _ in range(6):
        node.step()
        torch.cuda.synchronize()
        exp = torch.cat([torch.cat([f.u0, torch.zeros(4 - f.u0.shape[0], f.B, device=DEV), f.status.float()[None]])
                         for f in node.fleets], dim=1)
        assert torch.equal(node.gathered, exp)
    assert int(node.fail_cnt.sum()) == 0


def test_fused_statistics_equal_torch_ops(built):
    """The device statistics FleetNode accumulates inside the plant / renewal launch (nmpc_fleet_stats) equal the
    general torch form (accumulate_one) on the same closed loop: per-robot iteration sums and maxima, failures, the
    iteration histogram and the post-renewal (cold) counts, bit for bit. Short ttls make renewals frequent."""
    ren = dict(ttl_min=2, ttl_max=9)
    models = [("diff", 700), ("omni4", 300)]
    a = FleetNode(models, 40, SEED + 4, DEV, renew=ren)
    b = FleetNode(models, 40, SEED + 4, DEV, renew=ren)
    assert all(x is not None for x in a.fused)
    b.fused = [None] * len(b.fleets)
    for _ in range(15):
        a.step()
        b.step()
    a.join()
    b.join()
    torch.cuda.synchronize()
    for name in ("iters_sum", "iters_max", "fail_cnt", "cold_cnt", "cold_iters"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for ha, hb in zip(a.iter_hist, b.iter_hist):
        assert torch.equal(ha, hb)
    assert int(a.cold_cnt.sum()) > 0 and int(torch.stack(a.iter_hist).sum()) == 15 * a.B
    assert a.iter_stats() == b.iter_stats()
