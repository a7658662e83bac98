"""Seeded closed-loop regression harness: the batched counterpart of the reference's
scripts/test_scripts/acados_sim_*.py demos, which drive one acados solver in closed loop against its own model.

B robots of one model run T ticks entirely on the device: nmpc_batch_run (the wrapper's run: x0 packing, unwrap,
padding, terminal hack, SQP-RTI, vel-ref carry, inverse kinematics) then nmpc_fleet_sim_step (RK4 plant and new
references). Seeded resets ({name}_acados_reset, NMPCNavControlDiff.cpp:177-181) hit a fraction of the robots at
chosen ticks. At check ticks a robot sample is replayed through the fp64 oracle from the GPU's own pre-tick state
(iterate, carried vel-refs, measurements, references), which pins the multi-tick warm-start chain: no shift, the
x1 -> x0 carry (NMPCNavControlDiff.cpp:168-172) and the resets.

Test infrastructure (it calls the oracle): tests/test_gpu_sim_regress.py runs it small; as a script it writes a
JSON report:  python tests/sim_regress.py --model diff --N 40 --B 4096 --ticks 60 --out report.json
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(model, N, B, ticks, sample=64, check_every=10, reset_frac=0.02, reset_every=7, seed=20250824,
        kernel="team", device="cuda:0", dump=None):
    import torch

    from nmpc_nav_control_amd.batch import BatchSolver
    from nmpc_nav_control_amd.scenario import make_fleet
    from oracle.oracle import Oracle

    dev = torch.device(device)
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=dt)  # noqa
    host = lambda a: np.ascontiguousarray(a.cpu().numpy(), np.float64)  # noqa: E731
    fl = make_fleet(model, B, seed=seed)
    solver = BatchSolver(model, N, B, kernel=kernel)
    xv, uv, cv = solver.state()
    cv.copy_from(t(fl["carried"]))
    pose, vel, steer, path, s = t(fl["pose"]), t(fl["vel"]), t(fl["steer"]), t(fl["path"]), t(fl["s"])
    steer_arg = steer if model == "tric" else None
    traj = torch.zeros(N + 1, 3, B, device=dev)
    tlen = torch.zeros(B, dtype=torch.int32, device=dev)
    cmd = torch.zeros(3, B, device=dev)
    u0 = torch.zeros(solver.nu, B, device=dev)
    status = torch.zeros(B, dtype=torch.int32, device=dev)
    qp_iter = torch.zeros(B, dtype=torch.int32, device=dev)
    solver.fleet_sim_step(path, s, pose, vel, steer_arg, None, None, traj, tlen, advance=False)
    rng = np.random.default_rng([seed, 7])
    o = Oracle(model, N, rule="batched")
    S = min(sample, B)
    report = dict(model=model, N=N, B=B, ticks=ticks, sample=S, kernel=kernel, checks=[], failed=0, resets=0,
                  qp_iter_mean=0.0, qp_iter_max=0)
    it_sum = 0.0
    for tick in range(ticks):
        reset = None
        if reset_every and tick % reset_every == reset_every - 1:
            mask = (rng.uniform(size=B) < reset_frac).astype(np.uint8)
            mask[:S] |= (np.arange(S) % 8 == tick % 8).astype(np.uint8)  # sampled robots are reset too
            reset = t(mask, torch.uint8)
            report["resets"] += int(mask.sum())
        check = check_every and tick % check_every == check_every - 1
        if check:
            torch.cuda.synchronize()
            X, U, C = xv.to_tensor(), uv.to_tensor(), cv.to_tensor()
            args = (np.ascontiguousarray(host(pose[:, :S]).T), np.ascontiguousarray(host(vel[:, :S]).T),
                    host(steer[:S]) if model == "tric" else None,
                    np.ascontiguousarray(host(traj[:, :, :S]).transpose(2, 0, 1)),
                    np.ascontiguousarray(tlen[:S].cpu().numpy(), np.int32),
                    None if reset is None else reset[:S].cpu().numpy())
            carried = np.ascontiguousarray(host(C[:, :S]).T)
            xbar = np.ascontiguousarray(host(X[:, :S]).T.reshape(S, N + 1, o.nx))
            ubar = np.ascontiguousarray(host(U[:, :S]).T.reshape(S, N, o.nu))
        solver.run(pose, vel, traj, steer=steer_arg, traj_len=tlen, reset=reset, cmd=cmd, u0=u0, status=status,
                   qp_iter=qp_iter)
        torch.cuda.synchronize()
        st = status.cpu().numpy()
        qi = qp_iter.cpu().numpy()
        report["failed"] += int((st != 0).sum())
        it_sum += float(qi.mean())
        report["qp_iter_max"] = max(report["qp_iter_max"], int(qi.max()))
        if check:
            pre = (carried.copy(), xbar.copy(), ubar.copy())  # batch_tick advances them in place
            nf, cmd_o, u0_o, st_o, _ = o.batch_tick(*args, carried, xbar, ubar)
            ok = (st_o == 0) & (st[:S] == 0)
            eu = float(np.abs(u0[:, :S].cpu().numpy().T - u0_o)[ok].max()) if ok.any() else 0.0
            ec = float(np.abs(cmd[:, :S].cpu().numpy().T - cmd_o)[ok].max()) if ok.any() else 0.0
            report["checks"].append(dict(tick=tick, u0_err=eu, cmd_err=ec, oracle_failed=int(nf),
                                         status_mismatch=int((st_o != st[:S]).sum())))
            if dump is not None and eu > dump.get("u0_err", -1.0):
                err = np.abs(u0[:, :S].cpu().numpy().T - u0_o).max(axis=1)
                i = int(np.argmax(np.where(ok, err, -1.0)))
                dump.update(u0_err=eu, tick=tick, robot=i, pose=args[0][i], vel=args[1][i],
                            steer=0.0 if args[2] is None else args[2][i], traj=args[3][i], tlen=args[4][i],
                            reset=0 if args[5] is None else int(args[5][i]), carried=pre[0][i], xbar=pre[1][i],
                            ubar=pre[2][i], u0_gpu=u0[:, i].cpu().numpy(), u0_oracle=u0_o[i],
                            qp_iter_gpu=int(qi[i]))
        solver.fleet_sim_step(path, s, pose, vel, steer_arg, u0, status, traj, tlen, advance=True)
    report["qp_iter_mean"] = it_sum / max(ticks, 1)
    report["u0_err_max"] = max((c["u0_err"] for c in report["checks"]), default=0.0)
    report["cmd_err_max"] = max((c["cmd_err"] for c in report["checks"]), default=0.0)
    return report


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--model", default="diff", choices=["diff", "omni4", "tric"])
    ap.add_argument("--N", type=int, default=40)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=60)
    ap.add_argument("--sample", type=int, default=64)
    ap.add_argument("--check-every", type=int, default=10)
    ap.add_argument("--reset-frac", type=float, default=0.02)
    ap.add_argument("--reset-every", type=int, default=7)
    ap.add_argument("--kernel", default="team", choices=["team"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rep = run(a.model, a.N, a.B, a.ticks, a.sample, a.check_every, a.reset_frac, a.reset_every, kernel=a.kernel)
    line = json.dumps(rep)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if rep["failed"] == 0 and rep["u0_err_max"] <= 1e-3 else 1


if __name__ == "__main__":
    sys.exit(main())
