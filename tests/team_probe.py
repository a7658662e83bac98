"""One team-kernel solve of oracle closed-loop inputs, written to an npz (run as a child process of
tests/test_gpu_split.py::test_constant_rows_per_launch, so that each library -- the product's or the checker build
named by NMPC_AMD_LIB -- is the only libnmpc_amd.so in its process). usage: team_probe.py model N B ticks layout out"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from helpers import oracle_closed_loop  # noqa: E402

from nmpc_nav_control_amd._lib import default_params  # noqa: E402
from nmpc_nav_control_amd.batch import BatchSolver  # noqa: E402


def main():
    model, N, B, ticks, layout, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        sys.argv[5], sys.argv[6]
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device=dev, dtype=torch.float32)  # noqa: E731
    o, rec = oracle_closed_loop(model, N, B, ticks)
    os.environ["NMPC_AMD_ROWPAR_MAX"] = "0"  # the team kernel, unsplit, at this batch size
    os.environ["NMPC_AMD_SPLIT_MAX"] = "0"
    s = BatchSolver(model, N, B, params=default_params(model, N), record_layout=layout)
    assert s.plan_ex(B)["kernel"] == "team"
    xv, uv, _ = s.state()
    X, U = xv.to_tensor(), uv.to_tensor()
    X[:, :B] = t(np.stack([r[3] for r in rec]).reshape(B, -1).T)
    U[:, :B] = t(np.stack([r[4] for r in rec]).reshape(B, -1).T)
    xv.copy_from(X)
    uv.copy_from(U)
    xtraj = torch.zeros((N + 1) * o.nx, B, device=dev)
    utraj = torch.zeros(N * o.nu, B, device=dev)
    status = torch.full((B,), -7, dtype=torch.int32, device=dev)
    s.solve(t(np.stack([r[0] for r in rec]).T), t(np.stack([r[1] for r in rec]).transpose(1, 2, 0)),
            We=t(np.stack([r[2] for r in rec]).T), xtraj=xtraj, utraj=utraj, status=status)
    torch.cuda.synchronize()
    np.savez(out, xtraj=xtraj.cpu().numpy(), utraj=utraj.cpu().numpy(), status=status.cpu().numpy(),
             lib=os.environ.get("NMPC_AMD_LIB", ""))


if __name__ == "__main__":
    main()
