"""Reference-pose generation on the device: PathDiscretizer::getNextNPoses for B robots in one launch.

Mirrors include/nmpc_nav_control/PathDiscretizer.h:12-51 (constructor arguments, getNextNPoses) on top of
``nmpc_path_discretize`` (include/nmpc_amd/nmpc_path.h). The march itself runs only in the HIP kernel
(csrc/path_discretizer.hip); this module builds and packs path segments and owns the device buffers.

Path segments restate the part of parametric_trajectories_common::TPath that PathDiscretizer uses (the
library is not vendored by the reference): cubic polynomials x(u), y(u), theta_h(u) on u in [0, 1] plus a
signed speed. ``PathSegment.line / bezier / arc`` build the usual shapes.
"""
import ctypes
import math

import numpy as np
import torch

from ._lib import check, lib
from .controller import Pose

SEG_DOUBLES = 16  # sizeof(nmpc_path_segment) / sizeof(double)


class PathSegment:
    """One parametric segment: GetX/GetY/GetThetaHolomonic are cubics in u (ascending coefficients),
    GetVelocity() = v (negative: the robot drives the segment backwards)."""

    def __init__(self, x, y, th=(0.0, 0.0, 0.0, 0.0), v=0.0):
        self.x = np.asarray(x, np.float64).reshape(4)
        self.y = np.asarray(y, np.float64).reshape(4)
        self.th = np.asarray(th, np.float64).reshape(4)
        self.v = float(v)

    def GetVelocity(self):
        return self.v

    def pack(self):
        rec = np.zeros(SEG_DOUBLES)
        rec[0:4], rec[4:8], rec[8:12], rec[12] = self.x, self.y, self.th, self.v
        return rec

    @staticmethod
    def _heading(th0, th1, default):
        th0 = default if th0 is None else th0
        th1 = th0 if th1 is None else th1
        return (th0, th1 - th0, 0.0, 0.0)  # linear holonomic heading

    @classmethod
    def line(cls, p0, p1, v, th0=None, th1=None):
        (x0, y0), (x1, y1) = p0, p1
        d = math.atan2(y1 - y0, x1 - x0)
        return cls((x0, x1 - x0, 0, 0), (y0, y1 - y0, 0, 0), cls._heading(th0, th1, d), v)

    @classmethod
    def bezier(cls, p0, p1, p2, p3, v, th0=None, th1=None):
        """Cubic Bezier with control points p0..p3 in power form."""
        P = np.asarray([p0, p1, p2, p3], np.float64)
        c = np.stack([P[0], 3 * (P[1] - P[0]), 3 * (P[2] - 2 * P[1] + P[0]), P[3] - 3 * P[2] + 3 * P[1] - P[0]])
        d = math.atan2(*(P[1] - P[0])[::-1]) if np.any(P[1] != P[0]) else 0.0
        return cls(c[:, 0], c[:, 1], cls._heading(th0, th1, d), v)

    @classmethod
    def arc(cls, cx, cy, r, a0, a1, v, th0=None, th1=None):
        """Circular arc (centre, radius, polar angles a0 -> a1, |a1 - a0| <= pi/2) as its standard cubic
        Bezier approximation (radial error < 3e-4 r for a quarter circle)."""
        k = 4.0 / 3.0 * math.tan((a1 - a0) / 4.0)
        p0 = (cx + r * math.cos(a0), cy + r * math.sin(a0))
        p3 = (cx + r * math.cos(a1), cy + r * math.sin(a1))
        p1 = (p0[0] - k * r * math.sin(a0), p0[1] + k * r * math.cos(a0))
        p2 = (p3[0] + k * r * math.sin(a1), p3[1] - k * r * math.cos(a1))
        return cls.bezier(p0, p1, p2, p3, v, th0, th1)


def pack_paths(path_lists, max_segs=None):
    """[B][S][16] float64 segment records and int32 [B] counts of B path lists (S = longest list)."""
    S = max(max(len(p) for p in path_lists), 1) if max_segs is None else int(max_segs)
    segs = np.zeros((len(path_lists), S, SEG_DOUBLES))
    nseg = np.zeros(len(path_lists), np.int32)
    for i, pl in enumerate(path_lists):
        if not 1 <= len(pl) <= S:
            raise ValueError(f"path {i}: {len(pl)} segments (1..{S} allowed)")
        for j, s in enumerate(pl):
            segs[i, j] = s.pack()
        nseg[i] = len(pl)
    return segs, nseg


def _dev_ptr(t, dtype):
    if t is None:
        return None
    if not t.is_cuda or not t.is_contiguous() or t.dtype != dtype:
        raise ValueError(f"expected a contiguous {dtype} device tensor")
    return ctypes.c_void_p(t.data_ptr())


def discretize(segs, nseg, nearest_u, sample_period, num_poses, is_holonomic=False, traj=None, traj64=None,
               stream=None):
    """nmpc_path_discretize on device tensors: segs float64 [B][S][16], nseg int32 [B], nearest_u float64 [B].
    Writes traj float32 [num_poses][3][B] (allocated if None; the traj input of BatchSolver.run) and, if
    given, traj64 float64 [num_poses][3][B]. Returns traj."""
    B, S = int(segs.shape[0]), int(segs.shape[1])
    if segs.dim() != 3 or segs.shape[2] != SEG_DOUBLES:
        raise ValueError("segs must be [B][S][16]")
    if nseg.shape != (B,) or nearest_u.shape != (B,):
        raise ValueError("nseg and nearest_u must be [B]")
    if traj is None:
        traj = torch.empty((num_poses, 3, B), dtype=torch.float32, device=segs.device)
    for t in (traj, traj64):
        if t is not None and tuple(t.shape) != (num_poses, 3, B):
            raise ValueError("traj / traj64 must be [num_poses][3][B]")
    s = stream if stream is not None else torch.cuda.current_stream(segs.device)
    check(lib().nmpc_path_discretize(B, _dev_ptr(segs, torch.float64), S, _dev_ptr(nseg, torch.int32),
                                     _dev_ptr(nearest_u, torch.float64), float(sample_period), int(num_poses),
                                     1 if is_holonomic else 0, _dev_ptr(traj, torch.float32),
                                     _dev_ptr(traj64, torch.float64), ctypes.c_void_p(s.cuda_stream)),
          "nmpc_path_discretize")
    return traj


class PathDiscretizer:
    """PathDiscretizer(sample_period, num_poses, is_holonomic) (PathDiscretizer.cpp:5-12). getNextNPoses runs
    one robot on the device; discretize_batch runs many."""

    def __init__(self, sample_period, num_poses, is_holonomic=False, device="cuda"):
        self.sample_period = float(sample_period)
        self.num_poses = int(num_poses)
        self.is_holonomic = bool(is_holonomic)
        self.device = torch.device(device)

    def discretize_batch(self, path_lists, nearest_u):
        """[B][num_poses][3] float64 poses of B robots (path lists of PathSegment, nearest path parameters)."""
        segs, nseg = pack_paths(path_lists)
        dev = self.device
        t64 = torch.empty((self.num_poses, 3, len(path_lists)), dtype=torch.float64, device=dev)
        discretize(torch.from_numpy(segs).to(dev), torch.from_numpy(nseg).to(dev),
                   torch.as_tensor(np.asarray(nearest_u, np.float64)).to(dev), self.sample_period, self.num_poses,
                   self.is_holonomic, traj64=t64)
        return t64.permute(2, 0, 1).cpu().numpy()

    def getNextNPoses(self, path_list, nearest_sample_u, next_poses=None):
        """Appends num_poses poses to next_poses (a list; created if None) and returns it (PathDiscretizer.cpp:14)."""
        out = self.discretize_batch([list(path_list)], [nearest_sample_u])[0]
        next_poses = [] if next_poses is None else next_poses
        next_poses.extend(Pose(float(p[0]), float(p[1]), float(p[2])) for p in out)
        return next_poses
