"""Seeded synthetic robot fleets (SURVEY.md 8d "Synthetic inputs").

Every robot starts at x, y ~ U(-1, 1) m, theta ~ U(-pi, pi), wheel / speed / steering states ~ U(-0.5, 0.5)
and carried vel-ref states ~ U(-0.5, 0.5), except the tric steering reference alpha_ref ~ U(-0.78, 0.78) rad:
its rate bound (15 deg/s) keeps it within 23 deg of its start over the 1.5 s horizon, so the 45 deg bound
(NMPCNavControlTric.cpp:24-29) is active only for robots that start near it (measured on the fp64 oracle,
256 robots: 14-18 % of the fleet has alpha_ref on the bound at ticks 3-24, against 3-4 % with U(-0.5, 0.5);
BASELINE config 4 asks for >= 10 %). Half of the robots follow a circular-arc path (start within
0.2 m and 0.3 rad of the robot, curvature ~ U(-k, k) 1/m, |v| ~ U(0.2, 0.8) m/s, length ~ U(3, 5) m);
the other half drive to a goal pose (x, y ~ U(-1.5, 1.5) m, random heading), which repeats one pose
N+1 times and so triggers the diff terminal-weight hack (NMPCNavControlDiff.cpp:127-139).
Arrays are float32 in the instance-minor [field][B] layout of include/nmpc_amd/nmpc_batch.h.

Stationary closed loop (``RENEW``, nmpc_fleet_sim_step_renew): the reference's node solves only while it has a goal
or a path, gets new ones from its topics and calls reset_mpc on each (NMPCNavControlROS.cpp:304-327). The bench
fleet does the same: a robot that arrives, or whose goal / path has been active for its ttl (80-240 ticks, 2-6 s),
gets a new one drawn from (seed, global index, event count) and is reset on its next solve. The first ttl is
uniform in [1, ttl_max], so renewals are spread over the ticks from the start and the tick mix does not drift.
"""
import numpy as np

from ._lib import model_dims

DEFAULT_SEED = 20250824
PARAMS = {"diff": (0.270, 0.1, 0.0), "omni4": (0.535, 0.1, 0.0), "tric": (0.270, 0.1, 0.5)}
SPEED = {}  # path speed range per model (default U(0.2, 0.8) m/s)
ALPHA_REF0 = 0.78  # tric: initial steering-reference states up to the 45 deg bound (>= 10 % of the fleet on it)


BLOCK = 64  # robots per independently seeded block: a robot's data depends only on (seed, global index)

# goal / path renewal of the stationary bench loop (nmpc_fleet_renew); arrival tolerances are the shipped
# final_position_error / final_orientation_error (config/nmpc_nav_control.yaml:6-7)
RENEW = dict(ttl_min=80, ttl_max=240, goal_r_lo=0.3, goal_r_hi=1.5, len_lo=3.0, len_hi=5.0, pos_tol=0.01,
             ang_tol=float(np.deg2rad(1.0)))
_M32 = 0xFFFFFFFF


def _lowbias32(h):
    h = np.asarray(h, np.uint64) & _M32
    h ^= h >> 16
    h = (h * 0x7FEB352D) & _M32
    h ^= h >> 15
    h = (h * 0x846CA68B) & _M32
    h ^= h >> 16
    return h


def fleet_hash(seed, index, counter):
    """nmpc_fleet_hash (fleet_sim.hip) on uint32 values / arrays."""
    h = _lowbias32(_lowbias32(np.uint64(seed & _M32) ^ np.uint64(0x9E3779B9)) + np.asarray(index, np.uint64))
    return _lowbias32(h + np.asarray(counter, np.uint64))


def fleet_u(seed, index, event, j):
    """Draw j of renewal event `event` of robot `index`: (h >> 8) / 2^24, exact in fp32 and fp64."""
    return (fleet_hash(seed, index, 16 * np.asarray(event, np.uint64) + j) >> 8).astype(np.float64) / 16777216.0


def fleet_ttl(seed, index, event, lo, hi):
    """The ttl drawn at renewal event `event` (event 0: the initial one): lo + ((h >> 8) * (hi - lo + 1) >> 24)."""
    h = fleet_hash(seed, index, 16 * np.asarray(event, np.uint64) + 15) >> 8
    return (lo + ((h * np.uint64(hi - lo + 1)) >> 24)).astype(np.int32)


def kappa_max_of(model):
    return 2.5 if model == "tric" else 1.0


def _block(model, seed, blk, kappa_max, path_frac, p, speed):
    """Robots [blk*BLOCK, (blk+1)*BLOCK) of the global fleet, float64 [field][BLOCK]."""
    rng = np.random.default_rng([seed, blk])
    B = BLOCK
    nbx = model_dims(model)["nbx"]
    pose = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), rng.uniform(-np.pi, np.pi, B)])
    vel = np.zeros((3, B))
    steer = np.zeros(B)
    if model == "diff":
        vl, vr = rng.uniform(-0.5, 0.5, B), rng.uniform(-0.5, 0.5, B)
        vel[0] = 0.5 * (vl + vr)
        vel[2] = (vr - vl) / p[0]
    elif model == "omni4":
        w = rng.uniform(-0.5, 0.5, (4, B))
        vel[0] = 0.25 * (w[0] - w[1] + w[2] - w[3])
        vel[1] = 0.25 * (-w[0] - w[1] + w[2] + w[3])
        vel[2] = -(w[0] + w[1] + w[2] + w[3]) / (2.0 * p[0])
    else:
        vel[0] = rng.uniform(-0.5, 0.5, B)
        steer = rng.uniform(-0.5, 0.5, B)
    carried = rng.uniform(-0.5, 0.5, (nbx, B))
    if model == "tric":
        carried[1] = rng.uniform(-ALPHA_REF0, ALPHA_REF0, B)
    is_path = rng.uniform(0, 1, B) < path_frac
    path = np.zeros((6, B))
    # arcs
    r = rng.uniform(0, 0.2, B)
    a = rng.uniform(-np.pi, np.pi, B)
    path[0] = pose[0] + r * np.cos(a)
    path[1] = pose[1] + r * np.sin(a)
    path[2] = pose[2] + rng.uniform(-0.3, 0.3, B)
    path[3] = rng.uniform(-kappa_max, kappa_max, B)
    path[4] = rng.uniform(speed[0], speed[1], B)
    path[5] = rng.uniform(3.0, 5.0, B)
    # goals
    goal = np.stack([rng.uniform(-1.5, 1.5, B), rng.uniform(-1.5, 1.5, B), rng.uniform(-np.pi, np.pi, B)])
    path[:3, ~is_path] = goal[:, ~is_path]
    path[3:5, ~is_path] = 0.0
    path[5, ~is_path] = -1.0
    return dict(pose=pose, vel=vel, steer=steer, carried=carried, path=path, is_path=is_path)


def make_fleet(model, B, seed=DEFAULT_SEED, kappa_max=None, path_frac=0.5, p=None, start=0, speed=None):
    """Robots [start, start + B) of the seeded global fleet (so an instance shard of a multi-GPU run holds
    exactly the robots a single-GPU run of the whole fleet would give those indices)."""
    p = PARAMS[model] if p is None else p
    if kappa_max is None:
        kappa_max = kappa_max_of(model)
    if speed is None:
        speed = SPEED.get(model, (0.2, 0.8))
    b0, b1 = start // BLOCK, (start + B + BLOCK - 1) // BLOCK
    blocks = [_block(model, seed, k, kappa_max, path_frac, p, speed) for k in range(b0, b1)]
    lo = start - b0 * BLOCK
    cat = {k: np.concatenate([bl[k] for bl in blocks], axis=-1)[..., lo:lo + B] for k in blocks[0]} if blocks else \
        _block(model, seed, 0, kappa_max, path_frac, p, speed)
    f32 = lambda x: np.ascontiguousarray(x, dtype=np.float32)  # noqa: E731
    out = {k: f32(v) for k, v in cat.items() if k != "is_path"}
    if not blocks:
        out = {k: v[..., :0] for k, v in out.items()}
    out["s"] = np.zeros(B, np.float32)
    out["is_path"] = cat["is_path"][..., :B]
    # renewal state: no event yet, first ttl uniform in [1, ttl_max] (spread renewals from the first tick)
    out["ev"] = np.zeros(B, np.int32)
    out["ttl"] = fleet_ttl(seed, np.arange(start, start + B), 0, 1, RENEW["ttl_max"])
    return out


def renew_step(model, path, s, pose, ev, ttl, seed, start, i, renew=None, speed=None):
    """CPU mirror (fp64) of the renewal in k_fleet_sim for robot i after its plant step; returns the reset flag.
    path [6][B], s [B], ev / ttl [B] are updated in place."""
    R = dict(RENEW, **(renew or {}))
    speed = speed or SPEED.get(model, (0.2, 0.8))
    if path[5, i] < 0:
        end = np.array([path[0, i], path[1, i], path[2, i]], np.float64)
    else:
        end = arc_pose(path, i, float(path[5, i]))
    d2 = (pose[0] - end[0]) ** 2 + (pose[1] - end[1]) ** 2
    err = (pose[2] - end[2] + np.pi) % (2 * np.pi) - np.pi
    arrived = d2 <= R["pos_tol"] ** 2 and abs(err) <= R["ang_tol"]
    t = int(ttl[i]) - 1
    if not (arrived or t <= 0):
        ttl[i] = t
        return 0
    e = int(ev[i]) + 1
    gi = start + i
    u = [float(fleet_u(seed, gi, e, j)) for j in range(6)]
    ca, sa = np.cos(2 * np.pi * u[0]), np.sin(2 * np.pi * u[0])
    if path[5, i] < 0:
        rr = R["goal_r_lo"] + (R["goal_r_hi"] - R["goal_r_lo"]) * u[1]
        path[0, i], path[1, i], path[2, i] = pose[0] + rr * ca, pose[1] + rr * sa, np.pi * (2 * u[2] - 1)
    else:
        rr = 0.2 * u[1]
        km = kappa_max_of(model)
        path[0, i], path[1, i] = pose[0] + rr * ca, pose[1] + rr * sa
        path[2, i] = pose[2] + 0.3 * (2 * u[2] - 1)
        path[3, i] = km * (2 * u[3] - 1)
        path[4, i] = speed[0] + (speed[1] - speed[0]) * u[4]
        path[5, i] = R["len_lo"] + (R["len_hi"] - R["len_lo"]) * u[5]
        s[i] = 0.0
    ttl[i] = int(fleet_ttl(seed, gi, e, R["ttl_min"], R["ttl_max"]))
    ev[i] = e
    return 1


def arc_pose(path, i, s):
    """Pose at arc length s on robot i's path (same formula as fleet_sim.hip)."""
    x0, y0, th0, kap = (float(path[j, i]) for j in range(4))
    th = th0 + kap * s
    if abs(kap) > 1e-4:
        return np.array([x0 + (np.sin(th) - np.sin(th0)) / kap, y0 - (np.cos(th) - np.cos(th0)) / kap, th])
    return np.array([x0 + s * np.cos(th0), y0 + s * np.sin(th0), th])


def refs_for(path, i, pose, s_prev, N, dt):
    """Reference poses of robot i (CPU mirror of fleet_sim.hip, for CPU-only tests).
    Returns (traj [n][3], s_new)."""
    if path[5, i] < 0:
        return path[:3, i][None, :].astype(np.float64), s_prev
    length = float(path[5, i])
    sc = float(s_prev)
    for _ in range(3):
        q = arc_pose(path, i, sc)
        sc += (pose[0] - q[0]) * np.cos(q[2]) + (pose[1] - q[1]) * np.sin(q[2])
        sc = min(max(sc, 0.0), length)
    sc = max(sc, s_prev)
    spacing = abs(float(path[4, i])) * dt
    traj = np.stack([arc_pose(path, i, min(sc + (k + 1) * spacing, length)) for k in range(N + 1)])
    return traj, sc
