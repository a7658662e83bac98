"""Pure-Python restatement of PathDiscretizer (src/nmpc_nav_control/PathDiscretizer.cpp), line by line, used
to pin the C oracle (oracle/path_oracle.c) on small cases. Python floats are IEEE doubles and math.sqrt /
math.atan2 / math.floor are the C library's, so the two agree bit for bit.

Segments are the nmpc_path_segment records (include/nmpc_amd/nmpc_path.h): rec[0:4] x(u), rec[4:8] y(u),
rec[8:12] theta_h(u) coefficients, rec[12] signed speed.
"""
import math


class TPath:
    """The TPath interface PathDiscretizer uses, on one segment record."""

    def __init__(self, rec):
        self.c = [float(v) for v in rec]

    def _p(self, o, u):
        c = self.c
        return ((c[o + 3] * u + c[o + 2]) * u + c[o + 1]) * u + c[o]

    def _d(self, o, u):
        c = self.c
        return ((3.0 * c[o + 3]) * u + 2.0 * c[o + 2]) * u + c[o + 1]

    def GetX(self, u):
        return self._p(0, u)

    def GetY(self, u):
        return self._p(4, u)

    def GetDX(self, u):
        return self._d(0, u)

    def GetDY(self, u):
        return self._d(4, u)

    def GetTheta(self, u):
        return math.atan2(self.GetDY(u), self.GetDX(u))

    def GetThetaHolomonic(self, u):
        return self._p(8, u)

    def GetVelocity(self):
        return self.c[12]


class PathDiscretizer:
    def __init__(self, sample_period, num_poses, is_holonomic=False):  # :5-12
        self.sample_period = sample_period
        self.num_poses = num_poses
        self.is_holonomic = is_holonomic
        self.percent_error_dist_treshold = 1e-2
        self.num_points_per_cycle = 20 if sample_period >= 1.0 else 10

    def _index(self, a):
        # floor(a) as a list index; the reference leaves out-of-range / NaN undefined (nmpc_path.h)
        n = len(self.path_vector)
        if 0.0 <= a < n:
            return int(math.floor(a))
        return n - 1 if a >= n else 0

    def getNextNPoses(self, path_list, nearest_sample_u, max_steps=65536):  # :14-63
        self.path_vector = list(path_list)
        next_poses = []
        N = float(len(self.path_vector))
        vel = abs(self.path_vector[self._index(nearest_sample_u)].GetVelocity())
        goal_dist = vel * self.sample_period
        rel = goal_dist / self.num_points_per_cycle
        u = nearest_sample_u
        old_point = self.getPoseSample(nearest_sample_u)
        vx, vy = self.getVelSample(nearest_sample_u)
        step = _div(rel, math.sqrt(vx * vx + vy * vy))
        curr_dist = 0.0
        steps = 0
        while u < N and steps < max_steps:
            steps += 1
            u += step
            u = N if N < u else u
            new_point = self.getPoseSample(u)
            dx, dy = new_point[0] - old_point[0], new_point[1] - old_point[1]
            curr_dist += math.sqrt(dx * dx + dy * dy)
            if (goal_dist - curr_dist) <= self.percent_error_dist_treshold * goal_dist:
                next_poses.append(new_point)
                fu = math.floor(u) if math.isfinite(u) else u
                vel = abs(self.path_vector[self._index(N - 1 if N - 1 < fu else fu)].GetVelocity())
                goal_dist = vel * self.sample_period
                rel = goal_dist / self.num_points_per_cycle
                curr_dist = 0.0
            if self.num_poses == len(next_poses):
                break
            vx, vy = self.getVelSample(u)
            step = _div(rel, math.sqrt(vx * vx + vy * vy))
            old_point = new_point
        if self.num_poses > len(next_poses):
            last_point = self.getPoseSample(N)
            while self.num_poses > len(next_poses):
                next_poses.append(last_point)
        return next_poses, steps

    def _segment(self, sample_u):  # :67-76
        n = len(self.path_vector)
        if 0.0 <= sample_u < n:
            path_num = int(math.floor(sample_u))
            return path_num, sample_u - path_num
        if sample_u >= n:
            return n - 1, 1.0
        return 0, 0.0

    def getPoseSample(self, sample_u):  # :65-85
        k, u = self._segment(sample_u)
        path = self.path_vector[k]
        if not self.is_holonomic:
            th = path.GetTheta(u) if path.GetVelocity() >= 0 else path.GetTheta(u) + math.pi
        else:
            th = path.GetThetaHolomonic(u)
        return (path.GetX(u), path.GetY(u), th)

    def getVelSample(self, sample_u):  # :87-102
        k, u = self._segment(sample_u)
        path = self.path_vector[k]
        return path.GetDX(u), path.GetDY(u)


def _div(a, b):
    """IEEE division as C does it (x/0 -> +-inf or nan)."""
    try:
        return a / b
    except ZeroDivisionError:
        if a == 0.0 or math.isnan(a):
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
