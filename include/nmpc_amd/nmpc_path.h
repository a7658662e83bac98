/*
 * nmpc_path.h -- batched reference-pose generation on the device (libnmpc_amd.so), C ABI.
 *
 * nmpc_path_discretize is PathDiscretizer::getNextNPoses (src/nmpc_nav_control/PathDiscretizer.cpp:14-63,
 * include/nmpc_nav_control/PathDiscretizer.h:12-51) for B robots in one launch: the step the reference runs
 * per robot on the CPU right before NMPCNavControl*::run (NMPCNavControlROS.cpp:669-681). Its output is the
 * traj argument of nmpc_batch_run (nmpc_batch.h), so a path-following tick never leaves the GPU.
 *
 * The parametric path segments (parametric_trajectories_common::TPath) come from a library the reference does
 * not vendor; nmpc_path_segment restates the interface PathDiscretizer uses (GetX/GetY/GetDX/GetDY/GetTheta/
 * GetThetaHolomonic/GetVelocity) as cubic polynomials in the segment parameter u in [0, 1]:
 *   GetX(u) = x[0] + x[1] u + x[2] u^2 + x[3] u^3      (Horner order, no fused multiply-add)
 *   GetY(u) likewise with y[], GetThetaHolomonic(u) likewise with th[]
 *   GetDX(u), GetDY(u): the derivatives; GetTheta(u) = atan2(GetDY(u), GetDX(u)); GetVelocity() = v.
 * Lines, cubic Bezier / Hermite curves and polynomial approximations of arcs all fit this form.
 *
 * Conventions as in nmpc_batch.h: DEVICE pointers, asynchronous on `stream` (hipStream_t, NULL = default),
 * 0 on success or < 0 with nmpc_last_error().
 */
#ifndef NMPC_AMD_NMPC_PATH_H
#define NMPC_AMD_NMPC_PATH_H

#ifdef __cplusplus
extern "C" {
#endif

/* One parametric path segment (128 bytes). */
typedef struct nmpc_path_segment {
    double x[4];  /* GetX(u) coefficients, ascending powers of u */
    double y[4];  /* GetY(u) */
    double th[4]; /* GetThetaHolomonic(u) */
    double v;     /* GetVelocity(): signed segment speed; v < 0 drives the segment backwards (theta + pi) */
    double reserved[3];
} nmpc_path_segment;

/* getNextNPoses for robots [0, B):
 *   segs       [B][seg_stride] segments; robot i's path list is segs[i*seg_stride .. i*seg_stride+nseg[i]-1]
 *   nseg       [B] segments per robot (>= 1)
 *   nearest_u  [B] path parameter of the robot's nearest point (integer part = segment index)
 *   sample_period, num_poses, is_holonomic: the PathDiscretizer constructor arguments (num_poses <= 8192)
 *              (PathDiscretizer.cpp:5-12; the ROS node passes dt, N+1, false: NMPCNavControlROS.cpp:669)
 * outputs (either may be NULL):
 *   traj       [num_poses][3][B] float {x, y, theta}: the traj input of nmpc_batch_run
 *   traj64     [num_poses][3][B] double, the same poses unrounded
 * Differences from the reference, all on inputs where it is undefined: the segment index of the first
 * velocity lookup is clamped to [0, nseg-1] (PathDiscretizer.cpp:23 indexes without a check), a NaN path
 * parameter selects segment 0, and a robot stops after 65536 loop steps (the reference loop has no cap;
 * a non-degenerate path needs about 10 steps per pose). */
int nmpc_path_discretize(int B, const nmpc_path_segment* segs, int seg_stride, const int* nseg,
                         const double* nearest_u, double sample_period, int num_poses, int is_holonomic,
                         float* traj, double* traj64, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NMPC_AMD_NMPC_PATH_H */
