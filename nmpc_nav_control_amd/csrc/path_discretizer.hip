// path_discretizer.hip -- PathDiscretizer::getNextNPoses for B robots (include/nmpc_amd/nmpc_path.h).
//
// Reference: src/nmpc_nav_control/PathDiscretizer.cpp:14-63 (the march along the path), :65-104 (segment
// sampling). One lane per robot: the march is a sequential loop of ~10 steps per pose whose trip count depends
// on the robot's path, so lanes of a wave diverge only in their last few steps; the segments are 128-byte
// records read through the L1/L2 caches. The arithmetic is IEEE fp64 in the reference's operation order with
// contraction disabled, so x, y and every emit decision match a fp64 CPU run of PathDiscretizer.cpp bit for
// bit; theta differs only by the atan2 implementation's last-ulp rounding.
#include <hip/hip_runtime.h>

#include "nmpc_amd/nmpc_path.h"
#include "nmpc_kernels.hpp"

#pragma clang fp contract(off)  // and -ffp-contract=off in the Makefile

namespace nmpc {
namespace {

constexpr int kMaxSteps = 65536;  // safety exit of the march (see nmpc_path.h)

// floor(su) as a segment index with the reference's out-of-range handling (PathDiscretizer.cpp:67-76):
// k >= n -> last segment at u = 1, k < 0 (or NaN) -> first segment at u = 0
__device__ inline void seg_param(double su, int n, int* k, double* u)
{
    if (su >= 0.0 && su < (double)n) {
        *k = (int)floor(su);
        *u = su - (double)*k;
    } else if (su >= (double)n) {
        *k = n - 1;
        *u = 1.0;
    } else {
        *k = 0;
        *u = 0.0;
    }
}

__device__ inline double horner(const double* c, double u) { return ((c[3] * u + c[2]) * u + c[1]) * u + c[0]; }
__device__ inline double dhorner(const double* c, double u)
{
    return ((3.0 * c[3]) * u + 2.0 * c[2]) * u + c[1];
}

// |path_vector[idx].GetVelocity()| with idx = floor(a) clamped to the list
__device__ inline double seg_speed(const nmpc_path_segment* S, int n, double a)
{
    int k = (a >= 0.0 && a < (double)n) ? (int)floor(a) : ((a >= (double)n) ? n - 1 : 0);
    return fabs(S[k].v);
}

__global__ void __launch_bounds__(64) k_path_discretize(int B, const nmpc_path_segment* segs, int seg_stride,
                                                        const int* nseg, const double* nearest_u, double period,
                                                        int num_poses, int holo, float* traj, double* traj64)
{
    extern __shared__ double s_emit[];  // [num_poses][blockDim.x]: path parameter of every emitted pose
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    double* emit_u = s_emit + threadIdx.x;
    const int es = blockDim.x;
    const nmpc_path_segment* S = segs + (size_t)i * seg_stride;
    const int n = nseg[i];
    const double N = (double)n;
    const double npc = (period >= 1.0) ? 20.0 : 10.0;  // num_points_per_cycle_ (:9-10)
    const double thr = 1e-2;                           // percent_error_dist_treshold_ (:7)

    // The segment under the current path parameter stays in registers: the march crosses a segment boundary
    // about once per ten poses, so a step has no dependent load. The march only records the path parameter of
    // each pose (a divergent emit costs a few instructions); the poses are evaluated afterwards in lockstep.
    int ck = -1;
    double cx[4], cy[4], cgoal = 0.0, crel = 0.0;  // + goal_dist and rel of the segment's speed (:44-46)
    auto at = [&](double su) -> double {  // select the segment of su, return its local parameter
        int k;
        double uu;
        seg_param(su, n, &k, &uu);
        if (k != ck) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                cx[j] = S[k].x[j];
                cy[j] = S[k].y[j];
            }
            cgoal = fabs(S[k].v) * period;
            crel = cgoal / npc;
            ck = k;
        }
        return uu;
    };

    const double u0 = nearest_u[i];
    const double vel = seg_speed(S, n, u0);  // :23
    double goal_dist = vel * period;
    double rel = goal_dist / npc;
    double u = u0;
    double uu = at(u0);
    double ox = horner(cx, uu), oy = horner(cy, uu);
    double vx = dhorner(cx, uu), vy = dhorner(cy, uu);
    double step = rel / sqrt(vx * vx + vy * vy);
    double curr_dist = 0.0;
    int count = 0;
    for (int it = 0; u < N && it < kMaxSteps; it++) {  // :33
        u += step;
        u = (N < u) ? N : u;  // std::min(u, N)
        uu = at(u);
        const double nx = horner(cx, uu), ny = horner(cy, uu);
        const double dx = nx - ox, dy = ny - oy;
        curr_dist += sqrt(dx * dx + dy * dy);
        if ((goal_dist - curr_dist) <= thr * goal_dist) {  // :41-48
            emit_u[count * es] = u;
            count++;
            // path_vector[min(floor(u), N - 1)] is the segment of u (seg_param), already in registers
            goal_dist = cgoal;
            rel = crel;
            curr_dist = 0.0;
        }
        if (count == num_poses) break;  // :50
        vx = dhorner(cx, uu);
        vy = dhorner(cy, uu);
        step = rel / sqrt(vx * vx + vy * vy);  // :52-53
        ox = nx;
        oy = ny;
    }

    // getPoseSample of every emitted parameter, then the padding with the path end (:58-63)
    const size_t Bn = (size_t)B;
    for (int j = 0; j < num_poses; j++) {
        const double su = (j < count) ? emit_u[j * es] : N;
        int k;
        double w;
        seg_param(su, n, &k, &w);
        const nmpc_path_segment& g = S[k];
        const double x = horner(g.x, w), y = horner(g.y, w);
        double th;
        if (holo) {
            th = horner(g.th, w);
        } else {
            th = atan2(dhorner(g.y, w), dhorner(g.x, w));
            th = (g.v >= 0.0) ? th : th + M_PI;
        }
        const size_t o = (size_t)j * 3 * Bn + i;
        if (traj) {
            traj[o] = (float)x;
            traj[o + Bn] = (float)y;
            traj[o + 2 * Bn] = (float)th;
        }
        if (traj64) {
            traj64[o] = x;
            traj64[o + Bn] = y;
            traj64[o + 2 * Bn] = th;
        }
    }
}

}  // namespace

hipError_t launch_path_discretize(int B, const nmpc_path_segment* segs, int seg_stride, const int* nseg,
                                  const double* nearest_u, double period, int num_poses, int holo, float* traj,
                                  double* traj64, hipStream_t stream)
{
    if (B <= 0) return hipSuccess;
    // one wave per workgroup (the ~B/64 waves spread over the CUs); narrower when the emitted parameters of 64
    // robots would not fit 64 KB of LDS
    int block = 64;
    while (block > 1 && (size_t)block * num_poses * sizeof(double) > 65536) block /= 2;
    const size_t lds = (size_t)block * num_poses * sizeof(double);
    if (lds > 65536) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_path_discretize, dim3((B + block - 1) / block), dim3(block), lds, stream, B, segs,
                       seg_stride, nseg, nearest_u, period, num_poses, holo, traj, traj64);
    return hipGetLastError();
}

}  // namespace nmpc
