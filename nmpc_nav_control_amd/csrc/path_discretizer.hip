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
#include "path_march.hpp"

#pragma clang fp contract(off)  // and -ffp-contract=off in the Makefile

namespace nmpc {
namespace {

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

    // The march (path_march.hpp) only records the path parameter of each pose (a divergent emit costs a few
    // instructions); the poses are evaluated afterwards in lockstep.
    const int count = path_march(S, n, nearest_u[i], period, num_poses,
                                 [&](int j, double u) { emit_u[j * es] = u; });

    // getPoseSample of every emitted parameter, then the padding with the path end (:58-63)
    const size_t Bn = (size_t)B;
    for (int j = 0; j < num_poses; j++) {
        const double su = (j < count) ? emit_u[j * es] : N;
        double x, y, th;
        path_pose(S, n, su, holo, &x, &y, &th);
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
