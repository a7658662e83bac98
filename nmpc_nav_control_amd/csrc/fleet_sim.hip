// fleet_sim.hip -- closed-loop harness for benches and tests (not part of the reference's solve path).
//
// Per robot and tick: advance the plant (the same model, one RK4 step of length dt_ctrl with the
// applied input u0, SURVEY.md 8d "in closed loop the plant is integrated by RK4 with the same model"),
// read back the "measured" pose / velocity / steering angle the way getInputData() provides them
// (NMPCNavControlROS.cpp:545-553), and regenerate the N+1 reference poses:
//   path-following robots: nearest point on a circular-arc path, then samples spaced |v|*dt along it
//     (PathDiscretizer.cpp:25-47: first sample one spacing ahead, padding with the path end, :55-60);
//   go-to-pose robots: the goal pose alone (processGoToPose, NMPCNavControlROS.cpp:630-636).
#include "nmpc_kernels.hpp"

namespace nmpc {
namespace {

__device__ inline void arc_pose(const float* path, size_t Bn, int i, float s, float* out)
{
    const float x0 = path[i], y0 = path[Bn + i], th0 = path[2 * Bn + i], kap = path[3 * Bn + i];
    const float th = th0 + kap * s;
    float s1, c1;
    __sincosf(th, &s1, &c1);
    if (fabsf(kap) > 1e-4f) {
        float s0, c0;
        __sincosf(th0, &s0, &c0);
        out[0] = x0 + (s1 - s0) / kap;
        out[1] = y0 - (c1 - c0) / kap;
    } else {
        float s0, c0;
        __sincosf(th0, &s0, &c0);
        out[0] = x0 + s * c0;
        out[1] = y0 + s * s0;
    }
    out[2] = th;
}

template <class M>
__global__ void k_fleet_sim(KParams P, int B, int stride, const float* path, float* s, float* pose, float* vel,
                            float* steer, const float* u0, const int* status, const float* carried, float* traj,
                            int* traj_len, int advance)
{
    constexpr int NX = M::NX, NU = M::NU;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    const size_t Bn = (size_t)B;
    float ps[3] = {pose[i], pose[Bn + i], pose[2 * Bn + i]};
    if (advance && (!status || status[i] == 0)) {
        float v3[3] = {vel[i], vel[Bn + i], vel[2 * Bn + i]};
        float x[NX], u[NU], xn[NX];
        x[0] = ps[0];
        x[1] = ps[1];
        x[2] = ps[2];
        M::direct_kin(v3, steer ? steer[i] : 0.0f, P, x + 3);
#pragma unroll
        for (int j = 0; j < NU; j++) u[j] = u0[(size_t)j * Bn + i];
        // ref states at the solve's x0 = carried (already advanced by the post-solve) - u0 * dt_ctrl
#pragma unroll
        for (int j = 0; j < M::NBX; j++) x[M::idxbx(j)] = carried[(size_t)j * stride + i] - u[j] * P.dt_ctrl;
        rk4<M>(x, u, P, P.dt_ctrl, xn);
        ps[0] = xn[0];
        ps[1] = xn[1];
        ps[2] = xn[2];
        float nv[3];
        if (M::ID == kDiff) {
            nv[0] = 0.5f * (xn[3] + xn[4]);
            nv[1] = 0.0f;
            nv[2] = (xn[4] - xn[3]) / P.p[0];
        } else if (M::ID == kOmni4) {
            nv[0] = 0.25f * (xn[3] - xn[4] + xn[5] - xn[6]);
            nv[1] = 0.25f * (-xn[3] - xn[4] + xn[5] + xn[6]);
            nv[2] = -(xn[3] + xn[4] + xn[5] + xn[6]) / (2.0f * P.p[0]);
        } else {
            nv[0] = xn[3];
            nv[1] = 0.0f;
            nv[2] = 0.0f;
            if (steer) steer[i] = xn[4];
        }
#pragma unroll
        for (int j = 0; j < 3; j++) {
            pose[(size_t)j * Bn + i] = ps[j];
            vel[(size_t)j * Bn + i] = nv[j];
        }
    }
    const int N = P.N;
    const float len = path[5 * Bn + i];
    if (len < 0.0f) {
        // go-to-pose: the goal pose alone
        traj[i] = path[i];
        traj[Bn + i] = path[Bn + i];
        traj[2 * Bn + i] = path[2 * Bn + i];
        if (traj_len) traj_len[i] = 1;
        return;
    }
    // nearest point: a few projection steps from the previous progress (monotone, clamped to the path)
    float sc = s[i];
    for (int itn = 0; itn < 3; itn++) {
        float q[3];
        arc_pose(path, Bn, i, sc, q);
        float sn, cs;
        __sincosf(q[2], &sn, &cs);
        sc += (ps[0] - q[0]) * cs + (ps[1] - q[1]) * sn;
        sc = fminf(fmaxf(sc, 0.0f), len);
    }
    sc = fmaxf(sc, s[i]);
    s[i] = sc;
    const float spacing = fabsf(path[4 * Bn + i]) * P.dt_ctrl;
    for (int k = 0; k <= N; k++) {
        float q[3];
        arc_pose(path, Bn, i, fminf(sc + (k + 1) * spacing, len), q);
        traj[((size_t)k * 3 + 0) * Bn + i] = q[0];
        traj[((size_t)k * 3 + 1) * Bn + i] = q[1];
        traj[((size_t)k * 3 + 2) * Bn + i] = q[2];
    }
    if (traj_len) traj_len[i] = N + 1;
}

}  // namespace

template <class M>
hipError_t launch_fleet_sim(const KParams& P, int B, int stride, const float* path, float* s, float* pose, float* vel,
                            float* steer, const float* u0, const int* status, const float* carried, float* traj,
                            int* traj_len, int advance, hipStream_t stream)
{
    if (B <= 0) return hipSuccess;
    const int block = 256;
    hipLaunchKernelGGL(k_fleet_sim<M>, dim3((B + block - 1) / block), dim3(block), 0, stream, P, B, stride, path, s,
                       pose, vel, steer, u0, status, carried, traj, traj_len, advance);
    return hipGetLastError();
}

#define INST(M)                                                                                                      \
    template hipError_t launch_fleet_sim<M>(const KParams&, int, int, const float*, float*, float*, float*, float*, \
                                            const float*, const int*, const float*, float*, int*, int, hipStream_t);
INST(Diff2)
INST(Omni4)
INST(Tric3)
#undef INST

}  // namespace nmpc
