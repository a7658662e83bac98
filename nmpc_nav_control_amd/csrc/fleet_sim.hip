// fleet_sim.hip -- closed-loop harness for benches and tests (not part of the reference's solve path).
//
// Per robot and tick: advance the plant (the same model, one RK4 step of length dt_ctrl with the
// applied input u0, SURVEY.md 8d "in closed loop the plant is integrated by RK4 with the same model"),
// read back the "measured" pose / velocity / steering angle the way getInputData() provides them
// (NMPCNavControlROS.cpp:545-553), and regenerate the N+1 reference poses:
//   path-following robots: nearest point on a circular-arc path, then samples spaced |v|*dt along it
//     (PathDiscretizer.cpp:25-47: first sample one spacing ahead, padding with the path end, :55-60);
//   go-to-pose robots: the goal pose alone (processGoToPose, NMPCNavControlROS.cpp:630-636).
// With a renewal record (nmpc_fleet_sim_step_renew) the loop is stationary: after the plant step a robot that has
// arrived or whose goal / path has been active for its ttl gets a new one from the harness hash and is reset on
// its next solve (the goal / path callbacks, NMPCNavControlROS.cpp:304-327).
#include "nmpc_kernels.hpp"

namespace nmpc {

__host__ __device__ inline unsigned int lowbias32(unsigned int h)
{
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}
__host__ __device__ inline unsigned int fleet_hash(unsigned int seed, unsigned int index, unsigned int counter)
{
    return lowbias32(lowbias32(lowbias32(seed ^ 0x9e3779b9u) + index) + counter);
}

namespace {

// pose at arc length s of the arc path pp = {x0, y0, th0, kappa, ...}
__device__ inline void arc_pose(const float* pp, float s, float* out)
{
    const float x0 = pp[0], y0 = pp[1], th0 = pp[2], kap = pp[3];
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

__device__ inline float wrap_pi(float a)
{
    a = fmodf(a + kPi, 2.0f * kPi);
    return (a < 0.0f ? a + 2.0f * kPi : a) - kPi;
}

// draw j of event e of robot gi: a uniform in [0, 1) with 24 random bits (exact in fp32 and fp64)
__device__ inline float fleet_u(const nmpc_fleet_renew& R, unsigned int gi, int e, int j)
{
    return (float)(fleet_hash(R.seed, gi, 16u * (unsigned int)e + (unsigned int)j) >> 8) * (1.0f / 16777216.0f);
}

// 16 lanes per robot (kLanes robots per 256-thread block): lane 0 runs the robot's scalar work (statistics, plant
// step, renewal, nearest-point projection) and leaves the path parameters in LDS; then the robot's 16 lanes evaluate
// its N+1 reference poses (pose k on lane k mod 16). One lane per robot with a serial pose loop took 17.6 us per
// tick for 4096 robots on 16 CUs (profiles/r03/bench_metric_kernel_stats.csv).
constexpr int kFleetLanes = 16;
constexpr int kFleetBlock = 256;

template <class M>
__global__ __launch_bounds__(kFleetBlock) void k_fleet_sim(KParams P, int B, int stride, float* path, float* s,
                                                          float* pose, float* vel, float* steer, const float* u0,
                                                          const int* status, const float* carried, float* traj,
                                                          int* traj_len, int advance, nmpc_fleet_renew R,
                                                          nmpc_fleet_stats S)
{
    constexpr int NX = M::NX, NU = M::NU;
    constexpr int RPB = kFleetBlock / kFleetLanes;  // robots per block
    const int lane = threadIdx.x % kFleetLanes, slot = threadIdx.x / kFleetLanes;
    const int i = blockIdx.x * RPB + slot;
    const bool lead = lane == 0 && i < B;
    const size_t Bn = (size_t)B;
    __shared__ float sh_path[RPB][6], sh_sc[RPB];
    __shared__ unsigned int hist[64];  // block-local histogram of the statistics (S.qp_iter)
    if (threadIdx.x < 64) hist[threadIdx.x] = 0u;
    __syncthreads();
    if (lead) {
        // the lead lane loads everything first: as far as the compiler knows every array may alias every other, so
        // a load placed after a store waits for it (one memory round trip each)
        const bool renew = R.ev && advance;
        const int st_i = status ? status[i] : 0;
        const unsigned char rs_i = (S.qp_iter || renew) ? R.reset[i] : 0;
        float ps[3] = {pose[i], pose[Bn + i], pose[2 * Bn + i]};
        float v3[3] = {vel[i], vel[Bn + i], vel[2 * Bn + i]};
        const float st0 = steer ? steer[i] : 0.0f;
        float u[NU], cr[M::NBX], pp[6];
#pragma unroll
        for (int j = 0; j < NU; j++) u[j] = advance ? u0[(size_t)j * Bn + i] : 0.0f;
#pragma unroll
        for (int j = 0; j < M::NBX; j++) cr[j] = advance ? carried[(size_t)j * stride + i] : 0.0f;
#pragma unroll
        for (int j = 0; j < 6; j++) pp[j] = path[(size_t)j * Bn + i];
        float s_i = s[i];
        const int ev_i = renew ? R.ev[i] : 0, ttl_i = renew ? R.ttl[i] : 0;
        if (S.qp_iter) {
            // the statistics of the solve this step follows (bench harness; replaces a dozen small launches per
            // tick); `reset` still holds the flags that solve ran with
            const int it = S.qp_iter[i];
            const long long cold = rs_i ? 1 : 0;
            const long long isum = S.iters_sum[i], fcnt = S.fail_cnt[i], ccnt = S.cold_cnt[i];
            const long long citer = S.cold_iters[i];
            const int imax = S.iters_max[i];
            S.iters_sum[i] = isum + it;
            S.iters_max[i] = max(imax, it);
            S.fail_cnt[i] = fcnt + (st_i != 0 ? 1 : 0);
            S.cold_cnt[i] = ccnt + cold;
            S.cold_iters[i] = citer + cold * it;
            atomicAdd(&hist[min(max(it, 0), 63)], 1u);
        }
        if (advance && st_i == 0) {
            float x[NX], xn[NX];
            x[0] = ps[0];
            x[1] = ps[1];
            x[2] = ps[2];
            M::direct_kin(v3, st0, P, x + 3);
            // ref states at the solve's x0 = carried (already advanced by the post-solve) - u0 * dt_ctrl
#pragma unroll
            for (int j = 0; j < M::NBX; j++) x[M::idxbx(j)] = cr[j] - u[j] * P.dt_ctrl;
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
        if (renew) {
            // the fleet manager: arrival (the end-of-trajectory test of processGoToPose / processFollowPath,
            // NMPCNavControlROS.cpp:637-643 / :682-693; |heading error| where the reference compares the signed
            // normAngRad) or the ttl of the current goal / path ends -> a new one, and reset_mpc on the next solve
            float end[3];
            if (pp[5] < 0.0f) {
                end[0] = pp[0];
                end[1] = pp[1];
                end[2] = pp[2];
            } else {
                arc_pose(pp, pp[5], end);
            }
            const float dx = ps[0] - end[0], dy = ps[1] - end[1];
            const bool arrived = (dx * dx + dy * dy <= R.pos_tol * R.pos_tol) && fabsf(wrap_pi(ps[2] - end[2])) <= R.ang_tol;
            const int ttl = ttl_i - 1;
            if (arrived || ttl <= 0) {
                const int e = ev_i + 1;
                const unsigned int gi = (unsigned int)(R.start + i);
                const float ua = fleet_u(R, gi, e, 0), ub = fleet_u(R, gi, e, 1), uc = fleet_u(R, gi, e, 2);
                float sa, ca;
                __sincosf(2.0f * kPi * ua, &sa, &ca);
                if (pp[5] < 0.0f) {
                    const float rr = R.goal_r_lo + (R.goal_r_hi - R.goal_r_lo) * ub;
                    pp[0] = ps[0] + rr * ca;
                    pp[1] = ps[1] + rr * sa;
                    pp[2] = kPi * (2.0f * uc - 1.0f);
                } else {
                    const float rr = 0.2f * ub;
                    pp[0] = ps[0] + rr * ca;
                    pp[1] = ps[1] + rr * sa;
                    pp[2] = ps[2] + 0.3f * (2.0f * uc - 1.0f);
                    pp[3] = R.kappa_max * (2.0f * fleet_u(R, gi, e, 3) - 1.0f);
                    pp[4] = R.speed_lo + (R.speed_hi - R.speed_lo) * fleet_u(R, gi, e, 4);
                    pp[5] = R.len_lo + (R.len_hi - R.len_lo) * fleet_u(R, gi, e, 5);
                    s_i = 0.0f;
                }
#pragma unroll
                for (int j = 0; j < 6; j++) path[(size_t)j * Bn + i] = pp[j];
                const unsigned long long span = (unsigned long long)(R.ttl_max - R.ttl_min + 1);
                R.ttl[i] = R.ttl_min + (int)((unsigned long long)(fleet_hash(R.seed, gi, 16u * (unsigned int)e + 15u) >> 8) * span >> 24);
                R.ev[i] = e;
                R.reset[i] = 1;
            } else {
                R.ttl[i] = ttl;
                R.reset[i] = 0;
            }
        }
        const float len = pp[5];
        float sc = 0.0f;
        if (len < 0.0f) {
            // go-to-pose: the goal pose alone
            traj[i] = pp[0];
            traj[Bn + i] = pp[1];
            traj[2 * Bn + i] = pp[2];
            if (traj_len) traj_len[i] = 1;
        } else {
            // nearest point: a few projection steps from the previous progress (monotone, clamped to the path)
            sc = s_i;
            for (int itn = 0; itn < 3; itn++) {
                float q[3];
                arc_pose(pp, sc, q);
                float sn, cs;
                __sincosf(q[2], &sn, &cs);
                sc += (ps[0] - q[0]) * cs + (ps[1] - q[1]) * sn;
                sc = fminf(fmaxf(sc, 0.0f), len);
            }
            sc = fmaxf(sc, s_i);
            s[i] = sc;
            if (traj_len) traj_len[i] = P.N + 1;
        }
#pragma unroll
        for (int j = 0; j < 6; j++) sh_path[slot][j] = pp[j];
        sh_sc[slot] = sc;
    }
    __syncthreads();
    if (S.qp_iter && threadIdx.x < 64 && hist[threadIdx.x])
        atomicAdd((unsigned long long*)&S.hist[threadIdx.x], (unsigned long long)hist[threadIdx.x]);
    if (i >= B) return;
    const float* pp = sh_path[slot];
    const float len = pp[5];
    if (len < 0.0f) return;
    // the robot's N+1 reference poses on its 16 lanes
    const float sc = sh_sc[slot];
    const float spacing = fabsf(pp[4]) * P.dt_ctrl;
    for (int k = lane; k <= P.N; k += kFleetLanes) {
        float q[3];
        arc_pose(pp, fminf(sc + (k + 1) * spacing, len), q);
        traj[((size_t)k * 3 + 0) * Bn + i] = q[0];
        traj[((size_t)k * 3 + 1) * Bn + i] = q[1];
        traj[((size_t)k * 3 + 2) * Bn + i] = q[2];
    }
}

}  // namespace

template <class M>
hipError_t launch_fleet_sim(const KParams& P, int B, int stride, float* path, float* s, float* pose, float* vel,
                            float* steer, const float* u0, const int* status, const float* carried, float* traj,
                            int* traj_len, int advance, const nmpc_fleet_renew* renew, hipStream_t stream)
{
    if (B <= 0) return hipSuccess;
    constexpr int rpb = kFleetBlock / kFleetLanes;
    nmpc_fleet_renew R{};
    nmpc_fleet_stats S{};
    if (renew) R = *renew;
    if (renew && renew->stats) S = *renew->stats;
    R.stats = nullptr;  // host memory: the kernel gets S by value
    hipLaunchKernelGGL(k_fleet_sim<M>, dim3((B + rpb - 1) / rpb), dim3(kFleetBlock), 0, stream, P, B, stride, path, s,
                       pose, vel, steer, u0, status, carried, traj, traj_len, advance, R, S);
    return hipGetLastError();
}

#define INST(M)                                                                                                      \
    template hipError_t launch_fleet_sim<M>(const KParams&, int, int, float*, float*, float*, float*, float*,       \
                                            const float*, const int*, const float*, float*, int*, int,              \
                                            const nmpc_fleet_renew*, hipStream_t);
INST(Diff2)
INST(Omni4)
INST(Tric3)
#undef INST

}  // namespace nmpc

extern "C" unsigned int nmpc_fleet_hash(unsigned int seed, unsigned int index, unsigned int counter)
{
    return nmpc::fleet_hash(seed, index, counter);
}
