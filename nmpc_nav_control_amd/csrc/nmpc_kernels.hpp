// nmpc_kernels.hpp -- kernel-side interface shared by the HIP kernels and the C-ABI host code.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

#include "nmpc_amd/nmpc_batch.h"
#include "nmpc_amd/nmpc_path.h"
#include "nmpc_models.hpp"

// Internal to the library (acados_shim.cpp -> nmpc_batch.cpp, not part of the public ABI): nmpc_batch_solve_iterate
// for one robot whose I/O block the row-parallel kernel stages itself (KArgs::stage_*): it reads [in_d, in_d + in_n)
// from the host-mapped in_h at its start and writes [out_d, out_d + out_n) to the host-mapped out_h at its end.
// NMPC_ERR_ARG when the launch would not run the row-parallel kernel.
struct nmpc_stage_io {
    const float* in_h;
    float* in_d;
    int in_n;
    float* out_h;
    const float* out_d;
    int out_n;
};
extern "C" int nmpc_batch_solve_iterate_staged(nmpc_batch* b, const float* x0, const float* yref, int ny_in,
                                               const float* We, float* xbar, float* ubar, int* status, int* qp_iter,
                                               float* qp_res, void* stream, const nmpc_stage_io* io);

namespace nmpc {

constexpr float kPi = 3.14159265358979323846f;

enum KernelMode { kModeSolve = 0, kModeRun = 1 };

// Device pointers of one batched launch. Public inputs/outputs are [field][B] (instance-minor);
// the device-resident state (iterate, carried refs, scratch) is [field][stride], stride = capacity.
struct KArgs {
    int B, stride;   // stride: leading dimension of xbar / ubar / carried (the capacity, or the caller's ld)
    int sstride;     // the handle's capacity: row count of the scratch planes (DZ plane, dummy blocks), whatever stride is
    float* xbar;     // [(N+1)*NX][stride]   SQP iterate, warm start of the next tick
    float* ubar;     // [N*NU][stride]
    float* carried;  // [NBX][stride]        ref states carried between ticks (run mode)
    float* scratch;  // per-stage workspace
    // solve mode
    const float* x0;    // [NX][B]
    const float* yref;  // [N+1][ny_in][B]
    int ny_in;
    const float* We;  // [NX][B] or nullptr
    // run mode
    const float* pose;   // [3][B]
    const float* vel;    // [3][B]  {v, vn, w}
    const float* steer;  // [B] or nullptr
    const float* traj;   // [N+1][3][B]
    const int* traj_len; // [B] or nullptr (= N+1)
    const unsigned char* reset;  // [B] or nullptr
    // run mode from parametric paths (nmpc_batch_run_path): getNextNPoses in the kernel instead of traj
    const nmpc_path_segment* segs;  // [B][seg_stride] or nullptr
    int seg_stride, holo;
    const int* nseg;                // [B]
    const double* nearest_u;        // [B]
    double period;
    float* traj_out;                // [N+1][3][B] or nullptr: the poses the march produced
    // outputs (each may be nullptr)
    float* u0;     // [NU][B]
    float* x1;     // [NX][B]
    float* cmd;    // [3][B]
    int* status;   // [B]
    int* qp_iter;  // [B]
    float* qp_res; // [3][B] res_stat, res_ineq, mu at IPM exit
    float* xtraj;  // [(N+1)*NX][B]
    float* utraj;  // [N*NU][B]
    // team placement (schedule.hip): team slot -> instance, or nullptr (slot i = instance i)
    const int* order;
    int* iter_key;  // [stride] resident: executed IPM iterations of the last solve, or nullptr
    unsigned char* warm;  // [stride] resident: the robot's last solve succeeded and its records hold its multipliers
                          // in the layout tagged (NMPC_WARM_TAG_*), 0 otherwise; nullptr: cold start, nothing written
    int warm_tag;   // this launch's record layout tag: a robot starts warm only if warm[inst] == warm_tag
    int dense;      // the launch has more waves than the device has SIMDs (selects the team kernel variant)
    int rowpar;     // 0: team kernel; W > 0: k_sqp_rti_rowpar with W waves per robot
    int rec_split;  // team kernel, diff: split core / bound record planes (TeamRec::SPLIT_OK; tric always)
    int split;      // one 256-lane block per robot: P0's integrations spread over its 16 rows (4 waves, stage k on
                    // row k mod 16, joined by a block barrier); small batches
    int seg;        // k_sqp_rti_rowpar: horizon segments S (N % S == 0) whose Riccati sweeps run in parallel on S rows,
                    // joined by a master recursion over the segment boundaries; 0: the serial phases B / C
    // hybrid launch (A/B build -DNMPC_HYBRID only, nmpc_batch.cpp): the robots of the first hyb_n[0] ranks of `order`
    // (the hardest by last tick's IPM count) run the segmented row-parallel kernel on a second stream (role 2, at most
    // hyb_cap blocks), the rest the team kernel (role 1, team slot t -> order[hyb_n[0] + t]); role 0: a plain launch
    const int* hyb_n;
    int hyb_role, hyb_cap;
    // one-robot capsule solves (acados_shim.cpp, k_sqp_rti_rowpar only): the kernel copies the capsule's input block
    // from host-mapped memory into the device block at its start and the output block back at its end, in place of a
    // copy launch on each side (stage_in_n / stage_out_n = 0: nothing staged)
    const float* stage_in_h;
    float* stage_in_d;
    int stage_in_n;
    float* stage_out_h;
    const float* stage_out_d;
    int stage_out_n;
};

template <class M>
size_t team_scratch_floats(int N, int stride);
template <class M>
hipError_t launch_sqp_rti_team(const KParams& P, const KArgs& a, int mode, hipStream_t stream);
// small batches: one wave per robot, stage-parallel phases over its four rows (sqp_rti_rowpar.hip)
template <class M>
hipError_t launch_sqp_rti_rowpar(const KParams& P, const KArgs& a, int mode, hipStream_t stream);
template <class M>
size_t rowpar_lds_bytes(int N, int mode, int seg);
constexpr int kSegMax = 16;  // most horizon segments of the segmented row-parallel kernel
template <class M>
hipError_t launch_fleet_sim(const KParams& P, int B, int stride, float* path, float* s, float* pose, float* vel,
                            float* steer, const float* u0, const int* status, const float* carried, float* traj,
                            int* traj_len, int advance, const nmpc_fleet_renew* renew, hipStream_t stream);
hipError_t launch_team_order(const int* key, int B, int layout, int* sorted, int* order, hipStream_t stream);
#ifdef NMPC_HYBRID
// sorted order (hardest first) plus nhard[0] = min(#robots with key >= H, cap): the hybrid launch's split
hipError_t launch_hybrid_order(const int* key, int B, int H, int cap, int* order, int* nhard, hipStream_t stream);
#endif
hipError_t launch_path_discretize(int B, const nmpc_path_segment* segs, int seg_stride, const int* nseg,
                                  const double* nearest_u, double period, int num_poses, int holo, float* traj,
                                  double* traj64, hipStream_t stream);

}  // namespace nmpc
