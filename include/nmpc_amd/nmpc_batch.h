/*
 * nmpc_batch.h -- batched MI355X SQP-RTI solve path (libnmpc_amd.so), C ABI.
 *
 * The batched entry points behind which thousands of NMPCNavControl*::run() calls of the reference
 * (src/nmpc_nav_control/NMPCNavControl{Diff,Omni4,Tric}.cpp:82/91/88) execute as one device launch.
 * The per-robot acados-compatible ABI ({name}_acados_*, ocp_nlp_*) lives in acados_solver_{name}.h
 * and acados_c/ocp_nlp_interface.h and is implemented on top of these functions.
 *
 * Conventions
 *   - All array arguments of nmpc_batch_solve / nmpc_batch_run are DEVICE pointers (hipMalloc or torch
 *     CUDA tensors), fp32, instance-minor "[field][B]" layout so that lane i of a wave reads element i.
 *   - `stream` is a hipStream_t (NULL = default stream). Calls are asynchronous on that stream.
 *   - Return value: 0 on success, < 0 on an API error (see nmpc_last_error()). Per-instance solver
 *     status codes follow acados (0 success, 1 NaN detected, 4 QP failure) and are written to `status`.
 *   - Array outputs may be NULL when not wanted.
 */
#ifndef NMPC_AMD_NMPC_BATCH_H
#define NMPC_AMD_NMPC_BATCH_H

#include "nmpc_amd/nmpc_path.h"

#ifdef __cplusplus
extern "C" {
#endif

#define NMPC_MODEL_DIFF2AMR 0
#define NMPC_MODEL_OMNI4AMR 1
#define NMPC_MODEL_TRIC3AMR 2

#define NMPC_OK 0
#define NMPC_ERR_ARG (-1)
#define NMPC_ERR_HIP (-2)
#define NMPC_ERR_UNSUPPORTED (-3)

/* Model + OCP + solver configuration. Mirrors the two parameter surfaces of the reference:
 *   codegen yaml  config/nmpc_nav_control_acados_models.yaml  (N, dt = 1/freq; bakes the model)
 *   ROS yaml      config/nmpc_nav_control.yaml                (dt_ctrl = 1/control_freq, p, bounds, W) */
typedef struct nmpc_model_params {
    int model; /* NMPC_MODEL_* */
    int N;     /* horizon (common.py:6: N = ceil(tf_ini / dt)) */
    double dt;      /* solver time step */
    double dt_ctrl; /* wrapper time step used for vel_ref integration (NMPCNavControlDiff.cpp:155-157) */
    double p[3];    /* diff {b, tau_v}; omni4 {l1+l2, tau_v}; tric {d, tau_v, tau_a} */
    double lbx[4], ubx[4]; /* bounds of the ref states idxbx (stages 1..N) */
    double lbu[4], ubu[4]; /* bounds of the inputs idxbu (stages 0..N-1) */
    double W[15];   /* stage weight diagonal [Q_diag; R_diag] (NY entries) */
    double W_e[11]; /* terminal weight diagonal (NX entries); constructors set it to Q_diag */
    int terminal_hack; /* diff run(): x100 terminal pose weight when yref[N]==yref[N-1] (default 1 for diff) */
    int tric_sin_bug;  /* tric_amr_model.py:45 cos_alpha = sin(alpha) (default 1: reproduce) */
    int qp_iter_max;   /* 50 */
    double qp_tol_stat, qp_tol_ineq, qp_tol_comp; /* fp32 stopping rule, see DESIGN.md */
    double qp_mu0, qp_thr0, qp_tau;              /* IPM initial point and fraction-to-boundary */
    /* IPM direction rule: NMPC_IPM_SINGLE (default) one Newton direction per iteration with the centring
     * sigma = clamp((1 - alpha_prev)^2, qp_sigma_lo, qp_sigma_hi); NMPC_IPM_MEHROTRA predictor-corrector (the
     * fp64 oracle's rule). Both solve the same QP to the same stopping rule (DESIGN.md "Algorithm"). */
    int qp_ipm;
    double qp_sigma_lo, qp_sigma_hi; /* 0.01, 0.5 */
    /* IPM warm start (default 1): a robot whose previous solve on this handle succeeded starts its bound
     * multipliers at max(lambda_previous, qp_warm_kappa / t) instead of qp_mu0 / t (the QP solution is the same;
     * the IPM path is shorter, so qp_iter counts are not acados'). This departs from the reference, whose
     * generated HPIPM never sets qp_solver_warm_start (every QP there starts cold); 0 restores that. Reset robots,
     * nmpc_batch_init_iterate and nmpc_batch_forget_warm start cold. The multipliers live in the handle's slot i
     * of instance i: keep an instance's slot stable across calls (nmpc_batch_solve_iterate included) or clear it
     * with nmpc_batch_forget_warm. The capsule ABI warm-starts a capsule only while it still owns its engine slot
     * (its last solve there succeeded and no reset / create came in between), with kappa 0.01. */
    int qp_warm_start;
    double qp_warm_kappa; /* diff 0.2, omni4 / tric 0.01 */
    /* Warm-start only after a solve that converged within this many IPM iterations (default 12; 0 = qp_iter_max).
     * A robot whose QP was hard last tick starts its next IPM cold: warm-started multipliers speed up the easy
     * majority but lengthen exactly the hard QPs that set the launch time (DESIGN.md "Algorithm and precision"). */
    int qp_warm_iter_max;
    /* Early infeasibility exit (status 4): the IPM stops once its largest bound multiplier exceeds
     * qp_infeas_lambda * max(1, w_max / 10) (w_max: the largest stage or terminal weight of the robot, terminal
     * hack included) while the bound residual stays above 1e-3. HPIPM has no such test (a hard QP runs to
     * qp_iter_max, which acados' RTI accepts), so 0 switches it off; the batched default is 1e5, the capsule ABI
     * default 0 (acados semantics). */
    double qp_infeas_lambda;
} nmpc_model_params;

enum { NMPC_IPM_MEHROTRA = 0, NMPC_IPM_SINGLE = 1 };

typedef struct nmpc_batch nmpc_batch;

/* Dimensions of a model: nx, nu, ny (=nx+nu), nbx, nbu, np. Any pointer may be NULL. */
int nmpc_model_dims(int model, int* nx, int* nu, int* ny, int* nbx, int* nbu, int* np);
/* Defaults = the reference's shipped runtime configuration. */
int nmpc_model_params_default(int model, int N, nmpc_model_params* prm);
/* Bounds from the wrapper-constructor scalars (NMPCNavControlDiff.cpp:18-22, NMPCNavControlOmni4.cpp:18-22,
 * NMPCNavControlTric.cpp:18-29): ref states in [-v_max, v_max] (tric alpha_ref in [alpha_min, alpha_max]),
 * inputs in [-a_max, a_max] (tric dalpha_ref in [-dalpha_max, dalpha_max]); angles in radians. */
int nmpc_model_params_set_limits(nmpc_model_params* prm, double v_max, double a_max, double alpha_min,
                                 double alpha_max, double dalpha_max);

/* Create a batch engine for up to `capacity` instances on the current HIP device. The iterate is
 * initialised with {name}_acados_create semantics (x = [0,0,pi,0,...], u = 0) and carried refs = 0. */
int nmpc_batch_create(const nmpc_model_params* prm, int capacity, nmpc_batch** out);
int nmpc_batch_destroy(nmpc_batch* b);
/* Replace weights / bounds / parameters / QP options (model and N must not change). */
int nmpc_batch_set_params(nmpc_batch* b, const nmpc_model_params* prm);
int nmpc_batch_get_params(const nmpc_batch* b, nmpc_model_params* prm);
/* Re-initialise instances [0, B): mode 0 = create semantics (x = [0,0,pi,0,...], u = 0, carried ref states 0);
 * mode 1 = reset semantics ({name}_acados_reset: iterate zeroed, the carried ref states kept, like the
 * per-robot `reset` mask of nmpc_batch_solve / nmpc_batch_run). */
int nmpc_batch_init_iterate(nmpc_batch* b, int B, int mode, void* stream);

/* One SQP-RTI iteration ({name}_acados_solve) for instances [0, B) on caller-packed QP data:
 *   x0    [NX][B]          initial state (stage-0 lbx = ubx)
 *   yref  [N+1][ny_in][B]  stage references; entries j >= ny_in are 0 (ny_in = 3 pose-only or NY);
 *                          stage N uses entries 0..NX-1
 *   We    [NX][B] or NULL  per-instance terminal weight diagonal (NULL: params W_e)
 *   reset [B] or NULL      nonzero: zero the iterate before solving ({name}_acados_reset)
 * outputs: u0 [NU][B], x1 [NX][B], xtraj [(N+1)*NX][B], utraj [N*NU][B], status [B], qp_iter [B],
 *          qp_res [3][B] = {max |stationarity residual|, max |bound residual|, mu} at IPM exit. */
int nmpc_batch_solve(nmpc_batch* b, int B, const float* x0, const float* yref, int ny_in, const float* We,
                     const unsigned char* reset, float* u0, float* x1, float* xtraj, float* utraj, int* status,
                     int* qp_iter, float* qp_res, void* stream);

/* nmpc_batch_solve with the iterate held by the caller instead of the handle: xbar [(N+1)*NX][ld] and
 * ubar [N*NU][ld] (device) are read as the linearisation point and overwritten with the new iterate (a failed solve
 * keeps its own). Used by the capsule ABI, whose iterate travels with each call; the warm-start records are still
 * the handle's (slot i = instance i). */
int nmpc_batch_solve_iterate(nmpc_batch* b, int B, const float* x0, const float* yref, int ny_in, const float* We,
                             const unsigned char* reset, float* xbar, float* ubar, int ld, int* status, int* qp_iter,
                             float* qp_res, void* stream);

/* Batched NMPCNavControl*::run(): pre-solve + SQP-RTI + post-solve for B robots.
 *   pose  [3][B] {x, y, theta}; vel [3][B] {v, vn, w}; steer [B] (tric; NULL = 0)
 *   traj  [N+1][3][B] reference poses; traj_len [B] poses valid per robot (NULL = N+1; padded with the
 *         last valid pose, NMPCNavControlDiff.cpp:113-117)
 * outputs: cmd [3][B] (diff {v, w, 0}, omni4 {v, vn, w}, tric {v, alpha, 0}), u0 [NU][B], status, qp_iter,
 * qp_res [3][B] (as nmpc_batch_solve). The carried vel-ref states are kept on the device between calls
 * (NMPCNavControlDiff.cpp:168-172). A robot whose solve fails (status != 0) gets a zero (stop) cmd, keeps its
 * carried refs and its iterate: the reference throws there and the node publishes a stop command
 * (NMPCNavControl.cpp:14-23, NMPCNavControlROS.cpp:716-719). Failures stay on their robot: a NaN robot exits
 * its IPM at the first iteration and no other robot's arithmetic depends on it. */
int nmpc_batch_run(nmpc_batch* b, int B, const float* pose, const float* vel, const float* steer,
                   const float* traj, const int* traj_len, const unsigned char* reset, float* cmd, float* u0,
                   int* status, int* qp_iter, float* qp_res, void* stream);

/* A path-following tick in one launch: PathDiscretizer::getNextNPoses (nmpc_path.h, PathDiscretizer.cpp:14-63)
 * of every robot followed by nmpc_batch_run on those N+1 poses -- processFollowPath's discretize + run
 * (NMPCNavControlROS.cpp:666-668 -> :713) without the trip of the poses through a second launch. The march
 * runs in the solve kernel (fp64, the reference's operation order: the same poses as nmpc_path_discretize
 * with num_poses = N+1, bit for bit). Arguments as nmpc_path_discretize and nmpc_batch_run; traj_out
 * [N+1][3][B] receives the poses (NULL: not written). Every robot's reference has N+1 poses (padded with the
 * path end). nseg [B] >= 1. */
int nmpc_batch_run_path(nmpc_batch* b, int B, const float* pose, const float* vel, const float* steer,
                        const nmpc_path_segment* segs, int seg_stride, const int* nseg, const double* nearest_u,
                        double sample_period, int is_holonomic, const unsigned char* reset, float* traj_out,
                        float* cmd, float* u0, int* status, int* qp_iter, float* qp_res, void* stream);

/* Kernel variant: NMPC_KERNEL_TEAM (16-lane team per robot, DPP row exchange) is the only one; any other value
 * returns NMPC_ERR_UNSUPPORTED. (The round-1 one-lane-per-robot kernel was removed: its fp32 factor is not
 * accurate enough at bench scale, DESIGN.md "Algorithm and precision".) */
#define NMPC_KERNEL_TEAM 0
int nmpc_batch_set_kernel(nmpc_batch* b, int kernel);

/* Team placement of the team kernel (no effect on any result; DESIGN.md "Scheduling"). A robot's IPM iteration
 * count persists from tick to tick, so the handle keeps each robot's last count and, before a launch, orders the
 * robots by it (one small sort kernel on the same stream):
 *   NMPC_SCHED_OFF          robot i in team slot i;
 *   NMPC_SCHED_AUTO         (default) NMPC_SCHED_SORTED when the launch has more waves (B/4) than the device
 *                           has SIMDs, else OFF (with one wave per SIMD the slowest robot sets the time
 *                           whatever the placement);
 *   NMPC_SCHED_SORTED       hardest robots in the lowest slots (tric N=60 B=8192: 5.24 -> 5.06 ms per tick);
 *   NMPC_SCHED_INTERLEAVED  even 16-team blocks from the hard end, odd blocks from the easy end (best when
 *                           several models' launches share the GPU on concurrent streams: mixed fleet
 *                           4.44 -> 4.26 ms per tick). */
#define NMPC_SCHED_OFF 0
#define NMPC_SCHED_AUTO 1
#define NMPC_SCHED_SORTED 2
#define NMPC_SCHED_INTERLEAVED 3
#define NMPC_SCHED_SPREAD 4 /* the hardest 4 robots per block in its first wave, easy CU-mates (schedule.hip) */
int nmpc_batch_set_schedule(nmpc_batch* b, int mode);

/* Device pointers of the resident state: xbar [(N+1)*NX][stride], ubar [N*NU][stride],
 * carried [NBX][stride]; stride = capacity. */
int nmpc_batch_state(nmpc_batch* b, float** xbar, float** ubar, float** carried, int* stride);

/* Forget the IPM warm start of instances [0, B) where mask[i] != 0 (mask NULL: all of them): their next solve
 * starts its multipliers cold (qp_mu0 / t), as after a reset, while the iterate is kept. For callers that move
 * instances between slots (a slot's multipliers belong to whatever instance solved there last). mask: device. */
int nmpc_batch_forget_warm(nmpc_batch* b, int B, const unsigned char* mask, void* stream);

/* Device pointers of the IPM warm-start state (qp_warm_start): warm [capacity] per-robot flags and the scratch
 * records [scratch_bytes] that hold each robot's multipliers. A flag is 0 (the next solve starts cold) or the tag of
 * the record layout its multipliers were stored in (NMPC_WARM_TAG_*): a solve reads them only when its launch uses
 * the same layout, so a robot whose launches change kernel or layout (e.g. a handle whose batch crosses the
 * row-parallel kernel's limit) starts cold on its own, and no other robot is touched. With nmpc_batch_state this
 * is everything a solve reads from the handle, e.g. to checkpoint a fleet or to replay a tick bit for bit.
 * Checkpoints of this state are tied to the library version that wrote them: before round 5 a flag of 1 meant
 * "succeeded", whatever the layout, and now reads as NMPC_WARM_TAG_WIDE (a tric team-kernel record written then
 * was split-layout). After restoring a warm state saved by an older build, call nmpc_batch_forget_warm on the
 * restored robots: their first solve then starts cold (wrong warm multipliers would only be clamped, costing
 * IPM iterations, never a wrong solution). */
#define NMPC_WARM_TAG_WIDE 1     /* single-direction field order, one record per lane (team / row-parallel) */
#define NMPC_WARM_TAG_SPLIT 2    /* the team kernel's split core / bound planes */
#define NMPC_WARM_TAG_MEHROTRA 3 /* the Mehrotra rule's field order (NMPC_IPM_MEHROTRA) */
int nmpc_batch_warm_state(nmpc_batch* b, unsigned char** warm, float** scratch, size_t* scratch_bytes);

/* Record layout of the team kernel's single-direction scratch records, a per-handle choice fixed at create time
 * and changed only by this call (never by other handles):
 *   NMPC_REC_WIDE   one 64-B record per lane and stage (diff's default alone on a device: the metric fleet's
 *                   107 MB fit the Infinity Cache, and the issue-bound kernel is 1.2 % faster with it);
 *   NMPC_REC_SPLIT  core and bound planes (tric always; diff beside other resident fleets: the mixed fleet's
 *                   272 MB drop under the 256 MB Infinity Cache, 5.25 -> 5.70 M it/s);
 *   NMPC_REC_AUTO   the model's choice from this handle alone: tric SPLIT, omni4 WIDE, diff SPLIT when its own
 *                   records (capacity x (N+1) x 640 B) exceed 192 MB, else WIDE.
 * diff accepts all three; tric only SPLIT / AUTO and omni4 only WIDE / AUTO (NMPC_ERR_UNSUPPORTED otherwise). The
 * environment variable NMPC_AMD_REC_SPLIT (0 / 1) overrides the create-time choice (A/B runs). Changing the layout
 * leaves every robot's warm flag in place: each robot starts its next IPM cold because its tag no longer matches. */
#define NMPC_REC_AUTO (-1)
#define NMPC_REC_WIDE 0
#define NMPC_REC_SPLIT 1
int nmpc_batch_set_record_layout(nmpc_batch* b, int layout);

/* The warm-start rule the solve kernels apply (the parameters after the NMPC_AMD_WARM / NMPC_AMD_WARM_ITER_MAX
 * overrides): a robot's flag is set after a solve iff warm && status == 0 && iterations < iter_max &&
 * iterations <= warm_iter_max. Hosts that mirror the device flags (the capsule shim) use this, not their copy of
 * the parameters. Each output may be NULL. */
int nmpc_batch_warm_rule(const nmpc_batch* b, int* warm, int* warm_iter_max, int* iter_max);

/* The launch a call of B robots makes on this handle (nmpc_batch_plan_ex; nmpc_batch_plan: a solve launch):
 *   kernel          0 = k_sqp_rti_team (four robots per wave), 1 = k_sqp_rti_rowpar;
 *   waves_per_robot the row-parallel kernel's waves per robot (0 for the team kernel);
 *   segments        its horizon segments (0 = the serial phases, or the team kernel);
 *   record_layout   NMPC_REC_WIDE / NMPC_REC_SPLIT: the scratch record layout of the launch;
 *   warm_tag        the NMPC_WARM_TAG_* the launch reads and writes (nmpc_batch_warm_state);
 *   record_bytes    this handle's records touched per sweep over its capacity (the NMPC_REC_AUTO measure).
 * mode: NMPC_PLAN_SOLVE (nmpc_batch_solve / _solve_iterate), NMPC_PLAN_RUN (nmpc_batch_run: run mode keeps the
 * reference poses in LDS, which can push a long horizon off the row-parallel kernel) or NMPC_PLAN_RUN_PATH
 * (nmpc_batch_run_path: always the team kernel). */
#define NMPC_PLAN_SOLVE 0
#define NMPC_PLAN_RUN 1
#define NMPC_PLAN_RUN_PATH 2
typedef struct nmpc_launch_plan {
    int kernel, waves_per_robot, segments, record_layout, warm_tag;
    size_t record_bytes;
} nmpc_launch_plan;
int nmpc_batch_plan_ex(const nmpc_batch* b, int B, int mode, nmpc_launch_plan* plan);
int nmpc_batch_plan(const nmpc_batch* b, int B, int* kernel, int* waves_per_robot, int* segments);

/* Bench / test harness: closed-loop plant step and path-reference regeneration for B robots
 * (see DESIGN.md "Synthetic closed loop"). All device pointers, [field][B]:
 *   path [6][B] = {x0, y0, th0, kappa, speed, length} circular-arc paths; goal-pose robots have length < 0
 *   and {x0, y0, th0} is the goal. s [B] arc-length progress (in/out). pose/vel/steer in/out: advanced by
 *   one RK4 step of the plant with the applied input u0 [NU][B]; traj [N+1][3][B], traj_len [B] out. */
int nmpc_fleet_sim_step(nmpc_batch* b, int B, const float* path, float* s, float* pose, float* vel, float* steer,
                        const float* u0, const int* status, float* traj, int* traj_len, int advance, void* stream);

/* Stationary closed loop (bench / test harness): the fleet manager issues a robot a new goal or path when it
 * has arrived (the end-of-trajectory test of processGoToPose / processFollowPath, NMPCNavControlROS.cpp:637-643 /
 * :682-693, with |heading error|) or when its current one has been active for `ttl` ticks, and the node resets
 * the controller as its goal / path callbacks do (reset_mpc -> {name}_acados_reset, NMPCNavControlROS.cpp:304-327):
 * `reset` [B] is set for the next nmpc_batch_run. A new target depends only on (seed, start + robot index, event
 * count) and the robot's pose: draw j of event e is u = (h >> 8) / 2^24 with h = nmpc_fleet_hash(seed,
 * global index, 16 e + j) (the same 32-bit integer hash on host and device), so any sharding or stream grouping
 * issues the same targets. Goal robots (path length < 0) get a goal at distance U(goal_r_lo, goal_r_hi) in a
 * uniform direction with a uniform heading; path robots an arc starting within 0.2 m / 0.3 rad of the robot
 * (curvature U(-kappa_max, kappa_max), speed U(speed_lo, speed_hi), length U(len_lo, len_hi)), progress s = 0.
 * The new ttl is ttl_min + ((h >> 8) * (ttl_max - ttl_min + 1) >> 24).
 * `stats` (optional) accumulates the statistics of the solve that preceded this step in the same launch, before the
 * renewal rewrites `reset` (so `cold_*` count the solves that ran with reset set): */
typedef struct nmpc_fleet_stats {
    const int* qp_iter;         /* [B] in: the solve's executed IPM iterations */
    long long* iters_sum;       /* [B] += qp_iter */
    int* iters_max;             /* [B] = max(iters_max, qp_iter) */
    long long* fail_cnt;        /* [B] += (status != 0) */
    long long* hist;            /* [64] += robots per executed iteration count (clamped to [0, 63]) */
    long long* cold_cnt;        /* [B] += reset */
    long long* cold_iters;      /* [B] += reset * qp_iter */
} nmpc_fleet_stats;
typedef struct nmpc_fleet_renew {
    unsigned int seed;
    int start;                  /* global index of robot 0 of this call */
    int ttl_min, ttl_max;       /* ticks a goal / path stays active (inclusive range) */
    float goal_r_lo, goal_r_hi; /* m */
    float kappa_max, speed_lo, speed_hi, len_lo, len_hi;
    float pos_tol, ang_tol;     /* final_position_error (m) / final_orientation_error (rad), nmpc_nav_control.yaml:6-7 */
    int* ev;                    /* [B] events so far (in/out) */
    int* ttl;                   /* [B] ticks left (in/out) */
    unsigned char* reset;       /* [B] in: the flags the last solve ran with; out: 1 where this step issued a new
                                 * goal / path */
    const nmpc_fleet_stats* stats; /* NULL: no statistics (every pointer of a given one is required, and status) */
} nmpc_fleet_renew;
int nmpc_fleet_sim_step_renew(nmpc_batch* b, int B, float* path, float* s, float* pose, float* vel, float* steer,
                              const float* u0, const int* status, float* traj, int* traj_len,
                              const nmpc_fleet_renew* renew, void* stream);
/* The harness hash: lowbias32(lowbias32(lowbias32(seed ^ 0x9e3779b9) + index) + counter) (uint32 arithmetic). */
unsigned int nmpc_fleet_hash(unsigned int seed, unsigned int index, unsigned int counter);

const char* nmpc_last_error(void);
const char* nmpc_version(void);

#ifdef __cplusplus
}
#endif
#endif
