/*
 * path_oracle.c -- CPU restatement (fp64) of PathDiscretizer::getNextNPoses.
 *
 * TEST INFRASTRUCTURE ONLY (same rules as nmpc_oracle.h): the checker of nmpc_path_discretize.
 *
 * Follows src/nmpc_nav_control/PathDiscretizer.cpp line by line:
 *   constructor             :5-12   (num_points_per_cycle 20 if sample_period >= 1 else 10, 1 % threshold)
 *   getNextNPoses           :14-63  (march in the path parameter, emit a pose every goal_dist = |v| T,
 *                                    pad with the path end)
 *   getPoseSample           :65-85  (segment index = floor(u), out-of-range -> last at u = 1 / first at u = 0,
 *                                    theta = GetTheta (+pi for v < 0) or GetThetaHolomonic)
 *   getVelSample            :87-102
 * std::pow(d, 2) is written d * d and std::min(a, b) as (b < a) ? b : a. Compiled with -ffp-contract=off so
 * that no multiply-add is fused (the device kernel is compiled the same way).
 *
 * PARITY UNPINNED for the segment math: parametric_trajectories_common::TPath (GetX/GetY/GetDX/GetDY/GetTheta/
 * GetThetaHolomonic/GetVelocity) is an external library that the reference does not vendor; the segments are
 * the cubic polynomials of include/nmpc_amd/nmpc_path.h. The reference has no tests or fixtures for this path.
 * Inputs on which the reference is undefined are handled as documented in nmpc_path.h.
 */
#include <math.h>
#include <stddef.h>

typedef struct oc_path_segment {
    double x[4], y[4], th[4];
    double v;
    double reserved[3];
} oc_path_segment;

#define OC_PATH_MAX_STEPS 65536

static void seg_param(double su, int n, int* k, double* u)
{
    if (su >= 0.0 && su < (double)n) {
        *k = (int)floor(su);
        *u = su - (double)*k;
    } else if (su >= (double)n) { /* path_num >= path_vector.size() (:69-71) */
        *k = n - 1;
        *u = 1.0;
    } else { /* path_num < 0 (:72-74) */
        *k = 0;
        *u = 0.0;
    }
}

static double poly(const double* c, double u) { return ((c[3] * u + c[2]) * u + c[1]) * u + c[0]; }
static double dpoly(const double* c, double u) { return ((3.0 * c[3]) * u + 2.0 * c[2]) * u + c[1]; }

/* getPoseSample (:65-85) */
static void pose_sample(const oc_path_segment* S, int n, double su, int holo, double* p)
{
    int k;
    double u;
    seg_param(su, n, &k, &u);
    p[0] = poly(S[k].x, u);
    p[1] = poly(S[k].y, u);
    if (!holo) {
        const double th = atan2(dpoly(S[k].y, u), dpoly(S[k].x, u));
        p[2] = (S[k].v >= 0.0) ? th : th + M_PI;
    } else {
        p[2] = poly(S[k].th, u);
    }
}

/* getVelSample (:87-102), returned as sqrt(pow(vx, 2) + pow(vy, 2)) the way :31 and :52 use it */
static double vel_norm(const oc_path_segment* S, int n, double su)
{
    int k;
    double u;
    seg_param(su, n, &k, &u);
    const double vx = dpoly(S[k].x, u), vy = dpoly(S[k].y, u);
    return sqrt(vx * vx + vy * vy);
}

static double seg_speed(const oc_path_segment* S, int n, double a)
{
    const int k = (a >= 0.0 && a < (double)n) ? (int)floor(a) : ((a >= (double)n) ? n - 1 : 0);
    return fabs(S[k].v);
}

/* getNextNPoses (:14-63) for one robot; out[num_poses][3]. Returns the number of loop steps taken. */
int oc_path_next_n_poses(const oc_path_segment* S, int n, double nearest_u, double sample_period, int num_poses,
                         int holo, double* out)
{
    const double npc = (sample_period >= 1.0) ? 20.0 : 10.0;
    const double thr = 1e-2;
    const double N = (double)n;
    int count = 0, it = 0;
    double vel = seg_speed(S, n, nearest_u); /* :23 */
    double goal_dist = vel * sample_period;
    double rel = goal_dist / npc;
    double u = nearest_u;
    double old_p[3], new_p[3];
    pose_sample(S, n, nearest_u, holo, old_p);
    double step = rel / vel_norm(S, n, nearest_u);
    double curr_dist = 0.0;
    while (u < N && it < OC_PATH_MAX_STEPS) {
        it++;
        u += step;
        u = (N < u) ? N : u;
        pose_sample(S, n, u, holo, new_p);
        const double dx = new_p[0] - old_p[0], dy = new_p[1] - old_p[1];
        curr_dist += sqrt(dx * dx + dy * dy);
        if ((goal_dist - curr_dist) <= thr * goal_dist) {
            out[3 * count + 0] = new_p[0];
            out[3 * count + 1] = new_p[1];
            out[3 * count + 2] = new_p[2];
            count++;
            const double fu = floor(u), last = N - 1.0;
            vel = seg_speed(S, n, (last < fu) ? last : fu);
            goal_dist = vel * sample_period;
            rel = goal_dist / npc;
            curr_dist = 0.0;
        }
        if (count == num_poses) break;
        step = rel / vel_norm(S, n, u);
        old_p[0] = new_p[0];
        old_p[1] = new_p[1];
        old_p[2] = new_p[2];
    }
    if (count < num_poses) {
        double last_p[3];
        pose_sample(S, n, N, holo, last_p);
        while (count < num_poses) {
            out[3 * count + 0] = last_p[0];
            out[3 * count + 1] = last_p[1];
            out[3 * count + 2] = last_p[2];
            count++;
        }
    }
    return it;
}

/* B robots, segs [B][seg_stride], out [B][num_poses][3]. */
void oc_path_discretize(int B, const oc_path_segment* segs, int seg_stride, const int* nseg, const double* nearest_u,
                        double sample_period, int num_poses, int holo, double* out, int* steps)
{
    for (int i = 0; i < B; i++) {
        const int it = oc_path_next_n_poses(segs + (size_t)i * seg_stride, nseg[i], nearest_u[i], sample_period,
                                            num_poses, holo, out + (size_t)i * num_poses * 3);
        if (steps) steps[i] = it;
    }
}
