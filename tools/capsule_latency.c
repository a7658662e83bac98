/* capsule_latency.c -- per-tick latency of the drop-in acados capsule ABI for ONE robot, driven from C exactly
 * the way the reference's wrapper drives it every control tick (NMPCNavControlDiff::run,
 * src/nmpc_nav_control/NMPCNavControlDiff.cpp:82-172):
 *   ocp_nlp_constraints_model_set(0, "lbx"/"ubx", x0)          :98-103
 *   ocp_nlp_cost_model_set(i, "yref", yref[i]) for i = 0..N     :121-124
 *   ocp_nlp_cost_model_set(N, "W", W_e)  (terminal-weight hack) :127-139
 *   diff2amr_acados_solve                                       :142
 *   ocp_nlp_get("time_tot"), ocp_nlp_out_get(0, "u"), (1, "x")   :148-170
 * The robot follows a circle of radius 0.5 m in closed loop on a kinematic plant. No Python anywhere: this is
 * the latency a C++ ROS node linked against libacados_ocp_solver_diff2amr.so sees.
 * Prints one JSON line: wall ms per tick (mean, p50, p99), the solver's own time_tot, IPM iterations.
 * usage: build/capsule_latency [ticks=300] [cold|warm]
 *   cold (default): HPIPM's cold start every tick, acados' default and the reference's generated OCP's
 *         (scripts/diff/generate_c_code.py:68-74 sets no qp_warm_start), also the capsule's default
 *   warm: ocp_nlp_solver_opts_set(.., "qp_warm_start", 2) -- the capsule's multiplier (dual) warm start
 */
#include <string.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "acados_c/ocp_nlp_interface.h"
#include "acados_solver_diff2amr.h"

#define NX DIFF2AMR_NX
#define NU DIFF2AMR_NU
#define NY DIFF2AMR_NY
#define NYN DIFF2AMR_NYN

static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static int cmp(const void* a, const void* b)
{
    const double x = *(const double*)a, y = *(const double*)b;
    return (x > y) - (x < y);
}

int main(int argc, char** argv)
{
    const int ticks = argc > 1 ? atoi(argv[1]) : 300;
    const int warm = argc > 2 && !strcmp(argv[2], "warm");
    const double dt = 1.0 / 40.0, b = 0.270;  /* control period, wheel separation (NMPCNavControlDiff) */
    const double W[NY] = {10, 10, 5, 0, 0, 0, 0, 1, 1};
    diff2amr_solver_capsule* c = diff2amr_acados_create_capsule();
    if (diff2amr_acados_create(c) != 0) { fprintf(stderr, "create failed\n"); return 1; }
    const int N = c->nlp_dims->N;
    {
        int ws = warm ? 2 : 0;  /* acados: 2 = warm-start primal and dual */
        ocp_nlp_solver_opts_set(c->nlp_config, c->nlp_opts, "qp_warm_start", &ws);
    }
    /* constructor: stage weights (NMPCNavControlDiff.cpp:62-73) */
    double Wm[NY * NY] = {0}, We[NYN * NYN] = {0};
    for (int i = 0; i < NY; i++) Wm[i * NY + i] = W[i];
    for (int k = 0; k < N; k++) ocp_nlp_cost_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, k, "W", Wm);
    for (int i = 0; i < NYN; i++) We[i * NYN + i] = W[i];
    ocp_nlp_cost_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, N, "W", We);

    double pose[3] = {0.5, 0.0, M_PI / 2}, v = 0.0, w = 0.0, vref[2] = {0.0, 0.0};
    double* wall = malloc(sizeof(double) * ticks);
    double tot_sum = 0.0;
    int it_max = 0, it_sum = 0, fails = 0;
    double(*yref)[NY] = calloc((size_t)(N + 1), sizeof(double[NY]));
    for (int t = 0; t < ticks; t++) {
        const double t0 = now_ms();
        double x0[NX] = {pose[0], pose[1], pose[2], v - w * b / 2, v + w * b / 2, vref[0], vref[1]};
        ocp_nlp_constraints_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, c->nlp_out, 0, "lbx", x0);
        ocp_nlp_constraints_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, c->nlp_out, 0, "ubx", x0);
        double prev = pose[2];
        for (int k = 0; k <= N; k++) {
            const double s = 0.02 * (t + k + 1);
            double th = 0.6 * s + M_PI / 2;
            while (th - prev > M_PI) th -= 2 * M_PI;  /* unwrapAngle */
            while (th - prev < -M_PI) th += 2 * M_PI;
            prev = th;
            yref[k][0] = 0.5 * cos(0.6 * s);
            yref[k][1] = 0.5 * sin(0.6 * s);
            yref[k][2] = th;
            ocp_nlp_cost_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, k, "yref", yref[k]);
        }
        ocp_nlp_cost_model_set(c->nlp_config, c->nlp_dims, c->nlp_in, N, "W", We);
        const int st = diff2amr_acados_solve(c);
        double tt = 0.0, u0[NU], x1[NX];
        int qp_iter = 0;
        ocp_nlp_get(c->nlp_solver, "time_tot", &tt);
        ocp_nlp_get(c->nlp_solver, "qp_iter", &qp_iter);
        ocp_nlp_out_get(c->nlp_config, c->nlp_dims, c->nlp_out, 0, "u", u0);
        ocp_nlp_out_get(c->nlp_config, c->nlp_dims, c->nlp_out, 1, "x", x1);
        vref[0] = x0[5] + u0[0] * dt;
        vref[1] = x0[6] + u0[1] * dt;
        wall[t] = now_ms() - t0;
        if (st != 0) fails++;
        /* kinematic plant: apply (v, w) from the wheel refs for one period */
        v = 0.5 * (vref[0] + vref[1]);
        w = (vref[1] - vref[0]) / b;
        pose[0] += dt * v * cos(pose[2]);
        pose[1] += dt * v * sin(pose[2]);
        pose[2] += dt * w;
        if (t >= 10) {
            tot_sum += tt * 1e3;
            it_sum += qp_iter;
            if (qp_iter > it_max) it_max = qp_iter;
        }
    }
    const int n = ticks - 10;
    double mean = 0.0;
    for (int t = 10; t < ticks; t++) mean += wall[t];
    mean /= n;
    qsort(wall + 10, n, sizeof(double), cmp);
    printf("{\"N\": %d, \"ticks\": %d, \"run_wall_ms_mean\": %.4f, \"run_wall_ms_p50\": %.4f, \"run_wall_ms_p99\": %.4f, "
           "\"time_tot_ms_mean\": %.4f, \"qp_iter_mean\": %.2f, \"qp_iter_max\": %d, \"failed\": %d, "
           "\"qp_warm_start\": %d, \"driver\": \"C, NMPCNavControlDiff::run call sequence\"}\n",
           N, ticks, mean, wall[10 + n / 2], wall[10 + (int)(0.99 * (n - 1))], tot_sum / n, (double)it_sum / n, it_max,
           fails, warm);
    diff2amr_acados_free(c);
    diff2amr_acados_free_capsule(c);
    free(wall);
    free(yref);
    return fails ? 2 : 0;
}
