// ubench_master.hip -- unit check of the segmented-Riccati master's fused-DPP blocks (team_asm_gen.hpp mst_*,
// team_common.hpp rowchol) on one 16-lane row against a host fp64 reference: for a positive semidefinite G (= -Gam,
// full rank, rank 3 and zero), Q = Phat (I + G Phat)^-1 as Y Y', Y = L R^-T (L L' = Phat, R R' = I + L' G L),
// Phat' = Phat + F Q F', the vector blocks c = t + (-G) phat and w = phat + Q c. Prints one JSON line per case, and
// (first case) the cycles per step of chained master steps and of their parts (k_master_time).
// build: make -C nmpc_nav_control_amd/csrc ubench_master   run: build/ubench_master
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "team_common.hpp"

using namespace nmpc;
constexpr int NX = 7, NU = 2;

__global__ void k_master(const double* Ph, const double* G, const double* F, const double* vt, const double* vp,
                         double* oQ, double* oPn, double* oc, double* ow)
{
    __shared__ double sL[NX * NX];
    const int r = threadIdx.x & 15;
    const bool is_x = r >= NU && r < NU + NX;
    const int xi = is_x ? r - NU : 0;
    double Phr[NX], Lp[NX], Fr[NX], Gr[NX], Gn[NX], rdv[NX];
#pragma unroll
    for (int c = 0; c < NX; c++) {
        Phr[c] = Ph[xi * NX + c];
        Lp[c] = Phr[c];
        Fr[c] = F[xi * NX + c];
        Gr[c] = G[xi * NX + c];  // -Gam
        Gn[c] = -G[xi * NX + c];  // Gam
    }
    rowchol<NX, NU, true>(Lp, rdv, xi, 0.0, 1e-13);
    if (is_x)
        for (int c = 0; c < NX; c++) sL[xi * NX + c] = Lp[c];
    __syncthreads();
    double Lt[NX], V[NX], K[NX];
#pragma unroll
    for (int c = 0; c < NX; c++) {
        Lt[c] = sL[c * NX + xi];
        V[c] = 0.0;
        K[c] = (xi == c) ? 1.0 : 0.0;
    }
    mst_rowmul_lt<NX, NU>(V, Gr, Lp);  // as the kernel: L lower triangular, K's lower triangle only
    mst_rowmul_lt<NX, NU>(K, Lt, V);
    rowchol<NX, NU, false>(K, rdv, xi, 0.5);
    sfor<0, NX>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        const double y = Lp[j] * rdv[j];
        Lp[j] = y;
        if constexpr (j + 1 < NX) mst_trsv<NX, NU, j>(Lp, K[j], y);
    });
    double Q[NX], Wr[NX], Pn[NX];
#pragma unroll
    for (int c = 0; c < NX; c++) {
        Q[c] = 0.0;
        Wr[c] = 0.0;
        Pn[c] = Phr[c];
    }
    mst_rowdot<NX, NU>(Q, Lp, Lp);  // Q = Y Y'
    mst_rowmul<NX, NU>(Wr, Fr, Lp);  // W = F Y
    mst_rowdot<NX, NU>(Pn, Wr, Wr);  // Phat' = Phat + W W' (= Phat + F Q F')
    const double cv = mst_vdot<NX, NU>(vt[xi], vp[xi], Gn);
    const double w = mst_vdot<NX, NU>(vp[xi], cv, Q);
    if (is_x) {
        for (int c = 0; c < NX; c++) {
            oQ[xi * NX + c] = Q[c];
            oPn[xi * NX + c] = Pn[c];
        }
        oc[xi] = cv;
        ow[xi] = w;
    }
}

// Timing: a chain of `steps` dependent master steps on row 0 of one wave, the segment data in LDS as in the kernel.
// VAR 0: the kernel's backward step (qform + Phat_i = P + Phi Q Phi' + the vector terms); 1: one rowchol of Phat per
// step; 2: qform only (Phat <- P + Q); 3: the two products of the Phat update only. cyc[0, 1]: s_memtime and
// s_memrealtime (100 MHz) deltas of the chain.
template <int VAR, int UNR = 1>
__global__ void k_master_time(const double* Ph0, const double* G, const double* F, int steps,
                              unsigned long long* cyc, double* sink)
{
    __shared__ double sP[NX * NX], sG[NX * NX], sLw[4][NX * NX];
    double* const sL = sLw[threadIdx.x >> 6];
    __shared__ float sF[NX * NX], sV[2 * NX];
    for (int i = threadIdx.x; i < NX * NX; i += blockDim.x) {
        sP[i] = Ph0[i];
        sG[i] = -G[i];  // Gam
        sF[i] = (float)F[i];
    }
    for (int i = threadIdx.x; i < 2 * NX; i += blockDim.x) sV[i] = 0.01f * (float)i;
    __syncthreads();
    const int r = threadIdx.x & 15;
    const bool is_x = r >= NU && r < NU + NX;
    const int xi = is_x ? r - NU : 0;
    double Ph[NX], ph = 0.0;
#pragma unroll
    for (int c = 0; c < NX; c++) Ph[c] = sP[xi * NX + c];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll UNR
    for (int k = 0; k < steps; k++) {
        if constexpr (VAR == 0) {
            double Gn[NX], Q[NX];
#pragma unroll
            for (int c = 0; c < NX; c++) Gn[c] = -sG[xi * NX + c];
            mst_qform<NX, NU>(Ph, Gn, Q, sL, xi, is_x);
            double Fr[NX], Gr[NX], T[NX];
#pragma unroll
            for (int c = 0; c < NX; c++) {
                Fr[c] = (double)sF[xi * NX + c];
                Gr[c] = sG[xi * NX + c];
                T[c] = 0.0;
                Ph[c] = sP[xi * NX + c];
            }
            const double cv = mst_vdot<NX, NU>((double)sV[xi], ph, Gr);
            mst_rowdot<NX, NU>(T, Q, Fr);
            mst_rowmul<NX, NU>(Ph, Fr, T);
            const double w = mst_vdot<NX, NU>(ph, cv, Q);
            ph = mst_vdot<NX, NU>((double)sV[NX + xi], w, Fr);
        } else if constexpr (VAR == 7) {  // wave 0 the backward step, the other waves the dual step (other code)
            if (threadIdx.x < 64) {
                double Gn[NX], Q[NX];
#pragma unroll
                for (int c = 0; c < NX; c++) Gn[c] = -sG[xi * NX + c];
                mst_qform<NX, NU>(Ph, Gn, Q, sL, xi, is_x);
                double Fr[NX], Gr[NX], T[NX];
#pragma unroll
                for (int c = 0; c < NX; c++) {
                    Fr[c] = (double)sF[xi * NX + c];
                    Gr[c] = sG[xi * NX + c];
                    T[c] = 0.0;
                    Ph[c] = sP[xi * NX + c];
                }
                const double cv = mst_vdot<NX, NU>((double)sV[xi], ph, Gr);
                mst_rowdot<NX, NU>(T, Q, Fr);
                mst_rowmul<NX, NU>(Ph, Fr, T);
                const double w = mst_vdot<NX, NU>(ph, cv, Q);
                ph = mst_vdot<NX, NU>((double)sV[NX + xi], w, Fr);
            } else {
                double Pr[NX], Q[NX];
#pragma unroll
                for (int c = 0; c < NX; c++) Pr[c] = sP[xi * NX + c];
                mst_qform<NX, NU>(Ph, Pr, Q, sL, xi, is_x);
                const double e = mst_vdot<NX, NU>((double)sV[NX + xi], ph, Pr);
                const double u = mst_vdot<NX, NU>(ph, -e, Q);
                double Fc[NX], T[NX];
#pragma unroll
                for (int c = 0; c < NX; c++) {
                    Fc[c] = (double)sF[c * NX + xi];
                    Ph[c] = sG[xi * NX + c];
                    T[c] = 0.0;
                }
                mst_rowdot<NX, NU>(T, Q, Fc);
                mst_rowmul<NX, NU>(Ph, Fc, T);
                ph = mst_vdot<NX, NU>((double)sV[xi], u, Fc);
            }
        } else if constexpr (VAR == 1) {
            double Lp[NX], rdv[NX];
#pragma unroll
            for (int c = 0; c < NX; c++) Lp[c] = Ph[c];
            rowchol<NX, NU, true>(Lp, rdv, xi, 0.0, 1e-13);
#pragma unroll
            for (int c = 0; c < NX; c++) Ph[c] = sP[xi * NX + c] + 1e-3 * Lp[c];
        } else if constexpr (VAR == 4) {
            double Lp[NX], rdv[NX];
#pragma unroll
            for (int c = 0; c < NX; c++) Lp[c] = Ph[c];
            rowchol<NX, NU, true, true>(Lp, rdv, xi, 0.0, 1e-13);
#pragma unroll
            for (int c = 0; c < NX; c++) Ph[c] = sP[xi * NX + c] + 1e-3 * Lp[c];
        } else if constexpr (VAR == 5) {  // the LDS transpose round trip of qform alone
#pragma unroll
            for (int c = 0; c < NX; c++)
                if (is_x) sL[xi * NX + c] = Ph[c];
            lds_fence();
#pragma unroll
            for (int c = 0; c < NX; c++) Ph[c] = sL[c * NX + xi] * 0.999 + sP[xi * NX + c];
        } else if constexpr (VAR == 2) {
            double Gn[NX], Q[NX];
#pragma unroll
            for (int c = 0; c < NX; c++) Gn[c] = -sG[xi * NX + c];
            mst_qform<NX, NU>(Ph, Gn, Q, sL, xi, is_x);
#pragma unroll
            for (int c = 0; c < NX; c++) Ph[c] = sP[xi * NX + c] + Q[c];
        } else {
            double Fr[NX], T[NX], Q[NX];
#pragma unroll
            for (int c = 0; c < NX; c++) {
                Fr[c] = (double)sF[xi * NX + c];
                T[c] = 0.0;
                Q[c] = 1e-3 * Ph[c];
                Ph[c] = sP[xi * NX + c];
            }
            mst_rowdot<NX, NU>(T, Q, Fr);
            mst_rowmul<NX, NU>(Ph, Fr, T);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = r1 - r0;
    }
    double acc = ph;
#pragma unroll
    for (int c = 0; c < NX; c++) acc += Ph[c];
    sink[threadIdx.x] = acc;
}

// accuracy of the hardware fp64 reciprocal square root (v_rsq_f64) against 1 / sqrt in fp64
__global__ void k_rsq_acc(const double* x, double* out, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __builtin_amdgcn_rsq(x[i]);
}

static void rsq_accuracy()
{
    const int n = 1 << 16;
    std::vector<double> x(n), y(n);
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> ud(-30.0, 30.0);
    for (auto& v : x) v = std::pow(10.0, ud(rng) / 3.0);
    double *dx, *dy;
    (void)hipMalloc(&dx, n * 8);
    (void)hipMalloc(&dy, n * 8);
    (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rsq_acc, dim3(n / 256), dim3(256), 0, nullptr, dx, dy, n);
    (void)hipMemcpy(y.data(), dy, n * 8, hipMemcpyDeviceToHost);
    double worst = 0.0;
    for (int i = 0; i < n; i++) worst = std::fmax(worst, std::fabs(y[i] * std::sqrt(x[i]) - 1.0));
    std::printf("{\"rsq_f64_max_rel_err\": %.3e, \"samples\": %d}\n", worst, n);
    (void)hipFree(dx);
    (void)hipFree(dy);
}

template <int VAR, int UNR = 1>
static void time_variant(const double* dPh, const double* dG, const double* dF, const char* name, int threads = 64)
{
    unsigned long long* dc;
    double* ds;
    (void)hipMalloc(&dc, 2 * sizeof(unsigned long long));
    (void)hipMalloc(&ds, 64 * sizeof(double));
    const int steps = 256;
    unsigned long long c[2] = {0, 0};
    for (int rep = 0; rep < 3; rep++) {  // the last of three launches (the first ones warm the instruction cache)
        hipLaunchKernelGGL((k_master_time<VAR, UNR>), dim3(1), dim3(threads), 0, nullptr, dPh, dG, dF, steps, dc, ds);
        (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
    }
    const double ghz = c[1] ? (double)c[0] / ((double)c[1] * 10.0) : 0.0;
    std::printf("{\"timing\": \"%s\", \"unroll\": %d, \"waves\": %d, \"steps\": %d, \"cycles_per_step\": %.1f, "
                "\"ns_per_step\": %.1f, \"clock_ghz\": %.3f}\n", name, UNR, threads / 64, steps, (double)c[0] / steps,
                (double)c[1] * 10.0 / steps, ghz);
    (void)hipFree(dc);
    (void)hipFree(ds);
}

// host reference: A^-1 B by Gauss-Jordan with partial pivoting (n x n, row-major)
static void solve(std::vector<double> A, std::vector<double>& B, int n)
{
    for (int j = 0; j < n; j++) {
        int p = j;
        for (int i = j + 1; i < n; i++)
            if (std::fabs(A[i * n + j]) > std::fabs(A[p * n + j])) p = i;
        for (int c = 0; c < n; c++) {
            std::swap(A[j * n + c], A[p * n + c]);
            std::swap(B[j * n + c], B[p * n + c]);
        }
        const double d = A[j * n + j];
        for (int c = 0; c < n; c++) {
            A[j * n + c] /= d;
            B[j * n + c] /= d;
        }
        for (int i = 0; i < n; i++) {
            if (i == j) continue;
            const double f = A[i * n + j];
            for (int c = 0; c < n; c++) {
                A[i * n + c] -= f * A[j * n + c];
                B[i * n + c] -= f * B[j * n + c];
            }
        }
    }
}

int main()
{
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    const int n = NX, nn = NX * NX;
    int bad = 0;
    for (int cs = 0; cs < 6; cs++) {
        const int rank = (cs % 3 == 0) ? 7 : ((cs % 3 == 1) ? 3 : 0);
        const double pscale = (cs < 3) ? 1e2 : 1e8;
        std::vector<double> A(nn), H(n * 7), Ph(nn), G(nn, 0.0), F(nn), vt(n), vp(n);
        for (auto& v : A) v = nd(rng);
        for (auto& v : H) v = 3.0 * nd(rng);
        for (auto& v : F) v = nd(rng);
        for (auto& v : vt) v = nd(rng);
        for (auto& v : vp) v = nd(rng);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                double s = 0.0, g = 0.0;
                for (int l = 0; l < n; l++) s += A[i * n + l] * A[j * n + l];
                for (int l = 0; l < rank; l++) g += H[i * 7 + l] * H[j * 7 + l];
                Ph[i * n + j] = pscale * s;
                G[i * n + j] = (double)(float)g;  // the kernel's -Gam is an fp32 sum
            }
        for (int i = 0; i < n; i++)
            for (int j = 0; j < i; j++) G[i * n + j] = G[j * n + i];
        double *dPh, *dG, *dF, *dvt, *dvp, *dout;
        (void)hipMalloc(&dPh, nn * 8);
        (void)hipMalloc(&dG, nn * 8);
        (void)hipMalloc(&dF, nn * 8);
        (void)hipMalloc(&dvt, n * 8);
        (void)hipMalloc(&dvp, n * 8);
        (void)hipMalloc(&dout, (3 * nn + 2 * n) * 8);
        (void)hipMemcpy(dPh, Ph.data(), nn * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(dG, G.data(), nn * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(dF, F.data(), nn * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(dvt, vt.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(dvp, vp.data(), n * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_master, dim3(1), dim3(64), 0, nullptr, dPh, dG, dF, dvt, dvp, dout + nn, dout + 2 * nn,
                           dout + 3 * nn, dout + 3 * nn + n);
        if (cs == 0) {
            time_variant<0>(dPh, dG, dF, "backward_step");
            time_variant<1>(dPh, dG, dF, "rowchol");
            time_variant<2>(dPh, dG, dF, "qform");
            time_variant<3>(dPh, dG, dF, "phat_update_products");
            time_variant<4>(dPh, dG, dF, "rowchol_raw_rsq");
            time_variant<5>(dPh, dG, dF, "lds_transpose");
            // the same chain on every wave of one block (the waves of a CU running master steps side by side)
            time_variant<0>(dPh, dG, dF, "backward_step", 128);
            time_variant<0>(dPh, dG, dF, "backward_step", 256);
            time_variant<3>(dPh, dG, dF, "phat_update_products", 128);
            time_variant<1>(dPh, dG, dF, "rowchol", 128);
            time_variant<7>(dPh, dG, dF, "backward_beside_dual", 128);
            time_variant<7>(dPh, dG, dF, "backward_beside_dual", 256);
            // loop bodies of 4, 8 and 16 steps (about 20 / 40 / 80 KB of code): the instruction-cache footprint
            time_variant<0, 4>(dPh, dG, dF, "backward_step");
            time_variant<0, 8>(dPh, dG, dF, "backward_step");
            time_variant<0, 16>(dPh, dG, dF, "backward_step");
            rsq_accuracy();
        }
        std::vector<double> out(3 * nn + 2 * n);
        if (hipMemcpy(out.data(), dout, out.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) {
            std::fprintf(stderr, "hip error\n");
            return 2;
        }
        // reference: Q = Phat (I + G Phat)^-1 = ((I + G Phat)^-T Phat)^T; X' Q' = Phat with X = I + G Phat
        std::vector<double> Xt(nn), Qr(Ph), Ge(G);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                double s = (i == j) ? 1.0 : 0.0;
                for (int l = 0; l < n; l++) s += Ge[j * n + l] * Ph[l * n + i];  // (I + G Ph)^T [i][j]
                Xt[i * n + j] = s;
            }
        solve(Xt, Qr, n);  // Qr = X^-T Ph = Q^T (= Q)
        double eq = 0.0, mq = 0.0, ep = 0.0, mp = 0.0, ec = 0.0, ew = 0.0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                eq = std::fmax(eq, std::fabs(out[nn + i * n + j] - Qr[j * n + i]));
                mq = std::fmax(mq, std::fabs(Qr[i * n + j]));
                double fqf = 0.0;
                for (int a = 0; a < n; a++)
                    for (int b = 0; b < n; b++) fqf += F[i * n + a] * Qr[a * n + b] * F[j * n + b];
                const double pn = Ph[i * n + j] + fqf;
                ep = std::fmax(ep, std::fabs(out[2 * nn + i * n + j] - pn));
                mp = std::fmax(mp, std::fabs(pn));
            }
        std::vector<double> cref(n);
        for (int i = 0; i < n; i++) {
            double s = vt[i];
            for (int l = 0; l < n; l++) s -= G[i * n + l] * vp[l];
            cref[i] = s;
            ec = std::fmax(ec, std::fabs(out[3 * nn + i] - s) / (1.0 + std::fabs(s)));
        }
        for (int i = 0; i < n; i++) {
            double s = vp[i];
            for (int l = 0; l < n; l++) s += Qr[i * n + l] * cref[l];
            ew = std::fmax(ew, std::fabs(out[3 * nn + n + i] - s) / (1.0 + std::fabs(s)));
        }
        // (at Phat ~ 1e8 the host reference's own pivoted solve of X loses cond(X) x eps: 1e-5 there)
        const double tol = pscale > 1e4 ? 1e-5 : 1e-9;
        const bool ok = eq / mq < tol && ep / mp < tol && ec < 1e-9 && ew < 1e-4;
        bad += !ok;
        std::printf("{\"case\": %d, \"rank_G\": %d, \"phat_scale\": %g, \"Q_rel_err\": %.3e, \"Pnext_rel_err\": %.3e, "
                    "\"c_err\": %.3e, \"w_err\": %.3e, \"ok\": %s}\n",
                    cs, rank, pscale, eq / mq, ep / mp, ec, ew, ok ? "true" : "false");
        (void)hipFree(dPh);
        (void)hipFree(dG);
        (void)hipFree(dF);
        (void)hipFree(dvt);
        (void)hipFree(dvp);
        (void)hipFree(dout);
    }
    return bad ? 1 : 0;
}
