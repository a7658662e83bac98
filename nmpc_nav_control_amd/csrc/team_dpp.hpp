// team_dpp.hpp -- cross-lane primitives for 16-lane teams (one DPP row of a 64-wide CDNA4 wavefront).
//
// A team is one DPP row: lanes 16t..16t+15. row_newbcast:j broadcasts lane j of each row to the whole row
// (gfx90a+), so four independent teams in a wave exchange data without LDS. Row reductions use the
// quad_perm / row_half_mirror / row_mirror butterfly, which hipcc fuses into v_add_f32_dpp.
//
// The broadcast-multiply-accumulate chains of the Riccati recursion use the fused DPP forms
// v_fmac_f32_dpp / v_fmac_f64_dpp (one VALU op per term instead of a v_mov_dpp + FMA pair). hipcc does not
// form these for row_newbcast, so they are emitted as (non-volatile, freely scheduled) inline asm; the compiler's hazard recognizer does
// not see inside asm, so every block starts with the two wait states a VALU write -> DPP read needs (s_nop 1).
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

namespace nmpc {

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E). The DPP lane operand of the
// broadcasts below must be an immediate; a switch over a runtime index inside #pragma unroll loops blows up
// the unroller's size estimate (the loops then stay rolled and the switch becomes branches).
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Value of lane J (0..15) of this lane's 16-lane row.
template <int J>
__device__ __forceinline__ float bc(float v)
{
    return dpp_f<0x150 + J>(v);
}

// Runtime-index form (j must fold to a constant; prefer bc<J> inside loops).
__device__ __forceinline__ float bc16(float v, int j)
{
    switch (j & 15) {
    case 0: return dpp_f<0x150>(v);
    case 1: return dpp_f<0x151>(v);
    case 2: return dpp_f<0x152>(v);
    case 3: return dpp_f<0x153>(v);
    case 4: return dpp_f<0x154>(v);
    case 5: return dpp_f<0x155>(v);
    case 6: return dpp_f<0x156>(v);
    case 7: return dpp_f<0x157>(v);
    case 8: return dpp_f<0x158>(v);
    case 9: return dpp_f<0x159>(v);
    case 10: return dpp_f<0x15A>(v);
    case 11: return dpp_f<0x15B>(v);
    case 12: return dpp_f<0x15C>(v);
    case 13: return dpp_f<0x15D>(v);
    case 14: return dpp_f<0x15E>(v);
    default: return dpp_f<0x15F>(v);
    }
}

// ---- fused broadcast FMA (inline asm) ----------------------------------------------------------------------
// acc + bcast_J(a) * b   (S = -1: acc - bcast_J(a) * b)
template <int J, int S>
__device__ __forceinline__ float fmac_bc_t(float acc, float a, float b)
{
    if constexpr (S > 0)
        asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    else
        asm("s_nop 1\n\tv_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    return acc;
}

template <int J, int S>
__device__ __forceinline__ double fmac_bc64_t(double acc, double a, double b)
{
    if constexpr (S > 0)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    else
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    return acc;
}

template <int J>
__device__ __forceinline__ double bc64_t(double v)
{
    double r;
    asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "i"(J));
    return r;
}

template <int J>
__device__ __forceinline__ float fmac_bc(float acc, float a, float b) { return fmac_bc_t<J, 1>(acc, a, b); }
template <int J>
__device__ __forceinline__ float fnmac_bc(float acc, float a, float b) { return fmac_bc_t<J, -1>(acc, a, b); }
template <int J>
__device__ __forceinline__ double fmac_bc64(double acc, double a, double b) { return fmac_bc64_t<J, 1>(acc, a, b); }
template <int J>
__device__ __forceinline__ double fnmac_bc64(double acc, double a, double b) { return fmac_bc64_t<J, -1>(acc, a, b); }
template <int J>
__device__ __forceinline__ double bc64(double v) { return bc64_t<J>(v); }

// ---- grouped fused broadcast dot products ---------------------------------------------------------------------
// One asm block per group of up to 4 terms and one s_nop per block: inside a block only the accumulator is
// written, and it is never a DPP source, so the VALU-write -> DPP-read hazard can only involve instructions
// before the block.
#define NMPC_M " row_mask:0xf bank_mask:0xf"
#define NMPC_L(OP, NEG, B, J) "\n\t" OP " %0, " NEG "%1, %" #B " row_newbcast:%" #J NMPC_M
#define NMPC_P(OP, NEG, X, J) "\n\t" OP " %0, " NEG "%" #X ", %" #X " row_newbcast:%" #J NMPC_M

// same broadcast source a, lanes J0.., multipliers b0..
template <int J0, int J1, int J2, int J3, class T>
__device__ __forceinline__ T fmac4_lanes(T acc, T a, T b0, T b1, T b2, T b3)
{
    if constexpr (sizeof(T) == 8)
        asm("s_nop 1" NMPC_L("v_fmac_f64_dpp", "", 2, 6) NMPC_L("v_fmac_f64_dpp", "", 3, 7)
                         NMPC_L("v_fmac_f64_dpp", "", 4, 8) NMPC_L("v_fmac_f64_dpp", "", 5, 9)
                     : "+v"(acc) : "v"(a), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "i"(J0), "i"(J1), "i"(J2), "i"(J3));
    else
        asm("s_nop 1" NMPC_L("v_fmac_f32_dpp", "", 2, 6) NMPC_L("v_fmac_f32_dpp", "", 3, 7)
                         NMPC_L("v_fmac_f32_dpp", "", 4, 8) NMPC_L("v_fmac_f32_dpp", "", 5, 9)
                     : "+v"(acc) : "v"(a), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "i"(J0), "i"(J1), "i"(J2), "i"(J3));
    return acc;
}
template <int J0, int J1, int J2, class T>
__device__ __forceinline__ T fmac3_lanes(T acc, T a, T b0, T b1, T b2)
{
    if constexpr (sizeof(T) == 8)
        asm("s_nop 1" NMPC_L("v_fmac_f64_dpp", "", 2, 5) NMPC_L("v_fmac_f64_dpp", "", 3, 6)
                         NMPC_L("v_fmac_f64_dpp", "", 4, 7)
                     : "+v"(acc) : "v"(a), "v"(b0), "v"(b1), "v"(b2), "i"(J0), "i"(J1), "i"(J2));
    else
        asm("s_nop 1" NMPC_L("v_fmac_f32_dpp", "", 2, 5) NMPC_L("v_fmac_f32_dpp", "", 3, 6)
                         NMPC_L("v_fmac_f32_dpp", "", 4, 7)
                     : "+v"(acc) : "v"(a), "v"(b0), "v"(b1), "v"(b2), "i"(J0), "i"(J1), "i"(J2));
    return acc;
}
template <int J0, int J1, class T>
__device__ __forceinline__ T fmac2_lanes(T acc, T a, T b0, T b1)
{
    if constexpr (sizeof(T) == 8)
        asm("s_nop 1" NMPC_L("v_fmac_f64_dpp", "", 2, 4) NMPC_L("v_fmac_f64_dpp", "", 3, 5)
                     : "+v"(acc) : "v"(a), "v"(b0), "v"(b1), "i"(J0), "i"(J1));
    else
        asm("s_nop 1" NMPC_L("v_fmac_f32_dpp", "", 2, 4) NMPC_L("v_fmac_f32_dpp", "", 3, 5)
                     : "+v"(acc) : "v"(a), "v"(b0), "v"(b1), "i"(J0), "i"(J1));
    return acc;
}
template <int J, class T>
__device__ __forceinline__ T fmac1(T acc, T a, T b)
{
    if constexpr (sizeof(T) == 8) return fmac_bc64<J>(acc, a, b);
    else return fmac_bc<J>(acc, a, b);
}

// fp64 pairs: acc + S * sum_t bcast_J(x_t) * x_t
#define NMPC_PAIRS_BLOCK(NEG)                                                                                    \
    if constexpr (N4 == 4)                                                                                        \
        asm("s_nop 1" NMPC_P("v_fmac_f64_dpp", NEG, 1, 5) NMPC_P("v_fmac_f64_dpp", NEG, 2, 5)            \
                         NMPC_P("v_fmac_f64_dpp", NEG, 3, 5) NMPC_P("v_fmac_f64_dpp", NEG, 4, 5)                  \
                     : "+v"(acc) : "v"(x0), "v"(x1), "v"(x2), "v"(x3), "i"(J));                                   \
    else if constexpr (N4 == 3)                                                                                   \
        asm("s_nop 1" NMPC_P("v_fmac_f64_dpp", NEG, 1, 4) NMPC_P("v_fmac_f64_dpp", NEG, 2, 4)            \
                         NMPC_P("v_fmac_f64_dpp", NEG, 3, 4)                                                      \
                     : "+v"(acc) : "v"(x0), "v"(x1), "v"(x2), "i"(J));                                            \
    else if constexpr (N4 == 2)                                                                                   \
        asm("s_nop 1" NMPC_P("v_fmac_f64_dpp", NEG, 1, 3) NMPC_P("v_fmac_f64_dpp", NEG, 2, 3)            \
                     : "+v"(acc) : "v"(x0), "v"(x1), "i"(J));                                                     \
    else                                                                                                          \
        asm("s_nop 1" NMPC_P("v_fmac_f64_dpp", NEG, 1, 2) : "+v"(acc) : "v"(x0), "i"(J));

template <int J, int N4, int S>
__device__ __forceinline__ double fmacN_pairs(double acc, double x0, double x1, double x2, double x3)
{
    if constexpr (S > 0) {
        NMPC_PAIRS_BLOCK("")
    } else {
        NMPC_PAIRS_BLOCK("-")
    }
    return acc;
}
#undef NMPC_PAIRS_BLOCK
#undef NMPC_L
#undef NMPC_P
#undef NMPC_M

// ---- multi-accumulator blocks ---------------------------------------------------------------------------------
// c_t += S * bcast_{J_t}(a_t) * b_t for t < K: K independent FMAs per block (no dependent-issue stalls inside
// the block), one s_nop per block. Unused operands (t >= K) are ignored.
#define NMPC_M2 " row_mask:0xf bank_mask:0xf"
#define NMPC_T(OP, NEG, C, A, B, J) "\n\t" OP " %" #C ", " NEG "%" #A ", %" #B " row_newbcast:%" #J NMPC_M2
#define NMPC_MULTI(OP, NEG)                                                                                      \
    if constexpr (K == 4)                                                                                         \
        asm("s_nop 1" NMPC_T(OP, NEG, 0, 4, 8, 12) NMPC_T(OP, NEG, 1, 5, 9, 13) NMPC_T(OP, NEG, 2, 6, 10, 14)      \
                NMPC_T(OP, NEG, 3, 7, 11, 15)                                                                     \
            : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)                                                              \
            : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3), "i"(J0), "i"(J1), "i"(J2),  \
              "i"(J3));                                                                                           \
    else if constexpr (K == 3)                                                                                    \
        asm("s_nop 1" NMPC_T(OP, NEG, 0, 3, 6, 9) NMPC_T(OP, NEG, 1, 4, 7, 10) NMPC_T(OP, NEG, 2, 5, 8, 11)        \
            : "+v"(c0), "+v"(c1), "+v"(c2)                                                                        \
            : "v"(a0), "v"(a1), "v"(a2), "v"(b0), "v"(b1), "v"(b2), "i"(J0), "i"(J1), "i"(J2));                   \
    else if constexpr (K == 2)                                                                                    \
        asm("s_nop 1" NMPC_T(OP, NEG, 0, 2, 4, 6) NMPC_T(OP, NEG, 1, 3, 5, 7)                                      \
            : "+v"(c0), "+v"(c1)                                                                                  \
            : "v"(a0), "v"(a1), "v"(b0), "v"(b1), "i"(J0), "i"(J1));                                              \
    else if constexpr (K == 1)                                                                                    \
        asm("s_nop 1" NMPC_T(OP, NEG, 0, 1, 2, 3) : "+v"(c0) : "v"(a0), "v"(b0), "i"(J0));

template <int K, int S, int J0, int J1 = 0, int J2 = 0, int J3 = 0, class T>
__device__ __forceinline__ void fmac_multi(T& c0, T& c1, T& c2, T& c3, T a0, T a1, T a2, T a3, T b0, T b1, T b2,
                                           T b3)
{
    if constexpr (sizeof(T) == 8) {
        if constexpr (S > 0) {
            NMPC_MULTI("v_fmac_f64_dpp", "")
        } else {
            NMPC_MULTI("v_fmac_f64_dpp", "-")
        }
    } else {
        if constexpr (S > 0) {
            NMPC_MULTI("v_fmac_f32_dpp", "")
        } else {
            NMPC_MULTI("v_fmac_f32_dpp", "-")
        }
    }
}
#undef NMPC_MULTI
#undef NMPC_T
#undef NMPC_M2

// Outer-product style accumulation over a chunk of accumulators acc[I0 .. I0+K):
//   acc[I0+t] += S * bcast_{LANE(I0+t)}(A(I0+t)) * B(I0+t)
// with LANE a constexpr function of the index and A/B callables returning the operands.
template <int I0, int I1, int S, class T, class LaneF, class AF, class BF>
__device__ __forceinline__ void fmac_range(T* acc, LaneF lane, AF A, BF B)
{
    if constexpr (I0 < I1) {
        constexpr int K = (I1 - I0) < 4 ? (I1 - I0) : 4;
        constexpr int L0 = LaneF::template at<I0>();
        constexpr int L1 = LaneF::template at<(K > 1 ? I0 + 1 : I0)>();
        constexpr int L2 = LaneF::template at<(K > 2 ? I0 + 2 : I0)>();
        constexpr int L3 = LaneF::template at<(K > 3 ? I0 + 3 : I0)>();
        T d1 = T(0), d2 = T(0), d3 = T(0);
        T& c1 = (K > 1) ? acc[I0 + (K > 1 ? 1 : 0)] : d1;
        T& c2 = (K > 2) ? acc[I0 + (K > 2 ? 2 : 0)] : d2;
        T& c3 = (K > 3) ? acc[I0 + (K > 3 ? 3 : 0)] : d3;
        fmac_multi<K, S, L0, L1, L2, L3>(acc[I0], c1, c2, c3, A(I0), A(K > 1 ? I0 + 1 : I0), A(K > 2 ? I0 + 2 : I0),
                                         A(K > 3 ? I0 + 3 : I0), B(I0), B(K > 1 ? I0 + 1 : I0),
                                         B(K > 2 ? I0 + 2 : I0), B(K > 3 ? I0 + 3 : I0));
        fmac_range<I0 + K, I1, S>(acc, lane, A, B);
    }
}
// lane maps for fmac_range
template <int C>
struct LaneConst {
    template <int I>
    static constexpr int at() { return C; }
};
template <int OFF>
struct LaneIdx {
    template <int I>
    static constexpr int at() { return I + OFF; }
};

// acc + sum_{t<N} bcast_{J0+t}(a) * b[t]
template <int J0, int N, class T>
__device__ __forceinline__ T dot_lanes(T acc, T a, const T* b)
{
    if constexpr (N >= 4) {
        acc = fmac4_lanes<J0, J0 + 1, J0 + 2, J0 + 3>(acc, a, b[0], b[1], b[2], b[3]);
        return dot_lanes<J0 + 4, N - 4>(acc, a, b + 4);
    } else if constexpr (N == 3) {
        return fmac3_lanes<J0, J0 + 1, J0 + 2>(acc, a, b[0], b[1], b[2]);
    } else if constexpr (N == 2) {
        return fmac2_lanes<J0, J0 + 1>(acc, a, b[0], b[1]);
    } else if constexpr (N == 1) {
        return fmac1<J0>(acc, a, b[0]);
    } else {
        return acc;
    }
}

// acc + sum_{t<N} bcast_{J0+t}(a) * b[t], as two interleaved partial sums (halves the dependent chain)
template <int J0, int N, class T>
__device__ __forceinline__ T dot_lanes2(T acc, T a, const T* b)
{
    T p0 = acc, p1 = T(0), d2 = T(0), d3 = T(0);
    sfor<0, N / 2>([&](auto tc) {
        constexpr int t = 2 * decltype(tc)::value;
        fmac_multi<2, 1, J0 + t, J0 + t + 1>(p0, p1, d2, d3, a, a, a, a, b[t], b[t + 1], b[t], b[t]);
    });
    if constexpr (N % 2) p0 = fmac1<J0 + N - 1>(p0, a, b[N - 1]);
    return p0 + p1;
}

// acc + S * sum_{t<N} bcast_J(x[t]) * x[t]   (fp64)
template <int J, int N, int S>
__device__ __forceinline__ double dot_pairs(double acc, const double* x)
{
    if constexpr (N >= 4) {
        acc = fmacN_pairs<J, 4, S>(acc, x[0], x[1], x[2], x[3]);
        return dot_pairs<J, N - 4, S>(acc, x + 4);
    } else if constexpr (N >= 1) {
        return fmacN_pairs<J, N, S>(acc, x[0], N > 1 ? x[1] : 0.0, N > 2 ? x[2] : 0.0, 0.0);
    } else {
        return acc;
    }
}

// fp64 broadcast through two 32-bit row_newbcast moves (compiler-scheduled, no asm)
__device__ __forceinline__ double bc16d(double v, int j)
{
    return __hiloint2double(__float_as_int(bc16(__int_as_float(__double2hiint(v)), j)),
                            __float_as_int(bc16(__int_as_float(__double2loint(v)), j)));
}

// Sum over the 16 lanes of the row, result in every lane.
__device__ __forceinline__ float row_sum16(float v)
{
    v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);  // row_half_mirror
    v += dpp_f<0x140>(v);  // row_mirror
    return v;
}

__device__ __forceinline__ float row_max16(float v)
{
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    v = fmaxf(v, dpp_f<0x140>(v));
    return v;
}

__device__ __forceinline__ float row_min16(float v)
{
    v = fminf(v, dpp_f<0xB1>(v));
    v = fminf(v, dpp_f<0x4E>(v));
    v = fminf(v, dpp_f<0x141>(v));
    v = fminf(v, dpp_f<0x140>(v));
    return v;
}

// max that propagates NaN (fmaxf drops it)
__device__ __forceinline__ float nan_max(float a, float b) { return (b > a || b != b) ? b : a; }

// hardware reciprocal (1 ulp), used for the IPM's elementwise divisions
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// full-precision fp64 reciprocal square root: v_rsq_f64 seed + one Newton step
__device__ __forceinline__ double drsq(double x)
{
    double y = __builtin_amdgcn_rsq(x);
    return y * (1.5 - 0.5 * x * y * y);
}

}  // namespace nmpc
