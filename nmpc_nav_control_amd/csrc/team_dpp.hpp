// team_dpp.hpp -- cross-lane primitives for 16-lane teams (one DPP row of a 64-wide CDNA4 wavefront).
//
// A team is one DPP row: lanes 16t..16t+15. row_newbcast:j broadcasts lane j of each row to the whole row
// (gfx90a+), so four independent teams in a wave exchange data without LDS. Row reductions use the
// quad_perm / row_half_mirror / row_mirror butterfly, which hipcc fuses into v_add_f32_dpp.
//
// The broadcast-multiply-accumulate chains of the Riccati recursion use the fused DPP forms
// v_fmac_f32_dpp / v_fmac_f64_dpp (one VALU op per term instead of a v_mov_dpp + FMA pair). hipcc does not
// form these for row_newbcast, so they are emitted as inline asm; the compiler's hazard recognizer does not
// see inside asm, so every block starts with the two wait states a VALU write -> DPP read needs (s_nop 1).
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
        asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    else
        asm volatile("s_nop 1\n\tv_fmac_f32_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    return acc;
}

template <int J, int S>
__device__ __forceinline__ double fmac_bc64_t(double acc, double a, double b)
{
    if constexpr (S > 0)
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    else
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(acc) : "v"(a), "v"(b), "i"(J));
    return acc;
}

template <int J>
__device__ __forceinline__ double bc64_t(double v)
{
    double r;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "i"(J));
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
