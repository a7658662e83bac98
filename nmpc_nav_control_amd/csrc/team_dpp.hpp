// team_dpp.hpp -- cross-lane primitives for 16-lane teams (one DPP row of a 64-wide CDNA4 wavefront).
//
// A team is one DPP row: lanes 16t..16t+15. row_newbcast:j broadcasts lane j of each row to the whole row
// (gfx90a+), so four independent teams in a wave exchange data without LDS. Row reductions use the
// quad_perm / row_half_mirror / row_mirror butterfly, which hipcc fuses into v_add_f32_dpp.
#pragma once

#include <hip/hip_runtime.h>

namespace nmpc {

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Value of lane j (0..15) of this lane's 16-lane row. j must fold to a constant after unrolling.
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

}  // namespace nmpc
