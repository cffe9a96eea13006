// group_sum.h -- sums over lane groups on DPP (full-rate VALU lane moves, no
// LDS crossbar round trips): the reductions inside the one-sided Jacobi
// sweeps of init_models.hip and epnp_wave.h, which are long dependent chains
// where ds_bpermute's latency set the pace.
#pragma once

#include <hip/hip_runtime.h>

namespace orbgpu {

// DPP controls (gfx9 encoding)
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // lane i <- lane 7-i within each 8
constexpr int kDppMirror = 0x140;     // lane i <- lane 15-i within each 16

template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), Ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), Ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// sum over the lane's 16-lane row, in every lane of the row: quad sums (xor 1,
// xor 2), then the other quad of the half row (half mirror), then the other
// half (mirror).  The association order is fixed, so every lane of the row
// gets the same bits.
__device__ __forceinline__ double row16_sum(double x) {
    x += dpp_f64<kDppXor1>(x);
    x += dpp_f64<kDppXor2>(x);
    x += dpp_f64<kDppHalfMirror>(x);
    x += dpp_f64<kDppMirror>(x);
    return x;
}

// G in {16, 32, 64}: row sums on DPP, then xor shuffles across rows
template <int G>
__device__ __forceinline__ double group_sum_dpp(double x) {
    static_assert(G == 16 || G == 32 || G == 64, "group of 16, 32 or 64 lanes");
    x = row16_sum(x);
    if constexpr (G >= 32) x += __shfl_xor(x, 16, 64);
    if constexpr (G >= 64) x += __shfl_xor(x, 32, 64);
    return x;
}

// inclusive prefix sum over the 64 lanes of a wave (integer: exact in any
// order) on DPP: row_shr 1, 2, 4, 8 inside each 16-lane row, then row 0's
// total broadcast into rows 1 and 3 and rows 0-1's into rows 2 and 3
// (row_bcast:15 / :31).  Six full-rate VALU ops instead of six ds_bpermute
// round trips; every lane of the wave must be active.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false); // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false); // row_bcast:31 -> rows 2, 3
    return v;
}

}  // namespace orbgpu
