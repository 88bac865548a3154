// hsg_wave.h -- group sums for gfx950 wave64 on the VALU (DPP) instead of the LDS path.
// __shfl_xor lowers to ds_bpermute on gfx950: one LDS round trip per step.  Here the
// steps inside a 16-lane row are DPP lane permutes fused into the adds (quad permutes
// for xor 1 and xor 2, the half-row and row mirrors for the other quad / half of a row
// -- each step adds a value held by the partner group, so every lane of a group ends
// with the same sum).  Used by the GEMM / narrow-FFN epilogues whose per-row sums run
// once per output row (the rho partials of hsg_gemm_psw_elug_rho: 68.1 -> 64.9 us per
// launch against __shfl_xor).  The same change in the LayerNorm wave sums and the edge
// kernels' per-head sums measured neutral (profiles/r04_dev/step_kernels_r04l.txt).
#pragma once
#include <hip/hip_runtime.h>

template <int CTRL>
__device__ __forceinline__ float hsg_dpp(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}

// sum over each aligned group of G lanes (G a power of two <= 64), in every lane of it
template <int G>
__device__ __forceinline__ float hsg_group_sum(float x) {
    if constexpr (G >= 2) x += hsg_dpp<0xb1>(x);       // quad_perm [1,0,3,2]
    if constexpr (G >= 4) x += hsg_dpp<0x4e>(x);       // quad_perm [2,3,0,1]
    if constexpr (G >= 8) x += hsg_dpp<0x141>(x);      // row_half_mirror
    if constexpr (G >= 16) x += hsg_dpp<0x140>(x);     // row_mirror
    if constexpr (G >= 32) x += __shfl_xor(x, 16);
    if constexpr (G >= 64) x += __shfl_xor(x, 32);
    return x;
}
