// hsg_rng.h -- counter-based dropout masks (device side).
//
// keep(key, idx) = lowbias32((idx * K3) ^ key) >= floor(p * 2^32), with the 32-bit
// per-call key = fold(splitmix64(seed * K1 + offset * K2)) computed ONCE per thread
// (hsg_drop_key).  Stateless: the forward and the backward of one call regenerate
// the identical mask from (seed, offset, idx), so no mask tensor exists.  The
// effective drop probability is floor(p * 2^32) / 2^32 (|error| < 2.4e-10).
// Per element that is 3 32-bit multiplies and 7 logic ops; round 2's per-element
// splitmix64 of (seed, offset, idx) took ~12 (quarter-rate) 32-bit multiply pieces
// per element, which made the FFN LayerNorm kernels VALU-heavy.  idx < 2^32 (the
// host entry points check n * d).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint64_t hsg_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t hsg_drop_threshold(float p) {
    const double t = (double)p * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

// Chris Wellons' lowbias32 (bias ~0.17): 2 multiplies, 3 xor-shifts
__device__ __forceinline__ uint32_t hsg_lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// the 32-bit key of one dropout call (also the head-projection masks' key)
__device__ __forceinline__ uint32_t hsg_drop_key(uint64_t seed, uint32_t offset) {
    const uint64_t k64 = hsg_mix64(seed * 0x9E3779B97F4A7C15ull + (uint64_t)offset * 0xD1B54A32D192ED03ull);
    return (uint32_t)k64 ^ (uint32_t)(k64 >> 32);
}

__device__ __forceinline__ bool hsg_keep32(uint32_t key, uint32_t idx, uint32_t thr) {
    return hsg_lowbias32((idx * 0x85EBCA6Bu) ^ key) >= thr;
}
