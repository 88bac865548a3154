// hsg_rng.h -- counter-based dropout masks (device side).
//
// keep(seed, offset, idx) = splitmix64(seed ^ offset*K1 ^ idx*K2) >= p * 2^32 on its
// high 32 bits.  Stateless: the forward and the backward of one call regenerate
// the identical mask from (seed, offset, idx), so no mask tensor exists.  The
// effective drop probability is floor(p * 2^32) / 2^32 (|error| < 2.4e-10).
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

__device__ __forceinline__ bool hsg_keep(uint64_t seed, uint32_t offset, uint64_t idx, uint32_t thr) {
    const uint64_t z = hsg_mix64(seed * 0x9E3779B97F4A7C15ull + (uint64_t)offset * 0xD1B54A32D192ED03ull +
                                 idx * 0xA24BAED4963EE407ull);
    return (uint32_t)(z >> 32) >= thr;
}
