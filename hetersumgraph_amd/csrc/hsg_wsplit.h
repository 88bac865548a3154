// hsg_wsplit.h -- the weight limb split shared by hsg_gemm.hip (hsg_wsplit) and
// hsg_hproj.hip (hsg_step_prologue, which runs it inside the step's first launch).
//
// A weight operand B [N][K] (B = W or W^T) becomes three bf16 limb planes
// [3][Np][Kp] (zero padded, Np = N rounded up to 128, Kp = K rounded up to 32):
// x = x0 + x1 + x2, each limb the RNE bf16 of the remaining residual.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 hsg_bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void hsg_split3(float x, __bf16 &x0, __bf16 &x1, __bf16 &x2) {
    x0 = (__bf16)x;                       // v_cvt_pk_bf16_f32, RNE
    const float r = x - (float)x0;        // exact
    x1 = (__bf16)r;
    x2 = (__bf16)(r - (float)x1);         // exact difference, then RNE
}

// RNE split of 8 fp32 values into three bf16 limb vectors (two values per 32-bit word),
// x = l0 + l1 + l2 exactly: l0 = RNE(x) and l1 = RNE(x - l0) by v_cvt_pk_bf16_f32 (two
// values per instruction), l2 = x - l0 - l1 (at most 8 significant bits: exact in bf16,
// packed by v_perm_b32).  11 VALU per pair, limb magnitudes |l1| <= 2^-9 |x|,
// |l2| <= 2^-18 |x|: the dropped products a1 b2 + a2 b1 stay <= 2^-26 |ab|.  The
// subtractions are pinned to scalar v_sub_f32 (inline asm): SLP-packed v_pk_add_f32 beside
// MFMAs is an anti-lever on gfx950 (MI355X_MICROARCH.md, price of one filler).  The low
// element is unpacked by a byte permute, (a & 0xffff) << 16: written as a shift, the
// compiler saw through it and re-converted that element alone (v_cvt_pk_bf16_f32 x, 0).
typedef unsigned int hsg_u32x4_t __attribute__((ext_vector_type(4)));
typedef float hsg_f32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 hsg_bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void hsg_split_rne_pair(float va, float vb, unsigned &w0, unsigned &w1, unsigned &w2) {
    const unsigned a = __builtin_bit_cast(unsigned, hsg_bf16x2_t{(__bf16)va, (__bf16)vb});
    w0 = a;
    float ra, rb, sa, sb;
    asm("v_sub_f32 %0, %1, %2" : "=v"(ra) : "v"(va), "v"(__uint_as_float(__builtin_amdgcn_perm(0u, a, 0x01000c0cu))));
    asm("v_sub_f32 %0, %1, %2" : "=v"(rb) : "v"(vb), "v"(__uint_as_float(a & 0xFFFF0000u)));
    const unsigned b = __builtin_bit_cast(unsigned, hsg_bf16x2_t{(__bf16)ra, (__bf16)rb});
    w1 = b;
    asm("v_sub_f32 %0, %1, %2" : "=v"(sa) : "v"(ra), "v"(__uint_as_float(__builtin_amdgcn_perm(0u, b, 0x01000c0cu))));
    asm("v_sub_f32 %0, %1, %2" : "=v"(sb) : "v"(rb), "v"(__uint_as_float(b & 0xFFFF0000u)));
    w2 = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
}
__device__ __forceinline__ void hsg_split_rne8(const hsg_f32x4_t x, const hsg_f32x4_t y, hsg_u32x4_t &w0,
                                               hsg_u32x4_t &w1, hsg_u32x4_t &w2) {
    const float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        unsigned a, b, c;
        hsg_split_rne_pair(v[2 * p], v[2 * p + 1], a, b, c);
        w0[p] = a;
        w1[p] = b;
        w2[p] = c;
    }
}

struct HsgWSplitJobs {
    const float *W[4];
    __bf16 *out[4];
    int N[4], K[4], ldw[4], trans[4], Np[4], Kp[4];
    int start[5];                         // job q owns blocks [start[q], start[q + 1])
    int n;
};

// Block blk of the split (256 threads): one thread per (n, 8 consecutive k), three
// 16-B limb stores; for a transposed weight consecutive threads take consecutive n,
// so each of the 8 reads W[k][n] is coalesced across the wave.
__device__ __forceinline__ void hsg_wsplit_block(const HsgWSplitJobs &j, int blk) {
    int q = 0;
    while (q + 1 < j.n && blk >= j.start[q + 1]) ++q;
    const int u = (blk - j.start[q]) * 256 + (int)threadIdx.x;
    const int Kp = j.Kp[q], Np = j.Np[q], N = j.N[q], K = j.K[q], ldw = j.ldw[q];
    const int kc8 = Kp / 8;
    if (u >= Np * kc8) return;
    const bool tr = j.trans[q] != 0;
    const int n = tr ? u % Np : u / kc8, k0 = 8 * (tr ? u / Np : u % kc8);
    const float *W = j.W[q];
    hsg_bf16x8_t x0, x1, x2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = k0 + e;
        float v = 0.f;
        if (n < N && k < K) v = tr ? W[(size_t)k * ldw + n] : W[(size_t)n * ldw + k];
        __bf16 a, b, c;
        hsg_split3(v, a, b, c);
        x0[e] = a; x1[e] = b; x2[e] = c;
    }
    const size_t plane = (size_t)Np * Kp, o = (size_t)n * Kp + k0;
    *reinterpret_cast<hsg_bf16x8_t *>(j.out[q] + o) = x0;
    *reinterpret_cast<hsg_bf16x8_t *>(j.out[q] + plane + o) = x1;
    *reinterpret_cast<hsg_bf16x8_t *>(j.out[q] + 2 * plane + o) = x2;
}

// host: fill the job table (0, or 1001 = HSG_EINVAL for a bad job)
inline int hsg_wsplit_setup(HsgWSplitJobs &j, int njobs, const float *const *W, const int *N, const int *K,
                            const int *ldw, const int *trans, void *const *planes) {
    if (njobs < 0 || njobs > 4) return 1001;
    j.n = njobs;
    j.start[0] = 0;
    for (int q = 0; q < njobs; ++q) {
        if (!W[q] || !planes[q] || N[q] <= 0 || K[q] <= 0 || (((uintptr_t)planes[q]) & 15)) return 1001;
        if (ldw[q] < (trans[q] ? N[q] : K[q])) return 1001;
        j.W[q] = W[q];
        j.out[q] = reinterpret_cast<__bf16 *>(planes[q]);
        j.N[q] = N[q]; j.K[q] = K[q]; j.ldw[q] = ldw[q]; j.trans[q] = trans[q] != 0;
        j.Np[q] = (N[q] + 127) / 128 * 128;
        j.Kp[q] = (K[q] + 31) / 32 * 32;
        j.start[q + 1] = j.start[q] + (j.Np[q] * (j.Kp[q] / 8) + 255) / 256;     // blocks
    }
    return 0;
}
