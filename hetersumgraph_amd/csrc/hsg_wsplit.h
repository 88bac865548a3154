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
