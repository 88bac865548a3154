// hsg_ffn.hip -- the whole PositionwiseFeedForward forward in one launch, for the
// narrow FFN of the word->sentence layer (d = 64, d_hid = 512 at every config).
//
// Reference (module/GATLayer.py:35-44):
//     out = LayerNorm(Dropout(W2 relu(W1 x + b1) + b2) + x),  eps 1e-5
// On the W2S side the FFN runs over the sentence (and doc) nodes only -- 1,120 rows
// at config 2 -- so the split path (two hsg_gemm_f32 launches + hsg_ln_fwd) is
// three latency-bound launches with ~0.15 GFLOP between them.  Here one block of
// 8 waves owns 16 rows end to end, and every global operand of both GEMMs (the
// wave's W1 columns, its W2 K slice, the x tile) is requested at kernel start, so
// the block pays one memory latency rather than one per K chunk:
//   phase 1  H[16][d_hid] = relu(x W1^T + b1)    wave w: columns [w*d_hid/8, ...)
//            v_mfma_f32_16x16x4_f32, x from LDS; H is written to global (the
//            backward needs it) and kept in LDS
//   phase 2  y[16][d] = H W2^T + b2              wave w: K slice [w*d_hid/8, ...)
//            for all d/16 column tiles; the eight K-slice partials are added in
//            wave order through LDS (deterministic)
//   phase 3  out = LN(dropout(y) + x) per row    one wave per row, the same hash
//            dropout (hsg_rng.h, index r*d + c) and the same reductions as
//            hsg_ln_fwd, so hsg_ln_bwd consumes (y, mean, rstd) unchanged
// MFMA operand layout (16x16x4): lane (li = l&15, lk = l>>4) feeds k = k0 + 4lk + e
// to the e-th of 4 consecutive MFMAs, so every operand read is one 16-byte quad.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "../../include/hsg.h"
#include "hsg_rng.h"
#include "hsg_dev.h"
#include "hsg_wave.h"
#include <stdlib.h>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kRB = 16;          // rows per block

__device__ __forceinline__ float wsum(float v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int D, int HID>
__global__ __launch_bounds__(512) void k_ffn_small_fwd(int n, const float *__restrict__ x,
                                                       const float *__restrict__ w1, const float *__restrict__ b1,
                                                       const float *__restrict__ w2, const float *__restrict__ b2,
                                                       const float *__restrict__ gamma,
                                                       const float *__restrict__ beta, float eps, float p_drop,
                                                       const int64_t *__restrict__ seedp, uint32_t offset,
                                                       float *__restrict__ Hout, float *__restrict__ yout,
                                                       float *__restrict__ out, float *__restrict__ mean,
                                                       float *__restrict__ rstd) {
    constexpr int NW = 8;                    // waves per block
    constexpr int LX = D + 4, LH = HID + 4;
    constexpr int C1 = HID / NW;             // phase-1 columns per wave
    constexpr int CT1 = C1 / 16;             // ... as 16-wide MFMA tiles
    constexpr int KC1 = D / 16;              // phase-1 16-deep K chunks
    constexpr int KS2 = HID / NW;            // phase-2 K slice per wave
    constexpr int KC2 = KS2 / 16;
    constexpr int CT2 = D / 16;              // phase-2 column tiles
    __shared__ __attribute__((aligned(16))) float xs[kRB * LX];
    __shared__ __attribute__((aligned(16))) float hs[kRB * LH];
    __shared__ __attribute__((aligned(16))) float ps[NW][kRB * D];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int r0 = blockIdx.x * kRB;
    // every global operand of both GEMMs is requested up front (one memory latency
    // for the whole block instead of one per K chunk): this wave's W1 columns and
    // W2 K slice as MFMA operand quads, and the x tile
    const int cbase = w * C1, kb = w * KS2;
    f32x4 bw1[KC1][CT1], bw2[KC2][CT2];
#pragma unroll
    for (int kc = 0; kc < KC1; ++kc)
#pragma unroll
        for (int t = 0; t < CT1; ++t)
            bw1[kc][t] = *reinterpret_cast<const f32x4 *>(w1 + (size_t)(cbase + 16 * t + li) * D + 16 * kc + 4 * lk);
#pragma unroll
    for (int kc = 0; kc < KC2; ++kc)
#pragma unroll
        for (int t = 0; t < CT2; ++t)
            bw2[kc][t] = *reinterpret_cast<const f32x4 *>(w2 + (size_t)(16 * t + li) * HID + kb + 16 * kc + 4 * lk);
    for (int q = tid; q < kRB * D / 4; q += NW * 64) {
        const int r = q / (D / 4), c = (q % (D / 4)) * 4;
        const f32x4 v = r0 + r < n ? *reinterpret_cast<const f32x4 *>(x + (size_t)(r0 + r) * D + c)
                                   : f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4 *>(xs + r * LX + c) = v;
    }
    __syncthreads();
    // ---- phase 1: H = relu(x W1^T + b1), columns [cbase, cbase + C1)
    {
        f32x4 acc[CT1];
#pragma unroll
        for (int t = 0; t < CT1; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC1; ++kc) {
            const f32x4 a = *reinterpret_cast<const f32x4 *>(xs + li * LX + 16 * kc + 4 * lk);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int t = 0; t < CT1; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], bw1[kc][t][e], acc[t], 0, 0, 0);
        }
        // D layout: column li of the tile, rows 4lk .. 4lk+3
#pragma unroll
        for (int t = 0; t < CT1; ++t) {
            const int c = cbase + 16 * t + li;
            const float bb = b1[c];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * lk + e;
                const float v = fmaxf(acc[t][e] + bb, 0.f);
                hs[r * LH + c] = v;
                if (r0 + r < n) Hout[(size_t)(r0 + r) * HID + c] = v;
            }
        }
    }
    __syncthreads();
    // ---- phase 2: partial y over this wave's K slice, all column tiles
    {
        f32x4 acc[CT2];
#pragma unroll
        for (int t = 0; t < CT2; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC2; ++kc) {
            const f32x4 a = *reinterpret_cast<const f32x4 *>(hs + li * LH + kb + 16 * kc + 4 * lk);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int t = 0; t < CT2; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], bw2[kc][t][e], acc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < CT2; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) ps[w][(4 * lk + e) * D + 16 * t + li] = acc[t][e];
    }
    __syncthreads();
    // ---- phase 3: y = sum of the K slices (wave order) + b2; out = LN(dropout(y) + x)
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    constexpr int NPL = (D + 63) / 64;
    for (int r = w; r < kRB; r += NW) {
        const int gr = r0 + r;
        if (gr >= n) break;
        float s[NPL];
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const int c = lane + 64 * i;
            s[i] = 0.f;
            if (c < D) {
                const size_t o = (size_t)gr * D + c;
                float v = ps[0][r * D + c];
#pragma unroll
                for (int q = 1; q < NW; ++q) v += ps[q][r * D + c];
                v += b2[c];
                yout[o] = v;
                if (p_drop > 0.f) v = hsg_keep32(dkey, (uint32_t)o, thr) ? v * scale : 0.f;
                s[i] = v + xs[r * LX + c];
                acc += s[i];
            }
        }
        const float mu = wsum(acc) / D;
        float var = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i)
            if (lane + 64 * i < D) { const float t = s[i] - mu; var = fmaf(t, t, var); }
        const float rs = rsqrtf(wsum(var) / D + eps);
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const int c = lane + 64 * i;
            if (c < D) out[(size_t)gr * D + c] = (s[i] - mu) * rs * gamma[c] + beta[c];
        }
        if (lane == 0) { mean[gr] = mu; rstd[gr] = rs; }
    }
}

// Backward of the same FFN up to the weight gradients, one block of 8 waves per 16
// rows (the counterpart of hsg_ln_bwd + the dH and dx GEMMs of the split path):
//   phase A  LN + dropout backward per row (2 rows per wave, lane = column):
//            ds = dLN/ds (residual branch), dy = ds * mask / (1-p); block column
//            partials of dgamma, dbeta and dy (= db2) -> lnpart[block][3][d]
//   phase B  dH = (dy W2) * (H > 0)             wave w: columns [w*d_hid/8, ...)
//            written to global (for dW1 = dH^T x) and kept in LDS; its block
//            column sums -> hpart[block][d_hid] (db1)
//   phase C  dx = ds + dH W1                    wave w: K slice [w*d_hid/8, ...),
//            the eight partials added in wave order
// W2 / W1 / H operands are requested at kernel start (scalar MFMA operands: the
// reduction runs along the rows of W2 and W1).  dW1, dW2 stay hsg_gemm_f32 split-K
// GEMMs and the partials go through hsg_ffn_colsums, as in the split path.
template <int D, int HID>
__global__ __launch_bounds__(512) void k_ffn_small_bwd(int n, const float *__restrict__ dout,
                                                       const float *__restrict__ x, const float *__restrict__ H,
                                                       const float *__restrict__ y, const float *__restrict__ w1,
                                                       const float *__restrict__ w2,
                                                       const float *__restrict__ gamma,
                                                       const float *__restrict__ mean,
                                                       const float *__restrict__ rstd, float p_drop,
                                                       const int64_t *__restrict__ seedp, uint32_t offset,
                                                       float *__restrict__ dy, float *__restrict__ dH,
                                                       float *__restrict__ dx, float *__restrict__ lnpart,
                                                       float *__restrict__ hpart) {
    constexpr int NW = 8;
    constexpr int LY = D + 4, LH = HID + 4;
    constexpr int C1 = HID / NW, CT1 = C1 / 16, KC1 = D / 16;      // phase B
    constexpr int KS2 = HID / NW, KC2 = KS2 / 16, CT2 = D / 16;   // phase C
    static_assert(D == 64, "phase A maps one lane per column");
    __shared__ __attribute__((aligned(16))) float dys[kRB * LY];
    __shared__ __attribute__((aligned(16))) float dss[kRB * D];
    __shared__ __attribute__((aligned(16))) float dhs[kRB * LH];
    __shared__ __attribute__((aligned(16))) float ps[NW][kRB * D];
    __shared__ float red[NW][3][D];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int r0 = blockIdx.x * kRB;
    const int cb = w * C1, kb = w * KS2;
    // operands of phases B and C, requested first
    float bw2[KC1][CT1][4], bw1[KC2][CT2][4], hv[CT1][4];
#pragma unroll
    for (int kc = 0; kc < KC1; ++kc)
#pragma unroll
        for (int t = 0; t < CT1; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) bw2[kc][t][e] = w2[(size_t)(16 * kc + 4 * lk + e) * HID + cb + 16 * t + li];
#pragma unroll
    for (int kc = 0; kc < KC2; ++kc)
#pragma unroll
        for (int t = 0; t < CT2; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) bw1[kc][t][e] = w1[(size_t)(kb + 16 * kc + 4 * lk + e) * D + 16 * t + li];
#pragma unroll
    for (int t = 0; t < CT1; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int r = min(r0 + 4 * lk + e, n - 1);
            hv[t][e] = H[(size_t)r * HID + cb + 16 * t + li];
        }
    // ---- phase A: LayerNorm + dropout backward, rows w and w + 8
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    const float gam = gamma[lane];
    float dg = 0.f, db = 0.f, dyb = 0.f;
#pragma unroll
    for (int q = 0; q < kRB / NW; ++q) {
        const int r = w + NW * q, gr = r0 + r;
        const bool ok = gr < n;
        const size_t o = (size_t)(ok ? gr : 0) * D + lane;
        const float yv = y[o], xv = x[o], go = ok ? dout[o] : 0.f;
        const float mu = mean[ok ? gr : 0], rs = rstd[ok ? gr : 0];
        bool keep = true;
        float v = yv;
        if (p_drop > 0.f) {
            keep = hsg_keep32(dkey, (uint32_t)o, thr);
            v = keep ? v * scale : 0.f;
        }
        const float xh = (v + xv - mu) * rs;
        const float g = go * gam;
        const float mg = wsum(g) / D, mgx = wsum(g * xh) / D;
        const float ds = ok ? rs * (g - mg - xh * mgx) : 0.f;
        const float dyv = keep ? ds * scale : 0.f;
        if (ok) {
            dg = fmaf(go, xh, dg);
            db += go;
            dyb += dyv;
            dy[o] = dyv;
        }
        dys[r * LY + lane] = dyv;
        dss[r * D + lane] = ds;
    }
    red[w][0][lane] = dg;
    red[w][1][lane] = db;
    red[w][2][lane] = dyb;
    __syncthreads();
    if (tid < 3 * D) {
        const int which = tid / D, c = tid - which * D;
        float a = 0.f;
#pragma unroll
        for (int q = 0; q < NW; ++q) a += red[q][which][c];
        lnpart[(size_t)blockIdx.x * 3 * D + which * D + c] = a;
    }
    // ---- phase B: dH = (dy W2) * (H > 0), columns [cb, cb + C1)
    {
        f32x4 acc[CT1];
#pragma unroll
        for (int t = 0; t < CT1; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC1; ++kc) {
            const f32x4 a = *reinterpret_cast<const f32x4 *>(dys + li * LY + 16 * kc + 4 * lk);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int t = 0; t < CT1; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], bw2[kc][t][e], acc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < CT1; ++t) {
            const int c = cb + 16 * t + li;
            float cs = 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * lk + e;
                const float v = (r0 + r < n && hv[t][e] > 0.f) ? acc[t][e] : 0.f;
                dhs[r * LH + c] = v;
                if (r0 + r < n) dH[(size_t)(r0 + r) * HID + c] = v;
                cs += v;
            }
            // rows 4lk..4lk+3 here; the four lk groups of a column are lanes li + 16 lk
            cs += __shfl_xor(cs, 16);
            cs += __shfl_xor(cs, 32);
            if (lk == 0) hpart[(size_t)blockIdx.x * HID + c] = cs;
        }
    }
    __syncthreads();
    // ---- phase C: dx = ds + dH W1 (this wave's K slice, all column tiles)
    {
        f32x4 acc[CT2];
#pragma unroll
        for (int t = 0; t < CT2; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC2; ++kc) {
            const f32x4 a = *reinterpret_cast<const f32x4 *>(dhs + li * LH + kb + 16 * kc + 4 * lk);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int t = 0; t < CT2; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], bw1[kc][t][e], acc[t], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < CT2; ++t)
#pragma unroll
            for (int e = 0; e < 4; ++e) ps[w][(4 * lk + e) * D + 16 * t + li] = acc[t][e];
    }
    __syncthreads();
    for (int q = tid; q < kRB * D; q += NW * 64) {
        const int r = q / D, c = q - (q / D) * D;
        if (r0 + r >= n) continue;
        float v = ps[0][q];
#pragma unroll
        for (int k = 1; k < NW; ++k) v += ps[k][q];
        dx[(size_t)(r0 + r) * D + c] = dss[q] + v;
    }
}

// ---------------------------------------------------------- 4-row blocks ----
// (round 4) The same phases on blocks of 8 rows (two 4-row groups): cfg2's 1,120 W2S
// rows make 140 blocks instead of 70 of 16 (the 16-row blocks left 186 of 256 CUs idle:
// 15.3 / 12.7 us per fwd / bwd launch; 4-row blocks, 280 of them at one block per CU,
// ran in two rounds: 19.9 / 12.2 us).  The GEMMs run on v_mfma_f32_4x4x1_16b_f32: 16 independent 4x4 outer products per
// instruction that all take the block's 4 rows, one output column quad per product,
// so one instruction is 4 rows x 64 columns x 1 k at the f32 MFMA rate with nothing
// padded (the 16x16x4 form needs 16 rows).  Operand lanes (b = lane / 4): A[i] at
// lane 4b + i (row i's value, the same for every b), B[j] at lane 4b + j (column
// 4b + j, i.e. column = lane), D[i][j] in register i of lane 4b + j.  Each wave's 64
// weights per lane (a W1 row / a W2 K slice, or the columns of the backward) are
// requested at kernel start (the forward's row-per-lane weights through an LDS image,
// so the global loads stay coalesced); the k loop runs two accumulator chains per
// row group (k even / odd), added in chain order.  Deterministic: the K-slice partials of the second GEMM are
// added in wave order, the LN / bias partials per block as before.
constexpr int kRG = 2;           // 4-row groups per block of the 4x4x1 kernels
constexpr int kRB4 = 4 * kRG;    // their rows per block (cfg2 W2S: 140 blocks, one round)

// sum over each aligned 8-lane group, in every lane (DPP, hsg_wave.h)
__device__ __forceinline__ float row8_sum(float x) { return hsg_group_sum<8>(x); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

// RG row groups x 64 k steps: A from LDS rows (row group g at arow + g * 4 * lda;
// broadcast f32x4 reads), B per lane (one register per k, shared by the groups); two
// accumulator chains per group (k even / odd), added in chain order
template <int RG>
__device__ __forceinline__ void mfma4_k64(const float *arow, int lda, const f32x4 (&bq)[16], f32x4 (&out)[RG]) {
    f32x4 acc[RG][2];
#pragma unroll
    for (int g = 0; g < RG; ++g) acc[g][0] = acc[g][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
#pragma unroll
        for (int g = 0; g < RG; ++g) {
            const f32x4 a = *reinterpret_cast<const f32x4 *>(arow + g * 4 * lda + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[g][e & 1] = mfma4(a[e], bq[q][e], acc[g][e & 1]);
        }
    }
#pragma unroll
    for (int g = 0; g < RG; ++g) out[g] = acc[g][0] + acc[g][1];
}

// bq[q][e] = M[row0 + lane][c0 + 4q + e] of a row-major matrix: the wave loads the
// 64 x 64 block coalesced (4 rows x 256 B per instruction) into its LDS image and
// reads its own row back (pitch 68: a 16-lane group's b128 reads hit all 64 banks)
__device__ __forceinline__ void rows_via_lds(const float *__restrict__ M, int ld, int row0, int c0, float *img,
                                             int lane, f32x4 (&bq)[16]) {
    constexpr int P = 68;
    f32x4 t[16];
#pragma unroll
    for (int q = 0; q < 16; ++q)
        t[q] = *reinterpret_cast<const f32x4 *>(M + (size_t)(row0 + 4 * q + lane / 16) * ld + c0 + 4 * (lane % 16));
#pragma unroll
    for (int q = 0; q < 16; ++q) *reinterpret_cast<f32x4 *>(img + (4 * q + lane / 16) * P + 4 * (lane % 16)) = t[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int q = 0; q < 16; ++q) bq[q] = *reinterpret_cast<const f32x4 *>(img + lane * P + 4 * q);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");      // reads done before the image is reused
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int D, int HID>
__global__ __launch_bounds__(512) void k_ffn_small_fwd4(int n, const float *__restrict__ x,
                                                        const float *__restrict__ w1, const float *__restrict__ b1,
                                                        const float *__restrict__ w2, const float *__restrict__ b2,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta, float eps, float p_drop,
                                                        const int64_t *__restrict__ seedp, uint32_t offset,
                                                        float *__restrict__ Hout, float *__restrict__ yout,
                                                        float *__restrict__ out, float *__restrict__ mean,
                                                        float *__restrict__ rstd) {
    constexpr int NW = 8, LX = D + 4, LH = HID + 4;      // row pads: the 4 rows on distinct banks
    static_assert(D == 64 && HID == 64 * NW && kRB4 == NW, "one instruction spans 64 columns; a wave per row");
    __shared__ __attribute__((aligned(16))) float xs[kRB4 * LX];
    __shared__ __attribute__((aligned(16))) float hs[kRB4 * LH];
    // the weight images (dead after the staging barrier) hold the phase-2 partials
    __shared__ __attribute__((aligned(16))) float img[NW][64 * 68];
    float (*ps)[64 * 68] = img;
    static_assert(kRB4 * D <= 64 * 68, "partials fit a wave's image");
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i4 = lane & 3;
    const int r0 = blockIdx.x * kRB4;
    const int col = w * 64 + lane;                       // phase-1 column of this lane
    if (tid < kRB4 * D / 4) {
        const int r = tid / (D / 4), c = (tid % (D / 4)) * 4;
        const f32x4 v = r0 + r < n ? *reinterpret_cast<const f32x4 *>(x + (size_t)(r0 + r) * D + c)
                                   : f32x4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f32x4 *>(xs + r * LX + c) = v;
    }
    // W1[col][k] (the wave's 64 W1 rows) and W2[lane][w*64 + k] (its K slice), each
    // lane's row through the wave's LDS image: coalesced global loads
    f32x4 bw1[16], bw2[16];
    rows_via_lds(w1, D, w * 64, 0, img[w], lane, bw1);
    rows_via_lds(w2, HID, 0, w * 64, img[w], lane, bw2);
    __syncthreads();
    // ---- phase 1: H[:, col] = relu(x W1^T + b1)
    {
        f32x4 h[kRG];
        mfma4_k64<kRG>(xs + i4 * LX, LX, bw1, h);
        const float bb = b1[col];
#pragma unroll
        for (int g = 0; g < kRG; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * g + i;
                const float v = fmaxf(h[g][i] + bb, 0.f);
                hs[r * LH + col] = v;
                if (r0 + r < n) Hout[(size_t)(r0 + r) * HID + col] = v;
            }
    }
    __syncthreads();
    // ---- phase 2: y partial over this wave's K slice [w*64, w*64 + 64), column = lane
    {
        f32x4 y[kRG];
        mfma4_k64<kRG>(hs + i4 * LH + w * 64, LH, bw2, y);
#pragma unroll
        for (int g = 0; g < kRG; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) ps[w][(4 * g + i) * D + lane] = y[g][i];
    }
    __syncthreads();
    // ---- phase 3: row w (lane = column): y = K slices (wave order) + b2,
    // out = LN(dropout(y) + x) -- the hsg_ln_fwd reductions, as k_ffn_small_fwd
    const int gr = r0 + w;
    if (gr >= n) return;
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    const size_t o = (size_t)gr * D + lane;
    float v = ps[0][w * D + lane];
#pragma unroll
    for (int q = 1; q < NW; ++q) v += ps[q][w * D + lane];
    v += b2[lane];
    yout[o] = v;
    if (p_drop > 0.f) v = hsg_keep32(dkey, (uint32_t)o, thr) ? v * scale : 0.f;
    const float s = v + xs[w * LX + lane];
    const float mu = wsum(s) / D;
    const float t = s - mu;
    const float rs = rsqrtf(wsum(t * t) / D + eps);
    out[o] = t * rs * gamma[lane] + beta[lane];
    if (lane == 0) { mean[gr] = mu; rstd[gr] = rs; }
}

template <int D, int HID>
__global__ __launch_bounds__(512) void k_ffn_small_bwd4(int n, const float *__restrict__ dout,
                                                        const float *__restrict__ x, const float *__restrict__ H,
                                                        const float *__restrict__ y, const float *__restrict__ w1,
                                                        const float *__restrict__ w2,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ mean,
                                                        const float *__restrict__ rstd, float p_drop,
                                                        const int64_t *__restrict__ seedp, uint32_t offset,
                                                        float *__restrict__ dy, float *__restrict__ dH,
                                                        float *__restrict__ dx, float *__restrict__ lnpart,
                                                        float *__restrict__ hpart, const float *__restrict__ hg,
                                                        float *__restrict__ Gout, float *__restrict__ rho) {
    constexpr int NW = 8, LY = D + 4, LH = HID + 4;
    static_assert(D == 64 && HID == 64 * NW && kRB4 == NW, "one instruction spans 64 columns; a wave per row");
    __shared__ __attribute__((aligned(16))) float dys[kRB4 * LY];
    __shared__ __attribute__((aligned(16))) float dss[kRB4 * D];
    __shared__ __attribute__((aligned(16))) float dhs[kRB4 * LH];
    __shared__ __attribute__((aligned(16))) float ps[NW][kRB4 * D];
    __shared__ float red[kRB4][3][D];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i4 = lane & 3;
    const int r0 = blockIdx.x * kRB4;
    const int col = w * 64 + lane;                       // phase-B column of this lane
    // operands of phases B and C, requested first (lanes along a row: coalesced):
    // W2[k][col] (B: k = d), W1[w*64 + k][lane] (C: k = the wave's hidden slice), H
    f32x4 bw2[16], bw1[16];
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            bw2[q][e] = w2[(size_t)(4 * q + e) * HID + col];
            bw1[q][e] = w1[(size_t)(w * 64 + 4 * q + e) * D + lane];
        }
    float hv[kRB4];
#pragma unroll
    for (int r = 0; r < kRB4; ++r) hv[r] = H[(size_t)min(r0 + r, n - 1) * HID + col];
    // ---- phase A: LayerNorm + dropout backward, row w (lane = column)
    {
        const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
        const uint32_t thr = hsg_drop_threshold(p_drop);
        const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
        const int gr = r0 + w;
        const bool ok = gr < n;
        const size_t o = (size_t)(ok ? gr : 0) * D + lane;
        const float yv = y[o], xv = x[o], go = ok ? dout[o] : 0.f;
        const float mu = mean[ok ? gr : 0], rs = rstd[ok ? gr : 0];
        bool keep = true;
        float v = yv;
        if (p_drop > 0.f) {
            keep = hsg_keep32(dkey, (uint32_t)o, thr);
            v = keep ? v * scale : 0.f;
        }
        const float xh = (v + xv - mu) * rs;
        const float g = go * gamma[lane];
        const float mg = wsum(g) / D, mgx = wsum(g * xh) / D;
        const float ds = ok ? rs * (g - mg - xh * mgx) : 0.f;
        const float dyv = keep ? ds * scale : 0.f;
        if (ok) dy[o] = dyv;
        dys[w * LY + lane] = dyv;
        dss[w * D + lane] = ds;
        red[w][0][lane] = ok ? go * xh : 0.f;
        red[w][1][lane] = go;
        red[w][2][lane] = ok ? dyv : 0.f;
    }
    __syncthreads();
    if (tid < 3 * D) {                                   // block partials (row order)
        const int which = tid / D, c = tid - which * D;
        float a = 0.f;
#pragma unroll
        for (int r = 0; r < kRB4; ++r) a += red[r][which][c];
        lnpart[(size_t)blockIdx.x * 3 * D + which * D + c] = a;
    }
    // ---- phase B: dH[:, col] = (dy W2) * (H > 0), block column sums -> hpart (db1)
    {
        f32x4 acc[kRG];
        mfma4_k64<kRG>(dys + i4 * LY, LY, bw2, acc);
        float cs = 0.f;
#pragma unroll
        for (int g = 0; g < kRG; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = 4 * g + i;
                const float v = (r0 + r < n && hv[r] > 0.f) ? acc[g][i] : 0.f;
                dhs[r * LH + col] = v;
                if (r0 + r < n) dH[(size_t)(r0 + r) * HID + col] = v;
                cs += v;
            }
        hpart[(size_t)blockIdx.x * HID + col] = cs;
    }
    __syncthreads();
    // ---- phase C: dx partial over this wave's hidden slice, column = lane
    {
        f32x4 acc[kRG];
        mfma4_k64<kRG>(dhs + i4 * LH + w * 64, LH, bw1, acc);
#pragma unroll
        for (int g = 0; g < kRG; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) ps[w][(4 * g + i) * D + lane] = acc[g][i];
    }
    __syncthreads();
    if (r0 + w < n) {                                    // wave-uniform
        float v = ps[0][w * D + lane];
#pragma unroll
        for (int q = 1; q < NW; ++q) v += ps[q][w * D + lane];
        const size_t o = (size_t)(r0 + w) * D + lane;
        const float dxv = dss[w * D + lane] + v;
        dx[o] = dxv;
        if (Gout) {
            // the W2S edge layer's backward operands from this dx (= its dOut): G =
            // dOut * elu'(h) (elu'(h) = 1 for h > 0, else exp(h): as hsg_gat_bwd_dst) and
            // rho[row][k] = G_k . h_k over head k's 8 columns (lanes 8k .. 8k + 7)
            const float hv = hg[o];
            const float g = hv > 0.f ? dxv : dxv * __expf(hv);
            Gout[o] = g;
            const float gh = row8_sum(g * hv);
            if ((lane & 7) == 0) rho[(size_t)(r0 + w) * (D / 8) + lane / 8] = gh;
        }
    }
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// rows per block of the narrow FFN kernels: 8 (k_ffn_small_*4); 16 with
// HSG_FFN_RB=16 in the dev library (the round-3 kernels, for A/B)
int ffn_rows_per_block() {
    const char *e = HSG_DEV_ENV("HSG_FFN_RB");
    return e && atoi(e) == 16 ? kRB : kRB4;
}

}  // namespace

extern "C" {

int hsg_ffn_small_supported(int d, int d_hid) { return (d == 64 && d_hid == 512) ? 1 : 0; }

int hsg_ffn_small_fwd(int n, int d, int d_hid, const float *x, const float *w1, const float *b1, const float *w2,
                      const float *b2, const float *gamma, const float *beta, float eps, float p_drop,
                      const int64_t *seed, uint32_t offset, float *H, float *y, float *out, float *mean, float *rstd,
                      void *stream) {
    if (n < 0 || !hsg_ffn_small_supported(d, d_hid) || p_drop < 0.f || p_drop >= 1.f) return HSG_EINVAL;
    if (!x || !w1 || !b1 || !w2 || !b2 || !gamma || !beta || !H || !y || !out || !mean || !rstd) return HSG_EINVAL;
    if (p_drop > 0.f && (!seed || (long)n * d >= (1L << 32))) return HSG_EINVAL;   // 32-bit mask index
    if (!aligned16(x) || !aligned16(w1) || !aligned16(w2)) return HSG_EINVAL;
    if (n == 0) return 0;
    const int rb = ffn_rows_per_block();
    if (rb == kRB4)
        hipLaunchKernelGGL((k_ffn_small_fwd4<64, 512>), dim3((unsigned)((n + kRB4 - 1) / kRB4)), dim3(512), 0,
                           (hipStream_t)stream, n, x, w1, b1, w2, b2, gamma, beta, eps, p_drop, seed, offset, H, y,
                           out, mean, rstd);
    else
        hipLaunchKernelGGL((k_ffn_small_fwd<64, 512>), dim3((unsigned)((n + kRB - 1) / kRB)), dim3(512), 0,
                           (hipStream_t)stream, n, x, w1, b1, w2, b2, gamma, beta, eps, p_drop, seed, offset, H, y,
                           out, mean, rstd);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int hsg_ffn_small_bwd_blocks(int n) {
    const int rb = ffn_rows_per_block();
    return n > 0 ? (n + rb - 1) / rb : 0;
}

namespace {
int ffn_small_bwd(int n, int d, int d_hid, const float *dout, const float *x, const float *H, const float *y,
                  const float *w1, const float *w2, const float *gamma, const float *mean, const float *rstd,
                  float p_drop, const int64_t *seed, uint32_t offset, float *dy, float *dH, float *dx, float *lnpart,
                  float *hpart, const float *hg, float *G, float *rho, void *stream) {
    if (n < 0 || !hsg_ffn_small_supported(d, d_hid) || p_drop < 0.f || p_drop >= 1.f) return HSG_EINVAL;
    if (!dout || !x || !H || !y || !w1 || !w2 || !gamma || !mean || !rstd || !dy || !dH || !dx || !lnpart || !hpart)
        return HSG_EINVAL;
    if (p_drop > 0.f && (!seed || (long)n * d >= (1L << 32))) return HSG_EINVAL;   // 32-bit mask index
    if (G && (!hg || !rho || ffn_rows_per_block() != kRB4)) return HSG_EINVAL;
    if (n == 0) return 0;
    if (ffn_rows_per_block() == kRB4)
        hipLaunchKernelGGL((k_ffn_small_bwd4<64, 512>), dim3((unsigned)hsg_ffn_small_bwd_blocks(n)), dim3(512), 0,
                           (hipStream_t)stream, n, dout, x, H, y, w1, w2, gamma, mean, rstd, p_drop, seed, offset, dy,
                           dH, dx, lnpart, hpart, hg, G, rho);
    else
        hipLaunchKernelGGL((k_ffn_small_bwd<64, 512>), dim3((unsigned)hsg_ffn_small_bwd_blocks(n)), dim3(512), 0,
                           (hipStream_t)stream, n, dout, x, H, y, w1, w2, gamma, mean, rstd, p_drop, seed, offset, dy,
                           dH, dx, lnpart, hpart);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}
}  // namespace

int hsg_ffn_small_bwd(int n, int d, int d_hid, const float *dout, const float *x, const float *H, const float *y,
                      const float *w1, const float *w2, const float *gamma, const float *mean, const float *rstd,
                      float p_drop, const int64_t *seed, uint32_t offset, float *dy, float *dH, float *dx,
                      float *lnpart, float *hpart, void *stream) {
    return ffn_small_bwd(n, d, d_hid, dout, x, H, y, w1, w2, gamma, mean, rstd, p_drop, seed, offset, dy, dH, dx,
                         lnpart, hpart, nullptr, nullptr, nullptr, stream);
}

int hsg_ffn_small_bwd_gate(int n, int d, int d_hid, const float *dout, const float *x, const float *H,
                           const float *y, const float *w1, const float *w2, const float *gamma, const float *mean,
                           const float *rstd, float p_drop, const int64_t *seed, uint32_t offset, float *dy,
                           float *dH, float *dx, float *lnpart, float *hpart, const float *h_edge, float *G,
                           float *rho, void *stream) {
    if (!h_edge || !G || !rho) return HSG_EINVAL;
    return ffn_small_bwd(n, d, d_hid, dout, x, H, y, w1, w2, gamma, mean, rstd, p_drop, seed, offset, dy, dH, dx,
                         lnpart, hpart, h_edge, G, rho, stream);
}

}  // extern "C"
