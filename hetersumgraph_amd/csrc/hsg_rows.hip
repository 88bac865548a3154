// hsg_rows.hip -- row-wise epilogues of PositionwiseFeedForward for gfx950.
//
// Reference (module/GATLayer.py:35-44):
//     out = LayerNorm(Dropout(W2 relu(W1 x + b1) + b2) + x),  eps 1e-5
// The GEMMs run on MFMA (hsg_gemm.hip); this file fuses everything after the
// second GEMM into one pass over the rows (dropout, residual add, LayerNorm) and
// the matching backward (LayerNorm backward, dropout backward, residual split,
// per-block dgamma/dbeta partials -- no atomics, deterministic).
//
// Dropout masks come from a counter-based hash of (seed, offset, element) (hsg_rng.h:
// a per-call 32-bit key, then lowbias32 per element): seed is
// read from device memory (so a HIP-graph replay can advance it), offset is a
// per-call-site constant.  Forward and backward regenerate the same mask, so no
// mask tensor is stored.  One wave per row; lane owns columns lane + 64*i.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/hsg.h"
#include "hsg_dev.h"
#include "hsg_rng.h"

namespace {

constexpr int kMaxPerLane = 8;   // d <= 512

__device__ __forceinline__ float wsum(float v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <int NPL>
__global__ __launch_bounds__(256) void k_ln_fwd(int n, int d, const float *__restrict__ y,
                                                const float *__restrict__ x, const float *__restrict__ gamma,
                                                const float *__restrict__ beta, float eps, float p_drop,
                                                const int64_t *__restrict__ seedp, uint32_t offset,
                                                float *__restrict__ out, float *__restrict__ mean,
                                                float *__restrict__ rstd) {
    const int lane = threadIdx.x & 63;
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += gridDim.x * 4) {
        float s[NPL];
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const int c = lane + 64 * i;
            s[i] = 0.f;
            if (c < d) {
                const size_t o = (size_t)r * d + c;
                float v = y[o];
                if (p_drop > 0.f) v = hsg_keep32(dkey, (uint32_t)o, thr) ? v * scale : 0.f;
                s[i] = v + x[o];
                acc += s[i];
            }
        }
        const float mu = wsum(acc) / d;
        float var = 0.f;
#pragma unroll
        for (int i = 0; i < NPL; ++i)
            if (lane + 64 * i < d) { const float t = s[i] - mu; var = fmaf(t, t, var); }
        const float rs = rsqrtf(wsum(var) / d + eps);
#pragma unroll
        for (int i = 0; i < NPL; ++i) {
            const int c = lane + 64 * i;
            if (c < d) out[(size_t)r * d + c] = (s[i] - mu) * rs * gamma[c] + beta[c];
        }
        if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
    }
}

// Vector form (d % 4 == 0, 16-byte aligned rows): lane owns the column quads
// 4*lane + 256*i, i < NV, and each wave takes RPW rows whose loads are issued
// together (float4 loads: a quarter of the load instructions of k_ln_fwd).
typedef float f32x4r __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4r __attribute__((ext_vector_type(4)));
template <int NV, int RPW>
__global__ __launch_bounds__(256) void k_ln_fwd4(int n, int d, const float *__restrict__ y,
                                                 const float *__restrict__ x, const float *__restrict__ gamma,
                                                 const float *__restrict__ beta, float eps, float p_drop,
                                                 const int64_t *__restrict__ seedp, uint32_t offset,
                                                 float *__restrict__ out, float *__restrict__ mean,
                                                 float *__restrict__ rstd) {
    const int lane = threadIdx.x & 63;
    const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
    if (row0 >= n) return;
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    f32x4r s[RPW][NV];
    float acc[RPW];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int r = min(row0 + q, n - 1);
        acc[q] = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = 4 * lane + 256 * i;
            s[q][i] = f32x4r{0.f, 0.f, 0.f, 0.f};
            if (c < d) {
                const size_t o = (size_t)r * d + c;
                f32x4r v = *reinterpret_cast<const f32x4r *>(y + o);
                if (p_drop > 0.f) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = hsg_keep32(dkey, (uint32_t)(o + e), thr) ? v[e] * scale : 0.f;
                }
                s[q][i] = v + *reinterpret_cast<const f32x4r *>(x + o);
                acc[q] += (s[q][i][0] + s[q][i][1]) + (s[q][i][2] + s[q][i][3]);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int r = row0 + q;
        const float mu = wsum(acc[q]) / d;
        float var = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i)
            if (4 * lane + 256 * i < d)
#pragma unroll
                for (int e = 0; e < 4; ++e) { const float t = s[q][i][e] - mu; var = fmaf(t, t, var); }
        const float rs = rsqrtf(wsum(var) / d + eps);
        if (r >= n) continue;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = 4 * lane + 256 * i;
            if (c < d) {
                const f32x4r g = *reinterpret_cast<const f32x4r *>(gamma + c);
                const f32x4r b = *reinterpret_cast<const f32x4r *>(beta + c);
                *reinterpret_cast<f32x4r *>(out + (size_t)r * d + c) = (s[q][i] - mu) * rs * g + b;
            }
        }
        if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
    }
}

// Round 4 (257..512 columns, the S2W FFN at d = 300): k_ln_fwd4 on a persistent grid
// of kLnFwdPBlocks blocks, each wave walking row groups g, g + waves, ... with the next
// group's y / x loads issued before this group's reductions and stores, so the HBM read
// of one group overlaps the write of the previous one (k_ln_fwd4: one round of waves,
// every load first, then every store).  Same arithmetic per row (bitwise equal,
// tests/test_gpu_ffn.py).  cfg2 in-step at 1,536 blocks: 15.6-15.8 vs 17.7 us per launch
// (profiles/r04_dev/ln_fwdp/); dev: HSG_LN_FWDP=<blocks> (0: k_ln_fwd4), HSG_LN_FWDP_R=2.
// YBF (round 5, the bf16 GEMM mode): y -- the wide FFN's output, the LayerNorm input --
// comes as bf16 rows (pitch d), kept as raw quads until the row is consumed (a
// conversion at the load would wait for the prefetch at once).
// XBF (round 6): the residual x -- the edge layer's output elu(h) + origin -- comes as
// bf16 rows of pitch ldx (>= ceil8(d)), likewise kept raw until used.
template <int NV, int RPW, bool YBF = false, bool XBF = false>
__global__ __launch_bounds__(256) void k_ln_fwd4p(int n, int d, const float *__restrict__ y,
                                                  const float *__restrict__ x, const float *__restrict__ gamma,
                                                  const float *__restrict__ beta, float eps, float p_drop,
                                                  const int64_t *__restrict__ seedp, uint32_t offset,
                                                  float *__restrict__ out, float *__restrict__ mean,
                                                  float *__restrict__ rstd, int ldx = 0) {
    const int lane = threadIdx.x & 63;
    const int ng = (n + RPW - 1) / RPW, nw = gridDim.x * 4;
    int g = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= ng) return;
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    f32x4r yv[RPW][NV], xv[RPW][NV];
    bf16x4r yb[YBF ? RPW : 1][YBF ? NV : 1], xb[XBF ? RPW : 1][XBF ? NV : 1];
    auto load = [&](int gg) {
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int r = min(gg * RPW + q, n - 1);
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int c = min(4 * lane + 256 * i, d - 4);        // clamped: unused past d
                if constexpr (YBF)
                    yb[q][i] = *reinterpret_cast<const bf16x4r *>(reinterpret_cast<const __bf16 *>(y) + (size_t)r * d + c);
                else
                    yv[q][i] = *reinterpret_cast<const f32x4r *>(y + (size_t)r * d + c);
                if constexpr (XBF)
                    xb[q][i] = *reinterpret_cast<const bf16x4r *>(reinterpret_cast<const __bf16 *>(x) + (size_t)r * ldx + c);
                else
                    xv[q][i] = *reinterpret_cast<const f32x4r *>(x + (size_t)r * d + c);
            }
        }
    };
    load(g);
    for (; g < ng; g += nw) {
        f32x4r s[RPW][NV];
        float acc[RPW];
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int r = min(g * RPW + q, n - 1);
            acc[q] = 0.f;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int c = 4 * lane + 256 * i;
                s[q][i] = f32x4r{0.f, 0.f, 0.f, 0.f};
                if (c < d) {
                    const size_t o = (size_t)r * d + c;
                    f32x4r v;
                    if constexpr (YBF) v = f32x4r{(float)yb[q][i][0], (float)yb[q][i][1], (float)yb[q][i][2], (float)yb[q][i][3]};
                    else v = yv[q][i];
                    if (p_drop > 0.f) {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            v[e] = hsg_keep32(dkey, (uint32_t)(o + e), thr) ? v[e] * scale : 0.f;
                    }
                    if constexpr (XBF)
                        s[q][i] = v + f32x4r{(float)xb[q][i][0], (float)xb[q][i][1], (float)xb[q][i][2], (float)xb[q][i][3]};
                    else
                        s[q][i] = v + xv[q][i];
                    acc[q] += (s[q][i][0] + s[q][i][1]) + (s[q][i][2] + s[q][i][3]);
                }
            }
        }
        if (g + nw < ng) load(g + nw);
#pragma unroll
        for (int q = 0; q < RPW; ++q) {
            const int r = g * RPW + q;
            const float mu = wsum(acc[q]) / d;
            float var = 0.f;
#pragma unroll
            for (int i = 0; i < NV; ++i)
                if (4 * lane + 256 * i < d)
#pragma unroll
                    for (int e = 0; e < 4; ++e) { const float t = s[q][i][e] - mu; var = fmaf(t, t, var); }
            const float rs = rsqrtf(wsum(var) / d + eps);
            if (r >= n) continue;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int c = 4 * lane + 256 * i;
                if (c < d) {
                    const f32x4r gm = *reinterpret_cast<const f32x4r *>(gamma + c);
                    const f32x4r b = *reinterpret_cast<const f32x4r *>(beta + c);
                    *reinterpret_cast<f32x4r *>(out + (size_t)r * d + c) = (s[q][i] - mu) * rs * gm + b;
                }
            }
            if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
        }
    }
}

// Backward: one wave per row, two rows in flight per wave (their loads are
// issued together).  Per block, column partials of dgamma, dbeta and of dy (the
// gradient of W2's bias, b2) go to part[block][3][d].
template <int NPL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NPL <= 2 ? 6 : (NPL <= 4 ? 4 : 2), 8))) void k_ln_bwd(int n, int d, const float *__restrict__ dout,
                                                const float *__restrict__ y, const float *__restrict__ x,
                                                const float *__restrict__ gamma, const float *__restrict__ mean,
                                                const float *__restrict__ rstd, float p_drop,
                                                const int64_t *__restrict__ seedp, uint32_t offset,
                                                float *__restrict__ dy, float *__restrict__ dx,
                                                float *__restrict__ part) {
    __shared__ float s_red[4][kMaxPerLane * 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    float dg[NPL], db[NPL], dyb[NPL];
    float gam[NPL];
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
        dg[i] = db[i] = dyb[i] = 0.f;
        gam[i] = lane + 64 * i < d ? gamma[lane + 64 * i] : 0.f;
    }
    const int stride = gridDim.x * 4;
    for (int r0 = blockIdx.x * 4 + wid; r0 < n; r0 += 2 * stride) {
        const int rr[2] = {r0, r0 + stride};
        float yv[2][NPL], xv[2][NPL], gv[2][NPL], mu[2], rs[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const bool ok = rr[q] < n;
            const int r = ok ? rr[q] : r0;
            mu[q] = mean[r];
            rs[q] = rstd[r];
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int c = lane + 64 * i;
                const size_t o = (size_t)r * d + (c < d ? c : 0);
                yv[q][i] = y[o];
                xv[q][i] = x[o];
                gv[q][i] = (ok && c < d) ? dout[o] : 0.f;
            }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            if (rr[q] >= n) break;
            const size_t rb = (size_t)rr[q] * d;
            float xh[NPL], g[NPL];
            bool keep[NPL];
            float sg = 0.f, sgx = 0.f;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int c = lane + 64 * i;
                xh[i] = g[i] = 0.f;
                keep[i] = true;
                if (c < d) {
                    float v = yv[q][i];
                    if (p_drop > 0.f) {
                        keep[i] = hsg_keep32(dkey, (uint32_t)(rb + c), thr);
                        v = keep[i] ? v * scale : 0.f;
                    }
                    xh[i] = (v + xv[q][i] - mu[q]) * rs[q];
                    const float go = gv[q][i];
                    g[i] = go * gam[i];
                    sg += g[i];
                    sgx = fmaf(g[i], xh[i], sgx);
                    dg[i] = fmaf(go, xh[i], dg[i]);
                    db[i] += go;
                }
            }
            const float mg = wsum(sg) / d, mgx = wsum(sgx) / d;
#pragma unroll
            for (int i = 0; i < NPL; ++i) {
                const int c = lane + 64 * i;
                if (c < d) {
                    const float ds = rs[q] * (g[i] - mg - xh[i] * mgx);
                    const float dyv = keep[i] ? ds * scale : 0.f;
                    dx[rb + c] = ds;
                    dy[rb + c] = dyv;
                    dyb[i] += dyv;
                }
            }
        }
    }
    // block partials, three passes through one LDS slab (fixed order: deterministic)
    float *dst = part + (size_t)blockIdx.x * 3 * d;
#pragma unroll
    for (int which = 0; which < 3; ++which) {
#pragma unroll
        for (int i = 0; i < NPL; ++i) s_red[wid][lane + 64 * i] = which == 0 ? dg[i] : which == 1 ? db[i] : dyb[i];
        __syncthreads();
        for (int c = threadIdx.x; c < d; c += blockDim.x)
            dst[which * d + c] = s_red[0][c] + s_red[1][c] + s_red[2][c] + s_red[3][c];
        __syncthreads();
    }
}

// Vector backward (d % 4 == 0, 16-byte aligned rows, 257..512 columns): lane owns the
// column quads 4*lane + 256*i (float4 loads and stores: 6 instead of 15 row loads), each
// wave walks rows r, r + waves, ... with the next row's dout / y / x requested before
// this row's wave sums and stores (as k_ln_fwd4p).  Same per-element arithmetic as
// k_ln_bwd; the row sums add a lane's columns in another order (fp32 noise), and the
// block partials go to the same part[block][3][d] layout.  cfg2 in-step: 23.0-23.1 vs
// 24.6 us per launch at the 512-block cap (1,024 / 1,536 blocks: 25.3 / 24.0 us and
// larger partial slabs; profiles/r04_dev/ln_bwdp/).
// DYBF (round 5, the bf16 GEMM mode): dy -- a pure GEMM operand there (dH = dy W2,
// dW2 = dy^T H, both on bf16-rounded operands) -- is stored as bf16 rows of pitch ld_dy
// (>= ceil8(d)), the pad columns d .. ceil8(d) - 1 zero (the bf16-A contract of
// hsg_gemm_bf16_psw_io); db2 still sums the fp32 values.
// XBF (round 6): x as bf16 rows of pitch ldx (the forward's k_ln_fwd4p<..., XBF>).
template <int NV, bool DYBF = false, bool YBF = false, bool XBF = false, int PF = 1>
__global__ __launch_bounds__(256) void k_ln_bwd4p(int n, int d, const float *__restrict__ dout,
                                                  const float *__restrict__ y, const float *__restrict__ x,
                                                  const float *__restrict__ gamma, const float *__restrict__ mean,
                                                  const float *__restrict__ rstd, float p_drop,
                                                  const int64_t *__restrict__ seedp, uint32_t offset,
                                                  float *__restrict__ dy, float *__restrict__ dx,
                                                  float *__restrict__ part, int ld_dy = 0, int ldx = 0) {
    __shared__ __attribute__((aligned(16))) float s_red[4][kMaxPerLane * 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t dkey = p_drop > 0.f ? hsg_drop_key((uint64_t)seedp[0], offset) : 0u;
    const uint32_t thr = hsg_drop_threshold(p_drop);
    const float scale = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
    int cq[NV];
    bool cok[NV];
    f32x4r dg[NV], db[NV], dyb[NV], gam[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        cok[i] = 4 * lane + 256 * i < d;
        cq[i] = cok[i] ? 4 * lane + 256 * i : d - 4;               // clamped: loads unused past d
        dg[i] = db[i] = dyb[i] = f32x4r{0.f, 0.f, 0.f, 0.f};
        gam[i] = cok[i] ? *reinterpret_cast<const f32x4r *>(gamma + cq[i]) : f32x4r{0.f, 0.f, 0.f, 0.f};
    }
    const int nw = gridDim.x * 4;
    int r = blockIdx.x * 4 + wid;
    // PF row buffers (dev PF = 2: two rows of the wave's walk in flight; the buffer index
    // is a compile-time constant after unrolling, so the buffers stay in registers)
    f32x4r yv[PF][NV], xv[PF][NV], gv[PF][NV];
    bf16x4r yb[PF][YBF ? NV : 1];                                    // YBF: bf16 y rows, raw until used
    bf16x4r xb[PF][XBF ? NV : 1];                                    // XBF: bf16 x rows, likewise
    float mu[PF], rs[PF];
    auto load = [&](int rr, int bf) {
        mu[bf] = mean[rr];
        rs[bf] = rstd[rr];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const size_t o = (size_t)rr * d + cq[i];
            if constexpr (YBF) yb[bf][i] = *reinterpret_cast<const bf16x4r *>(reinterpret_cast<const __bf16 *>(y) + o);
            else yv[bf][i] = *reinterpret_cast<const f32x4r *>(y + o);
            if constexpr (XBF)
                xb[bf][i] = *reinterpret_cast<const bf16x4r *>(reinterpret_cast<const __bf16 *>(x) + (size_t)rr * ldx + cq[i]);
            else
                xv[bf][i] = *reinterpret_cast<const f32x4r *>(x + o);
            gv[bf][i] = *reinterpret_cast<const f32x4r *>(dout + o);
        }
    };
#pragma unroll
    for (int bf = 0; bf < PF; ++bf)
        if (r + bf * nw < n) load(r + bf * nw, bf);
    for (; r < n; r += PF * nw) {
#pragma unroll
        for (int bf = 0; bf < PF; ++bf) {
            const int rr = r + bf * nw;
            if (rr >= n) break;                                      // wave-uniform
            const size_t rb = (size_t)rr * d;
            f32x4r xh[NV], g[NV];
            uint32_t keep = 0xFFFFFFFFu;                             // bit 4 i + e
            float sg = 0.f, sgx = 0.f;
            const float rsr = rs[bf], mur = mu[bf];
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                xh[i] = g[i] = f32x4r{0.f, 0.f, 0.f, 0.f};
                if (cok[i]) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float v;
                        if constexpr (YBF) v = (float)yb[bf][i][e];
                        else v = yv[bf][i][e];
                        if (p_drop > 0.f) {
                            const bool k = hsg_keep32(dkey, (uint32_t)(rb + cq[i] + e), thr);
                            if (!k) keep &= ~(1u << (4 * i + e));
                            v = k ? v * scale : 0.f;
                        }
                        float xe;
                        if constexpr (XBF) xe = (float)xb[bf][i][e];
                        else xe = xv[bf][i][e];
                        xh[i][e] = (v + xe - mur) * rsr;
                        const float go = gv[bf][i][e];
                        g[i][e] = go * gam[i][e];
                        sg += g[i][e];
                        sgx = fmaf(g[i][e], xh[i][e], sgx);
                        dg[i][e] = fmaf(go, xh[i][e], dg[i][e]);
                        db[i][e] += go;
                    }
                }
            }
            if (rr + PF * nw < n) load(rr + PF * nw, bf);
            const float mg = wsum(sg) / d, mgx = wsum(sgx) / d;
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                if (cok[i]) {
                    f32x4r ds, dyv;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        ds[e] = rsr * (g[i][e] - mg - xh[i][e] * mgx);
                        dyv[e] = (keep >> (4 * i + e)) & 1u ? ds[e] * scale : 0.f;
                    }
                    *reinterpret_cast<f32x4r *>(dx + rb + cq[i]) = ds;
                    if constexpr (DYBF) {
                        *reinterpret_cast<bf16x4r *>(reinterpret_cast<__bf16 *>(dy) + (size_t)rr * ld_dy + cq[i]) =
                            bf16x4r{(__bf16)dyv[0], (__bf16)dyv[1], (__bf16)dyv[2], (__bf16)dyv[3]};
                    } else {
                        *reinterpret_cast<f32x4r *>(dy + rb + cq[i]) = dyv;
                    }
                    dyb[i] += dyv;
                } else if (DYBF && 4 * lane + 256 * i == d && d + 4 <= ld_dy) {   // the zero pad quad
                    *reinterpret_cast<bf16x4r *>(reinterpret_cast<__bf16 *>(dy) + (size_t)rr * ld_dy + d) =
                        bf16x4r{(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
                }
            }
        }
    }
    // block partials, three passes through one LDS slab (fixed order: deterministic)
    float *dst = part + (size_t)blockIdx.x * 3 * d;
#pragma unroll
    for (int which = 0; which < 3; ++which) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
            if (cok[i])
                *reinterpret_cast<f32x4r *>(&s_red[wid][cq[i]]) = which == 0 ? dg[i] : which == 1 ? db[i] : dyb[i];
        __syncthreads();
        for (int c = threadIdx.x; c < d; c += blockDim.x)
            dst[which * d + c] = s_red[0][c] + s_red[1][c] + s_red[2][c] + s_red[3][c];
        __syncthreads();
    }
}

// Column sums of the FFN backward's block-row partial slabs in one launch: the dH
// GEMM's column partials hpart[rows_h][d_hid] -> db1, and hsg_ln_bwd's
// part[rows_ln][3][d] -> dgamma, dbeta, db2.  Block = (32 columns) x (8 row
// groups); group g sums rows g, g+8, ... in order, then the 8 group sums are added
// in order -> deterministic.  accumulate: add into the outputs.
__global__ __launch_bounds__(256) void k_ffn_colsums(int rows_h, int d_hid, const float *__restrict__ hpart,
                                                     float *__restrict__ db1, int rows_ln, int d,
                                                     const float *__restrict__ lnpart, float *__restrict__ dgamma,
                                                     float *__restrict__ dbeta, float *__restrict__ db2, int nb0,
                                                     int accumulate) {
    __shared__ float red[8][33];
    const bool second = (int)blockIdx.x >= nb0;
    const int rows = second ? rows_ln : rows_h, cols = second ? 3 * d : d_hid;
    const float *P = second ? lnpart : hpart;
    const int cb = (second ? (int)blockIdx.x - nb0 : (int)blockIdx.x) * 32;
    const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int c = cb + cl;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (c < cols) {
        int r = g;
        for (; r + 24 < rows; r += 32) {
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q] += P[(size_t)(r + 8 * q) * cols + c];
        }
        for (; r < rows; r += 8) s[0] += P[(size_t)r * cols + c];
    }
    red[g][cl] = (s[0] + s[1]) + (s[2] + s[3]);
    __syncthreads();
    if (g == 0 && c < cols) {
        float a = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) a += red[q][cl];
        float *o;
        if (!second) o = db1 + c;
        else o = c < d ? dgamma + c : (c < 2 * d ? dbeta + (c - d) : db2 + (c - 2 * d));
        *o = accumulate ? *o + a : a;
    }
}

int grid_rows(int n, int cap) {
    int b = (n + 3) / 4;
    if (b < 1) b = 1;
    return b < cap ? b : cap;
}
constexpr int kLnBwdGridCap = 512;
constexpr bool kLnBwdVec = true;       // k_ln_bwd4p for 257..512 aligned columns (dev: HSG_LN_BWDP=0)
// the backward's grid cap: hsg_ln_bwd_blocks and hsg_ln_bwd must agree (part rows)
int ln_bwd_cap() {
    if (const char *e = HSG_DEV_ENV("HSG_LN_BWD_CAP")) return atoi(e) > 0 ? atoi(e) : kLnBwdGridCap;
    return kLnBwdGridCap;
}
constexpr int kLnFwdPBlocks = 1536;   // persistent LayerNorm forward: 6 waves per SIMD (768 / 1024 / 2048: slower)

int status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

int hsg_ln_bwd_blocks(int n) { return grid_rows(n, ln_bwd_cap()); }

int hsg_ln_fwd(int n, int d, const float *y, const float *x, const float *gamma, const float *beta, float eps,
               float p_drop, const int64_t *seed, uint32_t offset, float *out, float *mean, float *rstd,
               void *stream) {
    if (d < 1 || d > 64 * kMaxPerLane || p_drop < 0.f || p_drop >= 1.f || (p_drop > 0.f && !seed) ||
        (p_drop > 0.f && (long)n * d >= (1L << 32)))                      // 32-bit mask index
        return HSG_EINVAL;
    if (n == 0) return 0;
    const int npl = (d + 63) / 64;
    dim3 grid(grid_rows(n, 8192)), block(256);
    hipStream_t st = (hipStream_t)stream;
    int vec = d % 4 == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)out & 15) == 0 &&
              ((uintptr_t)gamma & 15) == 0 && ((uintptr_t)beta & 15) == 0;
    // rows per wave: 3 for 257..512 columns (cfg2 S2W, d = 300: 6,400 waves = one round
    // of resident waves, against 9,600 at 2; step -4 us in one A/B, 4 rows: -3 us)
    int rpw = (d + 255) / 256 == 2 ? 3 : 2;
    if (const char *e = HSG_DEV_ENV("HSG_LN_FWD")) {                   // dev A/B: 0 = scalar, 1-4 rows per wave
        rpw = atoi(e);
        vec = vec && rpw > 0;
    }
    int pblocks = HSG_DEV_ENV("HSG_LN_FWD") ? 0 : kLnFwdPBlocks, prow = 1;   // HSG_LN_FWD: k_ln_fwd4 / k_ln_fwd
    if (const char *e = HSG_DEV_ENV("HSG_LN_FWDP")) pblocks = atoi(e);
    if (const char *e = HSG_DEV_ENV("HSG_LN_FWDP_R")) prow = atoi(e);
    if (pblocks > 0 && vec && (d + 255) / 256 == 2) {
        const int ng = (n + prow - 1) / prow;
        const int blocks = pblocks < (ng + 3) / 4 ? pblocks : (ng + 3) / 4;
#ifdef HSG_DEV
        if (prow == 2) {
            hipLaunchKernelGGL((k_ln_fwd4p<2, 2>), dim3(blocks), block, 0, st, n, d, y, x, gamma, beta, eps, p_drop,
                               seed, offset, out, mean, rstd);
            return status();
        }
#endif
        hipLaunchKernelGGL((k_ln_fwd4p<2, 1>), dim3(blocks), block, 0, st, n, d, y, x, gamma, beta, eps, p_drop, seed,
                           offset, out, mean, rstd);
        return status();
    }
    if (vec) {
        const int nv = (d + 255) / 256;
        const dim3 g4((unsigned)((n + 4 * rpw - 1) / (4 * rpw)));
#define HSG_LNF4(NV_, R_)                                                                                  \
    if (nv == NV_ && rpw == R_) {                                                                          \
        hipLaunchKernelGGL((k_ln_fwd4<NV_, R_>), g4, block, 0, st, n, d, y, x, gamma, beta, eps, p_drop, seed, \
                           offset, out, mean, rstd);                                                       \
        return status();                                                                                   \
    }
        HSG_LNF4(1, 2) HSG_LNF4(2, 3)
#ifdef HSG_DEV
        HSG_LNF4(1, 1) HSG_LNF4(1, 4) HSG_LNF4(2, 1) HSG_LNF4(2, 2) HSG_LNF4(2, 4)
#endif
#undef HSG_LNF4
    }
#define HSG_LNF(K)                                                                                       \
    case K:                                                                                              \
        hipLaunchKernelGGL(k_ln_fwd<K>, grid, block, 0, st, n, d, y, x, gamma, beta, eps, p_drop, seed, \
                           offset, out, mean, rstd);                                                     \
        break;
    switch (npl) { HSG_LNF(1) HSG_LNF(2) HSG_LNF(3) HSG_LNF(4) HSG_LNF(5) HSG_LNF(6) HSG_LNF(7) HSG_LNF(8) }
#undef HSG_LNF
    return status();
}

int hsg_ln_bwd(int n, int d, const float *dout, const float *y, const float *x, const float *gamma,
               const float *mean, const float *rstd, float p_drop, const int64_t *seed, uint32_t offset,
               float *dy, float *dx, float *part, void *stream) {
    if (d < 1 || d > 64 * kMaxPerLane || p_drop < 0.f || p_drop >= 1.f || (p_drop > 0.f && !seed) || !part ||
        (p_drop > 0.f && (long)n * d >= (1L << 32)))
        return HSG_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid(grid_rows(n, ln_bwd_cap())), block(256);
    if (n == 0) return (int)hipMemsetAsync(part, 0, sizeof(float) * 3 * d * grid.x, st);
    const int npl = (d + 63) / 64;
    bool vec = kLnBwdVec;
    if (const char *e = HSG_DEV_ENV("HSG_LN_BWDP")) vec = atoi(e) != 0;            // dev A/B
    const auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
    if (vec && d % 4 == 0 && (d + 255) / 256 == 2 && al(dout) && al(y) && al(x) && al(gamma) && al(dy) && al(dx)) {
#ifdef HSG_DEV
        if (const char *e = HSG_DEV_ENV("HSG_LN_BWD_PF"); e && atoi(e) == 2) {   // dev A/B: two rows in flight
            hipLaunchKernelGGL((k_ln_bwd4p<2, false, false, false, 2>), grid, block, 0, st, n, d, dout, y, x, gamma,
                               mean, rstd, p_drop, seed, offset, dy, dx, part);
            return status();
        }
#endif
        hipLaunchKernelGGL((k_ln_bwd4p<2>), grid, block, 0, st, n, d, dout, y, x, gamma, mean, rstd, p_drop, seed,
                           offset, dy, dx, part);
        return status();
    }
#define HSG_LNB(K)                                                                                       \
    case K:                                                                                              \
        hipLaunchKernelGGL(k_ln_bwd<K>, grid, block, 0, st, n, d, dout, y, x, gamma, mean, rstd, p_drop, \
                           seed, offset, dy, dx, part);                                                  \
        break;
    switch (npl) { HSG_LNB(1) HSG_LNB(2) HSG_LNB(3) HSG_LNB(4) HSG_LNB(5) HSG_LNB(6) HSG_LNB(7) HSG_LNB(8) }
#undef HSG_LNB
    return status();
}

// hsg_ln_bwd with dy stored as bf16 rows (the bf16 GEMM mode's bf16 activations): the
// vector kernel's shapes only (d % 4 == 0, 257..512 columns, 16-byte aligned fp32 rows,
// ld_dy % 8 == 0 and >= ceil8(d), 16-byte aligned dy), HSG_EINVAL otherwise.
int hsg_ln_bwd_dy16(int n, int d, const float *dout, const void *y, int y_bf16, const float *x, const float *gamma,
                    const float *mean, const float *rstd, float p_drop, const int64_t *seed, uint32_t offset,
                    void *dy, int ld_dy, float *dx, float *part, void *stream) {
    const auto al = [](const void *q) { return ((uintptr_t)q & 15) == 0; };
    if (d % 4 || (d + 255) / 256 != 2 || d <= 256 || (ld_dy & 7) || ld_dy < (d + 7) / 8 * 8 || p_drop < 0.f ||
        p_drop >= 1.f || (p_drop > 0.f && !seed) || !part || (p_drop > 0.f && (long)n * d >= (1L << 32)) ||
        !al(dout) || !al(y) || !al(x) || !al(gamma) || !al(dy) || !al(dx))
        return HSG_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid(grid_rows(n, ln_bwd_cap())), block(256);
    if (n == 0) return (int)hipMemsetAsync(part, 0, sizeof(float) * 3 * d * grid.x, st);
    const float *yf = reinterpret_cast<const float *>(y);
    if (y_bf16)
        hipLaunchKernelGGL((k_ln_bwd4p<2, true, true>), grid, block, 0, st, n, d, dout, yf, x, gamma, mean, rstd,
                           p_drop, seed, offset, reinterpret_cast<float *>(dy), dx, part, ld_dy);
    else
        hipLaunchKernelGGL((k_ln_bwd4p<2, true>), grid, block, 0, st, n, d, dout, yf, x, gamma, mean, rstd, p_drop,
                           seed, offset, reinterpret_cast<float *>(dy), dx, part, ld_dy);
    return status();
}

// hsg_ln_fwd with y given as bf16 rows (pitch d; the bf16 GEMM mode's FFN output): the
// persistent vector kernel's shapes only (d % 4 == 0, 257..512 columns, 16-byte aligned
// fp32 rows, 8-byte aligned y), HSG_EINVAL otherwise.  out, mean, rstd as hsg_ln_fwd on
// the bf16 values of y.
int hsg_ln_fwd_y16(int n, int d, const void *y, const float *x, const float *gamma, const float *beta, float eps,
                   float p_drop, const int64_t *seed, uint32_t offset, float *out, float *mean, float *rstd,
                   void *stream) {
    const auto al = [](const void *q, uintptr_t a) { return ((uintptr_t)q & (a - 1)) == 0; };
    if (d % 4 || (d + 255) / 256 != 2 || d <= 256 || p_drop < 0.f || p_drop >= 1.f || (p_drop > 0.f && !seed) ||
        (p_drop > 0.f && (long)n * d >= (1L << 32)) || !al(y, 8) || !al(x, 16) || !al(out, 16) || !al(gamma, 16) ||
        !al(beta, 16))
        return HSG_EINVAL;
    if (n == 0) return 0;
    const int blocks = kLnFwdPBlocks < (n + 3) / 4 ? kLnFwdPBlocks : (n + 3) / 4;
    hipLaunchKernelGGL((k_ln_fwd4p<2, 1, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, d,
                       reinterpret_cast<const float *>(y), x, gamma, beta, eps, p_drop, seed, offset, out, mean, rstd);
    return status();
}

// The bf16 GEMM mode's bf16 x rows (round 6): hsg_ln_fwd_y16 / hsg_ln_bwd_dy16 with the
// residual x given as bf16 rows of pitch ldx (ldx % 8 == 0, >= ceil8(d), 16-byte aligned)
// -- the edge layer's output as hsg_gat_fwd_ws16 stores it.  y is bf16 (pitch d) in both,
// dy bf16 rows of pitch ld_dy in the backward.  HSG_EINVAL off those shapes.
int hsg_ln_fwd_x16(int n, int d, const void *y, const void *x, int ldx, const float *gamma, const float *beta,
                   float eps, float p_drop, const int64_t *seed, uint32_t offset, float *out, float *mean, float *rstd,
                   void *stream) {
    const auto al = [](const void *q, uintptr_t a) { return ((uintptr_t)q & (a - 1)) == 0; };
    if (d % 4 || (d + 255) / 256 != 2 || d <= 256 || (ldx & 7) || ldx < (d + 7) / 8 * 8 || p_drop < 0.f ||
        p_drop >= 1.f || (p_drop > 0.f && !seed) || (p_drop > 0.f && (long)n * d >= (1L << 32)) || !al(y, 8) ||
        !al(x, 16) || !al(out, 16) || !al(gamma, 16) || !al(beta, 16))
        return HSG_EINVAL;
    if (n == 0) return 0;
    const int blocks = kLnFwdPBlocks < (n + 3) / 4 ? kLnFwdPBlocks : (n + 3) / 4;
    hipLaunchKernelGGL((k_ln_fwd4p<2, 1, true, true>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, d,
                       reinterpret_cast<const float *>(y), reinterpret_cast<const float *>(x), gamma, beta, eps,
                       p_drop, seed, offset, out, mean, rstd, ldx);
    return status();
}

int hsg_ln_bwd_x16(int n, int d, const float *dout, const void *y, const void *x, int ldx, const float *gamma,
                   const float *mean, const float *rstd, float p_drop, const int64_t *seed, uint32_t offset, void *dy,
                   int ld_dy, float *dx, float *part, void *stream) {
    const auto al = [](const void *q, uintptr_t a) { return ((uintptr_t)q & (a - 1)) == 0; };
    if (d % 4 || (d + 255) / 256 != 2 || d <= 256 || (ld_dy & 7) || ld_dy < (d + 7) / 8 * 8 || (ldx & 7) ||
        ldx < (d + 7) / 8 * 8 || p_drop < 0.f || p_drop >= 1.f || (p_drop > 0.f && !seed) || !part ||
        (p_drop > 0.f && (long)n * d >= (1L << 32)) || !al(dout, 16) || !al(y, 8) || !al(x, 16) || !al(gamma, 16) ||
        !al(dy, 16) || !al(dx, 16))
        return HSG_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    dim3 grid(grid_rows(n, ln_bwd_cap())), block(256);
    if (n == 0) return (int)hipMemsetAsync(part, 0, sizeof(float) * 3 * d * grid.x, st);
    hipLaunchKernelGGL((k_ln_bwd4p<2, true, true, true>), grid, block, 0, st, n, d, dout,
                       reinterpret_cast<const float *>(y), reinterpret_cast<const float *>(x), gamma, mean, rstd,
                       p_drop, seed, offset, reinterpret_cast<float *>(dy), dx, part, ld_dy, ldx);
    return status();
}

int hsg_ffn_colsums(int rows_h, int d_hid, const float *hpart, float *db1, int rows_ln, int d, const float *lnpart,
                    float *dgamma, float *dbeta, float *db2, int accumulate, void *stream) {
    if (rows_h < 0 || d_hid < 0 || rows_ln < 0 || d < 0) return HSG_EINVAL;
    if ((d_hid && (!hpart || !db1)) || (d && (!lnpart || !dgamma || !dbeta || !db2))) return HSG_EINVAL;
    const int nb0 = (d_hid + 31) / 32, nb1 = (3 * d + 31) / 32;
    if (nb0 + nb1 == 0) return 0;
    hipLaunchKernelGGL(k_ffn_colsums, dim3(nb0 + nb1), dim3(256), 0, (hipStream_t)stream, rows_h, d_hid, hpart, db1,
                       rows_ln, d, lnpart, dgamma, dbeta, db2, nb0, accumulate);
    return status();
}

}  // extern "C"
