// hsg_gat.hip -- fused multi-head heterogeneous GAT edge kernels for gfx950 (MI355X).
//
// Replaces, for one WSGATLayer/SWGATLayer application with all heads at once
// (module/GATLayer.py:81-152, module/GATStackLayer.py:55-59, module/GAT.py:56-57):
//   * DGL apply_edges(edge_attention)  -> s_e = leaky(sigma[src] + tau[box])  
//   * DGL pull(message_func, reduce_func) with degree bucketing -> one wave per
//     destination, online softmax over its CSR segment, phantom in-edges folded in
//     as c_v * exp(-m_v), weighted aggregation of Z rows
//   * F.elu + residual
// and their backward (destination-centric CSR pass + source-centric CSC pass, no
// atomics on global memory, deterministic).
//
// Wave-level design (64-lane wavefronts):
//   (k,l) mapping: lane = k*LPH + l, LPH = 64 / nextpow2(H).  Lanes of head k split
//       that head's per-edge scalar work (scores, alphas, dot products) and reduce
//       with xor-shuffles inside their aligned LPH-lane group.
//   flat mapping:  lane owns features f = lane + 64*i (i < NF): every Z/G/out row
//       access is a contiguous 256-B wave transaction.
//   Per-wave LDS holds one 64-edge chunk of {alpha[j][k], neighbour rank[j]}.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/hsg.h"

#define HSG_HMAX 16          // max heads (reference: 8 for W2S, 6 for S2W)
#define HSG_NT 11            // tau table rows: 10 tf-idf boxes + zero row
#define HSG_WAVES 4          // waves per 256-thread block
#define HSG_CHUNK 64         // edges staged per LDS chunk

namespace {

__device__ __forceinline__ void wave_lds_sync() {
    // Order this wave's LDS writes before its own subsequent reads by other lanes.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float leaky(float x, float slope) { return x > 0.f ? x : x * slope; }

// merge two online-softmax partials (max, sum); -inf/-inf stays (-inf, 0)
__device__ __forceinline__ void lse_merge(float &m, float &s, float om, float os) {
    float M = fmaxf(m, om);
    if (M == -INFINITY) { m = M; s = 0.f; return; }
    s = s * __expf(m - M) + os * __expf(om - M);
    m = M;
}

__device__ __forceinline__ float group_sum(float x, int lph) {
    for (int o = lph >> 1; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

struct RelPtrs {
    int n_src, n_dst, n_edges;
    const int32_t *__restrict__ indptr;
    const int32_t *__restrict__ src;
    const uint8_t *__restrict__ tf;
    const int32_t *__restrict__ phantom;
    const int32_t *__restrict__ cindptr;
    const int32_t *__restrict__ cdst;
    const int32_t *__restrict__ cperm;
};

RelPtrs rel_ptrs(const hsg_rel *r) {
    return RelPtrs{r->n_src, r->n_dst, r->n_edges, r->indptr, r->src, r->tf, r->phantom,
                   r->cindptr, r->cdst, r->cperm};
}

template <int TAU_MODE>
__device__ __forceinline__ int tau_row(const RelPtrs &R, int e) {
    if constexpr (TAU_MODE == HSG_TAU_TABLE) return (int)R.tf[e];
    else return e;
}

// ---------------------------------------------------------------- forward ----
template <int NF, int TAU_MODE>
__global__ __launch_bounds__(256) void k_gat_fwd(RelPtrs R, int H, int D, int lph, float slope,
                                                const float *__restrict__ Z,
                                                const float *__restrict__ sigma,
                                                const float *__restrict__ tau,
                                                const float *__restrict__ origin,
                                                float *__restrict__ hout, float *__restrict__ out,
                                                float *__restrict__ mout, float *__restrict__ lout) {
    __shared__ float s_alpha[HSG_WAVES][HSG_CHUNK * HSG_HMAX];
    __shared__ int s_nb[HSG_WAVES][HSG_CHUNK];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    int fh[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) { int f = lane + 64 * i; fh[i] = f < HD ? f / D : 0; }
    float *sa = s_alpha[wid];
    int *sn = s_nb[wid];

    for (int v = blockIdx.x * HSG_WAVES + wid; v < R.n_dst; v += gridDim.x * HSG_WAVES) {
        const int beg = R.indptr[v], end = R.indptr[v + 1];
        const int c = R.phantom[v];
        // phase 1: online (max, sum) of this head's scores over edges j = l (mod lph)
        float mx = -INFINITY, sm = 0.f;
        if (kact) {
            for (int e = beg + l; e < end; e += lph) {
                const int u = R.src[e];
                const float s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                if (s > mx) { sm = sm * __expf(mx - s) + 1.f; mx = s; }
                else sm += __expf(s - mx);
            }
        }
        for (int o = lph >> 1; o >= 1; o >>= 1) {
            const float om = __shfl_xor(mx, o), os = __shfl_xor(sm, o);
            lse_merge(mx, sm, om, os);
        }
        if (c > 0) lse_merge(mx, sm, 0.f, (float)c);     // phantom in-edges: e = 0
        const bool any = end > beg;
        const float inv = any ? 1.f / sm : 0.f;

        // phase 2: stage alphas per 64-edge chunk, then flat-mapped aggregation
        float acc[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i] = 0.f;
        for (int cb = beg; cb < end; cb += HSG_CHUNK) {
            const int n = min(HSG_CHUNK, end - cb);
            if (kact) {
                for (int j = l; j < n; j += lph) {
                    const int e = cb + j;
                    const int u = R.src[e];
                    const float s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                    sa[j * H + k] = __expf(s - mx) * inv;
                    if (k == 0) sn[j] = u;
                }
            }
            wave_lds_sync();
#pragma unroll 4
            for (int j = 0; j < n; ++j) {
                const float *zr = Z + (size_t)sn[j] * HD;
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const int f = lane + 64 * i;
                    if (f < HD) acc[i] = fmaf(sa[j * H + fh[i]], zr[f], acc[i]);
                }
            }
            wave_lds_sync();
        }
        // epilogue: h, and elu(h) + origin (GAT.py:56-57)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int f = lane + 64 * i;
            if (f < HD) {
                const size_t o = (size_t)v * HD + f;
                const float hv = acc[i];
                hout[o] = hv;
                if (origin) out[o] = (hv > 0.f ? hv : expm1f(hv)) + origin[o];
            }
        }
        if (kact && l == 0) {
            mout[v * H + k] = any ? mx : 0.f;
            lout[v * H + k] = any ? sm : 1.f;
        }
    }
}

// ---------------------------------------------------- backward: dst-centric ----
template <int NE, int TAU_MODE>
__global__ __launch_bounds__(256) void k_gat_bwd_dst(RelPtrs R, int H, int D, int lph, int origin_mode,
                                                    float slope,
                                                    const float *__restrict__ Z,
                                                    const float *__restrict__ sigma,
                                                    const float *__restrict__ tau,
                                                    const float *__restrict__ hsv,
                                                    const float *__restrict__ mv,
                                                    const float *__restrict__ lv,
                                                    const float *__restrict__ dout,
                                                    float *__restrict__ G, float *__restrict__ dpre,
                                                    float *__restrict__ dtau_part) {
    __shared__ float s_dtau[HSG_WAVES][HSG_NT * HSG_HMAX];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    float *sd = s_dtau[wid];
    if constexpr (TAU_MODE == HSG_TAU_TABLE) {
        for (int i = lane; i < HSG_NT * HSG_HMAX; i += 64) sd[i] = 0.f;
        wave_lds_sync();
    }

    for (int v = blockIdx.x * HSG_WAVES + wid; v < R.n_dst; v += gridDim.x * HSG_WAVES) {
        const int beg = R.indptr[v], end = R.indptr[v + 1];
        float g[NE];
        float rho = 0.f;
#pragma unroll
        for (int i = 0; i < NE; ++i) {
            const int d = l + lph * i;
            g[i] = 0.f;
            if (kact && d < D) {
                const size_t o = (size_t)v * HD + k * D + d;
                const float hv = hsv[o], dv = dout[o];
                const float gv = origin_mode ? (hv > 0.f ? dv : dv * __expf(hv)) : dv;
                G[o] = gv;
                g[i] = gv;
                rho = fmaf(gv, hv, rho);
            }
        }
        if (end == beg) continue;   // uniform per wave: no typed in-edge, no gradient
        rho = group_sum(rho, lph);
        const float M = kact ? mv[v * H + k] : 0.f;
        const float inv = kact ? 1.f / lv[v * H + k] : 0.f;
        for (int e = beg; e < end; ++e) {
            const int u = R.src[e];
            const float *zr = Z + (size_t)u * HD + k * D;
            float dot = 0.f;
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                const int d = l + lph * i;
                if (kact && d < D) dot = fmaf(g[i], zr[d], dot);
            }
            dot = group_sum(dot, lph);
            if (kact && l == 0) {
                const int t = tau_row<TAU_MODE>(R, e);
                const float pre = sigma[u * H + k] + tau[t * H + k];
                const float alpha = __expf(leaky(pre, slope) - M) * inv;
                const float ds = alpha * (dot - rho);
                const float dp = pre > 0.f ? ds : ds * slope;
                dpre[(size_t)e * H + k] = dp;
                if constexpr (TAU_MODE == HSG_TAU_TABLE) sd[t * H + k] += dp;
            }
        }
    }
    if constexpr (TAU_MODE == HSG_TAU_TABLE) {
        __syncthreads();
        const int nt = HSG_NT * H;
        for (int i = threadIdx.x; i < nt; i += blockDim.x) {
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < HSG_WAVES; ++w) a += s_dtau[w][i];
            dtau_part[(size_t)blockIdx.x * nt + i] = a;
        }
    }
}

// ---------------------------------------------------- backward: src-centric ----
template <int NF, int TAU_MODE>
__global__ __launch_bounds__(256) void k_gat_bwd_src(RelPtrs R, int H, int D, int lph, float slope,
                                                    const float *__restrict__ sigma,
                                                    const float *__restrict__ tau,
                                                    const float *__restrict__ mv,
                                                    const float *__restrict__ lv,
                                                    const float *__restrict__ G,
                                                    const float *__restrict__ dpre,
                                                    const float *__restrict__ a1,
                                                    const float *__restrict__ Z,
                                                    float *__restrict__ dZ, float *__restrict__ dsigma,
                                                    float *__restrict__ da1_part) {
    __shared__ float s_alpha[HSG_WAVES][HSG_CHUNK * HSG_HMAX];
    __shared__ int s_nb[HSG_WAVES][HSG_CHUNK];
    __shared__ float s_dsig[HSG_WAVES][HSG_HMAX];
    __shared__ float s_da1[HSG_WAVES][64 * NF];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    int fh[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) { int f = lane + 64 * i; fh[i] = f < HD ? f / D : 0; }
    float *sa = s_alpha[wid];
    int *sn = s_nb[wid];
    float da1[NF];                       // this wave's share of sum_u dsigma[u,k] Z[u,k,:]
#pragma unroll
    for (int i = 0; i < NF; ++i) da1[i] = 0.f;

    for (int u = blockIdx.x * HSG_WAVES + wid; u < R.n_src; u += gridDim.x * HSG_WAVES) {
        const int beg = R.cindptr[u], end = R.cindptr[u + 1];
        const float sig = kact ? sigma[u * H + k] : 0.f;
        float dsig = 0.f;
        float acc[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i] = 0.f;
        for (int cb = beg; cb < end; cb += HSG_CHUNK) {
            const int n = min(HSG_CHUNK, end - cb);
            if (kact) {
                for (int j = l; j < n; j += lph) {
                    const int p = cb + j;
                    const int v = R.cdst[p];
                    const int e = R.cperm[p];
                    const float pre = sig + tau[tau_row<TAU_MODE>(R, e) * H + k];
                    sa[j * H + k] = __expf(leaky(pre, slope) - mv[v * H + k]) / lv[v * H + k];
                    dsig += dpre[(size_t)e * H + k];
                    if (k == 0) sn[j] = v;
                }
            }
            wave_lds_sync();
#pragma unroll 4
            for (int j = 0; j < n; ++j) {
                const float *gr = G + (size_t)sn[j] * HD;
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const int f = lane + 64 * i;
                    if (f < HD) acc[i] = fmaf(sa[j * H + fh[i]], gr[f], acc[i]);
                }
            }
            wave_lds_sync();
        }
        dsig = group_sum(dsig, lph);
        if (kact && l == 0) {
            if (dsigma) dsigma[u * H + k] = dsig;
            s_dsig[wid][k] = dsig;
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int f = lane + 64 * i;
            if (f < HD) {
                const float ds = s_dsig[wid][fh[i]];
                float r = acc[i];
                if (a1) r = fmaf(ds, a1[f], r);
                dZ[(size_t)u * HD + f] = r;
                if (da1_part) da1[i] = fmaf(ds, Z[(size_t)u * HD + f], da1[i]);
            }
        }
        wave_lds_sync();
    }
    if (da1_part) {                      // block partial of d a1 (fixed order: deterministic)
#pragma unroll
        for (int i = 0; i < NF; ++i) s_da1[wid][lane + 64 * i] = da1[i];
        __syncthreads();
        for (int f = threadIdx.x; f < HD; f += blockDim.x) {
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < HSG_WAVES; ++w) a += s_da1[w][f];
            da1_part[(size_t)blockIdx.x * HD + f] = a;
        }
    }
}

// ------------------------------------------------------ sigma = <Z_k, a1_k> ----
__global__ __launch_bounds__(256) void k_attn_src_logits(int n, int H, int D, int lph,
                                                        const float *__restrict__ Z,
                                                        const float *__restrict__ a1,
                                                        float *__restrict__ sigma) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const int HD = H * D;
    for (int u = blockIdx.x * HSG_WAVES + wid; u < n; u += gridDim.x * HSG_WAVES) {
        float s = 0.f;
        if (k < H)
            for (int d = l; d < D; d += lph) s = fmaf(Z[(size_t)u * HD + k * D + d], a1[k * D + d], s);
        s = group_sum(s, lph);
        if (k < H && l == 0) sigma[u * H + k] = s;
    }
}

// ------------------------------------------------------------ host helpers ----
int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }
int lanes_per_head(int H) { return 64 / next_pow2(H); }
int grid_for(int rows, int cap) {
    int b = (rows + HSG_WAVES - 1) / HSG_WAVES;
    if (b < 1) b = 1;
    return b < cap ? b : cap;
}
constexpr int kFwdGridCap = 8192;
constexpr int kBwdDstGridCap = 1024;   // bounds the dtau partial slab
constexpr int kBwdSrcGridCap = 2048;   // bounds the d a1 partial slab

bool shape_ok(int H, int D) { return H >= 1 && H <= HSG_HMAX && D >= 1 && H * D <= 512; }

int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int TAU>
int fwd_dispatch(int nf, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, float slope,
                 const float *Z, const float *sg, const float *tau, const float *org, float *h,
                 float *out, float *m, float *l) {
#define HSG_FWD(NF_)                                                                           \
    case NF_:                                                                                  \
        hipLaunchKernelGGL((k_gat_fwd<NF_, TAU>), grid, dim3(256), 0, st, R, H, D, lph, slope, Z, \
                           sg, tau, org, h, out, m, l);                                        \
        break;
    switch (nf) {
        HSG_FWD(1) HSG_FWD(2) HSG_FWD(3) HSG_FWD(4) HSG_FWD(5) HSG_FWD(6) HSG_FWD(7) HSG_FWD(8)
        default: return HSG_EINVAL;
    }
#undef HSG_FWD
    return launch_status();
}

template <int TAU>
int bwd_dst_dispatch(int ne, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, int om,
                     float slope, const float *Z, const float *sg, const float *tau, const float *h,
                     const float *m, const float *l, const float *dout, float *G, float *dpre,
                     float *dtp) {
#define HSG_BD(NE_)                                                                              \
    case NE_:                                                                                    \
        hipLaunchKernelGGL((k_gat_bwd_dst<NE_, TAU>), grid, dim3(256), 0, st, R, H, D, lph, om,   \
                           slope, Z, sg, tau, h, m, l, dout, G, dpre, dtp);                      \
        break;
    switch (ne) {
        HSG_BD(1) HSG_BD(2) HSG_BD(3) HSG_BD(4) HSG_BD(5) HSG_BD(6) HSG_BD(7) HSG_BD(8)
        HSG_BD(16) HSG_BD(32) HSG_BD(64)
        default: return HSG_EINVAL;
    }
#undef HSG_BD
    return launch_status();
}

int ne_bucket(int ne) {
    if (ne <= 8) return ne;
    if (ne <= 16) return 16;
    if (ne <= 32) return 32;
    if (ne <= 64) return 64;
    return -1;
}

template <int TAU>
int bwd_src_dispatch(int nf, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, float slope,
                     const float *sg, const float *tau, const float *m, const float *l, const float *G,
                     const float *dpre, const float *a1, const float *Z, float *dZ, float *dsig, float *da1p) {
#define HSG_BS(NF_)                                                                               \
    case NF_:                                                                                     \
        hipLaunchKernelGGL((k_gat_bwd_src<NF_, TAU>), grid, dim3(256), 0, st, R, H, D, lph, slope, \
                           sg, tau, m, l, G, dpre, a1, Z, dZ, dsig, da1p);                        \
        break;
    switch (nf) {
        HSG_BS(1) HSG_BS(2) HSG_BS(3) HSG_BS(4) HSG_BS(5) HSG_BS(6) HSG_BS(7) HSG_BS(8)
        default: return HSG_EINVAL;
    }
#undef HSG_BS
    return launch_status();
}

}  // namespace

extern "C" {

int hsg_gat_fwd(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                const float *sigma, const float *tau, const float *origin, float *h, float *out,
                float *m, float *l, void *stream) {
    if (!rel || !shape_ok(H, D) || (origin && !out)) return HSG_EINVAL;
    if (rel->n_dst == 0) return 0;
    const RelPtrs R = rel_ptrs(rel);
    const int nf = (H * D + 63) / 64;
    const dim3 grid(grid_for(rel->n_dst, kFwdGridCap));
    hipStream_t st = (hipStream_t)stream;
    if (tau_mode == HSG_TAU_TABLE)
        return fwd_dispatch<HSG_TAU_TABLE>(nf, grid, st, R, H, D, lanes_per_head(H), slope, Z, sigma,
                                           tau, origin, h, out, m, l);
    if (tau_mode == HSG_TAU_PER_EDGE)
        return fwd_dispatch<HSG_TAU_PER_EDGE>(nf, grid, st, R, H, D, lanes_per_head(H), slope, Z,
                                              sigma, tau, origin, h, out, m, l);
    return HSG_EINVAL;
}

int hsg_gat_bwd_blocks(const hsg_rel *rel) { return rel ? grid_for(rel->n_dst, kBwdDstGridCap) : 0; }

int hsg_gat_bwd_dst(const hsg_rel *rel, int H, int D, int tau_mode, int origin_mode, float slope,
                    const float *Z, const float *sigma, const float *tau, const float *h,
                    const float *m, const float *l, const float *dout, float *G, float *dpre,
                    float *dtau_part, void *stream) {
    if (!rel || !shape_ok(H, D)) return HSG_EINVAL;
    const int lph = lanes_per_head(H);
    const int ne = ne_bucket((D + lph - 1) / lph);
    if (ne < 0) return HSG_EINVAL;
    const RelPtrs R = rel_ptrs(rel);
    const dim3 grid(hsg_gat_bwd_blocks(rel));
    hipStream_t st = (hipStream_t)stream;
    if (rel->n_dst == 0) {
        if (tau_mode == HSG_TAU_TABLE && dtau_part)
            return (int)hipMemsetAsync(dtau_part, 0, sizeof(float) * HSG_NT * H * grid.x, st);
        return 0;
    }
    if (tau_mode == HSG_TAU_TABLE)
        return bwd_dst_dispatch<HSG_TAU_TABLE>(ne, grid, st, R, H, D, lph, origin_mode, slope, Z, sigma,
                                               tau, h, m, l, dout, G, dpre, dtau_part);
    if (tau_mode == HSG_TAU_PER_EDGE)
        return bwd_dst_dispatch<HSG_TAU_PER_EDGE>(ne, grid, st, R, H, D, lph, origin_mode, slope, Z,
                                                  sigma, tau, h, m, l, dout, G, dpre, dtau_part);
    return HSG_EINVAL;
}

int hsg_gat_bwd_src_blocks(const hsg_rel *rel) { return rel ? grid_for(rel->n_src, kBwdSrcGridCap) : 0; }

int hsg_gat_bwd_src(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *sigma,
                    const float *tau, const float *m, const float *l, const float *G,
                    const float *dpre, const float *a1, const float *Z, float *dZ, float *dsigma,
                    float *da1_part, void *stream) {
    if (!rel || !shape_ok(H, D) || (da1_part && !Z)) return HSG_EINVAL;
    const RelPtrs R = rel_ptrs(rel);
    const int nf = (H * D + 63) / 64;
    const dim3 grid(hsg_gat_bwd_src_blocks(rel));
    hipStream_t st = (hipStream_t)stream;
    if (rel->n_src == 0) {
        if (da1_part) return (int)hipMemsetAsync(da1_part, 0, sizeof(float) * H * D * grid.x, st);
        return 0;
    }
    if (tau_mode == HSG_TAU_TABLE)
        return bwd_src_dispatch<HSG_TAU_TABLE>(nf, grid, st, R, H, D, lanes_per_head(H), slope, sigma,
                                               tau, m, l, G, dpre, a1, Z, dZ, dsigma, da1_part);
    if (tau_mode == HSG_TAU_PER_EDGE)
        return bwd_src_dispatch<HSG_TAU_PER_EDGE>(nf, grid, st, R, H, D, lanes_per_head(H), slope,
                                                  sigma, tau, m, l, G, dpre, a1, Z, dZ, dsigma, da1_part);
    return HSG_EINVAL;
}

int hsg_attn_src_logits(int n, int H, int D, const float *Z, const float *a1, float *sigma,
                        void *stream) {
    if (!shape_ok(H, D)) return HSG_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_attn_src_logits, dim3(grid_for(n, kFwdGridCap)), dim3(256), 0,
                       (hipStream_t)stream, n, H, D, lanes_per_head(H), Z, a1, sigma);
    return launch_status();
}

const char *hsg_version(void) { return "hsg 0.1 gfx950 (fp32 WSWGAT edge kernels)"; }

}  // extern "C"
