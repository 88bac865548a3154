// hsg_attn.hip -- the per-layer attention parameters of a WSGAT/SWGAT application
// (module/GATLayer.py:84-93 / 123-131), folded into two one-block kernels.
//
// Per head k (D = head dim, F = feat_embed_size) the reference computes, per edge,
//   dfeat = feat_fc(tfidfembed_e)            (W_f [D,F], b_f [D] on S2W only)
//   e     = leaky_relu(attn_fc([z_src, z_dst, dfeat]))     attn_fc = [a1 | a2 | a3]
// tfidfembed_e is row t_e of the TF-IDF embedding table T [10, F]
// (HiGraph.py:52, 146-151) or zero (edges never written), and the z_dst part is
// zero (GATLayer.py:111).  So the edge-type term only takes 11 values per head:
//   tau[t][k] = <a3_k, W_f,k T[t] + b_f,k>   (t < 10),   tau[10][k] = <a3_k, b_f,k>
// hsg_attn_params_fwd builds that table (and a contiguous copy of a1 for the
// sigma kernel); hsg_attn_params_bwd reduces the per-block partials the edge
// kernels wrote (d tau, d a1; a 64-range stage kernel, then one workgroup per
// head plus one for dT) and produces every parameter gradient:
//   v[k][f]   = sum_d a3[k][d] W_f[k][d][f]
//   dv[k][f]  = sum_{t<10} dtau[t][k] T[t][f],   dc[k] = sum_{t<=10} dtau[t][k]
//   dT[t][f]  = sum_k dtau[t][k] v[k][f]
//   da3[k][d] = sum_f dv[k][f] W_f[k][d][f] + dc[k] b_f[k][d]
//   dW_f      = a3[k][d] dv[k][f],   db_f = a3[k][d] dc[k]
//   d attn    = [da1 | 0 | da3]
// All sums run in a fixed order (deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hsg.h"

namespace {

constexpr int kNT = 11;        // 10 tf-idf boxes + the zero row
constexpr int kHMax = 16;
constexpr int kFMax = 256;
constexpr int kDMax = 512;     // H*D bound of the edge kernels

constexpr int kWfLds = 8192;   // head slice W_f,k [D][F] staged in LDS when it fits

// v_k[f] = sum_d a3_k[d] W_f,k[d][f] for one head, all f (threads over f), with
// W_f,k staged in LDS (coalesced fill) when D*F fits, else read from global.
__device__ void head_v(int k, int D, int F, const float *__restrict__ attn, const float *__restrict__ wf,
                       float *wlds, float *a3s, float *vout) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const float *wk = wf + (size_t)k * D * F;
    const bool staged = D * F <= kWfLds;
    __syncthreads();
    if (staged)
        for (int i = tid; i < D * F; i += nt) wlds[i] = wk[i];
    for (int d = tid; d < D; d += nt) a3s[d] = attn[k * 3 * D + 2 * D + d];
    __syncthreads();
    const float *W = staged ? wlds : wk;
    for (int f = tid; f < F; f += nt) {
        float s = 0.f;
        for (int d = 0; d < D; ++d) s = fmaf(a3s[d], W[d * F + f], s);
        vout[f] = s;
    }
    __syncthreads();
}

// one workgroup per head k: v_k (W_f,k staged in LDS), then tau[:, k]; block 0
// also writes the contiguous a1 copy
__device__ __forceinline__ void attn_fwd_head(int k, int H, int D, int F, const float *__restrict__ attn,
                                              const float *__restrict__ wf, const float *__restrict__ bf,
                                              const float *__restrict__ T, float *__restrict__ a1,
                                              float *__restrict__ tau) {
    __shared__ float wlds[kWfLds];
    __shared__ float a3s[kDMax];
    __shared__ float v[kFMax];
    __shared__ float part[kNT][33];
    const int tid = threadIdx.x, nt = blockDim.x;
    if (k == 0)
        for (int i = tid; i < H * D; i += nt) {
            const int kk = i / D, d = i - (i / D) * D;
            a1[i] = attn[kk * 3 * D + d];
        }
    head_v(k, D, F, attn, wf, wlds, a3s, v);
    // tau[t][k] = <T[t], v_k> + <a3_k, bf_k>: 11 rows x 32 lanes, fixed-order sums
    const int ln = tid & 31;
    for (int t = tid >> 5; t < kNT; t += nt >> 5) {
        float s = 0.f;
        if (t < kNT - 1)
            for (int f = ln; f < F; f += 32) s = fmaf(T[t * F + f], v[f], s);
        if (bf)
            for (int d = ln; d < D; d += 32) s = fmaf(a3s[d], bf[k * D + d], s);
        part[t][ln] = s;
    }
    __syncthreads();
    if (tid < kNT) {
        float s = 0.f;
        for (int q = 0; q < 32; ++q) s += part[tid][q];
        tau[tid * H + k] = s;
    }
}

__global__ __launch_bounds__(256) void k_attn_params_fwd(int H, int D, int F, const float *__restrict__ attn,
                                                         const float *__restrict__ wf,
                                                         const float *__restrict__ bf,
                                                         const float *__restrict__ T, float *__restrict__ a1,
                                                         float *__restrict__ tau) {
    attn_fwd_head(blockIdx.x, H, D, F, attn, wf, bf, T, a1, tau);
}

// the tables of two layers (the stack's W2S and S2W, sharing T) in one launch:
// blocks [0, H0) are layer 0's heads, [H0, H0 + H1) layer 1's
// optional seed / snap: the step's dropout-seed advance (what k_seed_advance does:
// seed += 1, snap = the new value) rides in this launch, the first of the step's forward
struct AttnFwdPair {
    int H[2], D[2];
    const float *attn[2], *wf[2], *bf[2];
    float *a1[2], *tau[2];
    int64_t *seed, *snap;
};

__global__ __launch_bounds__(256) void k_attn_params_fwd_pair(AttnFwdPair j, int F, const float *__restrict__ T) {
    if (j.seed != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
        const int64_t s = j.seed[0] + 1;
        j.seed[0] = s;
        j.snap[0] = s;
    }
    const int q = (int)blockIdx.x >= j.H[0] ? 1 : 0;
    const int k = (int)blockIdx.x - (q ? j.H[0] : 0);
    attn_fwd_head(k, j.H[q], j.D[q], F, j.attn[q], j.wf[q], j.bf[q], T, j.a1[q], j.tau[q]);
}

// Stage 1 of the partial-slab reduction: blockIdx.y picks the slab (0: d tau
// partials [rows0][cols0], 1: d a1 partials [rows1][cols1]); block x sums its
// contiguous row range for every column into out[y][x][cols].  Rows within a
// range are added in order (deterministic).
constexpr int kStage = 64;     // row ranges per slab

__global__ __launch_bounds__(256) void k_colsum_stage(int rows0, int cols0, const float *__restrict__ p0, int rows1,
                                                      int cols1, const float *__restrict__ p1,
                                                      float *__restrict__ out0, float *__restrict__ out1,
                                                      int accumulate) {
    const int y = blockIdx.y;
    const int rows = y ? rows1 : rows0, cols = y ? cols1 : cols0;
    const float *p = y ? p1 : p0;
    float *out = y ? out1 : out0;
    const int per = (rows + kStage - 1) / kStage;
    const int r0 = blockIdx.x * per, r1 = min(rows, r0 + per);
    for (int c = threadIdx.x; c < cols; c += blockDim.x) {
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        int r = r0;
        for (; r + 4 <= r1; r += 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) s[q] += p[(size_t)(r + q) * cols + c];
        }
        for (; r < r1; ++r) s[0] += p[(size_t)r * cols + c];
        const float v = (s[0] + s[1]) + (s[2] + s[3]);
        out[(size_t)blockIdx.x * cols + c] = accumulate ? out[(size_t)blockIdx.x * cols + c] + v : v;
    }
}

// blocks 0..H-1: one head each (d attn row, dW_f,k, db_f,k); block H: dT
// d tau [11][H] of one layer, summed over the stage rows in order, into LDS
// (rows requested 32 at a time before any is added: the sum still runs in row order)
__device__ __forceinline__ float attn_bwd_dtau_col(int NTH, const float *__restrict__ dtau_st, int srows, int i) {
    float s = 0.f;
    for (int r0 = 0; r0 < srows; r0 += 32) {
        float v[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) v[q] = dtau_st[min(r0 + q, srows - 1) * NTH + i];
#pragma unroll
        for (int q = 0; q < 32; ++q)
            if (r0 + q < srows) s += v[q];
    }
    return s;
}

__device__ __forceinline__ void attn_bwd_dtau(int H, const float *__restrict__ dtau_st, int srows, float *dtau) {
    const int NTH = kNT * H;
    for (int i = threadIdx.x; i < NTH; i += blockDim.x) dtau[i] = attn_bwd_dtau_col(NTH, dtau_st, srows, i);
}

// the dT block's contribution of one layer: dT[t][f] (+)= sum_k dtau[t][k] v_k[f]
// (vall: LDS scratch [H][F])
__device__ __forceinline__ void attn_bwd_dT(int H, int D, int F, const float *dtau, const float *__restrict__ attn,
                                            const float *__restrict__ wf, float *vall, float *__restrict__ dT,
                                            bool acc) {
    const int tid = threadIdx.x, nt = blockDim.x;
    __syncthreads();                               // vall may hold the previous layer's v
    for (int i = tid; i < H * F; i += nt) {
        const int kk = i / F, f = i - (i / F) * F;
        const float *wk = wf + (size_t)kk * D * F;
        const float *a3 = attn + kk * 3 * D + 2 * D;
        float s = 0.f;
        // 32 weights requested at a time (coalesced across f), then added in d order
        for (int d0 = 0; d0 < D; d0 += 32) {
            float w[32], a[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) {
                const int d = min(d0 + q, D - 1);
                w[q] = wk[d * F + f];
                a[q] = a3[d];
            }
#pragma unroll
            for (int q = 0; q < 32; ++q)
                if (d0 + q < D) s = fmaf(a[q], w[q], s);
        }
        vall[i] = s;
    }
    __syncthreads();
    for (int i = tid; i < (kNT - 1) * F; i += nt) {
        const int t = i / F, f = i - (i / F) * F;
        float s = 0.f;
        for (int kk = 0; kk < H; ++kk) s = fmaf(dtau[t * H + kk], vall[kk * F + f], s);
        dT[i] = acc ? dT[i] + s : s;
    }
}

// head k of one layer: da1 (stage rows), da3, dWf, dbf
__device__ __forceinline__ void attn_bwd_head(int k, int H, int D, int F, const float *dtau,
                                              const float *__restrict__ da1_st, const float *__restrict__ attn,
                                              const float *__restrict__ wf, const float *__restrict__ bf,
                                              const float *__restrict__ T, float *__restrict__ dattn,
                                              float *__restrict__ dwf, float *__restrict__ dbf, int accumulate,
                                              int srows, float *wlds, float *a3s, float *dv) {
    const int tid = threadIdx.x, nt = blockDim.x;
    const float *wk = wf + (size_t)k * D * F;
    const bool staged = D * F <= kWfLds;
    if (staged)
        for (int i = tid; i < D * F; i += nt) wlds[i] = wk[i];
    for (int d = tid; d < D; d += nt) a3s[d] = attn[k * 3 * D + 2 * D + d];
    for (int f = tid; f < F; f += nt) {
        float s = 0.f;
        for (int t = 0; t < kNT - 1; ++t) s = fmaf(dtau[t * H + k], T[t * F + f], s);
        dv[f] = s;
    }
    float dc = 0.f;
    for (int t = 0; t < kNT; ++t) dc += dtau[t * H + k];
    __syncthreads();
    const float *W = staged ? wlds : wk;
    const int D3 = 3 * D;
    for (int d = tid; d < D; d += nt) {
        float s = 0.f;
        for (int f = 0; f < F; ++f) s = fmaf(dv[f], W[d * F + f], s);
        if (bf) {
            s = fmaf(dc, bf[k * D + d], s);
            if (dbf) dbf[k * D + d] = (accumulate & 1) ? dbf[k * D + d] + a3s[d] * dc : a3s[d] * dc;
        }
        float g = 0.f;                             // d a1: stage rows in order
        for (int r0 = 0; r0 < srows; r0 += 32) {
            float v[32];
#pragma unroll
            for (int q = 0; q < 32; ++q) v[q] = da1_st[(size_t)min(r0 + q, srows - 1) * H * D + k * D + d];
#pragma unroll
            for (int q = 0; q < 32; ++q)
                if (r0 + q < srows) g += v[q];
        }
        if (accumulate & 1) {
            dattn[k * D3 + d] += g;
            dattn[k * D3 + 2 * D + d] += s;
        } else {
            dattn[k * D3 + d] = g;
            dattn[k * D3 + D + d] = 0.f;
            dattn[k * D3 + 2 * D + d] = s;
        }
    }
    for (int i = tid; i < D * F; i += nt) {
        const int d = i / F, f = i - (i / F) * F;
        const float g = a3s[d] * dv[f];
        dwf[(size_t)k * D * F + i] = (accumulate & 1) ? dwf[(size_t)k * D * F + i] + g : g;
    }
}

__global__ __launch_bounds__(256) void k_attn_params_bwd(int H, int D, int F,
                                                         const float *__restrict__ dtau_st,   // [kStage][11*H]
                                                         const float *__restrict__ da1_st,    // [kStage][H*D]
                                                         const float *__restrict__ attn,
                                                         const float *__restrict__ wf,
                                                         const float *__restrict__ bf,
                                                         const float *__restrict__ T, float *__restrict__ dattn,
                                                         float *__restrict__ dwf, float *__restrict__ dbf,
                                                         float *__restrict__ dT, int accumulate, int srows) {
    __shared__ float wlds[kWfLds];
    __shared__ float a3s[kDMax];
    __shared__ float dv[kFMax];
    __shared__ float dtau[kNT * kHMax];
    attn_bwd_dtau(H, dtau_st, srows, dtau);
    __syncthreads();
    const int k = blockIdx.x;
    if (k == H) {                                  // dT[t][f] = sum_k dtau[t][k] v_k[f]
        attn_bwd_dT(H, D, F, dtau, attn, wf, wlds, dT, (accumulate & 2) != 0);
        return;
    }
    attn_bwd_head(k, H, D, F, dtau, da1_st, attn, wf, bf, T, dattn, dwf, dbf, accumulate, srows, wlds, a3s, dv);
}

// hsg_attn_params_finish of two layers sharing T in one launch: blocks [0, H0) and
// [H0, H0 + H1) are the layers' heads, the last block adds both layers' dT terms in
// layer order (layer 0's update of each element, then layer 1's: the same result as
// the two launches in that order, also when both write the same dT)
struct AttnBwdPair {
    int H[2], D[2], acc[2];
    const float *ws[2], *attn[2], *wf[2], *bf[2];
    float *dattn[2], *dwf[2], *dbf[2], *dT[2];
};

__global__ __launch_bounds__(256) void k_attn_params_bwd_pair(AttnBwdPair j, int F, const float *__restrict__ T,
                                                              int srows) {
    __shared__ float wlds[kWfLds];
    __shared__ float a3s[kDMax];
    __shared__ float dv[kFMax];
    __shared__ float dtau[2][kNT * kHMax];
    const int b = blockIdx.x;
    if (b == j.H[0] + j.H[1]) {                    // dT
        const int n0 = kNT * j.H[0], n1 = kNT * j.H[1];
        for (int i = threadIdx.x; i < n0 + n1; i += blockDim.x) {      // both layers' columns in one pass
            const int q = i >= n0 ? 1 : 0, c = i - (q ? n0 : 0);
            dtau[q][c] = attn_bwd_dtau_col(q ? n1 : n0, j.ws[q], srows, c);
        }
        __syncthreads();
        if ((j.H[0] + j.H[1]) * F <= kWfLds) {
            // both layers' v_k in ONE pass, then each dT element takes layer 0's update
            // and then layer 1's in one thread (the same values as the two passes in
            // that order, also when both layers write the same dT): half the dependent
            // load phases of this block, the launch's critical path
            const int n0v = j.H[0] * F, nv = n0v + j.H[1] * F;
            for (int i = threadIdx.x; i < nv; i += blockDim.x) {
                const int q = i >= n0v ? 1 : 0, ii = i - (q ? n0v : 0);
                const int kk = ii / F, f = ii - kk * F, D = j.D[q];
                const float *wk = j.wf[q] + (size_t)kk * D * F;
                const float *a3 = j.attn[q] + kk * 3 * D + 2 * D;
                float sv = 0.f;
                for (int d0 = 0; d0 < D; d0 += 32) {          // as attn_bwd_dT: 32 at a time, d order
                    float w[32], a[32];
#pragma unroll
                    for (int u = 0; u < 32; ++u) {
                        const int d = min(d0 + u, D - 1);
                        w[u] = wk[d * F + f];
                        a[u] = a3[d];
                    }
#pragma unroll
                    for (int u = 0; u < 32; ++u)
                        if (d0 + u < D) sv = fmaf(a[u], w[u], sv);
                }
                wlds[i] = sv;
            }
            __syncthreads();
            for (int i = threadIdx.x; i < (kNT - 1) * F; i += blockDim.x) {
                const int t = i / F, f = i - t * F;
                float s0 = 0.f, s1 = 0.f;
                for (int kk = 0; kk < j.H[0]; ++kk) s0 = fmaf(dtau[0][t * j.H[0] + kk], wlds[kk * F + f], s0);
                for (int kk = 0; kk < j.H[1]; ++kk) s1 = fmaf(dtau[1][t * j.H[1] + kk], wlds[n0v + kk * F + f], s1);
                j.dT[0][i] = (j.acc[0] & 2) ? j.dT[0][i] + s0 : s0;
                j.dT[1][i] = (j.acc[1] & 2) ? j.dT[1][i] + s1 : s1;
            }
            return;
        }
        for (int q = 0; q < 2; ++q)
            attn_bwd_dT(j.H[q], j.D[q], F, dtau[q], j.attn[q], j.wf[q], wlds, j.dT[q], (j.acc[q] & 2) != 0);
        return;
    }
    const int q = b >= j.H[0] ? 1 : 0, k = b - (q ? j.H[0] : 0);
    attn_bwd_dtau(j.H[q], j.ws[q], srows, dtau[0]);
    __syncthreads();
    const float *da1 = j.ws[q] + (size_t)kStage * kNT * j.H[q];
    attn_bwd_head(k, j.H[q], j.D[q], F, dtau[0], da1, j.attn[q], j.wf[q], j.bf[q], T, j.dattn[q], j.dwf[q], j.dbf[q],
                  j.acc[q], srows, wlds, a3s, dv);
}

int status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

bool dims_ok(int H, int D, int F) { return H >= 1 && H <= kHMax && D >= 1 && H * D <= kDMax && F >= 1 && F <= kFMax; }

}  // namespace

extern "C" {

int hsg_attn_params_fwd(int H, int D, int F, const float *attn, const float *wf, const float *bf, const float *T,
                        float *a1, float *tau, void *stream) {
    if (!dims_ok(H, D, F) || !attn || !wf || !T || !a1 || !tau) return HSG_EINVAL;
    hipLaunchKernelGGL(k_attn_params_fwd, dim3(H), dim3(256), 0, (hipStream_t)stream, H, D, F, attn, wf, bf, T,
                       a1, tau);
    return status();
}

int hsg_attn_params_fwd_pair(int H0, int D0, const float *attn0, const float *wf0, const float *bf0, float *a1_0,
                             float *tau0, int H1, int D1, const float *attn1, const float *wf1, const float *bf1,
                             float *a1_1, float *tau1, int F, const float *T, void *stream) {
    if (!dims_ok(H0, D0, F) || !dims_ok(H1, D1, F) || !attn0 || !wf0 || !a1_0 || !tau0 || !attn1 || !wf1 || !a1_1 ||
        !tau1 || !T)
        return HSG_EINVAL;
    return hsg_attn_params_fwd_pair_seed(H0, D0, attn0, wf0, bf0, a1_0, tau0, H1, D1, attn1, wf1, bf1, a1_1, tau1, F,
                                         T, nullptr, nullptr, stream);
}

int hsg_attn_params_fwd_pair_seed(int H0, int D0, const float *attn0, const float *wf0, const float *bf0,
                                  float *a1_0, float *tau0, int H1, int D1, const float *attn1, const float *wf1,
                                  const float *bf1, float *a1_1, float *tau1, int F, const float *T, int64_t *seed,
                                  int64_t *snap, void *stream) {
    if (!dims_ok(H0, D0, F) || !dims_ok(H1, D1, F) || !attn0 || !wf0 || !a1_0 || !tau0 || !attn1 || !wf1 || !a1_1 ||
        !tau1 || !T || (seed == nullptr) != (snap == nullptr))
        return HSG_EINVAL;
    AttnFwdPair j{{H0, H1}, {D0, D1}, {attn0, attn1}, {wf0, wf1}, {bf0, bf1}, {a1_0, a1_1}, {tau0, tau1}, seed, snap};
    hipLaunchKernelGGL(k_attn_params_fwd_pair, dim3(H0 + H1), dim3(256), 0, (hipStream_t)stream, j, F, T);
    return status();
}

size_t hsg_attn_params_bwd_workspace_floats(int H, int D) { return (size_t)kStage * (kNT * H + H * D); }

int hsg_attn_params_bwd(int H, int D, int F, int n_dtau_part, const float *dtau_part, int n_da1_part,
                        const float *da1_part, const float *attn, const float *wf, const float *bf, const float *T,
                        float *dattn, float *dwf, float *dbf, float *dT, float *workspace, int accumulate,
                        void *stream) {
    if (!dims_ok(H, D, F) || n_dtau_part < 0 || n_da1_part < 0 || !dtau_part || !da1_part || !attn || !wf ||
        !T || !dattn || !dwf || !dT || !workspace)
        return HSG_EINVAL;
    int rc = hsg_attn_params_stage(H, D, n_dtau_part, dtau_part, n_da1_part, da1_part, workspace, 0, stream);
    if (rc) return rc;
    return hsg_attn_params_finish(H, D, F, workspace, attn, wf, bf, T, dattn, dwf, dbf, dT, accumulate, stream);
}

int hsg_attn_params_stage(int H, int D, int n_dtau_part, const float *dtau_part, int n_da1_part,
                          const float *da1_part, float *workspace, int accumulate, void *stream) {
    if (H < 1 || H > kHMax || D < 1 || H * D > kDMax || n_dtau_part < 0 || n_da1_part < 0 || !dtau_part ||
        !da1_part || !workspace)
        return HSG_EINVAL;
    float *s0 = workspace, *s1 = workspace + (size_t)kStage * kNT * H;
    hipLaunchKernelGGL(k_colsum_stage, dim3(kStage, 2), dim3(256), 0, (hipStream_t)stream, n_dtau_part, kNT * H,
                       dtau_part, n_da1_part, H * D, da1_part, s0, s1, accumulate);
    return status();
}

int hsg_attn_params_finish(int H, int D, int F, const float *workspace, const float *attn, const float *wf,
                           const float *bf, const float *T, float *dattn, float *dwf, float *dbf, float *dT,
                           int accumulate, void *stream) {
    if (!dims_ok(H, D, F) || !workspace || !attn || !wf || !T || !dattn || !dwf || !dT) return HSG_EINVAL;
    const float *s0 = workspace, *s1 = workspace + (size_t)kStage * kNT * H;
    hipLaunchKernelGGL(k_attn_params_bwd, dim3(H + 1), dim3(256), 0, (hipStream_t)stream, H, D, F, s0, s1, attn, wf,
                       bf, T, dattn, dwf, dbf, dT, accumulate, kStage);
    return status();
}


int hsg_attn_params_finish_pair(int H0, int D0, const float *ws0, const float *attn0, const float *wf0,
                                const float *bf0, float *dattn0, float *dwf0, float *dbf0, float *dT0, int acc0,
                                int H1, int D1, const float *ws1, const float *attn1, const float *wf1,
                                const float *bf1, float *dattn1, float *dwf1, float *dbf1, float *dT1, int acc1,
                                int F, const float *T, void *stream) {
    if (!dims_ok(H0, D0, F) || !dims_ok(H1, D1, F) || !ws0 || !ws1 || !attn0 || !attn1 || !wf0 || !wf1 || !dattn0 ||
        !dattn1 || !dwf0 || !dwf1 || !dT0 || !dT1 || !T)
        return HSG_EINVAL;
    AttnBwdPair j{{H0, H1}, {D0, D1}, {acc0, acc1}, {ws0, ws1}, {attn0, attn1}, {wf0, wf1}, {bf0, bf1},
                  {dattn0, dattn1}, {dwf0, dwf1}, {dbf0, dbf1}, {dT0, dT1}};
    hipLaunchKernelGGL(k_attn_params_bwd_pair, dim3(H0 + H1 + 1), dim3(256), 0, (hipStream_t)stream, j, F, T,
                       kStage);
    return status();
}

}  // extern "C"
