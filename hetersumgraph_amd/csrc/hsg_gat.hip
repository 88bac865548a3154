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
#include <hip/hip_ext.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>

#include "../../include/hsg.h"
#include "hsg_dev.h"

#define HSG_HMAX 16          // max heads (reference: 8 for W2S, 6 for S2W)
#define HSG_NT 11            // tau table rows: 10 tf-idf boxes + zero row
#define HSG_WAVES 4          // waves per 256-thread block
#define HSG_CHUNK 64         // edges staged per LDS chunk

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void wave_lds_sync() {
    // Order this wave's LDS writes before its own subsequent reads by other lanes.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Raw buffer access (k_gat_fwd_b): the row offset goes in soffset (wave-uniform), the
// feature's byte offset in voffset; an offset past the descriptor's byte count reads 0
// and drops the store.  Descriptors are built from kernel arguments (wave-uniform).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *p, long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)voff, (int)soff, 0));
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, float x) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(x), r, (int)voff, (int)soff, 0);
}

__device__ __forceinline__ float leaky(float x, float slope) { return x > 0.f ? x : x * slope; }

// F.elu (GAT.py:56): x for x > 0, else exp(x) - 1 on v_exp_f32.  Absolute error
// <= ~2e-7 against expm1 (the reference's elu), far inside the 1e-5 fp64 parity
// bound; 4 VALU instead of the ~30 of a libm expm1f.
__device__ __forceinline__ float elu1(float x) { return x > 0.f ? x : __expf(x) - 1.f; }

// f / D for 0 <= f < 2^12, D >= 1, without an integer division: (f + 0.5) / D sits
// at least 0.5 / D away from the next integer, far more than the float rounding.
__device__ __forceinline__ int div_small(int f, float inv_d) { return (int)(((float)f + 0.5f) * inv_d); }

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
    int xcd;                 // 1: XCD-local node order (work_range)
    int n_dwork, n_swork;    // work lists (hsg_rel.dwork / swork; round 6), 0 = none
    int32_t *dwork;          // [n][4] items, then [n] arrival counters
    int32_t *swork;
};

// XCD-local node order (round 4).  The batched graph is a disjoint union of documents
// with node ids document by document (dataloader.py:480), so a node's neighbours --
// the rows its segment gathers -- lie in its own document, near it in rank order.
// Workgroup b is dispatched to XCD b % 8 (round robin; the map is not guaranteed, so
// this is for locality only and any placement stays correct): with a grid that is a
// multiple of 8, XCD x walks the contiguous eighth [s_x, e_x) of the n nodes, so each
// XCD's 4 MB L2 fetches only its own documents' rows instead of every XCD fetching
// all of them (S2W: the Z / sigma table 8 times over; W2S and the src passes: the
// rows shared by a document's nodes once per XCD that touches them).
struct WorkRange { int first, end, stride; };
__device__ __forceinline__ WorkRange work_range(int n, int npb, int slot, int xcd) {
    const int g = (int)gridDim.x, b = (int)blockIdx.x;
    if (!xcd || (g & 7)) return WorkRange{b * npb + slot, n, g * npb};
    const int x = b & 7, j = b >> 3, per = n >> 3, rem = n & 7;
    const int s = x * per + min(x, rem);
    return WorkRange{s + j * npb + slot, s + per + (x < rem ? 1 : 0), (g >> 3) * npb};
}

RelPtrs rel_ptrs(const hsg_rel *r) {
    int xcd = 1;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_XCD")) xcd = atoi(e);      // dev A/B
    return RelPtrs{r->n_src, r->n_dst, r->n_edges, r->indptr, r->src, r->tf, r->phantom,
                   r->cindptr, r->cdst, r->cperm, xcd, r->dwork ? r->n_dwork : 0, r->swork ? r->n_swork : 0,
                   r->dwork, r->swork};
}

template <int TAU_MODE>
__device__ __forceinline__ int tau_row(const RelPtrs &R, int e) {
    if constexpr (TAU_MODE == HSG_TAU_TABLE) return (int)R.tf[e];
    else return e;
}

// Work assignment.  WPN waves cooperate on one node: WPN = 1 -> a wave owns whole
// nodes (short edge segments, many nodes); WPN = 4 -> the block owns a node and
// wave w takes the w-th contiguous quarter of its segment (long segments, few
// nodes: the W2S destinations and S2W sources at config 2).  With WPN > 1 the node
// loop is block-uniform (it contains barriers) and partial results are combined
// through LDS in wave order (deterministic).
__device__ __forceinline__ void subrange(int beg, int end, int part, int wpn, int &eb, int &ee) {
    const int q = (end - beg + wpn - 1) / wpn;
    eb = min(end, beg + part * q);
    ee = min(end, eb + q);
}

// acc[i] += sum_j w[j][fh[i]] * X[rows[j], fo[i]] over the n staged edges of a
// chunk.  Rows are fetched GR at a time into registers before any is used, so a
// group's loads are in flight together; row indices past n are clamped and
// their weight is 0.  All loads are unconditional (no per-lane branches).
template <int NF>
__device__ __forceinline__ void gather_rows(const float *__restrict__ X, int HD, int n, const int *rows,
                                            const float *w, int H, const int (&fh)[NF], const int (&fo)[NF],
                                            float (&acc)[NF]) {
    // measured on the config-2 passes: grouping pays for narrow rows (NF <= 2);
    // for wide rows the extra registers cost more occupancy than they buy (two-row
    // groups in the S2W forward: 20.9 vs 18.4 us in-step, round 3)
    constexpr int GR = NF <= 2 ? 4 : 1;
    for (int j0 = 0; j0 < n; j0 += GR) {
        float xv[GR][NF];
#pragma unroll
        for (int q = 0; q < GR; ++q) {
            const float *xr = X + (size_t)rows[min(j0 + q, n - 1)] * HD;
#pragma unroll
            for (int i = 0; i < NF; ++i) xv[q][i] = xr[fo[i]];
        }
#pragma unroll
        for (int q = 0; q < GR; ++q) {
            const int j = j0 + q;
            if (j < n) {
#pragma unroll
                for (int i = 0; i < NF; ++i) acc[i] = fmaf(w[j * H + fh[i]], xv[q][i], acc[i]);
            }
        }
    }
}

// Merge of the pieces of long destinations (round 6).  The wave that merges a
// destination v (pieces first .. first + np - 1, in item order) combines their partials
// with v's phantoms -- exactly the online-softmax algebra of a whole destination: M =
// max(max_p m_p, 0 if c > 0), L = sum_p l_p e^(m_p - M) + c e^(-M), h = sum_p (l_p
// e^(m_p - M) / L) h_p, then elu(h) + origin and (m, l) = (M, L).  Lane = feature (flat
// mapping, as k_gat_fwd); the partials of kMergeBatch pieces are requested together (one
// round trip per batch).  Deterministic: the order is the items', whichever block merges.
// In the forward kernel the last piece block of v to arrive merges (in-kernel, below);
// the launch k_gat_fwd_merge (dev, HSG_PIECE_INLINE=0) does it as a second kernel.
constexpr int kMergeBatch = 8;

// the run of items with this code from `item` on (wave-wide: one ballot per 64 items)
__device__ __forceinline__ int piece_count(const int32_t *__restrict__ work, int n_work, int item, int code,
                                           int lane) {
    int np = 1;
    for (int base = item + 1;; base += 64) {
        const int j = base + lane;
        const unsigned long long same = __ballot(j < n_work && work[4 * j] == code);
        if (~same == 0ull) {
            np += 64;
            continue;
        }
        return np + __builtin_ctzll(~same);
    }
}

// block-cooperative: thread t takes features t, t + 256, ... one at a time (a loop,
// so the merge adds few registers to the kernels that call it in-kernel)
__device__ __forceinline__ void fwd_merge_block(const RelPtrs &R, int H, int D, const float *__restrict__ origin,
                                                const float *__restrict__ pws, int first, int np, int v,
                                                float *__restrict__ hout, float *__restrict__ out,
                                                float *__restrict__ mout, float *__restrict__ lout,
                                                __bf16 *__restrict__ out16 = nullptr, int ld16 = 0) {
    const int HD = H * D, W = HD + 2 * H;
    const float c = (float)R.phantom[v];
    const float *pw = pws + (size_t)first * W;
#pragma unroll 1
    for (int f = threadIdx.x; f < HD; f += blockDim.x) {
        const int k = f / D;
        // running max M, denominator L and weighted sum S of head k, batch by batch
        float M = c > 0.f ? 0.f : -INFINITY, L = c > 0.f ? c : 0.f, S = 0.f;     // c e^(0 - M), M = 0
#pragma unroll 1
        for (int p0 = 0; p0 < np; p0 += kMergeBatch) {
            float mv[kMergeBatch], lv[kMergeBatch], hv[kMergeBatch];
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j) {
                const int p = min(p0 + j, np - 1);      // clamped: weight 0 below
                mv[j] = pw[p * W + HD + k];
                lv[j] = pw[p * W + HD + H + k];
                hv[j] = pw[p * W + f];
            }
            float mb = M;
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j)
                if (p0 + j < np) mb = fmaxf(mb, mv[j]);
            const float sc = M == -INFINITY ? 0.f : __expf(M - mb);
            L *= sc;
            S *= sc;
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j) {
                if (p0 + j < np) {
                    const float w = lv[j] * __expf(mv[j] - mb);
                    L += w;
                    S = fmaf(w, hv[j], S);
                }
            }
            M = mb;
        }
        const float h = S / L;
        const size_t o = (size_t)v * HD + f;
        if (hout) hout[o] = h;
        if (origin) {
            const float xo = elu1(h) + origin[o];
            if (out16) out16[(size_t)v * ld16 + f] = (__bf16)xo;   // the bf16 x rows replace out
            else out[o] = xo;
        }
        if (f == k * D) {                                 // the head's first feature: its (m, l)
            mout[v * H + k] = M;
            lout[v * H + k] = L;
        }
    }
    if (out16)
        for (int f = HD + (int)threadIdx.x; f < ld16; f += blockDim.x) out16[(size_t)v * ld16 + f] = (__bf16)0.f;
}

// Piece hand-off (round 6): the partials are stored write-through (sc1: relaxed
// agent-scope atomic stores), every storing wave drains them (vmcnt(0)), the block
// meets at a barrier, and one lane adds to the node's arrival counter (relaxed, agent
// scope).  The block whose add completes a multiple of np merges, after an agent-scope
// acquire and a barrier (cdna_hip_programming.md §6 Guideline 16 R1: write-through
// stores + counter, the reducer reading them behind an acquire).  The counters start
// at 0 (hsg_rel_work) and every launch adds exactly np per node, so no reset is needed.
__device__ __forceinline__ void st_sc1(float *p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0 of the block: arrive; returns (block-wide, through *flag) whether it merges
__device__ __forceinline__ bool piece_arrive(int32_t *cnt, int np, int *flag) {
    __syncthreads();                                      // every wave's stores drained (vmcnt(0) before)
    if (threadIdx.x == 0) {
        const int old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = old % np == np - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        *flag = last;
    }
    __syncthreads();
    return *flag != 0;
}

// ---------------------------------------------------------------- forward ----
// PF (one destination per wave only): the next destination's indptr / phantom are
// requested one iteration ahead (vector loads, consumed by readfirstlane), and the
// residual row is requested before the score phase.  PF = 2 (round 4, the default): also
// the next destination's first lph edges -- (source, box) requested after this
// destination's score phase, their (sigma, tau) after its gather, before its stores
// (vmcnt retires in issue order: the next score phase then waits for neither the
// stores nor the next residual row) -- so its score phase starts with the scores.
// O16 (round 6, the bf16 GEMM mode's bf16 x rows): elu(h) + origin is stored as bf16
// rows of pitch ld16 (>= ceil8(H*D), pad columns zero) INSTEAD of the fp32 out -- the
// wide FFN's A operand, LayerNorm residual and dW1 operand (a template flag: the fp32
// kernels keep their registers)
template <int NF, int TAU_MODE, int WPN, int OCC = 1, int PF = 0, bool WL = false, bool O16 = false>
__global__ __launch_bounds__(256, OCC) void k_gat_fwd(RelPtrs R, int H, int D, int lph, float slope,
                                                const float *__restrict__ Z,
                                                const float *__restrict__ sigma,
                                                const float *__restrict__ tau,
                                                const float *__restrict__ origin,
                                                float *__restrict__ hout, float *__restrict__ out,
                                                float *__restrict__ mout, float *__restrict__ lout,
                                                float *__restrict__ pws, int pinline,
                                                __bf16 *__restrict__ out16, int ld16) {
    constexpr int NPB = HSG_WAVES / WPN;
    __shared__ int s_flag[1];
    __shared__ float s_alpha[HSG_WAVES][HSG_CHUNK * HSG_HMAX];
    __shared__ int s_nb[HSG_WAVES][HSG_CHUNK];
    __shared__ float s_ml[HSG_WAVES][2 * HSG_HMAX];
    __shared__ float s_acc[WPN > 1 ? HSG_WAVES : 1][WPN > 1 ? 64 * NF : 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    const int part = wid % WPN, w0 = wid - part;
    const bool writer = part == 0;
    // fh: head of feature f; fo: f clamped into the row, so every gather load is
    // unconditional (lanes past H*D compute values that are never stored) and the
    // compiler can keep a chunk's loads in flight together
    int fh[NF], fo[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int f = lane + 64 * i;
        fh[i] = f < HD ? div_small(f, 1.f / (float)D) : 0;
        fo[i] = f < HD ? f : HD - 1;
    }
    float *sa = s_alpha[wid];
    int *sn = s_nb[wid];

    static_assert(PF == 0 || WPN == 1, "prefetch: one destination per wave");
    // round 6: with the relation's CSR work list (and the piece scratch pws) the loop
    // walks its items -- whole destinations, and pieces of the long ones, whose (max,
    // sum, partial h) go to pws for k_gat_fwd_merge (multi-wave form only)
    // (WL: a template flag, so the kernel without a list keeps its registers)
    constexpr bool wl = WL && WPN > 1;
    const WorkRange wr = work_range(wl ? R.n_dwork : R.n_dst, NPB, wid / WPN, R.xcd);
    const int vstride = wr.stride;
    int pf_beg = 0, pf_end = 0, pf_c = 0;
    int pu = 0, pt = 0;                                   // PF = 2: next destination, edge l
    float psg = 0.f, ptu = 0.f;
    bool pok = false;
    if constexpr (PF) {
        const int v0 = wr.first;
        if (v0 < wr.end) { pf_beg = R.indptr[v0]; pf_end = R.indptr[v0 + 1]; pf_c = R.phantom[v0]; }
    }
    // PF = 2: the scores of edge l of the next destination (pok: it exists)
    auto pf_edges = [&](int nb, int ne) {
        pok = kact && nb + l < ne;
        if (pok) {
            pu = R.src[nb + l];
            pt = tau_row<TAU_MODE>(R, nb + l);
        }
    };
    auto pf_scores = [&]() {
        if (pok) {
            psg = sigma[pu * H + k];
            ptu = tau[pt * H + k];
        }
    };
    float org_next[PF == 3 ? NF : 1];                     // PF = 3: the next destination's residual row
    if constexpr (PF >= 2) {
        if (wr.first < wr.end) {
            pf_edges(__builtin_amdgcn_readfirstlane(pf_beg), __builtin_amdgcn_readfirstlane(pf_end));
            pf_scores();
            if constexpr (PF == 3) {
                const int v0 = __builtin_amdgcn_readfirstlane(wr.first);
#pragma unroll
                for (int i = 0; i < NF; ++i) org_next[i] = origin ? origin[(size_t)v0 * HD + fo[i]] : 0.f;
            }
        }
    }
    for (int v_ = wr.first; v_ < wr.end; v_ += vstride) {
        const int item = __builtin_amdgcn_readfirstlane(v_);   // scalar loads of indptr / phantom
        int v = item;
        bool piece = false;
        int beg, end, c;
        float org[NF];
        if constexpr (PF) {
            beg = __builtin_amdgcn_readfirstlane(pf_beg);
            end = __builtin_amdgcn_readfirstlane(pf_end);
            c = __builtin_amdgcn_readfirstlane(pf_c);
            // the residual row first: measured 17.3 us against 18.5 us with the row
            // requested after the score loads (cfg2 S2W, in-step), although vmcnt counts
            // in issue order and the score chain then also waits for this HBM row
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                if constexpr (PF == 3) org[i] = org_next[i];
                else org[i] = origin ? origin[(size_t)v * HD + fo[i]] : 0.f;
            }
            const int vn = v_ + vstride;
            if (vn < wr.end) { pf_beg = R.indptr[vn]; pf_end = R.indptr[vn + 1]; pf_c = R.phantom[vn]; }
        } else if (wl) {
            const int code = R.dwork[4 * item];
            beg = R.dwork[4 * item + 1];
            end = R.dwork[4 * item + 2];
            piece = code < 0;
            v = piece ? -code - 1 : code;
            c = piece ? 0 : R.phantom[v];                      // a piece's phantoms: in the merge
        } else {
            beg = R.indptr[v];
            end = R.indptr[v + 1];
            c = R.phantom[v];
        }
        int eb, ee;
        subrange(beg, end, part, WPN, eb, ee);
        const int n1 = ee - eb;
        const bool single = n1 <= HSG_CHUNK;      // scores stay in LDS between the phases
        // phase 1: online (max, sum) of this head's scores over edges j = l (mod lph)
        float mx = -INFINITY, sm = 0.f;
        if (kact) {
            for (int j = l; j < n1; j += lph) {
                const int e = eb + j;
                int u;
                float s;
                if (PF >= 2 && j == l && pok) {            // prefetched last iteration
                    u = pu;
                    s = leaky(psg + ptu, slope);
                } else {
                    u = R.src[e];
                    s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                }
                if (single) {
                    sa[j * H + k] = s;
                    if (k == 0) sn[j] = u;
                }
                if (s > mx) { sm = sm * __expf(mx - s) + 1.f; mx = s; }
                else sm += __expf(s - mx);
            }
        }
        for (int o = lph >> 1; o >= 1; o >>= 1) {
            const float om = __shfl_xor(mx, o), os = __shfl_xor(sm, o);
            lse_merge(mx, sm, om, os);
        }
        if constexpr (WPN > 1) {
            if (kact && l == 0) { s_ml[wid][k] = mx; s_ml[wid][HSG_HMAX + k] = sm; }
            __syncthreads();
            mx = -INFINITY;
            sm = 0.f;
            if (kact) {
#pragma unroll
                for (int p = 0; p < WPN; ++p) lse_merge(mx, sm, s_ml[w0 + p][k], s_ml[w0 + p][HSG_HMAX + k]);
            }
        }
        if (c > 0) lse_merge(mx, sm, 0.f, (float)c);     // phantom in-edges: e = 0
        if constexpr (PF >= 2) {                          // the next destination's (src, box)
            if (v_ + vstride < wr.end)
                pf_edges(__builtin_amdgcn_readfirstlane(pf_beg), __builtin_amdgcn_readfirstlane(pf_end));
            else
                pok = false;
        }
        const bool any = end > beg;
        const float inv = any ? 1.f / sm : 0.f;
        // the residual row: independent of the gathers below
        if constexpr (PF == 0) {
#pragma unroll
            for (int i = 0; i < NF; ++i) org[i] = (origin && writer && !piece) ? origin[(size_t)v * HD + fo[i]] : 0.f;
        }

        // PF = 3: the next destination's (sigma, tau) and residual row, requested once
        bool issued = false;
        auto pf3_next = [&]() {
            if constexpr (PF == 3) {
                const int vn = v_ + vstride;
                if (vn < wr.end) {
                    pf_scores();
                    const int vs = __builtin_amdgcn_readfirstlane(vn);
#pragma unroll
                    for (int i = 0; i < NF; ++i) org_next[i] = origin ? origin[(size_t)vs * HD + fo[i]] : 0.f;
                }
            }
        };
        // phase 2: alphas per 64-edge chunk, then flat-mapped aggregation
        float acc[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i] = 0.f;
        for (int cb = eb; cb < ee; cb += HSG_CHUNK) {
            const int n = min(HSG_CHUNK, ee - cb);
            if (kact) {
                for (int j = l; j < n; j += lph) {
                    float s;
                    if (single) {
                        s = sa[j * H + k];                 // written by this same lane
                    } else {
                        const int e = cb + j;
                        const int u = R.src[e];
                        s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                        if (k == 0) sn[j] = u;
                    }
                    sa[j * H + k] = __expf(s - mx) * inv;
                }
            }
            wave_lds_sync();
            if constexpr (PF == 3) {
                // after the first row's loads the next destination's (sigma, tau) and
                // residual row are requested, so (vmcnt in issue order) the FMAs wait for
                // the L2 rows only and the next destination's HBM residual row has a whole
                // iteration to arrive
                for (int j = 0; j < n; ++j) {
                    float xv[NF];
                    const float *xr = Z + (size_t)sn[j] * HD;
#pragma unroll
                    for (int i = 0; i < NF; ++i) xv[i] = xr[fo[i]];
                    if (!issued) {
                        issued = true;
                        pf3_next();
                    }
#pragma unroll
                    for (int i = 0; i < NF; ++i) acc[i] = fmaf(sa[j * H + fh[i]], xv[i], acc[i]);
                }
            } else {
                gather_rows<NF>(Z, HD, n, sn, sa, H, fh, fo, acc);
            }
            wave_lds_sync();
        }
        if constexpr (PF == 3) {
            if (!issued) pf3_next();                        // no edges
        }
        if constexpr (WPN > 1) {
#pragma unroll
            for (int i = 0; i < NF; ++i) s_acc[wid][lane + 64 * i] = acc[i];
            __syncthreads();
            if (writer) {
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int p = 0; p < WPN; ++p) a += s_acc[w0 + p][lane + 64 * i];
                    acc[i] = a;
                }
            }
        }
        if constexpr (PF == 2) pf_scores();              // ... and its (sigma, tau), before the stores
        // epilogue: h, and elu(h) + origin (GAT.py:56-57); a piece: its partial h (normalised
        // by its own sum), max and sum, [HD | H | H] per item
        if (writer && piece) {
            float *pw = pws + (size_t)item * (HD + 2 * H);
            if (pinline) {                                // write-through: the hand-off below
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const int f = lane + 64 * i;
                    if (f < HD) st_sc1(&pw[f], acc[i]);
                }
                if (kact && l == 0) {
                    st_sc1(&pw[HD + k], mx);
                    st_sc1(&pw[HD + H + k], sm);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            } else {
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const int f = lane + 64 * i;
                    if (f < HD) pw[f] = acc[i];
                }
                if (kact && l == 0) {
                    pw[HD + k] = mx;
                    pw[HD + H + k] = sm;
                }
            }
        } else if (writer) {
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                const int f = lane + 64 * i;
                if (f < HD) {
                    const size_t o = (size_t)v * HD + f;
                    const float hv = acc[i];
                    if (hout) hout[o] = hv;
                    if (origin) {
                        const float xo = elu1(hv) + org[i];
                        if constexpr (O16) out16[(size_t)v * ld16 + f] = (__bf16)xo;
                        else out[o] = xo;
                    }
                } else if (O16 && f < ld16) {             // the zero pad columns
                    out16[(size_t)v * ld16 + f] = (__bf16)0.f;
                }
            }
            if (kact && l == 0) {
                mout[v * H + k] = any ? mx : 0.f;
                lout[v * H + k] = any ? sm : 1.f;
            }
        }
        if constexpr (WPN > 1) {
            // a piece, merged in-kernel (round 6): the last of v's pieces to arrive merges
            // them (wave 0); item, piece and the node are block-uniform here
            if (wl && piece && pinline) {
                const int first = R.dwork[4 * item + 3];
                const int np = __builtin_amdgcn_readfirstlane(piece_count(R.dwork, R.n_dwork, first,
                                                                          R.dwork[4 * first], lane));
                if (piece_arrive(R.dwork + 4 * R.n_dwork + first, np, &s_flag[0]))
                    fwd_merge_block(R, H, D, origin, pws, first, np, v, hout, out, mout, lout,
                                    O16 ? out16 : nullptr, ld16);
            }
            __syncthreads();                              // s_ml / s_acc / s_flag are reused
        }
    }
}

__global__ __launch_bounds__(256) void k_gat_fwd_merge(RelPtrs R, int H, int D, const float *__restrict__ origin,
                                                       const float *__restrict__ pws, float *__restrict__ hout,
                                                       float *__restrict__ out, float *__restrict__ mout,
                                                       float *__restrict__ lout, __bf16 *__restrict__ out16,
                                                       int ld16) {
    const int item = (int)blockIdx.x;                     // one block per item (dev: HSG_PIECE_INLINE=0)
    const int code = R.dwork[4 * item];
    if (code >= 0 || R.dwork[4 * item + 3] != item) return;   // not a first piece
    __shared__ int s_np;
    if (threadIdx.x < 64) {
        const int np = piece_count(R.dwork, R.n_dwork, item, code, (int)threadIdx.x);
        if (threadIdx.x == 0) s_np = np;
    }
    __syncthreads();
    fwd_merge_block(R, H, D, origin, pws, item, s_np, -code - 1, hout, out, mout, lout, out16, ld16);
}

#ifdef HSG_DEV
// ---------------------------------------------------- forward, destination tiles ----
// (round 6, dev: measured slower -- 24.1 / 27.7 us with 48- / 24-destination tiles
// against 16.3 us for k_gat_fwd on the cfg2 S2W pass) The short-segment
// forward (one destination per wave, the S2W words: ~2
// sentence edges each) by tiles of kTileW consecutive destinations per block.  The
// block first stages everything its destinations' edges will read -- their indptr
// range, the (source, box) of every edge, and the source rows Z and logits sigma of
// the window [s0, s0 + kTileZ) around the smallest source the tile touches (documents
// are contiguous in node order, so one document's sentences cover a tile) -- with
// coalesced loads, then its 8 waves walk the tile's destinations reading scores and
// gathered rows from LDS: the per-destination chain has no dependent global load
// left (the residual row is requested one destination ahead).  Sources outside the
// window and edges past kTileE are read from global memory (flat pointers), so any
// graph is covered.  Per destination the arithmetic is k_gat_fwd's (WPN = 1): the same
// score order, online (max, sum) merge and gather order -- bitwise equal results.
// blocks b run on XCD b % 8: XCD x takes the contiguous run x of the tiles (a bijection)
__device__ __forceinline__ int xcd_run(int b, int total) {
    const int x = b & 7, j = b >> 3, per = total >> 3, rem = total & 7;
    return x * per + min(x, rem) + j;
}

constexpr int kTileW = 48;                 // destinations per block
constexpr int kTileZ = 48;                 // staged source rows
constexpr int kTileE = 512;                // staged edges
constexpr int kTileCh = 16;                // edges per score / gather chunk
constexpr int kTileWaves = 8;

template <int NF, int TAU_MODE, bool O16 = false, int TW = kTileW>
__global__ __launch_bounds__(512, 4) void k_gat_fwd_tile(RelPtrs R, int H, int D, int lph, float slope,
                                                         const float *__restrict__ Z,
                                                         const float *__restrict__ sigma,
                                                         const float *__restrict__ tau,
                                                         const float *__restrict__ origin,
                                                         float *__restrict__ hout, float *__restrict__ out,
                                                         float *__restrict__ mout, float *__restrict__ lout,
                                                         __bf16 *__restrict__ out16, int ld16, int ntiles) {
    constexpr int HDP = 64 * NF;           // staged row pitch (floats)
    __shared__ __attribute__((aligned(16))) float sZ[kTileZ * HDP];
    __shared__ float sSig[kTileZ * HSG_HMAX];
    __shared__ int sSrc[kTileE];
    __shared__ int sTau[kTileE];
    __shared__ int sPtr[TW + 1];
    __shared__ float s_alpha[kTileWaves][kTileCh * HSG_HMAX];
    __shared__ int s_nb[kTileWaves][kTileCh];
    __shared__ int s_min[kTileWaves];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int t = xcd_run((int)blockIdx.x, ntiles);       // XCD-local runs of tiles
    const int v0 = t * TW, v1 = min(R.n_dst, v0 + TW), nv = v1 - v0;
    // 1. the tile's indptr range, then its edges' (source, box) and the source window
    for (int i = threadIdx.x; i <= nv; i += blockDim.x) sPtr[i] = R.indptr[v0 + i];
    __syncthreads();
    const int e0 = sPtr[0], ne = sPtr[nv] - e0, nes = min(ne, kTileE);
    int mn = 0x7fffffff;
    for (int i = threadIdx.x; i < nes; i += blockDim.x) {
        const int u = R.src[e0 + i];
        sSrc[i] = u;
        sTau[i] = tau_row<TAU_MODE>(R, e0 + i);
        mn = min(mn, u);
    }
    for (int o = 32; o >= 1; o >>= 1) mn = min(mn, __shfl_xor(mn, o));
    if (lane == 0) s_min[wid] = mn;
    __syncthreads();
    int s0 = s_min[0];
#pragma unroll
    for (int w = 1; w < kTileWaves; ++w) s0 = min(s0, s_min[w]);
    if (nes == 0) s0 = 0;
    const int nz = nes > 0 ? min(kTileZ, R.n_src - s0) : 0;  // window rows [s0, s0 + nz)
    if (HD % 4 == 0) {
        const int q = HD / 4;                                  // float4 quads per row
        for (int i = threadIdx.x; i < nz * q; i += blockDim.x) {
            const int r = i / q, c = (i - r * q) * 4;
            *reinterpret_cast<float4 *>(&sZ[r * HDP + c]) =
                *reinterpret_cast<const float4 *>(Z + (size_t)(s0 + r) * HD + c);
        }
    } else {
        for (int i = threadIdx.x; i < nz * HD; i += blockDim.x) {
            const int r = i / HD, c = i - r * HD;
            sZ[r * HDP + c] = Z[(size_t)(s0 + r) * HD + c];
        }
    }
    for (int i = threadIdx.x; i < nz * H; i += blockDim.x) sSig[i] = sigma[(size_t)s0 * H + i];
    __syncthreads();

    // 2. the destinations, one per wave at a time
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    int fh[NF], fo[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int f = lane + 64 * i;
        fh[i] = f < HD ? div_small(f, 1.f / (float)D) : 0;
        fo[i] = f < HD ? f : HD - 1;
    }
    float *sa = s_alpha[wid];
    int *sn = s_nb[wid];
    // a source row / logit: from the window when staged, else from global memory
    auto zrow = [&](int u) -> const float * {
        return (unsigned)(u - s0) < (unsigned)nz ? &sZ[(u - s0) * HDP] : Z + (size_t)u * HD;
    };
    auto sig = [&](int u, int kk) -> float {
        return (unsigned)(u - s0) < (unsigned)nz ? sSig[(u - s0) * H + kk] : sigma[(size_t)u * H + kk];
    };
    auto edge = [&](int e, int &u, int &tr) {               // e relative to e0
        if (e < kTileE) { u = sSrc[e]; tr = sTau[e]; }
        else { u = R.src[e0 + e]; tr = tau_row<TAU_MODE>(R, e0 + e); }
    };
    float orgn[NF];
    int vv = v0 + wid;
    if (origin && vv < v1) {
#pragma unroll
        for (int i = 0; i < NF; ++i) orgn[i] = origin[(size_t)vv * HD + fo[i]];
    }
    for (; vv < v1; vv += kTileWaves) {
        const int v = __builtin_amdgcn_readfirstlane(vv);
        const int beg = sPtr[v - v0] - e0, end = sPtr[v - v0 + 1] - e0;
        const int c = R.phantom[v];
        float org[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) org[i] = orgn[i];
        const int vn = v + kTileWaves;                       // the next destination's residual row
        if (origin && vn < v1) {
#pragma unroll
            for (int i = 0; i < NF; ++i) orgn[i] = origin[(size_t)vn * HD + fo[i]];
        }
        const int n1 = end - beg;
        const bool single = n1 <= kTileCh;
        float mx = -INFINITY, sm = 0.f;
        if (kact) {
            for (int j = l; j < n1; j += lph) {
                int u, tr;
                edge(beg + j, u, tr);
                const float s = leaky(sig(u, k) + tau[tr * H + k], slope);
                if (single) {
                    sa[j * H + k] = s;
                    if (k == 0) sn[j] = u;
                }
                if (s > mx) { sm = sm * __expf(mx - s) + 1.f; mx = s; }
                else sm += __expf(s - mx);
            }
        }
        for (int o = lph >> 1; o >= 1; o >>= 1) {
            const float om = __shfl_xor(mx, o), os = __shfl_xor(sm, o);
            lse_merge(mx, sm, om, os);
        }
        if (c > 0) lse_merge(mx, sm, 0.f, (float)c);
        const bool any = end > beg;
        const float inv = any ? 1.f / sm : 0.f;
        float acc[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i] = 0.f;
        for (int cb = 0; cb < n1; cb += kTileCh) {
            const int n = min(kTileCh, n1 - cb);
            if (kact) {
                for (int j = l; j < n; j += lph) {
                    float s;
                    if (single) {
                        s = sa[j * H + k];
                    } else {
                        int u, tr;
                        edge(beg + cb + j, u, tr);
                        s = leaky(sig(u, k) + tau[tr * H + k], slope);
                        if (k == 0) sn[j] = u;
                    }
                    sa[j * H + k] = __expf(s - mx) * inv;
                }
            }
            wave_lds_sync();
            for (int j = 0; j < n; ++j) {
                const float *xr = zrow(sn[j]);
                float xv[NF];
#pragma unroll
                for (int i = 0; i < NF; ++i) xv[i] = xr[fo[i]];
#pragma unroll
                for (int i = 0; i < NF; ++i) acc[i] = fmaf(sa[j * H + fh[i]], xv[i], acc[i]);
            }
            wave_lds_sync();
        }
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int f = lane + 64 * i;
            if (f < HD) {
                const size_t o = (size_t)v * HD + f;
                const float hv = acc[i];
                if (hout) hout[o] = hv;
                if (origin) {
                    const float xo = elu1(hv) + org[i];
                    if constexpr (O16) out16[(size_t)v * ld16 + f] = (__bf16)xo;
                    else out[o] = xo;
                }
            } else if (O16 && f < ld16) {
                out16[(size_t)v * ld16 + f] = (__bf16)0.f;
            }
        }
        if (kact && l == 0) {
            mout[v * H + k] = any ? mx : 0.f;
            lout[v * H + k] = any ? sm : 1.f;
        }
    }
}

// Launch floor probe (dev, round 6): the same grid as the edge launch
// it replaces, every wave reads its first index word and stores nothing, so the step
// trace shows what dispatch, ramp and drain of that grid cost in the step.
__global__ __launch_bounds__(256) void k_launch_floor(const int32_t *__restrict__ p, int n, int32_t *__restrict__ sink) {
    const int i = (int)blockIdx.x;
    if (i < n && p[i] == -0x7fffffff && sink) sink[0] = i;      // never true: no store
}
int launch_floor_mode() {
    const char *e = HSG_DEV_ENV("HSG_GAT_FLOOR");               // 1: W2S forward, 2: W2S backward
    return e ? atoi(e) : 0;
}
#endif

// ------------------------------------------------ forward, single pass (round 5) ----
// Narrow rows (H * D <= 64: the W2S sentence destinations, ~36 word in-edges each at
// cfg2).  k_gat_fwd runs a destination as two phases -- the scores' online (max, sum)
// over the lanes of each head, merged across the block's 4 waves through LDS and a
// barrier, then the alphas staged in LDS and the Z rows gathered -- i.e. four dependent
// memory round trips and two block barriers per destination.  Here one wave owns a
// destination and lane f its feature f (head f / D) end to end: lane j loads edge j's
// (source, box) for up to 64 edges at once; then per sub-batch of EB edges every lane
// requests, for each edge (source and box broadcast by readlane into SGPRs), its head's
// sigma and its Z feature by buffer loads (scalar row offset, per-lane feature offset:
// no address VALU) and reads tau from the block's LDS copy of the table.  The loads
// are unconditional (edges past the segment repeat the last one, weight 0) so a
// sub-batch's 2 EB loads issue back to back, and the next sub-batch's loads are issued
// before this one's arithmetic.  The softmax is online per lane over the sub-batch (one
// rescale per sub-batch), h = sum_e p_e Z_u / l: no alpha staging, no cross-lane
// reduction.  Same numbers as k_gat_fwd up to fp32 summation order; m, l as it writes.
// Measured (dev, HSG_GAT_FWD_SP=16 | 8): 25.5 / 30.4 us per cfg2 W2S launch against 7.9
// us for k_gat_fwd's four waves per destination -- 1,120 destinations are ~one wave per
// SIMD here, so each wave's whole issue stream (readlanes, 2 loads and ~10 VALU per edge)
// and its round trips are exposed; the first round-5 form (a per-edge branch that made
// every edge wait for its own loads) ran 16-17 us.  Dev only.
template <int TAU_MODE, int EB>
__global__ __launch_bounds__(256) void k_gat_fwd_sp(RelPtrs R, int H, int D, float slope,
                                                    const float *__restrict__ Z,
                                                    const float *__restrict__ sigma,
                                                    const float *__restrict__ tau,
                                                    const float *__restrict__ origin,
                                                    float *__restrict__ hout, float *__restrict__ out,
                                                    float *__restrict__ mout, float *__restrict__ lout) {
    static_assert(TAU_MODE == HSG_TAU_TABLE, "the tau table staged in LDS");
    __shared__ float s_tau[HSG_NT * HSG_HMAX];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const bool fok = lane < HD;
    const int f = fok ? lane : HD - 1;
    const int kf = div_small(f, 1.f / (float)D);
    for (int i = threadIdx.x; i < HSG_NT * H; i += blockDim.x) s_tau[i] = tau[i];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t zr = buf_rsrc(Z, (long)R.n_src * HD * 4);
    const __amdgpu_buffer_rsrc_t sr = buf_rsrc(sigma, (long)R.n_src * H * 4);
    const unsigned fb = 4u * (unsigned)f, kb = 4u * (unsigned)kf;
    const WorkRange wr = work_range(R.n_dst, HSG_WAVES, wid, R.xcd);
    for (int v_ = wr.first; v_ < wr.end; v_ += wr.stride) {
        const int v = __builtin_amdgcn_readfirstlane(v_);
        const int beg = R.indptr[v], end = R.indptr[v + 1], c = R.phantom[v];
        const float org = origin ? origin[(size_t)v * HD + f] : 0.f;
        float m = -INFINITY, l = 0.f, acc = 0.f;
        for (int e0 = beg; e0 < end; e0 += 64) {
            const int nb = min(64, end - e0);
            const int ej = e0 + min(lane, nb - 1);              // lanes past the chunk repeat its last edge
            const int uj = R.src[ej], tj = tau_row<TAU_MODE>(R, ej);
            float sg[2][EB], zz[2][EB];
            int tt[2][EB];
            auto issue = [&](int b, float (&sgb)[EB], float (&zzb)[EB], int (&ttb)[EB]) {
#pragma unroll
                for (int j = 0; j < EB; ++j) {
                    const int jj = min(b * EB + j, 63);
                    const int u = __builtin_amdgcn_readlane(uj, jj);
                    ttb[j] = __builtin_amdgcn_readlane(tj, jj);
                    sgb[j] = buf_ld(sr, kb, (unsigned)u * H * 4u);
                    zzb[j] = buf_ld(zr, fb, (unsigned)u * HD * 4u);
                }
            };
            const int nsb = (nb + EB - 1) / EB;
            issue(0, sg[0], zz[0], tt[0]);
            for (int b = 0; b < nsb; ++b) {
                const int cur = b & 1;
                if (b + 1 < nsb) {
                    if (cur == 0) issue(b + 1, sg[1], zz[1], tt[1]);
                    else issue(b + 1, sg[0], zz[0], tt[0]);
                }
                float sc[EB];
                float bm = m;
#pragma unroll
                for (int j = 0; j < EB; ++j) {
                    const bool ok = b * EB + j < nb;                 // wave-uniform
                    const float x = leaky((cur ? sg[1][j] : sg[0][j]) + s_tau[(cur ? tt[1][j] : tt[0][j]) * H + kf],
                                          slope);
                    sc[j] = ok ? x : -INFINITY;
                    bm = fmaxf(bm, sc[j]);
                }
                const float r = __expf(m - bm);                      // m = -inf on the first batch: 0
                acc *= r;
                l *= r;
#pragma unroll
                for (int j = 0; j < EB; ++j) {
                    const float pj = __expf(sc[j] - bm);             // 0 past the segment
                    l += pj;
                    acc = fmaf(pj, cur ? zz[1][j] : zz[0][j], acc);
                }
                m = bm;
            }
        }
        if (c > 0) {                                             // phantom in-edges: e = 0, no message
            const float bm = fmaxf(m, 0.f), r = __expf(m - bm);
            acc *= r;
            l = l * r + (float)c * __expf(-bm);
            m = bm;
        }
        const bool any = end > beg;
        const float hv = any ? acc / l : 0.f;
        if (fok) {
            const size_t o = (size_t)v * HD + f;
            if (hout) hout[o] = hv;
            if (origin) out[o] = elu1(hv) + org;
        }
        if (fok && f - kf * D == 0) {
            mout[v * H + kf] = any ? m : 0.f;
            lout[v * H + kf] = any ? l : 1.f;
        }
    }
}

// ---------------------------------------- forward, destination batches (round 5) ----
// Short segments, wide rows (S2W at cfg2: ~2.1 in-edges per word, H*D = 300).
// k_gat_fwd spends a wave on one destination: its (k, l) score lanes are mostly idle
// at two edges, and the per-destination fixed work -- the butterfly (max, sum) merge,
// one precise division per lane, the 64-bit address arithmetic of every gathered
// row -- made it VALU-issue-heavy (SQ_INSTS_VALU 753 per wave, ~281 per destination;
// the VALU was busy ~60 % of the kernel).  Here a wave takes a batch of up to DB
// consecutive destinations whose edges fit one LDS chunk (CH edges; a destination
// with more edges runs alone over several chunks):
//   stage:   lane q loads edge q's (source, box) (one coalesced load of the batch's
//            contiguous CSR range), then lanes p = (q, k) over all (edge, head) pairs
//            load (sigma, tau) -> scores in LDS, pairs two at a time in flight;
//   softmax: lane (d, k) walks destination d's scores of head k serially (online
//            max / sum, no cross-lane merge), folds the phantom edges, writes m / l
//            (coalesced over the batch) and turns its scores into alphas in place;
//   gather:  per destination (wave-uniform loop) the source rows are scalar bases
//            (readfirstlane of the staged index), so every row load is saddr + a
//            per-lane feature offset, two rows in flight, alphas from LDS; then
//            elu(h) + origin (the residual row requested with the rows).
// Chain per batch: indptr -> (src, box) -> (sigma, tau) -> rows -> stores.  Same
// arithmetic as k_gat_fwd (alpha = exp(s - m) / l, gathers in CSR order) up to the
// summation order of (m, l).
template <int NF, int TAU_MODE, int DB>
__global__ __launch_bounds__(256, 7) void k_gat_fwd_b(RelPtrs R, int H, int D, float slope,
                                                      const float *__restrict__ Z,
                                                      const float *__restrict__ sigma,
                                                      const float *__restrict__ tau,
                                                      const float *__restrict__ origin,
                                                      float *__restrict__ hout, float *__restrict__ out,
                                                      float *__restrict__ mout, float *__restrict__ lout) {
    constexpr int CH = HSG_CHUNK;
    __shared__ float s_sc[HSG_WAVES][CH * HSG_HMAX];    // scores, then alphas: [edge][head]
    __shared__ int s_u[HSG_WAVES][CH];                  // staged source rows
    __shared__ int s_t[HSG_WAVES][CH];                  // staged tau rows
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const float invH = 1.f / (float)H;
    // byte offset of feature f (clamped into the row) and its head.  Rows are read and
    // written by buffer instructions: scalar row offset (soffset) + this per-lane byte
    // offset, so a row access costs no VALU address arithmetic
    unsigned fb[NF];
    int fa[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int f = lane + 64 * i;
        fb[i] = 4u * (unsigned)(f < HD ? f : HD - 1);
        fa[i] = f < HD ? div_small(f, 1.f / (float)D) : 0;
    }
    const unsigned rowb = 4u * (unsigned)HD;
    const __amdgpu_buffer_rsrc_t zr = buf_rsrc(Z, (long)R.n_src * rowb);
    const __amdgpu_buffer_rsrc_t orr = buf_rsrc(origin, origin ? (long)R.n_dst * rowb : 0);
    const __amdgpu_buffer_rsrc_t outr = buf_rsrc(out, origin ? (long)R.n_dst * rowb : 0);
    const __amdgpu_buffer_rsrc_t hr = buf_rsrc(hout, hout ? (long)R.n_dst * rowb : 0);
    const int ndmax = min(DB, 64 / H);
    const int sd = div_small(lane, invH), sk = lane - sd * H;    // softmax lane: (destination, head)
    float *sc = s_sc[wid];
    int *su = s_u[wid], *st = s_t[wid];

    // scores of the chunk's edges [cb, cb + n) into sc[q * H + k]
    auto stage = [&](int cb, int n) {
        if (lane < n) {
            su[lane] = R.src[cb + lane];
            st[lane] = tau_row<TAU_MODE>(R, cb + lane);
        }
        wave_lds_sync();
        const int np = n * H;
        for (int p0 = 0; p0 < np; p0 += 128) {
            const int pa = min(p0 + lane, np - 1), pb = min(p0 + 64 + lane, np - 1);
            const int qa = div_small(pa, invH), qb = div_small(pb, invH);
            const int ka = pa - qa * H, kb = pb - qb * H;
            const float xa = sigma[su[qa] * H + ka] + tau[st[qa] * H + ka];
            const float xb = sigma[su[qb] * H + kb] + tau[st[qb] * H + kb];
            if (p0 + lane < np) sc[pa] = leaky(xa, slope);
            if (p0 + 64 + lane < np) sc[pb] = leaky(xb, slope);
        }
        wave_lds_sync();
    };

    const int nbat = (R.n_dst + DB - 1) / DB;
    const WorkRange wr = work_range(nbat, HSG_WAVES, wid, R.xcd);
    for (int b = wr.first; b < wr.end; b += wr.stride) {
        int v = __builtin_amdgcn_readfirstlane(b * DB);
        const int bend = min(R.n_dst, v + DB);
        while (v < bend) {
            const int rem = min(bend - v, ndmax);
            const int ip = R.indptr[v + min(lane, rem)];
            const int beg0 = __builtin_amdgcn_readlane(ip, 0);
            // destinations [v, v + nd) whose edges fit one chunk (ip is monotone: a prefix)
            const bool fit = lane >= 1 && lane <= rem && ip - beg0 <= CH;
            int nd = __builtin_popcountll(__ballot(fit));
            nd = __builtin_amdgcn_readfirstlane(nd > 0 ? nd : 1);
            const int endB = __builtin_amdgcn_readlane(ip, nd);
            const bool multi = endB - beg0 > CH;        // one destination over several chunks
            const bool sact = lane < nd * H;
            const int dbeg = __shfl(ip, sd), dend = __shfl(ip, sd + 1);
            const int c = sact ? R.phantom[v + sd] : 0;

            // softmax state of (destination sd, head sk)
            float mx = -INFINITY, sm = 0.f;
            for (int cb = beg0; cb < endB; cb += CH) {
                const int n = min(CH, endB - cb);
                stage(cb, n);
                if (sact) {
                    const int e1 = min(dend, cb + n);
                    for (int e = max(dbeg, cb); e < e1; ++e) {
                        const float s = sc[(e - cb) * H + sk];
                        if (s > mx) { sm = sm * __expf(mx - s) + 1.f; mx = s; }
                        else sm += __expf(s - mx);
                    }
                }
                wave_lds_sync();
            }
            if (c > 0) lse_merge(mx, sm, 0.f, (float)c);     // phantom in-edges: e = 0
            const bool any = dend > dbeg;
            const float inv = any ? 1.f / sm : 0.f;
            if (sact) {
                mout[(v + sd) * H + sk] = any ? mx : 0.f;
                lout[(v + sd) * H + sk] = any ? sm : 1.f;
            }

            float acc[NF];
#pragma unroll
            for (int i = 0; i < NF; ++i) acc[i] = 0.f;
            int d = 0;
            int cb = beg0;
            do {                                   // at least once: a batch may have no edges
                const int n = min(CH, endB - cb);
                if (multi) stage(cb, n);
                if (sact) {
                    const int e1 = min(dend, cb + n);
                    for (int e = max(dbeg, cb); e < e1; ++e) {
                        float *p = sc + (e - cb) * H + sk;
                        *p = __expf(*p - mx) * inv;
                    }
                }
                wave_lds_sync();
                for (; d < nd; ++d) {
                    const int e0 = __builtin_amdgcn_readlane(ip, d), e1 = __builtin_amdgcn_readlane(ip, d + 1);
                    const bool fin = e1 <= cb + n;              // the destination ends in this chunk
                    const int vd = v + d;
                    // rows two at a time; the residual row is requested right after the
                    // first pair (vmcnt retires in issue order: the pair's FMAs then wait
                    // for the L2 rows only, the HBM residual row just before the stores).
                    // No branches around the loads: the first pair runs even for an empty
                    // segment (weights 0, row 0), a null origin / out / h has a 0-byte
                    // descriptor (loads read 0, stores are dropped)
                    float org[NF];
                    const int qe = min(e1, cb + n) - cb;
                    auto pair = [&](int q, bool first) {
                        const bool one = q < qe, two = q + 1 < qe;          // wave-uniform
                        const int u0 = one ? __builtin_amdgcn_readfirstlane(su[q]) : 0;
                        const int u1 = two ? __builtin_amdgcn_readfirstlane(su[q + 1]) : u0;
                        float x0[NF], x1[NF];
#pragma unroll
                        for (int i = 0; i < NF; ++i) {
                            x0[i] = buf_ld(zr, fb[i], u0 * rowb);
                            x1[i] = buf_ld(zr, fb[i], u1 * rowb);
                        }
                        if (first) {
#pragma unroll
                            for (int i = 0; i < NF; ++i) org[i] = buf_ld(orr, fb[i], vd * rowb);
                        }
                        const float *a0 = sc + (one ? q : 0) * H, *a1 = sc + (two ? q + 1 : 0) * H;
#pragma unroll
                        for (int i = 0; i < NF; ++i) {
                            acc[i] = fmaf(one ? a0[fa[i]] : 0.f, x0[i], acc[i]);
                            acc[i] = fmaf(two ? a1[fa[i]] : 0.f, x1[i], acc[i]);
                        }
                    };
                    const int q0 = max(e0, cb) - cb;
                    pair(q0, true);
                    for (int q = q0 + 2; q < qe; q += 2) pair(q, false);
                    if (!fin) break;                            // continues in the next chunk
#pragma unroll
                    for (int i = 0; i < NF; ++i) {
                        if (lane + 64 * i < HD) {
                            buf_st(hr, fb[i], vd * rowb, acc[i]);
                            buf_st(outr, fb[i], vd * rowb, elu1(acc[i]) + org[i]);
                        }
                        acc[i] = 0.f;
                    }
                }
                wave_lds_sync();
                cb += CH;
            } while (cb < endB);
            v += nd;
        }
    }
}

// Grouped forward for short segments and wide rows (S2W: ~2 in-edges per word,
// H*D = 300): a wave carries 64/LPN destinations at once, one per LPN-lane group,
// so each wave has that many independent index -> score -> gather chains in flight
// and the grid needs 64/LPN times fewer waves.  Same arithmetic as k_gat_fwd with
// WPN = 1, group-local everything: lane = k*lph + l inside the group (lph =
// LPN / nextpow2(H)), features f = gl + LPN*i (LPN*4-byte contiguous segments per
// row), LDS chunk of kGrpChunk edges per group.
constexpr int kGrpChunk = 32;
template <int NF, int TAU_MODE, int LPN>
__global__ __launch_bounds__(256) void k_gat_fwd_grp(RelPtrs R, int H, int D, int lph, float slope,
                                                    const float *__restrict__ Z,
                                                    const float *__restrict__ sigma,
                                                    const float *__restrict__ tau,
                                                    const float *__restrict__ origin,
                                                    float *__restrict__ hout, float *__restrict__ out,
                                                    float *__restrict__ mout, float *__restrict__ lout) {
    constexpr int NG = 256 / LPN;                       // groups per block
    __shared__ float s_alpha[NG][kGrpChunk * HSG_HMAX];
    __shared__ int s_nb[NG][kGrpChunk];
    const int grp = threadIdx.x / LPN, gl = threadIdx.x % LPN;
    const int HD = H * D;
    const int k = gl / lph, l = gl - (gl / lph) * lph;
    const bool kact = k < H;
    int fh[NF], fo[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int f = gl + LPN * i;
        fh[i] = f < HD ? div_small(f, 1.f / (float)D) : 0;
        fo[i] = f < HD ? f : HD - 1;
    }
    float *sa = s_alpha[grp];
    int *sn = s_nb[grp];

    for (int v = blockIdx.x * NG + grp; v < R.n_dst; v += gridDim.x * NG) {
        const int beg = R.indptr[v], end = R.indptr[v + 1];
        const int c = R.phantom[v];
        // the residual row: independent of everything else, issued first
        float org[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) org[i] = origin ? origin[(size_t)v * HD + fo[i]] : 0.f;
        const int n1 = end - beg;
        const bool single = n1 <= kGrpChunk;
        float mx = -INFINITY, sm = 0.f;
        if (kact) {
            for (int j = l; j < n1; j += lph) {
                const int e = beg + j;
                const int u = R.src[e];
                const float s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                if (single) {
                    sa[j * H + k] = s;
                    if (k == 0) sn[j] = u;
                }
                if (s > mx) { sm = sm * __expf(mx - s) + 1.f; mx = s; }
                else sm += __expf(s - mx);
            }
        }
        for (int o = lph >> 1; o >= 1; o >>= 1) {
            const float om = __shfl_xor(mx, o), os = __shfl_xor(sm, o);
            lse_merge(mx, sm, om, os);
        }
        if (c > 0) lse_merge(mx, sm, 0.f, (float)c);
        const bool any = end > beg;
        const float inv = any ? 1.f / sm : 0.f;
        float acc[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i] = 0.f;
        for (int cb = beg; cb < end; cb += kGrpChunk) {
            const int n = min(kGrpChunk, end - cb);
            if (kact) {
                for (int j = l; j < n; j += lph) {
                    float s;
                    if (single) {
                        s = sa[j * H + k];
                    } else {
                        const int e = cb + j;
                        const int u = R.src[e];
                        s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                        if (k == 0) sn[j] = u;
                    }
                    sa[j * H + k] = __expf(s - mx) * inv;
                }
            }
            wave_lds_sync();
            gather_rows<NF>(Z, HD, n, sn, sa, H, fh, fo, acc);
            wave_lds_sync();
        }
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int f = gl + LPN * i;
            if (f < HD) {
                const size_t o = (size_t)v * HD + f;
                const float hv = acc[i];
                if (hout) hout[o] = hv;
                if (origin) out[o] = elu1(hv) + org[i];
            }
        }
        if (kact && l == 0) {
            mout[v * H + k] = any ? mx : 0.f;
            lout[v * H + k] = any ? sm : 1.f;
        }
    }
}

// Row-tile forward for short segments (S2W at config 2: ~2 in-edges per word,
// H*D = 300).  A block owns RT consecutive destinations, i.e. one contiguous
// RT*H*D-float band of origin / h / out, and streams it as float4 slots
// (slot q -> row q / (HD/4), columns 4(q % (HD/4)) .. +3; a slot may straddle two
// heads, so each component carries its own head index).  Every phase is parallel
// over the block, so one block runs ONE dependent chain for all its rows:
//   step 0:  the origin band (independent of everything, issued first), indptr and
//            the phantom counts of the RT rows -> LDS;
//   phase A1: thread p over the (edge j, head k) pairs of the block's contiguous
//            edge range: src / tf -> sigma / tau -> score in LDS (two round trips
//            for all edges at once, coalesced src / tf);
//   phase A2: thread p < RT*H owns (row, head): online (max, sum) over the row's
//            scores from LDS in CSR edge order, the phantom fold, m / l out, and
//            the alphas in place;
//   phase B: every slot sums alpha * Z[src] (float4 gathers) over its row's edges
//            in CSR order, then writes h and elu(h) + origin with float4 stores.
// Block edge ranges longer than the LDS chunk run A1 / A2 per chunk to get the
// softmax state first, then recompute each chunk's alphas (rows found by a binary
// search over the staged indptr) before its gathers.
constexpr int kRowsThreads = 256;
constexpr int kRowsEcap = 512;            // edges staged per chunk
constexpr int kRowsAlpha = 4096;          // floats of staged scores / alphas (ecap x H <= this, < 2^12)
constexpr int kRowsMaxPairs = kRowsThreads;   // RT * H bound: one (row, head) pair per thread

template <int NQ, int TAU_MODE>
__global__ __launch_bounds__(kRowsThreads) void k_gat_fwd_rows(RelPtrs R, int H, int D, int RT, float slope,
                                                               const float *__restrict__ Z,
                                                               const float *__restrict__ sigma,
                                                               const float *__restrict__ tau,
                                                               const float *__restrict__ origin,
                                                               float *__restrict__ hout, float *__restrict__ out,
                                                               float *__restrict__ mout, float *__restrict__ lout) {
    __shared__ int s_ptr[kRowsMaxPairs + 1];
    __shared__ int s_ph[kRowsMaxPairs];
    __shared__ int s_src[kRowsEcap];
    __shared__ float s_alpha[kRowsAlpha];
    __shared__ float s_m[kRowsMaxPairs], s_inv[kRowsMaxPairs];
    const int HD = H * D, HD4 = HD >> 2;
    const float inv_h = 1.f / (float)H;
    const int ecap = min(kRowsEcap, kRowsAlpha / H);
    const int t = threadIdx.x;
    const int v0 = blockIdx.x * RT;
    const int rows = min(RT, R.n_dst - v0);
    const int nslot = rows * HD4;
    // step 0: slot geometry and the residual band, issued first
    // skh: head k0 of the slot's first column and the component b from which the
    // columns belong to head k0 + 1 (b = 4: none), packed as k0 * 8 + b
    int srow[NQ], scol[NQ], skh[NQ];
    f32x4_t org[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const int q = t + kRowsThreads * i;
        const int qc = q < nslot ? q : nslot - 1;          // clamped (never stored)
        srow[i] = qc / HD4;
        scol[i] = (qc - srow[i] * HD4) * 4;
        const int k0 = scol[i] / D;
        skh[i] = k0 * 8 + min(4, (k0 + 1) * D - scol[i]);
        org[i] = origin ? *reinterpret_cast<const f32x4_t *>(origin + (size_t)(v0 + srow[i]) * HD + scol[i])
                        : f32x4_t{0.f, 0.f, 0.f, 0.f};
    }
    for (int r = t; r <= rows; r += kRowsThreads) s_ptr[r] = R.indptr[v0 + r];
    if (t < rows) s_ph[t] = R.phantom[v0 + t];
    __syncthreads();
    const int E0 = s_ptr[0], E1 = s_ptr[rows];
    const bool single = E1 - E0 <= ecap;
    // the (row, head) pair this thread owns in A2
    const int pr = div_small(t, inv_h), pk = t - pr * H;
    const bool pown = t < rows * H;
    const int pbeg = pown ? s_ptr[pr] : 0, pend = pown ? s_ptr[pr + 1] : 0;
    float mx = -INFINITY, sm = 0.f;
    for (int c0 = E0; c0 < E1; c0 += ecap) {
        const int c1 = min(E1, c0 + ecap), ne = c1 - c0;
        if (c0 > E0) __syncthreads();                    // A2 of the previous chunk is done
        // A1: scores of every (edge, head) pair of the chunk
        for (int p = t; p < ne * H; p += kRowsThreads) {
            const int j = div_small(p, inv_h), k = p - j * H;
            const int e = c0 + j;
            const int u = R.src[e];
            s_alpha[p] = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
            if (k == 0) s_src[j] = u;
        }
        __syncthreads();
        // A2: online (max, sum) of the owned pair over its edges in this chunk
        if (pown) {
            const int b = max(pbeg, c0), en = min(pend, c1);
            for (int e = b; e < en; ++e) {
                const float s = s_alpha[(e - c0) * H + pk];
                if (s > mx) { sm = sm * __expf(mx - s) + 1.f; mx = s; }
                else sm += __expf(s - mx);
            }
        }
    }
    if (pown) {
        const int c = s_ph[pr];
        if (c > 0) lse_merge(mx, sm, 0.f, (float)c);
        const bool any = pend > pbeg;
        const float inv = any ? 1.f / sm : 0.f;
        mout[(v0 + pr) * H + pk] = any ? mx : 0.f;
        lout[(v0 + pr) * H + pk] = any ? sm : 1.f;
        if (single) {
            for (int e = pbeg; e < pend; ++e) s_alpha[(e - E0) * H + pk] = __expf(s_alpha[(e - E0) * H + pk] - mx) * inv;
        } else {
            s_m[t] = mx;
            s_inv[t] = inv;
        }
    }
    __syncthreads();
    f32x4_t acc[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) acc[i] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    for (int c0 = E0; c0 < E1; c0 += ecap) {
        const int c1 = min(E1, c0 + ecap);
        if (!single) {                                   // recompute this chunk's alphas
            if (c0 > E0) __syncthreads();                // the previous chunk is gathered
            for (int p = t; p < (c1 - c0) * H; p += kRowsThreads) {
                const int j = div_small(p, inv_h), k = p - j * H;
                const int e = c0 + j;
                int lo = 0, hi = rows - 1;               // row: last r with s_ptr[r] <= e
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (s_ptr[mid] <= e) lo = mid; else hi = mid - 1;
                }
                const int u = R.src[e];
                const float s = leaky(sigma[u * H + k] + tau[tau_row<TAU_MODE>(R, e) * H + k], slope);
                s_alpha[p] = __expf(s - s_m[lo * H + k]) * s_inv[lo * H + k];
                if (k == 0) s_src[j] = u;
            }
            __syncthreads();
        }
        // phase B: edge jj of every slot's row in one step, so a thread's NQ gathers
        // are in flight together; per slot the sum still runs in CSR edge order
        int sb[NQ], sn[NQ], nmax = 0;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            sb[i] = max(s_ptr[srow[i]], c0);
            sn[i] = max(0, min(s_ptr[srow[i] + 1], c1) - sb[i]);
            nmax = max(nmax, sn[i]);
        }
        for (int jj = 0; jj < nmax; ++jj) {
            f32x4_t z[NQ];
            int j[NQ];
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                j[i] = (jj < sn[i] ? sb[i] + jj : c0) - c0;      // clamped to a staged edge
                z[i] = *reinterpret_cast<const f32x4_t *>(Z + (size_t)s_src[j[i]] * HD + scol[i]);
            }
#pragma unroll
            for (int i = 0; i < NQ; ++i) {
                if (jj < sn[i]) {
                    const int k0 = skh[i] >> 3, b = skh[i] & 7;
                    const float w0 = s_alpha[j[i] * H + k0], w1 = s_alpha[j[i] * H + min(k0 + 1, H - 1)];
#pragma unroll
                    for (int q = 0; q < 4; ++q) acc[i][q] = fmaf(q < b ? w0 : w1, z[i][q], acc[i][q]);
                }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const int q = t + kRowsThreads * i;
        if (q < nslot) {
            const size_t o = (size_t)(v0 + srow[i]) * HD + scol[i];
            if (hout) *reinterpret_cast<f32x4_t *>(hout + o) = acc[i];
            if (origin) {
                f32x4_t y;
#pragma unroll
                for (int j = 0; j < 4; ++j) y[j] = elu1(acc[i][j]) + org[i][j];
                *reinterpret_cast<f32x4_t *>(out + o) = y;
            }
        }
    }
}

// ---------------------------------------------------- backward: dst-centric ----
// Shared by both variants:  G = origin_mode ? dOut * elu'(h) : dOut,  rho = G.h,
//   dpre[e,k] = alpha (G_v.Z_u - rho) * leaky'(pre),  dtau partials per block.
//
// Edge-parallel variant (D <= 16): every lane of head k holds the whole G_v,k
// (DV registers) and handles its own edges e = l (mod lph) end to end -- no
// shuffles per edge, independent loads.  The d tau contributions go to 11
// per-lane registers (one per tau row), reduced once at the end.
template <int DV, int TAU_MODE, int WPN>
__global__ __launch_bounds__(256) void k_gat_bwd_dst_ep(RelPtrs R, int H, int D, int lph, int origin_mode,
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
    constexpr int NPB = HSG_WAVES / WPN;
    __shared__ float s_dtau[HSG_WAVES][HSG_NT * HSG_HMAX];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    const int part = wid % WPN;
    float dt[HSG_NT];
#pragma unroll
    for (int t = 0; t < HSG_NT; ++t) dt[t] = 0.f;

    const WorkRange wr = work_range(R.n_dst, NPB, wid / WPN, R.xcd);
    for (int v_ = wr.first; v_ < wr.end; v_ += wr.stride) {
        const int v = __builtin_amdgcn_readfirstlane(v_);      // scalar loads of indptr / phantom
        const int beg = R.indptr[v], end = R.indptr[v + 1];
        const float M = kact ? mv[v * H + k] : 0.f;             // issued early: independent
        const float lvv = kact ? lv[v * H + k] : 1.f;
        float g[DV];
        float rho = 0.f;
        const int kc = kact ? k : H - 1;
#pragma unroll
        for (int d = 0; d < DV; ++d) {           // clamped, unconditional loads; masked values
            const size_t o = (size_t)v * HD + kc * D + min(d, D - 1);
            const float hv = hsv[o], dv = dout[o];
            const bool ok = kact && d < D;
            const float gv = ok ? (origin_mode ? (hv > 0.f ? dv : dv * __expf(hv)) : dv) : 0.f;
            g[d] = gv;
            rho = fmaf(gv, hv, rho);
        }
        if (part == 0 && kact) {
#pragma unroll
            for (int d = 0; d < DV; ++d)
                if (d < D && d % lph == l) G[(size_t)v * HD + k * D + d] = g[d];
        }
        if (end == beg || !kact) continue;
        const float inv = 1.f / lvv;
        int eb, ee;
        subrange(beg, end, part, WPN, eb, ee);
#pragma unroll 2
        for (int e = eb + l; e < ee; e += lph) {
            const int u = R.src[e];
            const int t = tau_row<TAU_MODE>(R, e);
            const float *zr = Z + (size_t)u * HD + k * D;
            float dot = 0.f;
#pragma unroll
            for (int d = 0; d < DV; ++d) dot = fmaf(g[d], zr[min(d, D - 1)], dot);   // g[d] = 0 past D
            const float pre = sigma[u * H + k] + tau[t * H + k];
            const float alpha = __expf(leaky(pre, slope) - M) * inv;
            const float ds = alpha * (dot - rho);
            const float dp = pre > 0.f ? ds : ds * slope;
            dpre[(size_t)e * H + k] = dp;
            if constexpr (TAU_MODE == HSG_TAU_TABLE) {
#pragma unroll
                for (int tt = 0; tt < HSG_NT; ++tt) dt[tt] += t == tt ? dp : 0.f;
            }
        }
    }
    if constexpr (TAU_MODE == HSG_TAU_TABLE) {
#pragma unroll
        for (int tt = 0; tt < HSG_NT; ++tt) {
            const float a = group_sum(dt[tt], lph);
            if (kact && l == 0) s_dtau[wid][tt * H + k] = a;
        }
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

// Feature-split variant (any D <= 512, short segments): lane l of head k owns
// features d = l + lph*i; per edge the G.Z dot is a group sum.  The first lph
// edges' (src, pre) are loaded before the G/h/dOut rows so that chain overlaps
// them, then broadcast to the head group with a lane shuffle.
// NOH (no saved h; fused-stack S2W, origin present): G takes elu'(h) from
// e = x - origin = elu(h) (1 for e > 0, else e + 1 = exp(h); continuous at 0, so the
// rounding of x - origin moves G by ~ulp(x)), and rho = G_v.h_v = sum_e alpha_e
// (G_v.Z_u) over the typed edges (h_v = sum_e alpha_e Z_u; phantoms carry no message)
// is summed in a first pass over the edges whose dots are staged in LDS (the first
// kCh edges; later ones are recomputed in the second pass).
// GIN (with NOH): the G rows are given (hsg_gemm_f32_psw_elug produced them in the
// FFN backward's epilogue): read instead of dOut / x / origin, and not written.
constexpr int kCh = 16;
template <int NE, int TAU_MODE, int OCC = 1, bool NOH = false, bool GIN = false>
__global__ __launch_bounds__(256, OCC) void k_gat_bwd_dst(RelPtrs R, int H, int D, int lph, int origin_mode,
                                                    float slope,
                                                    const float *__restrict__ Z,
                                                    const float *__restrict__ sigma,
                                                    const float *__restrict__ tau,
                                                    const float *__restrict__ hsv,
                                                    const float *__restrict__ mv,
                                                    const float *__restrict__ lv,
                                                    const float *__restrict__ dout,
                                                    float *__restrict__ G, float *__restrict__ dpre,
                                                    float *__restrict__ dtau_part,
                                                    const float *__restrict__ xo,
                                                    const float *__restrict__ org) {
    __shared__ float s_dtau[HSG_WAVES][HSG_NT * HSG_HMAX];
    __shared__ float s_g[HSG_WAVES][512];                           // G_v, flat (H*D <= 512)
    __shared__ float s_gh[NOH ? 1 : HSG_WAVES][NOH ? 1 : 512];      // G_v * h_v
    __shared__ float s_dot[NOH ? HSG_WAVES : 1][NOH ? kCh * HSG_HMAX : 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    float *sd = s_dtau[wid];
    float *sg = s_g[wid], *sgh = s_gh[NOH ? 0 : wid], *sdt = s_dot[NOH ? wid : 0];
    if constexpr (TAU_MODE == HSG_TAU_TABLE) {
        for (int i = lane; i < HSG_NT * HSG_HMAX; i += 64) sd[i] = 0.f;
        wave_lds_sync();
    }

    const WorkRange wr = work_range(R.n_dst, HSG_WAVES, wid, R.xcd);
    for (int v_ = wr.first; v_ < wr.end; v_ += wr.stride) {
        const int v = __builtin_amdgcn_readfirstlane(v_);
        const int beg = R.indptr[v], end = R.indptr[v + 1];
        // softmax state of v: independent of everything below, issued first
        const float M = kact ? mv[v * H + k] : 0.f;
        const float lvv = kact ? lv[v * H + k] : 1.f;
        // prefetch edge j = l of this head: source rank, tau row and pre-activation
        int u0 = 0, t0 = 0;
        float pre0 = 0.f;
        if (kact && beg + l < end) {
            u0 = R.src[beg + l];
            t0 = tau_row<TAU_MODE>(R, beg + l);
            pre0 = sigma[u0 * H + k] + tau[t0 * H + k];
        }
        // G = dOut * elu'(h) over the row with the flat lane mapping (every access a
        // contiguous 256-B wave transaction), staged in LDS (with G*h); the (k, l) lanes
        // then pick their head's features from there
        constexpr int NF = 8;                     // 64 * NF >= H*D (<= 512)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int f = lane + 64 * i;
            if (f < HD) {
                const size_t o = (size_t)v * HD + f;
                float gv;
                if constexpr (GIN) {
                    gv = G[o];
                } else if constexpr (NOH) {
                    const float dv = dout[o];
                    const float e = xo[o] - org[o];
                    gv = e > 0.f ? dv : dv * (e + 1.f);
                } else {
                    const float dv = dout[o];
                    const float hv = hsv[o];
                    gv = origin_mode ? (hv > 0.f ? dv : dv * __expf(hv)) : dv;
                    sgh[f] = gv * hv;
                }
                if constexpr (!GIN) G[o] = gv;
                sg[f] = gv;
            }
        }
        wave_lds_sync();
        float g[NE];
        float rho = 0.f;
        const int kc = kact ? k : H - 1;
#pragma unroll
        for (int i = 0; i < NE; ++i) {
            const int d = l + lph * i;
            const bool ok = kact && d < D;
            const int f = kc * D + min(d, D - 1);
            g[i] = ok ? sg[f] : 0.f;
            if constexpr (!NOH) rho += ok ? sgh[f] : 0.f;
        }
        wave_lds_sync();                          // the next destination rewrites the stage
        if (end == beg) continue;   // uniform per wave: no typed in-edge, no gradient
        if constexpr (!NOH) rho = group_sum(rho, lph);
        const float inv = kact ? 1.f / lvv : 0.f;
        const int gl = k * lph;                         // first lane of this head group
        // one pair of edges: (src, tau row, pre) of both, then both Z rows fetched before
        // either dot is reduced -- or the dots from the stage (NOH second pass)
        auto edge_pair = [&](int e0, bool staged, float (&dot)[2], int (&t)[2], float (&pre)[2]) {
            int u[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int e = min(e0 + q, end - 1);
                const int j = e - beg;
                if (j < lph) {                          // wave-uniform branch
                    u[q] = __shfl(u0, gl + j);
                    t[q] = __shfl(t0, gl + j);
                    pre[q] = __shfl(pre0, gl + j);
                } else {
                    u[q] = R.src[e];
                    t[q] = tau_row<TAU_MODE>(R, e);
                    pre[q] = kact ? sigma[u[q] * H + k] + tau[t[q] * H + k] : 0.f;
                }
            }
            if (staged) {
#pragma unroll
                for (int q = 0; q < 2; ++q) dot[q] = sdt[min(e0 + q - beg, kCh - 1) * H + kc];
                return;
            }
            float zv[2][NE];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float *zr = Z + (size_t)u[q] * HD + kc * D;
#pragma unroll
                for (int i = 0; i < NE; ++i) zv[q][i] = zr[min(l + lph * i, D - 1)];
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                dot[q] = 0.f;
#pragma unroll
                for (int i = 0; i < NE; ++i) dot[q] = fmaf(g[i], zv[q][i], dot[q]);   // g = 0 past D
                dot[q] = group_sum(dot[q], lph);
            }
        };
        if constexpr (NOH) {
            if (end - beg <= 2) {                 // one pair: dots stay in registers, one pass
                float dot[2], pre[2];
                int t[2];
                edge_pair(beg, false, dot, t, pre);
                float al[2], rs = 0.f;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    al[q] = __expf(leaky(pre[q], slope) - M) * inv;
                    if (beg + q < end) rs = fmaf(al[q], dot[q], rs);
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int e = beg + q;
                    if (e < end && kact && l == 0) {
                        const float ds = al[q] * (dot[q] - rs);
                        const float dp = pre[q] > 0.f ? ds : ds * slope;
                        dpre[(size_t)e * H + k] = dp;
                        if constexpr (TAU_MODE == HSG_TAU_TABLE) sd[t[q] * H + k] += dp;
                    }
                }
                continue;
            }
        }
        if constexpr (NOH) {                      // pass 1: rho = sum_e alpha_e dot_e, dots staged
            float rs = 0.f;
            for (int e0 = beg; e0 < end; e0 += 2) {
                float dot[2], pre[2];
                int t[2];
                edge_pair(e0, false, dot, t, pre);
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int e = e0 + q;
                    if (e < end) {
                        rs = fmaf(__expf(leaky(pre[q], slope) - M) * inv, dot[q], rs);
                        if (kact && l == 0 && e - beg < kCh) sdt[(e - beg) * H + k] = dot[q];
                    }
                }
            }
            rho = rs;
            wave_lds_sync();
        }
        for (int e0 = beg; e0 < end; e0 += 2) {
            float dot[2], pre[2];
            int t[2];
            edge_pair(e0, NOH && e0 + 1 - beg < kCh, dot, t, pre);
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int e = e0 + q;
                if (e < end && kact && l == 0) {
                    const float alpha = __expf(leaky(pre[q], slope) - M) * inv;
                    const float ds = alpha * (dot[q] - rho);
                    const float dp = pre[q] > 0.f ? ds : ds * slope;
                    dpre[(size_t)e * H + k] = dp;
                    if constexpr (TAU_MODE == HSG_TAU_TABLE) sd[t[q] * H + k] += dp;
                }
            }
        }
        if constexpr (NOH) wave_lds_sync();       // the next destination restages the dots
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
template <int NF, int TAU_MODE, int WPN, int OCC = 1>
__global__ __launch_bounds__(256, OCC) void k_gat_bwd_src(RelPtrs R, int H, int D, int lph, float slope,
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
    constexpr int NPB = HSG_WAVES / WPN;
    __shared__ float s_alpha[HSG_WAVES][HSG_CHUNK * HSG_HMAX];
    __shared__ int s_nb[HSG_WAVES][HSG_CHUNK];
    __shared__ float s_dsig[HSG_WAVES][HSG_HMAX];
    __shared__ float s_dsum[HSG_WAVES][HSG_HMAX];
    __shared__ float s_da1[HSG_WAVES][64 * NF];
    __shared__ float s_acc[WPN > 1 ? HSG_WAVES : 1][WPN > 1 ? 64 * NF : 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    const int part = wid % WPN, w0 = wid - part;
    const bool writer = part == 0;
    int fh[NF], fo[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int f = lane + 64 * i;
        fh[i] = f < HD ? div_small(f, 1.f / (float)D) : 0;
        fo[i] = f < HD ? f : HD - 1;
    }
    float *sa = s_alpha[wid];
    int *sn = s_nb[wid];
    float da1[NF];                       // this wave's share of sum_u dsigma[u,k] Z[u,k,:]
#pragma unroll
    for (int i = 0; i < NF; ++i) da1[i] = 0.f;

    const WorkRange wr = work_range(R.n_src, NPB, wid / WPN, R.xcd);
    for (int u_ = wr.first; u_ < wr.end; u_ += wr.stride) {
        const int u = __builtin_amdgcn_readfirstlane(u_);
        const int beg = R.cindptr[u], end = R.cindptr[u + 1];
        int eb, ee;
        subrange(beg, end, part, WPN, eb, ee);
        const float sig = kact ? sigma[u * H + k] : 0.f;
        float zrow[NF];                  // Z row for d a1, issued early
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int f = lane + 64 * i;
            zrow[i] = (da1_part && writer && f < HD) ? Z[(size_t)u * HD + fo[i]] : 0.f;
        }
        float dsig = 0.f;
        float acc[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) acc[i] = 0.f;
        for (int cb = eb; cb < ee; cb += HSG_CHUNK) {
            const int n = min(HSG_CHUNK, ee - cb);
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
            gather_rows<NF>(G, HD, n, sn, sa, H, fh, fo, acc);
            wave_lds_sync();
        }
        dsig = group_sum(dsig, lph);
        if (kact && l == 0) s_dsig[wid][k] = dsig;
        if constexpr (WPN > 1) {
#pragma unroll
            for (int i = 0; i < NF; ++i) s_acc[wid][lane + 64 * i] = acc[i];
            __syncthreads();
            if (writer) {
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    float a = 0.f;
#pragma unroll
                    for (int p = 0; p < WPN; ++p) a += s_acc[w0 + p][lane + 64 * i];
                    acc[i] = a;
                }
                if (kact && l == 0) {
                    float a = 0.f;
#pragma unroll
                    for (int p = 0; p < WPN; ++p) a += s_dsig[w0 + p][k];
                    s_dsum[wid][k] = a;
                }
            }
        } else {
            if (kact && l == 0) s_dsum[wid][k] = dsig;
        }
        wave_lds_sync();
        if (writer) {
            if (dsigma && kact && l == 0) dsigma[u * H + k] = s_dsum[wid][k];
#pragma unroll
            for (int i = 0; i < NF; ++i) {
                const int f = lane + 64 * i;
                if (f < HD) {
                    const float ds = s_dsum[wid][fh[i]];
                    float r = acc[i];
                    if (a1) r = fmaf(ds, a1[f], r);
                    dZ[(size_t)u * HD + f] = r;
                    if (da1_part) da1[i] = fmaf(ds, zrow[i], da1[i]);
                }
            }
        }
        if constexpr (WPN > 1) __syncthreads();
        else wave_lds_sync();
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

// Merge of the pieces of long sources (round 6): the merging wave sums the pieces'
// partials in item order: dsigma_u,k = sum_p ds_p,k, dZ_u = sum_p dZ_p + dsigma_u * a1
// (the partials of kMergeBatch pieces requested together).  In-kernel by the last piece
// block to arrive (k_gat_bwd_src_g), or k_gat_bwd_src_g_merge as a second launch (dev).
// block-cooperative, one feature per thread per iteration (see fwd_merge_block)
__device__ __forceinline__ void bwd_merge_block(int H, int D, const float *__restrict__ pws, int first, int np, int u,
                                                const float *__restrict__ a1, float *__restrict__ dZ,
                                                float *__restrict__ dsigma) {
    const int HD = H * D, W = HD + H;
    const float *pw = pws + (size_t)first * W;
#pragma unroll 1
    for (int f = threadIdx.x; f < HD; f += blockDim.x) {
        const int k = f / D;
        float A = 0.f, DS = 0.f;
#pragma unroll 1
        for (int p0 = 0; p0 < np; p0 += kMergeBatch) {
            float av[kMergeBatch], dv[kMergeBatch];
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j) {
                const int p = min(p0 + j, np - 1);
                av[j] = pw[p * W + f];
                dv[j] = pw[p * W + HD + k];
            }
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j)
                if (p0 + j < np) {
                    A += av[j];
                    DS += dv[j];
                }
        }
        dZ[(size_t)u * HD + f] = a1 ? fmaf(DS, a1[f], A) : A;
        if (dsigma && f == k * D) dsigma[u * H + k] = DS;
    }
}

// ------------------------------------ backward: one source-centric pass (S2W) ----
// (round 4) The edge backward without its destination pass.  The softmax backward of
// edge e = (u -> v), head k, needs rho_v,k = G_v,k . h_v,k (G = dOut * elu'(h), h the
// aggregated message; GATLayer.py:118-131 under autograd): the FFN backward GEMM that
// makes G (hsg_gemm_psw_elug_rho) also writes rho as per-64-column partials, so
//   dpre_e,k = alpha_e,k (G_v,k . Z_u,k - rho_v,k) * leaky'(pre_e,k)
// is local to the edge and everything runs over the CSC segments.  Per source u the
// block's 4 waves split its out-edges (subrange); in blocks of lph edges lane (k, l)
// fetches edge l's destination, box, alpha and rho for head k, then per edge (4 rows in
// flight) the lph lanes of head k form G_v,k . Z_u,k over their NE features and every
// lane of the head accumulates alpha * G_v,k into its features of dZ_u, dpre into
// dsigma_u,k and (one lane) the box's d tau.  The waves' partials are combined in wave
// order; d tau and d a1 leave as per-block partials: deterministic.  Replaces the
// hsg_gat_bwd_dst_g + hsg_gat_bwd_src pair (G read once, no dpre round trip).
// GBF (round 5, the bf16 GEMM mode): G comes as bf16 rows (hsg_gemm_bf16_psw_elug_rho_a16
// with g_bf16), held raw until the edge uses them.
template <int NE, int OCC = 1, int EQ = 4, bool GBF = false, bool WL = false, bool PIN = false>
__global__ __launch_bounds__(256, OCC) void k_gat_bwd_src_g(RelPtrs R, int H, int D, int lph, float slope,
                                                      const float *__restrict__ sigma,
                                                      const float *__restrict__ tau,
                                                      const float *__restrict__ mv,
                                                      const float *__restrict__ lv,
                                                      const float *__restrict__ G,
                                                      const float *__restrict__ rhop, int rgroups, int rgw,
                                                      const float *__restrict__ a1,
                                                      const float *__restrict__ Z,
                                                      float *__restrict__ dZ, float *__restrict__ dsigma,
                                                      float *__restrict__ da1_part,
                                                      float *__restrict__ dtau_part,
                                                      float *__restrict__ pws, int pinline) {
    constexpr int WPN = HSG_WAVES;
    __shared__ int s_flag[1];
    __shared__ float s_acc[HSG_WAVES][512];
    __shared__ float s_dsig[HSG_WAVES][HSG_HMAX];
    __shared__ float s_dtau[HSG_WAVES][HSG_NT * HSG_HMAX];
    // the list kernel on fp32 G keeps wave 0's d a1 sums in LDS: in registers it spilled
    constexpr bool LDA1 = WL && !GBF;
    __shared__ float s_da1[LDA1 ? 512 : 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int k = lane / lph, l = lane - (lane / lph) * lph;
    const bool kact = k < H;
    const int kc = kact ? k : H - 1, gl = kc * lph, c0 = kc * D;
    float *sd = s_dtau[wid];
    for (int i = lane; i < HSG_NT * HSG_HMAX; i += 64) sd[i] = 0.f;
    if constexpr (LDA1)
        if (wid == 0)
            for (int i = lane; i < 512; i += 64) s_da1[i] = 0.f;
    wave_lds_sync();
    // rho partial addresses of head kc: rgw-column groups r0 (and r1 when the head
    // straddles two; D <= rgw), slot = head - first head of the group
    const int r0 = c0 / rgw, r1 = (c0 + D - 1) / rgw;
    const int o0 = r0 * 3 + (kc - (rgw * r0) / D), o1 = r1 * 3 + (kc - (rgw * r1) / D);
    float da1[LDA1 ? 1 : NE];                       // wave 0: sum_u dsigma[u,k] Z[u,k,:], (k, l) features
    int fo[NE];                                   // the lane's features c0 + d, clamped to the head
#pragma unroll
    for (int i = 0; i < NE; ++i) {
        if constexpr (!LDA1) da1[i] = 0.f;
        fo[i] = c0 + min(l + lph * i, D - 1);
    }

    // round 6: with the relation's CSC work list (and the piece scratch pws) the loop walks
    // its items -- whole sources, and pieces of the long ones (the HDSG doc supernodes),
    // whose dZ / dsigma partials go to pws for k_gat_bwd_src_g_merge
    // (WL: a template flag, so the kernel without a list keeps its registers)
    constexpr bool wl = WL;
    const WorkRange wr = work_range(wl ? R.n_swork : R.n_src, 1, 0, R.xcd);
    for (int u_ = wr.first; u_ < wr.end; u_ += wr.stride) {
        const int item = __builtin_amdgcn_readfirstlane(u_);
        // opaque per source: the compiler would otherwise hoist a 64-bit address per
        // feature and array (Z, a1, dZ, s_acc) out of the source loop and spill them
#pragma unroll
        for (int i = 0; i < NE; ++i) asm volatile("" : "+v"(fo[i]));
        int u = item, beg, end;
        bool piece = false;
        if (wl) {
            const int code = R.swork[4 * item];
            beg = R.swork[4 * item + 1];
            end = R.swork[4 * item + 2];
            piece = code < 0;
            u = piece ? -code - 1 : code;
        } else {
            beg = R.cindptr[u];
            end = R.cindptr[u + 1];
        }
        int eb, ee;
        subrange(beg, end, wid, WPN, eb, ee);
        const float sig = kact ? sigma[u * H + k] : 0.f;
        float zk[NE], acc[NE];
#pragma unroll
        for (int i = 0; i < NE; ++i) {
            zk[i] = kact && l + lph * i < D ? Z[(size_t)u * HD + fo[i]] : 0.f;
            acc[i] = 0.f;
        }
        float dsig = 0.f;
        #pragma unroll 1
        for (int jb = eb; jb < ee; jb += lph) {
            const int nb = min(lph, ee - jb);
            int vA = 0, tA = 0;
            float aA = 0.f, rA = 0.f, pA = 0.f;
            if (l < nb) {                                  // edge jb + l, head k
                const int p = jb + l;
                vA = R.cdst[p];
                tA = (int)R.tf[R.cperm[p]];
                if (kact) {
                    const float *rr = rhop + (size_t)vA * rgroups * 3;
                    rA = rr[o0] + (r1 != r0 ? rr[o1] : 0.f);
                    pA = sig + tau[tA * H + k];
                    aA = __expf(leaky(pA, slope) - mv[vA * H + k]) / lv[vA * H + k];
                }
            }
            #pragma unroll 1
            for (int j0 = 0; j0 < nb; j0 += EQ) {
                float gv[EQ][NE];
                __bf16 gb[GBF ? EQ : 1][GBF ? NE : 1];
#pragma unroll
                for (int q = 0; q < EQ; ++q) {
                    // lane j = (head 0, l = j) holds edge j's destination; scalar row base,
                    // per-lane feature offsets shared by every row (saddr + voffset loads)
                    const int v = __builtin_amdgcn_readfirstlane(__shfl(vA, min(j0 + q, nb - 1)));
                    if constexpr (GBF) {
                        const __bf16 *gr = reinterpret_cast<const __bf16 *>(G) + (size_t)v * HD;
#pragma unroll
                        for (int i = 0; i < NE; ++i) gb[q][i] = gr[fo[i]];
                    } else {
                        const float *gr = G + (size_t)v * HD;
#pragma unroll
                        for (int i = 0; i < NE; ++i) gv[q][i] = gr[fo[i]];
                    }
                }
#pragma unroll
                for (int q = 0; q < EQ; ++q) {
                    const int j = j0 + q;
                    if (j >= nb) break;                        // wave-uniform
                    if constexpr (GBF) {
#pragma unroll
                        for (int i = 0; i < NE; ++i) gv[q][i] = (float)gb[q][i];
                    }
                    float dot = 0.f;
#pragma unroll
                    for (int i = 0; i < NE; ++i) dot = fmaf(gv[q][i], zk[i], dot);     // zk = 0 past D
                    dot = group_sum(dot, lph);
                    const float a = __shfl(aA, gl + j), r = __shfl(rA, gl + j), pr = __shfl(pA, gl + j);
                    const int t = __shfl(tA, gl + j);
                    const float ds = a * (dot - r);
                    const float dp = pr > 0.f ? ds : ds * slope;
#pragma unroll
                    for (int i = 0; i < NE; ++i) acc[i] = fmaf(a, gv[q][i], acc[i]);
                    dsig += dp;
                    if (kact && l == 0) sd[t * H + k] += dp;
                }
            }
        }
        // combine the 4 waves' partials in wave order
#pragma unroll
        for (int i = 0; i < NE; ++i)
            if (kact && l + lph * i < D) s_acc[wid][fo[i]] = acc[i];
        if (kact && l == 0) s_dsig[wid][k] = dsig;
        __syncthreads();
        if (wid == 0) {
            float ds = 0.f;
#pragma unroll
            for (int w = 0; w < WPN; ++w) ds += s_dsig[w][kc];
            // a piece: its dZ partial without the ds * a1 term and its ds to pws
            // ([HD | H] per item), for the merge; its ds * Z_u into d a1 as any source's
            // (written through, sc1, when the last piece block merges in-kernel)
            float *pw = piece ? pws + (size_t)item * (HD + H) : nullptr;
            const bool pin = PIN && pinline;              // the merge launch's kernel: plain stores
            if (kact && l == 0) {
                if (piece) {
                    if (pin) st_sc1(&pw[HD + k], ds);
                    else pw[HD + k] = ds;
                } else if (dsigma) {
                    dsigma[u * H + k] = ds;
                }
            }
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                if (kact && l + lph * i < D) {
                    const int f = fo[i];
                    float a = 0.f;
#pragma unroll
                    for (int w = 0; w < WPN; ++w) a += s_acc[w][f];
                    if (piece) {
                        if (pin) st_sc1(&pw[f], a);
                        else pw[f] = a;
                    } else {
                        if (a1) a = fmaf(ds, a1[f], a);
                        dZ[(size_t)u * HD + f] = a;
                    }
                    if constexpr (LDA1) s_da1[f] = fmaf(ds, zk[i], s_da1[f]);    // lane-private slots
                    else da1[i] = fmaf(ds, zk[i], da1[i]);
                }
            }
            if (piece && pin) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if constexpr (WL && PIN) {
            // a piece, merged in-kernel (round 6): the last of u's pieces to arrive sums them
            // (wave 0); item and piece are block-uniform
            if (piece && pinline) {
                const int first = R.swork[4 * item + 3];
                const int np = __builtin_amdgcn_readfirstlane(piece_count(R.swork, R.n_swork, first,
                                                                          R.swork[4 * first], lane));
                if (piece_arrive(R.swork + 4 * R.n_swork + first, np, &s_flag[0]))
                    bwd_merge_block(H, D, pws, first, np, u, a1, dZ, dsigma);
            }
        }
        __syncthreads();                                   // s_acc / s_dsig / s_flag reused by the next source
    }
    if (wid == 0 && da1_part) {                            // block partial of d a1
#pragma unroll
        for (int i = 0; i < NE; ++i)
            if (kact && l + lph * i < D)
                da1_part[(size_t)blockIdx.x * HD + fo[i]] = LDA1 ? s_da1[fo[i]] : da1[LDA1 ? 0 : i];
    }
    // block partial of d tau (s_dtau written by lane (k, 0) of each wave; the loop's
    // last barrier orders them, this one covers a block without sources)
    __syncthreads();
    const int nt = HSG_NT * H;
    for (int i = threadIdx.x; i < nt; i += blockDim.x) {
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < HSG_WAVES; ++w) a += s_dtau[w][i];
        dtau_part[(size_t)blockIdx.x * nt + i] = a;
    }
}

__global__ __launch_bounds__(256) void k_gat_bwd_src_g_merge(RelPtrs R, int H, int D, const float *__restrict__ pws,
                                                             const float *__restrict__ a1, float *__restrict__ dZ,
                                                             float *__restrict__ dsigma) {
    const int item = (int)blockIdx.x;                     // one block per item (dev: HSG_PIECE_INLINE=0)
    const int code = R.swork[4 * item];
    if (code >= 0 || R.swork[4 * item + 3] != item) return;   // not a first piece
    __shared__ int s_np;
    if (threadIdx.x < 64) {
        const int np = piece_count(R.swork, R.n_swork, item, code, (int)threadIdx.x);
        if (threadIdx.x == 0) s_np = np;
    }
    __syncthreads();
    bwd_merge_block(H, D, pws, item, s_np, -code - 1, a1, dZ, dsigma);
}

// Head-lane src pass for narrow heads (D = DV = 8, short CSC segments: the W2S word
// sources, ~2 sentence edges each at config 2).  Lane = (source slot s, head k) with
// hp = nextpow2(H) lanes per source, so a wave carries 64 / hp sources at once and each
// lane owns its head's D features end to end: the per-edge alpha, dpre and the G-row
// quads are the lane's own loads -- no LDS staging of alphas, no cross-lane sums -- and
// the grid needs 64 / hp times fewer waves than one source per wave (cfg2 W2S: 2,400
// waves, all resident, instead of 19,200 in 2.3 rounds of dependent chains).  Edge
// pairs are requested together; accumulation is in edge order (fmaf per edge, as
// gather_rows), dsigma in edge order.  d a1 block partials are summed over the
// block's sources in (wave, slot) order: deterministic.
// RHO (round 4, table mode): the whole edge backward in this pass, as
// k_gat_bwd_src_g does for S2W: rho[v][k] = G_v,k . h_v,k comes from the narrow FFN's
// backward epilogue (hsg_ffn_small_bwd_gate, beside G), so each edge's
// dpre = alpha (G_v,k . Z_u,k - rho_v,k) * leaky'(pre) is formed here from the G quads
// the lane loads anyway and its own Z quads; d tau per box goes to per-lane registers
// (one add per box under a select) and leaves as per-block partials summed over the
// block's lanes in (wave, slot) order.  The dst pass is not launched.
template <int DV, int TAU_MODE, bool RHO = false>
__global__ __launch_bounds__(256) void k_gat_bwd_src_hl(RelPtrs R, int H, int D, int hp, float slope,
                                                        const float *__restrict__ sigma,
                                                        const float *__restrict__ tau,
                                                        const float *__restrict__ mv,
                                                        const float *__restrict__ lv,
                                                        const float *__restrict__ G,
                                                        const float *__restrict__ dpre,
                                                        const float *__restrict__ a1,
                                                        const float *__restrict__ Z,
                                                        float *__restrict__ dZ, float *__restrict__ dsigma,
                                                        float *__restrict__ da1_part,
                                                        const float *__restrict__ rho,
                                                        float *__restrict__ dtau_part) {
    static_assert(DV % 4 == 0, "features move as float4");
    static_assert(!RHO || TAU_MODE == HSG_TAU_TABLE, "per-box d tau partials: table mode");
    typedef float f4 __attribute__((ext_vector_type(4)));
    constexpr int NQ = DV / 4;
    __shared__ float s_tau[HSG_NT * HSG_HMAX];
    // d a1 partial rows padded to DV + 4 floats: the lanes' 16-byte stores then fall on
    // 16 distinct 4-bank slots per 16-lane group (at DV = 8, 32 B apart, they were 2-way)
    constexpr int DA = DV + 4;
    __shared__ __attribute__((aligned(16))) float s_da1[HSG_WAVES][64 * DA];
    // d tau lane partials box-major, rows of 264: the reduction's reads of one (wave,
    // slot) across lanes (t = i / 8, head i % 8) then sit on banks 8 t + head, distinct
    // within a wave (thread-major with 11 per thread they collided 2-way: 1.6e5
    // SQ_LDS_BANK_CONFLICT per launch)
    constexpr int DTS = 264;
    __shared__ float s_dt[RHO ? DTS * HSG_NT : 1];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int HD = H * D;
    const int sl = lane / hp, k = lane - sl * hp;
    const bool kact = k < H;
    const int wpw = 64 / hp;                                  // sources per wave
    if constexpr (TAU_MODE == HSG_TAU_TABLE) {
        for (int i = threadIdx.x; i < HSG_NT * H; i += blockDim.x) s_tau[i] = tau[i];
        __syncthreads();
    }
    const int kc = kact ? k : 0;
    f4 a1v[NQ], da1[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        a1v[q] = a1 ? *reinterpret_cast<const f4 *>(a1 + kc * D + 4 * q) : f4{0.f, 0.f, 0.f, 0.f};
        da1[q] = f4{0.f, 0.f, 0.f, 0.f};
    }
    float dt[RHO ? HSG_NT : 1];                               // RHO: this lane's d tau per box
#pragma unroll
    for (int t = 0; t < (RHO ? HSG_NT : 1); ++t) dt[t] = 0.f;
    const WorkRange wr = work_range((R.n_src + wpw - 1) / wpw, HSG_WAVES, wid, R.xcd);   // in wave groups
    for (int q0 = wr.first; q0 < wr.end; q0 += wr.stride) {
        const int u0 = q0 * wpw;
        const int u = u0 + sl;
        const bool act = kact && u < R.n_src;
        const int uc = act ? u : 0;
        const int beg = act ? R.cindptr[uc] : 0, end = act ? R.cindptr[uc + 1] : 0;
        const float sig = sigma[uc * H + kc];
        f4 zr[NQ], acc[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            zr[q] = (RHO || da1_part) ? *reinterpret_cast<const f4 *>(Z + (size_t)uc * HD + kc * D + 4 * q)
                                      : f4{0.f, 0.f, 0.f, 0.f};
            acc[q] = f4{0.f, 0.f, 0.f, 0.f};
        }
        float dsig = 0.f;
        for (int p = beg; p < end; p += 2) {
            const bool two = p + 1 < end;
            const int p1 = two ? p + 1 : p;
            const int v0 = R.cdst[p], e0 = R.cperm[p], v1 = R.cdst[p1], e1 = R.cperm[p1];
            const int t0 = tau_row<TAU_MODE>(R, e0), t1 = tau_row<TAU_MODE>(R, e1);
            const float M0 = mv[v0 * H + k], L0 = lv[v0 * H + k], M1 = mv[v1 * H + k], L1 = lv[v1 * H + k];
            float d0, d1, r0v = 0.f, r1v = 0.f;
            if constexpr (RHO) {
                r0v = rho[v0 * H + k];
                r1v = rho[v1 * H + k];
            } else {
                d0 = dpre[(size_t)e0 * H + k];
                d1 = dpre[(size_t)e1 * H + k];
            }
            f4 g0[NQ], g1[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                g0[q] = *reinterpret_cast<const f4 *>(G + (size_t)v0 * HD + k * D + 4 * q);
                g1[q] = *reinterpret_cast<const f4 *>(G + (size_t)v1 * HD + k * D + 4 * q);
            }
            float tv0, tv1;
            if constexpr (TAU_MODE == HSG_TAU_TABLE) { tv0 = s_tau[t0 * H + k]; tv1 = s_tau[t1 * H + k]; }
            else { tv0 = tau[(size_t)t0 * H + k]; tv1 = tau[(size_t)t1 * H + k]; }
            const float al0 = __expf(leaky(sig + tv0, slope) - M0) / L0;
            const float al1 = __expf(leaky(sig + tv1, slope) - M1) / L1;
            if constexpr (RHO) {
                float dot0 = 0.f, dot1 = 0.f;
#pragma unroll
                for (int q = 0; q < NQ; ++q)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        dot0 = fmaf(g0[q][j], zr[q][j], dot0);
                        dot1 = fmaf(g1[q][j], zr[q][j], dot1);
                    }
                const float s0 = al0 * (dot0 - r0v), s1 = al1 * (dot1 - r1v);
                d0 = sig + tv0 > 0.f ? s0 : s0 * slope;
                d1 = sig + tv1 > 0.f ? s1 : s1 * slope;
#pragma unroll
                for (int t = 0; t < HSG_NT; ++t) {
                    dt[t] += t == t0 ? d0 : 0.f;
                    if (two) dt[t] += t == t1 ? d1 : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[q][j] = fmaf(al0, g0[q][j], acc[q][j]);
            dsig += d0;
            if (two) {
#pragma unroll
                for (int q = 0; q < NQ; ++q)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[q][j] = fmaf(al1, g1[q][j], acc[q][j]);
                dsig += d1;
            }
        }
        if (act) {
            if (dsigma) dsigma[u * H + k] = dsig;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                f4 r = acc[q];
                if (a1) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) r[j] = fmaf(dsig, a1v[q][j], r[j]);
                }
                *reinterpret_cast<f4 *>(dZ + (size_t)u * HD + k * D + 4 * q) = r;
#pragma unroll
                for (int j = 0; j < 4; ++j) da1[q][j] = fmaf(dsig, zr[q][j], da1[q][j]);
            }
        }
    }
    if (da1_part) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) *reinterpret_cast<f4 *>(&s_da1[wid][lane * DA + 4 * q]) = da1[q];
        __syncthreads();
        for (int f = threadIdx.x; f < HD; f += blockDim.x) {
            const int kk = f / D, d = f - kk * D;
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < HSG_WAVES; ++w)
                for (int ss = 0; ss < wpw; ++ss) a += s_da1[w][(ss * hp + kk) * DA + d];
            da1_part[(size_t)blockIdx.x * HD + f] = a;
        }
    }
    if constexpr (RHO) {                     // d tau block partials, lanes in (wave, slot) order
#pragma unroll
        for (int t = 0; t < HSG_NT; ++t) s_dt[t * DTS + threadIdx.x] = dt[t];
        __syncthreads();
        const int nt = HSG_NT * H;
        for (int i = threadIdx.x; i < nt; i += blockDim.x) {
            const int t = i / H, kk = i - t * H;
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < HSG_WAVES; ++w)
                for (int ss = 0; ss < wpw; ++ss) a += s_dt[t * DTS + w * 64 + ss * hp + kk];
            dtau_part[(size_t)blockIdx.x * nt + i] = a;
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
constexpr int kFwdGridCap = 8192;
constexpr int kFwdPersistentCap = 1792;
// bounds the dtau partial slab; 1,536 = 256 CUs x the 6 resident blocks of the
// feature-split dst pass (w = 6): one persistent wave of blocks (cfg2 S2W dst pass
// 55.6 -> 49.9 us per step against 1,024; 2,048 / 4,800: 52.0 / 50.6)
constexpr int kBwdDstGridCap = 1536;
constexpr int kBwdSrcGridCap = 2048;   // bounds the d a1 partial slab
constexpr int kLongSegment = 16;       // mean segment length from which 4 waves share a node

// waves per node for a set of n nodes sharing n_edges edges
int wpn_for(int n, int n_edges) { return n > 0 && n_edges >= kLongSegment * n ? 4 : 1; }
int grid_nodes(int n, int wpn, int cap) {
    if (const char *e = HSG_DEV_ENV("HSG_GAT_CAP")) cap = atoi(e) < cap ? atoi(e) : cap;   // dev sweep
    int b = wpn == 4 ? n : (n + HSG_WAVES - 1) / HSG_WAVES;
    if (b < 1) b = 1;
    return b < cap ? b : cap;
}
int grid_for(int rows, int cap) { return grid_nodes(rows, 1, cap); }

bool shape_ok(int H, int D) { return H >= 1 && H <= HSG_HMAX && D >= 1 && H * D <= 512; }

int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// Measurement hook (bench.py's in-step kernel clock, hsg_kclock_arm): armed events are
// recorded by the next edge kernels' own dispatch packets (hipExtLaunchKernel) --
// start by the first kernel of an entry point, stop by its last -- so the measured
// interval is the kernels themselves, without event packets around them.  One-shot.
// The armed state is THREAD-LOCAL and bound to one stream: only launches from the
// arming thread onto that stream consume it, so entry points called from other
// threads, or on other streams of the same thread, never see it (the C ABI stays
// reentrant across threads and streams).
struct KClock {
    hipStream_t stream = nullptr;
    hipEvent_t start = nullptr, stop = nullptr;
};
thread_local KClock t_kc;
hipEvent_t kc_take(hipEvent_t &e, bool use) {
    if (!use) return nullptr;
    hipEvent_t r = e;
    e = nullptr;
    return r;
}
#define HSG_KLAUNCH(FIRST, LAST, KERNEL, GRID, BLOCK, ST, ...)                                              \
    do {                                                                                                    \
        if (t_kc.stream == (ST) && (((FIRST) && t_kc.start) || ((LAST) && t_kc.stop))) {                  \
            hipEvent_t e0_ = kc_take(t_kc.start, FIRST), e1_ = kc_take(t_kc.stop, LAST);                    \
            hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, 0, ST, e0_, e1_, 0, __VA_ARGS__);                    \
        } else {                                                                                            \
            hipLaunchKernelGGL(KERNEL, GRID, BLOCK, 0, ST, __VA_ARGS__);                                    \
        }                                                                                                   \
    } while (0)

template <int TAU, int WPN, int OCC = 1, int PF = 0, bool WL = false, bool O16 = false>
int fwd_dispatch(int nf, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, float slope,
                 const float *Z, const float *sg, const float *tau, const float *org, float *h,
                 float *out, float *m, float *l, float *pws = nullptr, bool last = true, int pinline = 0,
                 __bf16 *out16 = nullptr, int ld16 = 0) {
#define HSG_FWD(NF_)                                                                                     \
    case NF_:                                                                                            \
        HSG_KLAUNCH(true, last, (k_gat_fwd<NF_, TAU, WPN, OCC, PF, WL, O16>), grid, dim3(256), st, R, H, D, lph, slope, Z, \
                    sg, tau, org, h, out, m, l, pws, pinline, out16, ld16);                              \
        break;
    switch (nf) {
        HSG_FWD(1) HSG_FWD(2) HSG_FWD(3) HSG_FWD(4) HSG_FWD(5) HSG_FWD(6) HSG_FWD(7) HSG_FWD(8)
        default: return HSG_EINVAL;
    }
#undef HSG_FWD
    return launch_status();
}

// grouped forward: NF rounded up to an instantiated bucket (extra features are
// clamped loads that are never stored)
int grp_nf_bucket(int nf, int lpn) {
    static const int b32[] = {2, 4, 8, 10, 12, 16}, b16[] = {4, 8, 12, 16, 20, 32};
    const int *b = lpn == 32 ? b32 : b16;
    for (int i = 0; i < 6; ++i)
        if (nf <= b[i]) return b[i];
    return -1;
}

template <int TAU, int LPN>
int fwd_grp_dispatch(int nf, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, float slope,
                     const float *Z, const float *sg, const float *tau, const float *org, float *h, float *out,
                     float *m, float *l) {
#define HSG_FG(NF_)                                                                                      \
    case NF_:                                                                                            \
        hipLaunchKernelGGL((k_gat_fwd_grp<NF_, TAU, LPN>), grid, dim3(256), 0, st, R, H, D, lph, slope, Z, \
                           sg, tau, org, h, out, m, l);                                                  \
        break;
    if constexpr (LPN == 32) {
        switch (grp_nf_bucket(nf, LPN)) {
            HSG_FG(2) HSG_FG(4) HSG_FG(8) HSG_FG(10) HSG_FG(12) HSG_FG(16)
            default: return HSG_EINVAL;
        }
    } else {
        switch (grp_nf_bucket(nf, LPN)) {
            HSG_FG(4) HSG_FG(8) HSG_FG(12) HSG_FG(16) HSG_FG(20) HSG_FG(32)
            default: return HSG_EINVAL;
        }
    }
#undef HSG_FG
    return launch_status();
}

// lanes per destination for the forward: 64 (k_gat_fwd, one destination per
// wave) by default.  HSG_GAT_LPN=32/16 selects the grouped kernel; on the cfg2
// S2W pass (2.1 in-edges per word, H*D = 300) it measured 24.3 / 31.6 us against
// 23.5 us for one destination per wave (tools/gat_fwd_lpn.py), so more
// destinations per wave do not buy memory-level parallelism there.
int fwd_lanes_per_node(const hsg_rel *r, int H, int D) {
    int lpn = 64;
    const int HD = H * D;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_LPN")) lpn = atoi(e);
    if (lpn != 16 && lpn != 32) lpn = 64;
    if (lpn < 64 && (grp_nf_bucket((HD + lpn - 1) / lpn, lpn) < 0 || next_pow2(H) > lpn)) lpn = 64;
    return lpn;
}

// Row-tile forward plan: float4 slots per thread (NQ) and rows per block (RT) with
// the least idle slots; 0 when the shape or alignment does not allow it.
struct RowsPlan { int nq, rt; };
RowsPlan rows_plan(int H, int D, bool aligned) {
    RowsPlan best{0, 0};
    // opt-in (HSG_GAT_ROWS = -1: auto NQ, n > 0: NQ = n).  On the cfg2 S2W pass it
    // measured 25.3 us at NQ = 3 and 28.5 us at the auto NQ = 5 against 23.4 us for
    // one destination per wave (tools/gat_fwd_lpn.py): the per-(row, head) index ->
    // score chain of phase A costs more latency than the float4 band saves.
    int force = 0;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_ROWS")) force = atoi(e);
    if (force == 0) return best;
    const int HD = H * D;
    // a 4-column slot must not span more than two heads: D >= 2 (D = 2 slots are head-aligned)
    if (HD % 4 || D < 2 || !aligned) return best;
    const int hd4 = HD / 4;
    static const int nqs[] = {1, 2, 3, 4, 5, 6, 8};
    double best_u = 0.0;
    int rt_force = 0;                                   // dev sweep: rows per block
    if (const char *e = HSG_DEV_ENV("HSG_GAT_ROWS_RT")) rt_force = atoi(e);
    for (int nq : nqs) {
        if (force > 0 && nq != force) continue;
        int rt = kRowsThreads * nq / hd4;
        if (rt_force > 0 && rt_force < rt) rt = rt_force;
        if (rt > kRowsMaxPairs / H) rt = kRowsMaxPairs / H;
        if (rt < 1) continue;
        const double u = (double)rt * hd4 / (kRowsThreads * nq);
        if (u > best_u + 1e-9) { best_u = u; best = RowsPlan{nq, rt}; }
    }
    return best;
}

template <int TAU>
int fwd_rows_dispatch(RowsPlan pl, hipStream_t st, RelPtrs R, int H, int D, float slope, const float *Z,
                      const float *sg, const float *tau, const float *org, float *h, float *out, float *m,
                      float *l) {
    const dim3 grid((unsigned)((R.n_dst + pl.rt - 1) / pl.rt));
#define HSG_FR(NQ_)                                                                                     \
    case NQ_:                                                                                           \
        HSG_KLAUNCH(true, true, (k_gat_fwd_rows<NQ_, TAU>), grid, dim3(kRowsThreads), st, R, H, D, pl.rt, \
                    slope, Z, sg, tau, org, h, out, m, l);                                               \
        break;
    switch (pl.nq) {
        HSG_FR(1) HSG_FR(2) HSG_FR(3) HSG_FR(4) HSG_FR(5) HSG_FR(6) HSG_FR(8)
        default: return HSG_EINVAL;
    }
#undef HSG_FR
    return launch_status();
}

bool aligned16p(const void *p) { return ((uintptr_t)p & 15) == 0; }

// occupancy hints of the feature-split dst pass (6 waves per SIMD: 88 -> 79 VGPRs,
// no spill) and of the 4-waves-per-node src pass (5: 101 -> 90); HSG_GAT_BWD_OCC=0
// drops them.  cfg2 S2W backward 61.2 -> 56.1 us per step in one A/B.
bool bwd_occ() {
    const char *e = HSG_DEV_ENV("HSG_GAT_BWD_OCC");
    return !(e && atoi(e) == 0);
}

// next-destination prefetch in the one-destination-per-wave forward: cfg2 S2W
// forward 17.8 -> 17.2 us in-step, step 1.3084 -> 1.3049 ms in one A/B (round 3);
// HSG_GAT_FWD_PF=0 drops it
// round 4: two-level prefetch by default (S2W forward 16.53 / 16.59 -> 16.09 / 16.14 us
// per launch in two alternations of rocprofv3 step traces, profiles/r04_dev/pf{1,2}_step_*.txt);
// HSG_GAT_FWD_PF=1 / 0 (dev) restore one level / none.  Round 5, PF = 3 (dev): the next
// destination's residual row requested right after this one's first gathered row, i.e.
// a whole iteration ahead (6 waves per SIMD for its registers): 16.9 vs 16.0 us per
// launch in step traces, 16.2 vs 16.0 back to back -- the residual row is not what the
// forward waits on (without any residual read, h instead of out: 14.0 us).  The score
// lanes per head (HSG_GAT_FWD_LPH, dev) at 8 / 4 / 2 / 1: 15.6 / 15.9 / 17.2 / 19.6 us.
// the pieces of long nodes merged in-kernel by their last arrival (round 6, default) or by
// a second launch (dev A/B: HSG_PIECE_INLINE=0)
// bit 0: the forward, bit 1: the backward (default 1: the forward merges in-kernel)
int piece_inline() {
    const char *e = HSG_DEV_ENV("HSG_PIECE_INLINE");
    return e ? atoi(e) : 1;
}

#ifdef HSG_DEV
// the destination-tile forward (k_gat_fwd_tile) for short segments; dev: HSG_GAT_FWD_TILE
int fwd_tile() {
    int v = 0;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_FWD_TILE")) v = atoi(e);
    return v;
}

template <int TAU, bool O16>
int tile_dispatch(int nf, hipStream_t st, RelPtrs R, int H, int D, int lph, float slope, const float *Z,
                  const float *sg, const float *tau, const float *org, float *h, float *out, float *m, float *l,
                  __bf16 *out16, int ld16) {
    const int tw = fwd_tile() == 2 ? 24 : kTileW;
    const int ntiles = (R.n_dst + tw - 1) / tw;
#define HSG_FT(NF_)                                                                                        \
    case NF_:                                                                                              \
        if (tw == 24)                                                                                      \
            HSG_KLAUNCH(true, true, (k_gat_fwd_tile<NF_, TAU, O16, 24>), dim3((unsigned)ntiles), dim3(512), st, R, H, \
                        D, lph, slope, Z, sg, tau, org, h, out, m, l, out16, ld16, ntiles);                \
        else                                                                                               \
            HSG_KLAUNCH(true, true, (k_gat_fwd_tile<NF_, TAU, O16>), dim3((unsigned)ntiles), dim3(512), st, R, H, \
                        D, lph, slope, Z, sg, tau, org, h, out, m, l, out16, ld16, ntiles);                \
        break;
    switch (nf) {
        HSG_FT(1) HSG_FT(2) HSG_FT(3) HSG_FT(4) HSG_FT(5)
        default: return HSG_EINVAL;
    }
#undef HSG_FT
    return launch_status();
}
#endif

int fwd_pf() {
    const char *e = HSG_DEV_ENV("HSG_GAT_FWD_PF");
    return e ? (atoi(e) == 0 ? 0 : atoi(e) == 1 ? 1 : atoi(e) == 3 ? 3 : 2) : 2;
}

// occupancy hint of the one-destination-per-wave forward: 7 waves per SIMD (73 -> 64
// VGPRs, no spill; the SGPR count admits 7 blocks per CU); HSG_GAT_FWD_OCC=1 drops it
int fwd_occ() {
    int o = 7;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_FWD_OCC")) o = atoi(e);
    return o == 7 || o == 8 ? o : 1;
}

template <int TAU, int WPN>
int bwd_dst_ep_dispatch(int D, dim3 grid, hipStream_t st, RelPtrs R, int H, int lph, int om, float slope,
                        const float *Z, const float *sg, const float *tau, const float *h, const float *m,
                        const float *l, const float *dout, float *G, float *dpre, float *dtp) {
#define HSG_EP(DV_)                                                                                    \
    HSG_KLAUNCH(true, false, (k_gat_bwd_dst_ep<DV_, TAU, WPN>), grid, dim3(256), st, R, H, D, lph, om, slope, \
                Z, sg, tau, h, m, l, dout, G, dpre, dtp)
    if (D <= 4) HSG_EP(4);
    else if (D <= 8) HSG_EP(8);
    else HSG_EP(16);
#undef HSG_EP
    return launch_status();
}

template <int TAU, int OCC = 1, bool NOH = false, bool GIN = false>
int bwd_dst_dispatch(int ne, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, int om,
                     float slope, const float *Z, const float *sg, const float *tau, const float *h,
                     const float *m, const float *l, const float *dout, float *G, float *dpre,
                     float *dtp, const float *x = nullptr, const float *org = nullptr) {
#define HSG_BD(NE_)                                                                                        \
    case NE_:                                                                                              \
        HSG_KLAUNCH(true, false, (k_gat_bwd_dst<NE_, TAU, OCC, NOH, GIN>), grid, dim3(256), st, R, H, D, lph, \
                    om, slope, Z, sg, tau, h, m, l, dout, G, dpre, dtp, x, org);                           \
        break;
    if constexpr (NOH) {                 // the shapes the fused stack's S2W pass uses
        switch (ne) {
            HSG_BD(4) HSG_BD(5) HSG_BD(6) HSG_BD(7) HSG_BD(8) HSG_BD(16)
            default: return HSG_EINVAL;
        }
    } else {
        switch (ne) {
            HSG_BD(1) HSG_BD(2) HSG_BD(3) HSG_BD(4) HSG_BD(5) HSG_BD(6) HSG_BD(7) HSG_BD(8)
            HSG_BD(16) HSG_BD(32) HSG_BD(64)
            default: return HSG_EINVAL;
        }
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

template <int TAU, int WPN, int OCC = 1>
int bwd_src_dispatch(int nf, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, int lph, float slope,
                     const float *sg, const float *tau, const float *m, const float *l, const float *G,
                     const float *dpre, const float *a1, const float *Z, float *dZ, float *dsig, float *da1p) {
#define HSG_BS(NF_)                                                                                        \
    case NF_:                                                                                              \
        HSG_KLAUNCH(false, true, (k_gat_bwd_src<NF_, TAU, WPN, OCC>), grid, dim3(256), st, R, H, D, lph, slope, \
                    sg, tau, m, l, G, dpre, a1, Z, dZ, dsig, da1p);                                     \
        break;
    switch (nf) {
        HSG_BS(1) HSG_BS(2) HSG_BS(3) HSG_BS(4) HSG_BS(5) HSG_BS(6) HSG_BS(7) HSG_BS(8)
        default: return HSG_EINVAL;
    }
#undef HSG_BS
    return launch_status();
}

// dst-side launch shape (fwd and bwd_dst share it; the d tau slab has one row per block)
int dst_wpn(const hsg_rel *r) { return wpn_for(r->n_dst, r->n_edges); }
// single-pass narrow-row forward (k_gat_fwd_sp): its sub-batch of edges, 0 = off.  Measured
// slower than the 4-wave k_gat_fwd on the cfg2 W2S destinations (see the kernel): dev
// opt-in (HSG_GAT_FWD_SP=16|8)
int fwd_sp() {
    const char *e = HSG_DEV_ENV("HSG_GAT_FWD_SP");
    const int eb = e ? atoi(e) : 0;
    return eb == 0 ? 0 : (eb == 8 ? 8 : 16);
}
int src_wpn(const hsg_rel *r) { return wpn_for(r->n_src, r->n_edges); }
// destinations per wave batch of the short-segment forward (k_gat_fwd_b, dev only); 0 =
// the one-destination-per-wave k_gat_fwd.  Measured slower on the cfg2 S2W pass
// (rocprofv3 step traces, two alternations: 17.3 / 17.3 / 21.0 us with 4 / 2 / 8
// destinations per batch against 15.9 us; back to back 17.0 vs 16.0 us, gat_fwd_diag):
// the wave walks its batch's destinations one gather round trip after another, and
// fewer waves hide less.  HSG_GAT_FWD_B=2|4|8
int fwd_batch() {
    const char *e = HSG_DEV_ENV("HSG_GAT_FWD_B");
    const int b = e ? atoi(e) : 0;
    return b == 2 || b == 4 || b == 8 ? b : 0;
}

template <int TAU, int DB>
int fwd_b_dispatch(int nf, dim3 grid, hipStream_t st, RelPtrs R, int H, int D, float slope, const float *Z,
                   const float *sg, const float *tau, const float *org, float *h, float *out, float *m, float *l) {
#define HSG_FB(NF_)                                                                                      \
    case NF_:                                                                                            \
        HSG_KLAUNCH(true, true, (k_gat_fwd_b<NF_, TAU, DB>), grid, dim3(256), st, R, H, D, slope, Z, sg, tau, \
                    org, h, out, m, l);                                                                  \
        break;
    switch (nf) {
        HSG_FB(1) HSG_FB(2) HSG_FB(3) HSG_FB(4) HSG_FB(5) HSG_FB(6) HSG_FB(7) HSG_FB(8)
        default: return HSG_EINVAL;
    }
#undef HSG_FB
    return launch_status();
}

}  // namespace

extern "C" {

int hsg_gat_fwd(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                const float *sigma, const float *tau, const float *origin, float *h, float *out,
                float *m, float *l, void *stream) {
    return hsg_gat_fwd_ws(rel, H, D, tau_mode, slope, Z, sigma, tau, origin, h, out, m, l, nullptr, stream);
}

size_t hsg_gat_fwd_ws_floats(const hsg_rel *rel, int H, int D) {
    if (!rel || !shape_ok(H, D) || !rel->dwork || rel->n_dwork <= 0 || rel->n_dst == 0 || dst_wpn(rel) != 4)
        return 0;
    return (size_t)rel->n_dwork * (size_t)(H * D + 2 * H);
}

static int gat_fwd_impl(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                        const float *sigma, const float *tau, const float *origin, float *h, float *out, float *m,
                        float *l, float *ws, __bf16 *out16, int ld16, void *stream) {
    if (!rel || !shape_ok(H, D) || (origin && !out && !out16) || (!origin && !h)) return HSG_EINVAL;
    if (out16 && (!origin || ld16 < (H * D + 7) / 8 * 8 || ld16 % 8 || ((uintptr_t)out16 & 15))) return HSG_EINVAL;
    if (tau_mode != HSG_TAU_TABLE && tau_mode != HSG_TAU_PER_EDGE) return HSG_EINVAL;
    if (rel->n_dst == 0) return 0;
    const RelPtrs R = rel_ptrs(rel);
    hipStream_t st = (hipStream_t)stream;
#ifdef HSG_DEV
    const int lpn = fwd_lanes_per_node(rel, H, D);
    if (lpn < 64 && !out16) {
        const int ng = 256 / lpn;
        int b = (rel->n_dst + ng - 1) / ng;
        const dim3 g(b < kFwdGridCap ? b : kFwdGridCap);
        const int nfg = (H * D + lpn - 1) / lpn, lphg = lpn / next_pow2(H);
#define HSG_G(TAU, L) fwd_grp_dispatch<TAU, L>(nfg, g, st, R, H, D, lphg, slope, Z, sigma, tau, origin, h, out, m, l)
        if (tau_mode == HSG_TAU_TABLE) return lpn == 32 ? HSG_G(HSG_TAU_TABLE, 32) : HSG_G(HSG_TAU_TABLE, 16);
        return lpn == 32 ? HSG_G(HSG_TAU_PER_EDGE, 32) : HSG_G(HSG_TAU_PER_EDGE, 16);
#undef HSG_G
    }
#endif
    const int nf = (H * D + 63) / 64;
    const int wpn = dst_wpn(rel);
#ifdef HSG_DEV
    if (launch_floor_mode() == 1 && wpn == 4 && nf == 1) {      // dev probe: the W2S forward's grid, no work
        HSG_KLAUNCH(true, true, k_launch_floor, dim3(grid_nodes(rel->n_dst, 4, kFwdGridCap)), dim3(256), st,
                    rel->indptr, rel->n_dst, (int32_t *)nullptr);
        return launch_status();
    }
#endif
    if (nf == 1 && fwd_sp() && tau_mode == HSG_TAU_TABLE && !out16 &&
        (long)rel->n_src * H * D * 4 < 0x7fffffffL) {  // narrow rows: one single-pass wave per destination
        const dim3 g(grid_nodes(rel->n_dst, 1, kFwdGridCap));
        const int eb = fwd_sp();
#define HSG_SP(TAU, EB_) HSG_KLAUNCH(true, true, (k_gat_fwd_sp<TAU, EB_>), g, dim3(256), st, R, H, D, slope, Z, sigma, \
                                     tau, origin, h, out, m, l)
        if (eb == 8) HSG_SP(HSG_TAU_TABLE, 8);
        else HSG_SP(HSG_TAU_TABLE, 16);
#undef HSG_SP
        return launch_status();
    }
#ifdef HSG_DEV
    // (k_gat_fwd_b addresses rows by 32-bit buffer offsets)
    const bool b32 = (long)rel->n_src * H * D * 4 < 0x7fffffffL && (long)rel->n_dst * H * D * 4 < 0x7fffffffL;
    if (wpn == 1 && fwd_batch() && b32 && !out16) {   // short segments: destination batches per wave (dev A/B)
        const int db = fwd_batch();
        const dim3 g(grid_nodes((rel->n_dst + db - 1) / db, 1, kFwdPersistentCap));
#define HSG_B(DB_) (tau_mode == HSG_TAU_TABLE                                                                \
                        ? fwd_b_dispatch<HSG_TAU_TABLE, DB_>(nf, g, st, R, H, D, slope, Z, sigma, tau, origin, h, \
                                                             out, m, l)                                   \
                        : fwd_b_dispatch<HSG_TAU_PER_EDGE, DB_>(nf, g, st, R, H, D, slope, Z, sigma, tau, origin, \
                                                                h, out, m, l))
        if (db == 2) return HSG_B(2);
        if (db == 8) return HSG_B(8);
        return HSG_B(4);
#undef HSG_B
    }
    if (wpn == 1 && !out16) {            // short segments: row-tile float4 kernel
        const bool al = aligned16p(Z) && aligned16p(h) && (!origin || (aligned16p(origin) && aligned16p(out)));
        const RowsPlan pl = rows_plan(H, D, al);
        if (pl.nq > 0) {
            if (tau_mode == HSG_TAU_TABLE)
                return fwd_rows_dispatch<HSG_TAU_TABLE>(pl, st, R, H, D, slope, Z, sigma, tau, origin, h, out, m, l);
            return fwd_rows_dispatch<HSG_TAU_PER_EDGE>(pl, st, R, H, D, slope, Z, sigma, tau, origin, h, out, m, l);
        }
    }
#endif
    // one destination per wave: one persistent wave of blocks (256 CUs x the 7 blocks
    // the w = 7 kernel keeps resident; cfg2 S2W forward 24.8 -> 22.4 us per step)
    int fcap = wpn == 1 && fwd_occ() == 7 ? kFwdPersistentCap : kFwdGridCap;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_FWD_CAP")) fcap = atoi(e) > 0 ? atoi(e) : fcap;   // dev sweep
    const dim3 grid(grid_nodes(rel->n_dst, wpn, fcap));
    int lph = lanes_per_head(H);
    if (const char *e = HSG_DEV_ENV("HSG_GAT_FWD_LPH")) {      // dev sweep: score lanes per head (power of 2)
        const int v = atoi(e);
        if (v >= 1 && v <= lph && (v & (v - 1)) == 0 && wpn == 1) lph = v;
    }
    const int occ = wpn == 1 ? fwd_occ() : 1;
    if (occ > 1) {
        const int pf = fwd_pf();
        if (pf != 0 || occ != 8) {
#ifdef HSG_DEV
            if (out16 && pf != 2) return HSG_EINVAL;
            if (pf == 3) {                                 // residual row one destination ahead (dev A/B)
                // 6 waves per SIMD (the next row's registers): one persistent wave of 1,536 blocks
                const dim3 g6(grid_nodes(rel->n_dst, 1, 1536));
                if (tau_mode == HSG_TAU_TABLE)
                    return fwd_dispatch<HSG_TAU_TABLE, 1, 6, 3>(nf, g6, st, R, H, D, lph, slope, Z, sigma, tau,
                                                                origin, h, out, m, l, nullptr, true, 0, out16, ld16);
                return fwd_dispatch<HSG_TAU_PER_EDGE, 1, 6, 3>(nf, g6, st, R, H, D, lph, slope, Z, sigma, tau,
                                                               origin, h, out, m, l, nullptr, true, 0, out16, ld16);
            }
            if (pf == 1) {                                 // one-level prefetch (dev A/B)
                if (tau_mode == HSG_TAU_TABLE)
                    return fwd_dispatch<HSG_TAU_TABLE, 1, 7, 1>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau,
                                                                origin, h, out, m, l, nullptr, true, 0, out16, ld16);
                return fwd_dispatch<HSG_TAU_PER_EDGE, 1, 7, 1>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau,
                                                               origin, h, out, m, l, nullptr, true, 0, out16, ld16);
            }
            if (pf == 0) {
                if (tau_mode == HSG_TAU_TABLE)
                    return fwd_dispatch<HSG_TAU_TABLE, 1, 7>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau,
                                                             origin, h, out, m, l, nullptr, true, 0, out16, ld16);
                return fwd_dispatch<HSG_TAU_PER_EDGE, 1, 7>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau,
                                                            origin, h, out, m, l, nullptr, true, 0, out16, ld16);
            }
#endif
#ifdef HSG_DEV
            if (fwd_tile() && nf <= 5 && lph <= 64) {          // destination tiles (round 6, dev)
                const bool tt = tau_mode == HSG_TAU_TABLE;
                return tt ? (out16 ? tile_dispatch<HSG_TAU_TABLE, true>(nf, st, R, H, D, lph, slope, Z, sigma, tau,
                                                                       origin, h, out, m, l, out16, ld16)
                                   : tile_dispatch<HSG_TAU_TABLE, false>(nf, st, R, H, D, lph, slope, Z, sigma, tau,
                                                                        origin, h, out, m, l, out16, ld16))
                          : (out16 ? tile_dispatch<HSG_TAU_PER_EDGE, true>(nf, st, R, H, D, lph, slope, Z, sigma,
                                                                          tau, origin, h, out, m, l, out16, ld16)
                                   : tile_dispatch<HSG_TAU_PER_EDGE, false>(nf, st, R, H, D, lph, slope, Z, sigma,
                                                                           tau, origin, h, out, m, l, out16, ld16));
            }
#endif
#define HSG_F2(TAU, O16_) fwd_dispatch<TAU, 1, 7, 2, false, O16_>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau, \
                                                             origin, h, out, m, l, nullptr, true, 0, out16, ld16)
            if (tau_mode == HSG_TAU_TABLE) return out16 ? HSG_F2(HSG_TAU_TABLE, true) : HSG_F2(HSG_TAU_TABLE, false);
            return out16 ? HSG_F2(HSG_TAU_PER_EDGE, true) : HSG_F2(HSG_TAU_PER_EDGE, false);
#undef HSG_F2
        }
#ifdef HSG_DEV
#define HSG_FO(TAU, O) fwd_dispatch<TAU, 1, O>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau, origin, h, out, m, l, \
                                               nullptr, true, 0, out16, ld16)
        if (out16) return HSG_EINVAL;
        if (tau_mode == HSG_TAU_TABLE) return HSG_FO(HSG_TAU_TABLE, 8);
        return HSG_FO(HSG_TAU_PER_EDGE, 8);
#undef HSG_FO
#endif
    }
#define HSG_F(TAU, W) fwd_dispatch<TAU, W>(nf, grid, st, R, H, D, lph, slope, Z, sigma, tau, origin, h, out, m, l, \
                                           nullptr, true, 0, out16, ld16)
#ifdef HSG_DEV
    if (wpn == 1 && out16) return HSG_EINVAL;
    if (wpn == 1) return tau_mode == HSG_TAU_TABLE ? HSG_F(HSG_TAU_TABLE, 1) : HSG_F(HSG_TAU_PER_EDGE, 1);
#endif
#undef HSG_F
    // wpn == 1 took the w = 7 kernel above.  Multi-wave destinations: with the CSR work
    // list (and its scratch) the items of the list, then the merge of the long
    // destinations' pieces (round 6)
    const bool wl = ws && R.n_dwork > 0;
    const dim3 g4(grid_nodes(wl ? R.n_dwork : rel->n_dst, 4, fcap));
    float *pws = wl ? ws : nullptr;
    const int pin = piece_inline() & 1;
#define HSG_F4(TAU, O16_) fwd_dispatch<TAU, 4, 1, 0, false, O16_>(nf, g4, st, R, H, D, lph, slope, Z, sigma, tau, \
                                                             origin, h, out, m, l, nullptr, true, 0, out16, ld16)
#define HSG_FW(TAU, O16_) fwd_dispatch<TAU, 4, 6, 0, true, O16_>(nf, g4, st, R, H, D, lph, slope, Z, sigma, tau, \
                                                            origin, h, out, m, l, pws, pin, pin, out16, ld16)
    const bool tt = tau_mode == HSG_TAU_TABLE;
    const int rc = !wl ? (tt ? (out16 ? HSG_F4(HSG_TAU_TABLE, true) : HSG_F4(HSG_TAU_TABLE, false))
                             : (out16 ? HSG_F4(HSG_TAU_PER_EDGE, true) : HSG_F4(HSG_TAU_PER_EDGE, false)))
                       : (tt ? (out16 ? HSG_FW(HSG_TAU_TABLE, true) : HSG_FW(HSG_TAU_TABLE, false))
                             : (out16 ? HSG_FW(HSG_TAU_PER_EDGE, true) : HSG_FW(HSG_TAU_PER_EDGE, false)));
#undef HSG_F4
#undef HSG_FW
    if (rc != 0 || !wl || pin) return rc;
    HSG_KLAUNCH(false, true, k_gat_fwd_merge, dim3((unsigned)R.n_dwork), dim3(256), st, R, H, D, origin, pws, h, out,
                m, l, out16, ld16);
    return launch_status();
}

int hsg_gat_fwd_ws(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                   const float *sigma, const float *tau, const float *origin, float *h, float *out, float *m,
                   float *l, float *ws, void *stream) {
    return gat_fwd_impl(rel, H, D, tau_mode, slope, Z, sigma, tau, origin, h, out, m, l, ws, nullptr, 0, stream);
}

int hsg_gat_fwd_ws16(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                     const float *sigma, const float *tau, const float *origin, float *h, float *out, float *m,
                     float *l, float *ws, void *out16, int ld16, void *stream) {
    if (!out16) return HSG_EINVAL;
    return gat_fwd_impl(rel, H, D, tau_mode, slope, Z, sigma, tau, origin, h, out, m, l, ws,
                        reinterpret_cast<__bf16 *>(out16), ld16, stream);
}

int hsg_gat_bwd_blocks(const hsg_rel *rel) {
    if (!rel) return 0;
    int cap = kBwdDstGridCap;
    if (const char *e = HSG_DEV_ENV("HSG_GAT_BWD_CAP")) cap = atoi(e) > 0 ? atoi(e) : cap;   // dev sweep
    return grid_nodes(rel->n_dst, dst_wpn(rel), cap);
}

int hsg_gat_bwd_dst(const hsg_rel *rel, int H, int D, int tau_mode, int origin_mode, float slope,
                    const float *Z, const float *sigma, const float *tau, const float *h,
                    const float *m, const float *l, const float *dout, float *G, float *dpre,
                    float *dtau_part, void *stream) {
    if (!rel || !shape_ok(H, D)) return HSG_EINVAL;
    if (tau_mode != HSG_TAU_TABLE && tau_mode != HSG_TAU_PER_EDGE) return HSG_EINVAL;
    const int lph = lanes_per_head(H);
    const RelPtrs R = rel_ptrs(rel);
    const dim3 grid(hsg_gat_bwd_blocks(rel));
    hipStream_t st = (hipStream_t)stream;
    if (rel->n_dst == 0) {
        if (tau_mode == HSG_TAU_TABLE && dtau_part)
            return (int)hipMemsetAsync(dtau_part, 0, sizeof(float) * HSG_NT * H * grid.x, st);
        return 0;
    }
    const int wpn = dst_wpn(rel);
    if (D <= 16) {                       // edge-parallel: whole G_v,k per lane
#define HSG_E(TAU, W) bwd_dst_ep_dispatch<TAU, W>(D, grid, st, R, H, lph, origin_mode, slope, Z, sigma, tau, h, \
                                                  m, l, dout, G, dpre, dtau_part)
        if (tau_mode == HSG_TAU_TABLE) return wpn == 4 ? HSG_E(HSG_TAU_TABLE, 4) : HSG_E(HSG_TAU_TABLE, 1);
        return wpn == 4 ? HSG_E(HSG_TAU_PER_EDGE, 4) : HSG_E(HSG_TAU_PER_EDGE, 1);
#undef HSG_E
    }
    // feature-split variant (one wave per destination; with long segments it runs on
    // the same grid as above, the d tau slab's row count, with some idle waves)
    const int ne = ne_bucket((D + lph - 1) / lph);
    if (ne < 0) return HSG_EINVAL;
#ifdef HSG_DEV
    if (!bwd_occ()) {
        if (tau_mode == HSG_TAU_TABLE)
            return bwd_dst_dispatch<HSG_TAU_TABLE>(ne, grid, st, R, H, D, lph, origin_mode, slope, Z, sigma,
                                                   tau, h, m, l, dout, G, dpre, dtau_part);
        return bwd_dst_dispatch<HSG_TAU_PER_EDGE>(ne, grid, st, R, H, D, lph, origin_mode, slope, Z,
                                                  sigma, tau, h, m, l, dout, G, dpre, dtau_part);
    }
#endif
    if (tau_mode == HSG_TAU_TABLE)
        return bwd_dst_dispatch<HSG_TAU_TABLE, 6>(ne, grid, st, R, H, D, lph, origin_mode, slope, Z, sigma,
                                                  tau, h, m, l, dout, G, dpre, dtau_part);
    return bwd_dst_dispatch<HSG_TAU_PER_EDGE, 6>(ne, grid, st, R, H, D, lph, origin_mode, slope, Z,
                                                 sigma, tau, h, m, l, dout, G, dpre, dtau_part);
}

int hsg_gat_bwd_dst_noh_supported(const hsg_rel *rel, int H, int D) {
    if (!rel || !shape_ok(H, D) || D <= 16 || dst_wpn(rel) != 1) return 0;
    const int ne = ne_bucket((D + lanes_per_head(H) - 1) / lanes_per_head(H));
    return (ne >= 4 && ne <= 8) || ne == 16;
}

int hsg_gat_bwd_dst_noh(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                        const float *sigma, const float *tau, const float *x, const float *origin,
                        const float *m, const float *l, const float *dout, float *G, float *dpre,
                        float *dtau_part, void *stream) {
    if (!hsg_gat_bwd_dst_noh_supported(rel, H, D) || !x || !origin) return HSG_EINVAL;
    if (tau_mode != HSG_TAU_TABLE && tau_mode != HSG_TAU_PER_EDGE) return HSG_EINVAL;
    const int lph = lanes_per_head(H);
    const RelPtrs R = rel_ptrs(rel);
    const dim3 grid(hsg_gat_bwd_blocks(rel));
    hipStream_t st = (hipStream_t)stream;
    if (rel->n_dst == 0) {
        if (tau_mode == HSG_TAU_TABLE && dtau_part)
            return (int)hipMemsetAsync(dtau_part, 0, sizeof(float) * HSG_NT * H * grid.x, st);
        return 0;
    }
    const int ne = ne_bucket((D + lph - 1) / lph);
#ifdef HSG_DEV
    const char *oe = HSG_DEV_ENV("HSG_GAT_NOH_OCC");                      // dev A/B
    if (oe && atoi(oe) == 5 && tau_mode == HSG_TAU_TABLE)
        return bwd_dst_dispatch<HSG_TAU_TABLE, 5, true>(ne, grid, st, R, H, D, lph, 1, slope, Z, sigma, tau,
                                                        nullptr, m, l, dout, G, dpre, dtau_part, x, origin);
#endif
    if (tau_mode == HSG_TAU_TABLE)
        return bwd_dst_dispatch<HSG_TAU_TABLE, 6, true>(ne, grid, st, R, H, D, lph, 1, slope, Z, sigma, tau,
                                                        nullptr, m, l, dout, G, dpre, dtau_part, x, origin);
    return bwd_dst_dispatch<HSG_TAU_PER_EDGE, 6, true>(ne, grid, st, R, H, D, lph, 1, slope, Z, sigma, tau,
                                                       nullptr, m, l, dout, G, dpre, dtau_part, x, origin);
}

int hsg_gat_bwd_dst_g(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *Z,
                      const float *sigma, const float *tau, const float *m, const float *l, const float *G,
                      float *dpre, float *dtau_part, void *stream) {
    if (!hsg_gat_bwd_dst_noh_supported(rel, H, D) || !G) return HSG_EINVAL;
    if (tau_mode != HSG_TAU_TABLE && tau_mode != HSG_TAU_PER_EDGE) return HSG_EINVAL;
    const int lph = lanes_per_head(H);
    const RelPtrs R = rel_ptrs(rel);
    const dim3 grid(hsg_gat_bwd_blocks(rel));
    hipStream_t st = (hipStream_t)stream;
    if (rel->n_dst == 0) {
        if (tau_mode == HSG_TAU_TABLE && dtau_part)
            return (int)hipMemsetAsync(dtau_part, 0, sizeof(float) * HSG_NT * H * grid.x, st);
        return 0;
    }
    const int ne = ne_bucket((D + lph - 1) / lph);
    float *Gw = const_cast<float *>(G);                 // read only (GIN)
    if (tau_mode == HSG_TAU_TABLE)
        return bwd_dst_dispatch<HSG_TAU_TABLE, 6, true, true>(ne, grid, st, R, H, D, lph, 1, slope, Z, sigma, tau,
                                                              nullptr, m, l, nullptr, Gw, dpre, dtau_part);
    return bwd_dst_dispatch<HSG_TAU_PER_EDGE, 6, true, true>(ne, grid, st, R, H, D, lph, 1, slope, Z, sigma, tau,
                                                             nullptr, m, l, nullptr, Gw, dpre, dtau_part);
}

int hsg_gat_bwd_src_blocks(const hsg_rel *rel) {
    if (!rel) return 0;
    return grid_nodes(rel->n_src, src_wpn(rel), kBwdSrcGridCap);
}

int hsg_gat_bwd_src(const hsg_rel *rel, int H, int D, int tau_mode, float slope, const float *sigma,
                    const float *tau, const float *m, const float *l, const float *G,
                    const float *dpre, const float *a1, const float *Z, float *dZ, float *dsigma,
                    float *da1_part, void *stream) {
    if (!rel || !shape_ok(H, D) || (da1_part && !Z)) return HSG_EINVAL;
    if (tau_mode != HSG_TAU_TABLE && tau_mode != HSG_TAU_PER_EDGE) return HSG_EINVAL;
    const RelPtrs R = rel_ptrs(rel);
    const int nf = (H * D + 63) / 64;
    const dim3 grid(hsg_gat_bwd_src_blocks(rel));
    hipStream_t st = (hipStream_t)stream;
    if (rel->n_src == 0) {
        if (da1_part) return (int)hipMemsetAsync(da1_part, 0, sizeof(float) * H * D * grid.x, st);
        return 0;
    }
    const int wpn = src_wpn(rel), lph = lanes_per_head(H);
    // narrow heads over short segments: the head-lane kernel (HSG_GAT_SRC_HL=0: off)
    const char *hl = HSG_DEV_ENV("HSG_GAT_SRC_HL");
    if (wpn == 1 && D == 8 && H <= 8 && !(hl && atoi(hl) == 0) && (((uintptr_t)G | (uintptr_t)dZ | (uintptr_t)Z |
                                                                 (uintptr_t)a1) & 15) == 0) {
        const int hp = next_pow2(H);
        if (tau_mode == HSG_TAU_TABLE)
            HSG_KLAUNCH(false, true, (k_gat_bwd_src_hl<8, HSG_TAU_TABLE>), grid, dim3(256), st, R, H, D, hp, slope,
                        sigma, tau, m, l, G, dpre, a1, Z, dZ, dsigma, da1_part, nullptr, nullptr);
        else
            HSG_KLAUNCH(false, true, (k_gat_bwd_src_hl<8, HSG_TAU_PER_EDGE>), grid, dim3(256), st, R, H, D, hp, slope,
                        sigma, tau, m, l, G, dpre, a1, Z, dZ, dsigma, da1_part, nullptr, nullptr);
        return launch_status();
    }
    if (wpn == 4 && bwd_occ()) {
        if (tau_mode == HSG_TAU_TABLE)
            return bwd_src_dispatch<HSG_TAU_TABLE, 4, 5>(nf, grid, st, R, H, D, lph, slope, sigma, tau, m, l, G,
                                                         dpre, a1, Z, dZ, dsigma, da1_part);
        return bwd_src_dispatch<HSG_TAU_PER_EDGE, 4, 5>(nf, grid, st, R, H, D, lph, slope, sigma, tau, m, l, G,
                                                        dpre, a1, Z, dZ, dsigma, da1_part);
    }
#define HSG_S(TAU, W) bwd_src_dispatch<TAU, W>(nf, grid, st, R, H, D, lph, slope, sigma, tau, m, l, G, dpre, a1, \
                                               Z, dZ, dsigma, da1_part)
#ifdef HSG_DEV
    if (wpn == 4) return tau_mode == HSG_TAU_TABLE ? HSG_S(HSG_TAU_TABLE, 4) : HSG_S(HSG_TAU_PER_EDGE, 4);
#endif
    if (tau_mode == HSG_TAU_TABLE) return HSG_S(HSG_TAU_TABLE, 1);      // wpn == 4 took the w = 5 kernel above
    return HSG_S(HSG_TAU_PER_EDGE, 1);
#undef HSG_S
}

// the two shapes of the one-pass edge backward: wide heads over long CSC segments
// (S2W; rho as 64-column-group partials) and D = 8 heads over short ones (W2S: the
// head-lane kernel; rho per head)
// the one-pass wide kernel splits each source's out-edges over a block's 4 waves; it
// takes any segment length, so it stands in for the dst + src pair from a mean CSC
// segment of 4 on (cfg5's 14 words per sentence ran the two-pass backward while the
// condition was the 16 of the 4-wave forward / dst passes: 42 vs ~17 us per S2W
// application)
bool srcg_wide(const hsg_rel *rel, int H, int D) {
    return D >= 32 && D <= 64 && rel->n_src > 0 && rel->n_edges >= 4 * rel->n_src &&
           (D + lanes_per_head(H) - 1) / lanes_per_head(H) <= 8;
}
bool srcg_narrow(const hsg_rel *rel, int H, int D) { return D == 8 && H <= 8 && src_wpn(rel) == 1; }

int hsg_gat_bwd_src_g_supported(const hsg_rel *rel, int H, int D) {
    if (!rel || !shape_ok(H, D)) return 0;
    return srcg_wide(rel, H, D) || srcg_narrow(rel, H, D);
}

int hsg_gat_bwd_src_g_blocks(const hsg_rel *rel, int H, int D) {
    if (!hsg_gat_bwd_src_g_supported(rel, H, D)) return 0;
    const char *e = HSG_DEV_ENV("HSG_SRCG_GRID");                         // dev A/B: 0 = the src grid
    if (srcg_narrow(rel, H, D) && !(e && atoi(e) == 0)) {
        // the head-lane kernel takes 64 / nextpow2(H) sources per wave: one block per 4
        // such wave groups (cfg2 W2S: 600 blocks of busy waves instead of 2,048 blocks of
        // which 70 % of the waves had no source -- and 600 partial rows to reduce)
        const int groups = (rel->n_src + 64 / next_pow2(H) - 1) / (64 / next_pow2(H));
        const int b = (groups + HSG_WAVES - 1) / HSG_WAVES;
        return b < 1 ? 1 : (b < kBwdSrcGridCap ? b : kBwdSrcGridCap);
    }
    // one source (or CSC work item, round 6) per block per iteration; the work-list grid
    // whether or not the caller passes the piece scratch (a larger grid only adds
    // partial rows of zeros), so the slabs are sized alike for both entry points
    const int items = rel->swork && rel->n_swork > 0 ? rel->n_swork : rel->n_src;
    return grid_nodes(items, 4, kBwdSrcGridCap);
}

size_t hsg_gat_bwd_src_g_ws_floats(const hsg_rel *rel, int H, int D) {
    if (!hsg_gat_bwd_src_g_supported(rel, H, D) || !srcg_wide(rel, H, D) || !rel->swork || rel->n_swork <= 0)
        return 0;
    return (size_t)rel->n_swork * (size_t)(H * D + H);
}

// the wide one-pass kernel on bf16 G rows (the bf16 GEMM mode): g_bf16 != 0 needs the
// wide form (rho_groups > 0); HSG_EINVAL otherwise
int hsg_gat_bwd_src_g_io(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                         const float *m, const float *l, const void *G, int g_bf16, const float *rho, int rho_groups,
                         const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                         float *dtau_part, void *stream);

int hsg_gat_bwd_src_g(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                      const float *m, const float *l, const float *G, const float *rho, int rho_groups,
                      const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                      float *dtau_part, void *stream) {
    return hsg_gat_bwd_src_g_io(rel, H, D, slope, sigma, tau, m, l, G, 0, rho, rho_groups, a1, Z, dZ, dsigma,
                                da1_part, dtau_part, stream);
}

int hsg_gat_bwd_src_g_io(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                         const float *m, const float *l, const void *Gv, int g_bf16, const float *rho, int rho_groups,
                         const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                         float *dtau_part, void *stream) {
    return hsg_gat_bwd_src_g_ws(rel, H, D, slope, sigma, tau, m, l, Gv, g_bf16, rho, rho_groups, a1, Z, dZ, dsigma,
                                da1_part, dtau_part, nullptr, stream);
}

int hsg_gat_bwd_src_g_ws(const hsg_rel *rel, int H, int D, float slope, const float *sigma, const float *tau,
                         const float *m, const float *l, const void *Gv, int g_bf16, const float *rho, int rho_groups,
                         const float *a1, const float *Z, float *dZ, float *dsigma, float *da1_part,
                         float *dtau_part, float *ws, void *stream) {
    const float *G = reinterpret_cast<const float *>(Gv);
    if (g_bf16 && rho_groups == 0) return HSG_EINVAL;
    if (!hsg_gat_bwd_src_g_supported(rel, H, D) || !G || !rho || !Z || !dZ || !dtau_part) return HSG_EINVAL;
    const RelPtrs R = rel_ptrs(rel);
    const dim3 grid(hsg_gat_bwd_src_g_blocks(rel, H, D));
    hipStream_t st = (hipStream_t)stream;
    if (rho_groups == 0) {                   // per-head rho: the narrow head-lane kernel
        if (!srcg_narrow(rel, H, D) || ((uintptr_t)G | (uintptr_t)dZ | (uintptr_t)Z | (uintptr_t)a1) & 15)
            return HSG_EINVAL;
        if (rel->n_src == 0) {
            if (da1_part && hipMemsetAsync(da1_part, 0, sizeof(float) * H * D * grid.x, st) != hipSuccess)
                return HSG_EINVAL;
            return (int)hipMemsetAsync(dtau_part, 0, sizeof(float) * HSG_NT * H * grid.x, st);
        }
#ifdef HSG_DEV
        if (launch_floor_mode() == 2) {                         // dev probe: the W2S backward's grid, no work
            HSG_KLAUNCH(true, true, k_launch_floor, grid, dim3(256), st, rel->cindptr, rel->n_src, (int32_t *)nullptr);
            return launch_status();
        }
#endif
        HSG_KLAUNCH(true, true, (k_gat_bwd_src_hl<8, HSG_TAU_TABLE, true>), grid, dim3(256), st, R, H, D,
                    next_pow2(H), slope, sigma, tau, m, l, G, nullptr, a1, Z, dZ, dsigma, da1_part, rho, dtau_part);
        return launch_status();
    }
    // the group width of the rho partials (hsg_gemm_psw_elug_rho_gw): 64, or 112 (the dx
    // GEMM's 112-wide tiles), told apart by the count: the GEMM picks 112 only where the
    // counts differ (elug_gw), and where they are equal (H*D <= 64: one group, the same
    // layout; 113..128: 64 by that rule) 64 is the layout written
    const int rgw = rho_groups == (H * D + 63) / 64 ? 64 : rho_groups == (H * D + 111) / 112 ? 112 : 0;
    if (!srcg_wide(rel, H, D) || rgw == 0 || D > rgw) return HSG_EINVAL;
    const int lph = lanes_per_head(H), ne = (D + lph - 1) / lph;
    // the CSC work list with its scratch: pieces of the long sources, merged below (round 6)
    const bool wl = ws && R.n_swork > 0;
    float *pws = wl ? ws : nullptr;
    // the backward's pieces: a second launch merges them by default (the in-kernel
    // hand-off cost its kernel two spills and the fences: 31.0 vs 25.0 + 5.0 us per cfg4
    // application, profiles/r06/ab_piece_inline_cfg4/); dev HSG_PIECE_INLINE=3: in-kernel
    const int pin = piece_inline() >= 2 ? 1 : 0;
#define HSG_SG1(NE_, OCC_, EQ_, GBF_, WL_, PIN_)                                                             \
    HSG_KLAUNCH(true, !wl || pin, (k_gat_bwd_src_g<NE_, OCC_, EQ_, GBF_, WL_, PIN_>), grid, dim3(256), st, R, H, \
                D, lph, slope, sigma, tau, m, l, G, rho, rho_groups, rgw, a1, Z, dZ, dsigma, da1_part, dtau_part,  \
                pws, pin)
#ifdef HSG_DEV
#define HSG_SGW(NE_, OCC_, EQ_, GBF_)                                                                        \
    do {                                                                                                     \
        if (pin) HSG_SG1(NE_, OCC_, EQ_, GBF_, true, true);                                                  \
        else HSG_SG1(NE_, OCC_, EQ_, GBF_, true, false);                                                     \
    } while (0)
#else
#define HSG_SGW(NE_, OCC_, EQ_, GBF_) HSG_SG1(NE_, OCC_, EQ_, GBF_, true, false)
#endif
#define HSG_SG(NE_, OCC_, EQ_)                                                                               \
    do {                                                                                                     \
        if (g_bf16) {                                                                                        \
            if (wl) HSG_SGW(NE_, OCC_, EQ_, true);                                                           \
            else HSG_SG1(NE_, OCC_, EQ_, true, false, false);                                                \
        } else {                                                                                             \
            if (wl) HSG_SGW(NE_, OCC_, EQ_, false);                                                          \
            else HSG_SG1(NE_, OCC_, EQ_, false, false, false);                                               \
        }                                                                                                    \
    } while (0)
    // EQ: destination rows in flight per wave, as many as fit 5 blocks per CU unspilled
#ifdef HSG_DEV
    const char *eq = HSG_DEV_ENV("HSG_SRCG_EQ");                               // dev A/B
    if (eq && atoi(eq) == 4 && ne > 4 && ne <= 7) HSG_SG(7, 4, 4);
    else if (eq && atoi(eq) == 1 && ne > 4 && ne <= 7) HSG_SG(7, 5, 1);
    else
#endif
    if (ne <= 4) HSG_SG(4, 5, 4);
    else if (ne <= 7) HSG_SG(7, 5, 2);
    else HSG_SG(8, 5, 1);
#undef HSG_SG
#undef HSG_SGW
#undef HSG_SG1
    const int rc = launch_status();
    if (rc != 0 || !wl || pin) return rc;
    HSG_KLAUNCH(false, true, k_gat_bwd_src_g_merge, dim3((unsigned)R.n_swork), dim3(256), st, R, H, D, pws, a1, dZ,
                dsigma);
    return launch_status();
}

int hsg_attn_src_logits(int n, int H, int D, const float *Z, const float *a1, float *sigma,
                        void *stream) {
    if (!shape_ok(H, D)) return HSG_EINVAL;
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_attn_src_logits, dim3(grid_for(n, kFwdGridCap)), dim3(256), 0,
                       (hipStream_t)stream, n, H, D, lanes_per_head(H), Z, a1, sigma);
    return launch_status();
}

int hsg_kclock_arm(void *stream, void *start_event, void *stop_event) {
    t_kc.stream = (hipStream_t)stream;
    t_kc.start = (hipEvent_t)start_event;
    t_kc.stop = (hipEvent_t)stop_event;
    return 0;
}

int hsg_kclock_pending(void) { return (t_kc.start ? 1 : 0) + (t_kc.stop ? 2 : 0); }

#ifdef HSG_DEV
const char *hsg_version(void) { return "hsg 0.1 gfx950 (fp32 WSWGAT edge kernels) dev"; }
#else
const char *hsg_version(void) { return "hsg 0.1 gfx950 (fp32 WSWGAT edge kernels)"; }
#endif

}  // extern "C"
