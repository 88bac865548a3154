// hsg_hproj.hip -- head projection with per-head input dropout, for gfx950.
//
// Reference (module/GATStackLayer.py:56, GATLayer.py:110/146): in training, every
// head k sees its own dropout of the layer input,  z_k = fc_k(dropout(h)).  Done
// literally that is H copies of the [n, in] input (PyTorch: 8 x 19,200 x 300 for
// W2S) and a batched GEMM.  Here:
//   hsg_dropmask   writes the H keep-masks once as bits, 32 rows per word, words
//                  contiguous along the input column:
//                    bits[(k*NWI + i/32)*LDC + c] bit (i%32) = keep(i, k, c)
//                  NWI = ceil(n/32), LDC = in rounded up to 4 (0.7 MB for W2S)
//   hsg_hproj_fwd  Z[i, kD+d] = s * sum_c bit(i,k,c) X[i,c] W[kD+d, c]
//   hsg_hproj_dx   dX[i, c]   = s * sum_k bit(i,k,c) sum_d dZ[i,kD+d] W[kD+d, c]
//   hsg_hproj_dw   dW[kD+d,c] = s * sum_i dZ[i,kD+d] bit(i,k,c) X[i,c]
// All three are f32 MFMA kernels.  The mask changes with the head, so a head's
// outputs form their own tile ("slot" = up to 16 (fwd/dw) or DP (dx) outputs of
// one head); the mask is applied to the MFMA operand that carries (i, c) (fwd,
// dw) or to the per-head product before it is accumulated (dx).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/hsg.h"
#include "hsg_dev.h"

#ifdef HSG_DEV
#define HSG_PF_DEV 1
#else
#define HSG_PF_DEV 0
#endif
#include "hsg_rng.h"
#include "hsg_wsplit.h"

namespace {

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t lowbias32(uint32_t x) { return hsg_lowbias32(x); }

// 16-bit uniforms, two heads per hash: drop probability resolution 2^-16.
__device__ __forceinline__ uint32_t thr16(float p) {
    const float t = p * 65536.f;
    return t >= 65535.f ? 65535u : (uint32_t)t;
}

__host__ __device__ __forceinline__ int mask_ldc(int in) { return (in + 3) & ~3; }

// Buffer loads: an offset past the descriptor's byte count reads 0, so edge
// handling is a select on the OFFSET (kOOB) and the load itself is unconditional
// -- a select on a loaded value lets the compiler sink the load into a branch and
// serialise it.  Descriptors are built from kernel arguments (wave-uniform).
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
constexpr uint32_t kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, long bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float bld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ uint32_t bldu(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0);
}
__device__ __forceinline__ u32x4v bld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
}

// one thread = (head pair, 32-row word, column c); c fastest so stores coalesce.
// Columns in [in, LDC) get zero words.  The thread's 64 16-bit uniforms (32 rows
// x 2 heads) come from one lowbias32 hash of (key, word index) that seeds a
// xorshift64 stream (shifts and xors only: 32-bit integer multiplies run at a
// quarter of the VALU rate on CDNA, and one hash per word instead of per row
// removes most of them), read bit-sliced: 16 steps give the 16 bit planes of both
// heads' 32 uniforms, compared against the threshold with two or three logic ops
// per plane instead of a compare and a shift per row.
__device__ __forceinline__ uint32_t drop_key(const int64_t *seedp, uint32_t offset) {
    return hsg_drop_key((uint64_t)seedp[0], offset);
}

// thread unit t of one mask: (head pair kp, 32-row word iw, column c), c fastest
__device__ __forceinline__ void dropmask_unit(int n, int in, int H, uint32_t thr, uint32_t key, long t,
                                              uint32_t *__restrict__ bits) {
    const uint32_t NWI = (uint32_t)(n + 31) / 32;
    const uint32_t LDC = (uint32_t)mask_ldc(in);
    const uint32_t tu = (uint32_t)t;                   // < 2^31 (host-checked sizes): 32-bit division
    const int c = (int)(tu % LDC);
    const uint32_t r = tu / LDC;
    const int iw = (int)(r % NWI);
    const int kp = (int)(r / NWI);
    uint32_t b0 = 0, b1 = 0;
    if (c < in) {
        const uint32_t w = (uint32_t)(((long)kp * NWI + iw) * in + c);
        uint64_t x = ((uint64_t)lowbias32(key ^ (w * 0x9E3779B1u)) << 32) |
                     lowbias32(key + 0x7F4A7C15u + w * 0x85EBCA6Bu);
        x |= 1ull;                                     // xorshift state must be non-zero
        const int jmax = min(32, n - iw * 32);
        // bit-sliced compare of the 32 rows' 16-bit uniforms against thr, most significant
        // bit first: bit j of the b-th word is bit b of row j's uniform (one xorshift64
        // step gives the b-th word of both heads); keep = u >= thr = gt | eq at the end
        uint32_t eq0 = 0xFFFFFFFFu, gt0 = 0u, eq1 = 0xFFFFFFFFu, gt1 = 0u;
#pragma unroll
        for (int b = 15; b >= 0; --b) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            const uint32_t r0 = (uint32_t)x, r1 = (uint32_t)(x >> 32);
            if ((thr >> b) & 1u) {
                eq0 &= r0;
                eq1 &= r1;
            } else {
                gt0 |= eq0 & r0;
                eq0 &= ~r0;
                gt1 |= eq1 & r1;
                eq1 &= ~r1;
            }
            // every row of every lane decided (no eq bit left): the lower planes cannot
            // change gt | eq, so the wave stops drawing them (bitwise the same masks;
            // ~12 of 16 planes on average for the 4,096 row bits of a wave)
            if (b > 0 && !__any((eq0 | eq1) != 0u)) break;
        }
        const uint32_t rows = jmax >= 32 ? 0xFFFFFFFFu : ((1u << jmax) - 1u);
        b0 = (gt0 | eq0) & rows;
        b1 = (gt1 | eq1) & rows;
    }
    const int k0 = 2 * kp;
    bits[((long)k0 * NWI + iw) * LDC + c] = b0;
    if (k0 + 1 < H) bits[((long)(k0 + 1) * NWI + iw) * LDC + c] = b1;
}

__global__ __launch_bounds__(256) void k_dropmask(int n, int in, int H, float p, const int64_t *seedp,
                                                  uint32_t offset, uint32_t *__restrict__ bits) {
    const uint32_t key = drop_key(seedp, offset), thr = thr16(p);
    const long total = (long)((H + 1) / 2) * ((n + 31) / 32) * mask_ldc(in);
    for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x)
        dropmask_unit(n, in, H, thr, key, t, bits);
}

// Several masks (e.g. every head projection of one fused-stack forward) in one
// launch: job q owns blocks [start[q], start[q+1]), the same units and bits as
// hsg_dropmask(n[q], in[q], H[q], p[q], seed, offset[q], bits[q]).
struct DropJobs {
    int n[8], in[8], H[8];
    float p[8];
    uint32_t offset[8];
    uint32_t *bits[8];
    int start[9];
    int njobs;
    int upt;                                         // units per thread (blocks of 256 * upt units)
    // optional: the narrow-head projection's weight transpose (hsg_hproj_wt) in the
    // blocks after the masks' (W == nullptr: none)
    const float *W;
    float *Wt;
    int wH, wD, wIn;
    // optional: the wide FFN's weight limb planes (hsg_wsplit) in the blocks after those
    HsgWSplitJobs ws;
    int ws_first;                                    // first block of the split
};

// The step's dropout seed: seed += 1 and the backward-stable snapshot of the new value
// in one launch (was an in-place add plus a clone: two graph nodes).
__global__ __launch_bounds__(64) void k_seed_advance(int64_t *seed, int64_t *snap) {
    if (threadIdx.x == 0) {
        const int64_t s = seed[0] + 1;
        seed[0] = s;
        snap[0] = s;
    }
}

__device__ __forceinline__ void hproj_wt_block(int k, int c0, int D, int in, const float *__restrict__ W,
                                               float *__restrict__ Wt) {
    for (int e = threadIdx.x; e < 64 * D; e += 256) {
        const int d = e >> 6, c = c0 + (e & 63);
        if (c < in) Wt[((size_t)k * in + c) * D + d] = W[((size_t)k * D + d) * in + c];
    }
}

__global__ __launch_bounds__(256) void k_dropmask_multi(DropJobs j, const int64_t *seedp) {
    if ((int)blockIdx.x >= j.ws_first) {                // the weight limb split blocks
        hsg_wsplit_block(j.ws, (int)blockIdx.x - j.ws_first);
        return;
    }
    if ((int)blockIdx.x >= j.start[j.njobs]) {          // the weight-transpose blocks
        const int b = (int)blockIdx.x - j.start[j.njobs], nct = (j.wIn + 63) / 64;
        hproj_wt_block(b / nct, (b % nct) * 64, j.wD, j.wIn, j.W, j.Wt);
        return;
    }
    int q = 0;
    while (q + 1 < j.njobs && (int)blockIdx.x >= j.start[q + 1]) ++q;
    // upt units per thread (256 apart: each pass stays coalesced), so the per-wave
    // prologue -- the job search, the seed load, the key -- is paid once per upt units
    const long t0 = (long)((int)blockIdx.x - j.start[q]) * 256 * j.upt + threadIdx.x;
    const long total = (long)((j.H[q] + 1) / 2) * ((j.n[q] + 31) / 32) * mask_ldc(j.in[q]);
    if (t0 >= total) return;
    const uint32_t thr = thr16(j.p[q]), key = drop_key(seedp, j.offset[q]);
    for (int u = 0; u < j.upt; ++u) {
        const long t = t0 + 256L * u;
        if (t >= total) break;
        dropmask_unit(j.n[q], j.in[q], j.H[q], thr, key, t, j.bits[q]);
    }
}

// ---------------------------------------------------------------- forward ----
// v_mfma_f32_16x16x4_f32, no LDS.  One wave = one 16-row tile x SG slots (slot =
// 16 outputs [d0, d0+16) of head k, zero-padded past D).  The reduction index c
// is assigned so that every operand load is a 16-byte vector: in the 16-column
// chunk at c0, lane (li = l&15, lk = l>>4) holds columns c0+4lk .. c0+4lk+3 and
// feeds them to 4 consecutive MFMAs:
//   A[i = li][kk] = bit(i, k, c) X[i0+li, c]      (X float4, mask uint4)
//   B[kk][j = li] = W[kD + d0 + li, c]             (W row float4)
// Loads for chunk t+1 are issued before the MFMAs of chunk t.  All loads are
// unconditional from clamped addresses followed by a select, so the compiler can
// keep them in flight together.  VEC: in % 4 == 0 and 16-byte aligned rows.
// Optional fused epilogue (a1 != nullptr): the source logits of the attention,
// sigma[i, k] = <Z[i, kD:(k+1)D], a1_k> (module/GATLayer.py:91-92 / 130-131, the
// hsg_attn_src_logits of the split path), from the Z values just stored: per slot a
// 16-lane butterfly over the slot's columns, then the wave's slots of one head are
// added in slot order.  Needs every head's slots inside one wave's slot group
// (SG % SPH == 0, checked by the host).
template <int SG, bool VEC, int PF = 1>
__global__ __launch_bounds__(256) void k_hproj_fwd(int n, int in, int H, int D, const float *__restrict__ X,
                                                   int ldx, const float *__restrict__ W,
                                                   const uint32_t *__restrict__ bits, float scale,
                                                   float *__restrict__ Z, int ldz, const float *__restrict__ a1,
                                                   float *__restrict__ sigma) {
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int SPH = (D + 15) / 16, NS = H * SPH, NG = (NS + SG - 1) / SG;
    const int lane = threadIdx.x & 63;
    const int task = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int rt = task / NG, gq = task - rt * NG;
    const int i0 = rt * 16;
    if (i0 >= n) return;                          // whole wave: no barriers in this kernel
    const int li = lane & 15, lk = lane >> 4;
    const int i = i0 + li;
    const int ibit = i & 31;
    const auto rX = rsrc(X, (long)n * ldx * 4);
    const auto rW = rsrc(W, (long)H * D * in * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    const uint32_t xbase = i < n ? (uint32_t)i * ldx * 4 : kOOB;
    uint32_t wbase[SG], mbase[SG];
#pragma unroll
    for (int q = 0; q < SG; ++q) {
        const int slot = gq * SG + q;
        const int k = min(slot, NS - 1) / SPH;
        const int j = (min(slot, NS - 1) - k * SPH) * 16 + li;
        wbase[q] = (slot < NS && j < D) ? (uint32_t)(k * D + j) * in * 4 : kOOB;
        mbase[q] = (uint32_t)((k * NWI + i0 / 32) * LDC) * 4;
    }
    // operand quads for the 16-column chunk whose lane columns start at c
    auto load4 = [&](__amdgpu_buffer_rsrc_t r, uint32_t base, int c) -> f32x4v {
        if (VEC) {
            const u32x4v v = bld4(r, (c < in && base != kOOB) ? base + c * 4 : kOOB);
            return f32x4v{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
        }
        f32x4v v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = bld(r, (c + e < in && base != kOOB) ? base + (c + e) * 4 : kOOB);
        return v;
    };
    auto loadm = [&](uint32_t base, int c) -> u32x4v { return bld4(rM, c < LDC ? base + c * 4 : kOOB); };
    f32x4v acc[SG];
#pragma unroll
    for (int q = 0; q < SG; ++q) acc[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
    // PF-deep register ring of 16-column chunks: chunk t+PF is requested as soon as
    // chunk t's MFMAs are issued, so PF chunks of X / W / mask are in flight per wave
    f32x4v xv[PF], wv[PF][SG];
    u32x4v mv[PF][SG];
    auto fetch = [&](int u, int cc) {
        xv[u] = load4(rX, xbase, cc);
#pragma unroll
        for (int q = 0; q < SG; ++q) {
            wv[u][q] = load4(rW, wbase[q], cc);
            mv[u][q] = loadm(mbase[q], cc);
        }
    };
#pragma unroll
    for (int u = 0; u < PF; ++u) {
        fetch(u, 4 * lk + 16 * u);
        if constexpr (PF > 1) __builtin_amdgcn_sched_barrier(0);   // issue order = slot order
    }
    // whole rings only (chunks past `in` read zeros): a break inside the ring makes the
    // compiler wait vmcnt(0) at the loop head and the ring collapses to depth 1
    const int in_pad = (in + 16 * PF - 1) / (16 * PF) * (16 * PF);
    for (int c0 = 0; c0 < in_pad; c0 += 16 * PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
#pragma unroll
            for (int q = 0; q < SG; ++q) {             // slots past NS carry zero W
                acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(((mv[u][q].x >> ibit) & 1u) ? xv[u][0] : 0.f,
                                                              wv[u][q][0], acc[q], 0, 0, 0);
                acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(((mv[u][q].y >> ibit) & 1u) ? xv[u][1] : 0.f,
                                                              wv[u][q][1], acc[q], 0, 0, 0);
                acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(((mv[u][q].z >> ibit) & 1u) ? xv[u][2] : 0.f,
                                                              wv[u][q][2], acc[q], 0, 0, 0);
                acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(((mv[u][q].w >> ibit) & 1u) ? xv[u][3] : 0.f,
                                                              wv[u][q][3], acc[q], 0, 0, 0);
            }
            fetch(u, c0 + 16 * (u + PF) + 4 * lk);     // past `in`: OOB offsets read 0
            // keep the next slot's mask / operand work out of this step: hoisted, it
            // makes the loop head wait for every load of the ring (vmcnt(0))
            if constexpr (PF > 1) __builtin_amdgcn_sched_barrier(0);
        }
    }
    // D layout: col = lane & 15 (slot output j), row = (lane >> 4) * 4 + r
#pragma unroll
    for (int q = 0; q < SG; ++q) {
        const int slot = gq * SG + q;
        if (slot >= NS) continue;
        const int k = slot / SPH;
        const int j = (slot - k * SPH) * 16 + li;
        if (j >= D) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int gi = i0 + lk * 4 + r;
            if (gi < n) Z[(long)gi * ldz + k * D + j] = acc[q][r] * scale;
        }
    }
    if (a1) {
        float sg[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < SG; ++q) {
            const int slot = gq * SG + q;                    // wave-uniform
            if (slot >= NS) break;
            const int k = slot / SPH;
            const int j = (slot - k * SPH) * 16 + li;
            const float a = j < D ? a1[k * D + j] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = (acc[q][r] * scale) * a;
                v += __shfl_xor(v, 1);
                v += __shfl_xor(v, 2);
                v += __shfl_xor(v, 4);
                v += __shfl_xor(v, 8);
                sg[r] += v;
            }
            if ((slot + 1) % SPH == 0) {                     // last slot of head k
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int gi = i0 + lk * 4 + r;
                    if (li == 0 && gi < n) sigma[(long)gi * H + k] = sg[r];
                    sg[r] = 0.f;
                }
            }
        }
    }
}

// ----------------------------------------------------- forward, narrow heads ----
// VALU form for D = 8 (the W2S projection, 8 heads x 8): the 16x16x4 MFMA pads a
// head's 8 outputs to 16 columns, so its floor is twice the f32 FLOP floor.  One
// wave = 64 rows (one per lane) x one head x one K part.  The head's weights come
// transposed, Wt[k][c][d] (hsg_hproj_wt, once per forward), so W[kD+d, c..c+3] is 32
// contiguous wave-uniform floats (two s_load_dwordx16 per quad of columns) and each
// fmaf takes its weight as the SGPR operand.  The keep bit is one v_bfe_i32 + v_and
// on the X value.  The block (HB heads x KS K parts of one 64-row tile) stages X
// and the keep words through LDS, 32 columns per part per step (coalesced loads;
// lanes walking their own rows straight from memory thrash L1: 64 lines per load),
// the next step's loads in flight during this one.  K parts are added in part order
// through LDS (deterministic).  Blocks of one row tile sit on one XCD (block b runs
// on XCD b % 8), so their X rows are L2 hits.
// cfg2 W2S shape, rocprofv3: 22.7 us in-step against 32 us for the MFMA kernel
// (the staging alone, no FMA work: 5.2 us).
// Wt[k][c][d] = W[kD+d][c]: block (c-tile of 64, head k); thread (c, d) pairs, reads
// coalesced along c, 32-bit index arithmetic only.
__global__ __launch_bounds__(256) void k_hproj_wt(int H, int D, int in, const float *__restrict__ W,
                                                  float *__restrict__ Wt) {
    hproj_wt_block(blockIdx.y, blockIdx.x * 64, D, in, W, Wt);
}

template <int HB, int KS>
__global__ __launch_bounds__(64 * HB * KS) void k_hproj_fwd_v8(int n, int in, int H, const float *__restrict__ X,
                                                              int ldx, const float *__restrict__ Wt,
                                                              const uint32_t *__restrict__ bits, float scale,
                                                              float *__restrict__ Z, int ldz,
                                                              const float *__restrict__ a1,
                                                              float *__restrict__ sigma) {
    constexpr int D = 8, T = 64 * HB * KS, NS = KS * 512 / T, RS = 36;
    static_assert(NS >= 1 && KS * 512 % T == 0, "staging split");
    __shared__ __attribute__((aligned(16))) float sX[KS][64][RS];     // 64 rows x 32 columns per part
    __shared__ __attribute__((aligned(16))) float s_part[KS > 1 ? (KS - 1) * HB : 1][64 * D];
    __shared__ __attribute__((aligned(16))) uint32_t sM[HB][KS][2][32];       // keep words of the step
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int nrt = (n + 63) / 64, bpr = (H + HB - 1) / HB;
    // XCD-aware block -> (row tile, head group)
    const int b = blockIdx.x, xcd = b & 7, idx = b >> 3;
    const int rt = (idx / bpr) * 8 + xcd, hg = idx % bpr;
    if (rt >= nrt) return;                                       // block-uniform
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kp = wv % KS, hb = wv / KS;
    const int k = hg * HB + hb;
    const bool kok = k < H;                                      // wave-uniform
    const int r0 = rt * 64, i = r0 + lane;
    const int sh = i & 31;
    const auto rX = rsrc(X, (long)n * ldx * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    const int nq = in / 4, pq0 = kp * nq / KS, pq1 = (kp + 1) * nq / KS;
    const int steps = ((nq + KS - 1) / KS + 7) / 8;
    // staging: thread unit e = (part p, row r, quad u) loads X[r0 + r][4 (p nq/KS + 8t + u) ..]
    uint32_t goff[NS];
    float *ldst[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int e = tid + T * s, p = e / 512, f = e % 512, r = f / 8, u = f % 8;
        goff[s] = r0 + r < n ? (uint32_t)((r0 + r) * ldx + 4 * (p * nq / KS + u)) * 4 : kOOB;
        ldst[s] = &sX[p][r][4 * u];
    }
    f32x4v sr[NS];
    auto stage_load = [&](int t) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const u32x4v v = bld4(rX, goff[s] + t * 128);        // past the row / buffer: unused / 0
            sr[s] = f32x4v{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
        }
    };
    // keep words: thread tid stages word (head hg*HB + mh, row group r0/32 + mg, column
    // 4 pq0(mp) + 32 t + mw) of every step: one word per thread
    const int mw = tid & 31, mg = (tid >> 5) & 1, mp = (tid >> 6) % KS, mh = tid / (64 * KS);
    const int mk = hg * HB + mh;
    const uint32_t moff = mk < H ? (uint32_t)(((mk * NWI + r0 / 32 + mg) * LDC + 4 * (mp * nq / KS) + mw) * 4) : kOOB;
    uint32_t mr = 0;
    auto mask_load = [&](int t) { mr = bldu(rM, moff != kOOB ? moff + t * 128 : kOOB); };
    // this head's W^T [in][8] (wave-uniform: 32 floats per quad, two s_load_dwordx16)
    const f32x16 *wt = reinterpret_cast<const f32x16 *>(Wt + (size_t)min(k, H - 1) * in * D);
    // two accumulator sets (even / odd quads): 16 independent fmaf chains.  Plain
    // v_fmac_f32 with the weight as the SGPR operand (this file is built with
    // -fno-slp-vectorize: a packed v_pk_fma_f32 issues slower than two v_fma_f32)
    float acc2[2][D];
#pragma unroll
    for (int d = 0; d < D; ++d) acc2[0][d] = acc2[1][d] = 0.f;
    auto quad = [&](f32x16 w0, f32x16 w1, f32x4v x, u32x4v m, float (&a)[D]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int keep = __builtin_amdgcn_sbfe((int)m[j], sh, 1);         // 0 or -1
            const float xm = __int_as_float(__float_as_int(x[j]) & keep);
#pragma unroll
            for (int d = 0; d < D; ++d) a[d] = fmaf(xm, j < 2 ? w0[(j & 1) * 8 + d] : w1[(j & 1) * 8 + d], a[d]);
        }
    };
    // one step: the staged chunk t -> LDS, chunk t+1 requested, then the 8 quads of
    // this wave's part: X rows (row = lane) read from LDS up front, W two quads at a
    // time (one scalar-load wait per pair), mask words loaded one step ahead
    auto run_step = [&](int t) {
        __syncthreads();                                         // previous step's LDS reads done
#pragma unroll
        for (int s = 0; s < NS; ++s) *reinterpret_cast<f32x4v *>(ldst[s]) = sr[s];
        sM[mh][mp][mg][mw] = mr;
        __syncthreads();
        if (t + 1 < steps) {
            stage_load(t + 1);
            mask_load(t + 1);
        }
        if (kok) {
#pragma unroll
            for (int u = 0; u < 8; u += 2) {
                const int q = pq0 + 8 * t + u;
                if (q >= pq1) break;
                const f32x4v x0 = *reinterpret_cast<const f32x4v *>(&sX[kp][lane][4 * u]);
                const f32x4v x1 = *reinterpret_cast<const f32x4v *>(&sX[kp][lane][4 * u + 4]);
                const u32x4v m0 = *reinterpret_cast<const u32x4v *>(&sM[hb][kp][lane >> 5][4 * u]);
                const u32x4v m1 = *reinterpret_cast<const u32x4v *>(&sM[hb][kp][lane >> 5][4 * u + 4]);
                const f32x16 w0 = wt[2 * q], w1 = wt[2 * q + 1];
                if (q + 1 < pq1) {
                    const f32x16 w2 = wt[2 * q + 2], w3 = wt[2 * q + 3];
                    quad(w0, w1, x0, m0, acc2[0]);
                    quad(w2, w3, x1, m1, acc2[1]);
                } else {
                    quad(w0, w1, x0, m0, acc2[0]);
                }
            }
        }
    };
    stage_load(0);
    mask_load(0);
    for (int t = 0; t < steps; ++t) run_step(t);
    float acc[D];
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = acc2[0][d] + acc2[1][d];
    if constexpr (KS > 1) {
        if (kp > 0) {
#pragma unroll
            for (int d = 0; d < D; ++d) s_part[(kp - 1) * HB + hb][d * 64 + lane] = acc[d];
        }
        __syncthreads();
        if (kp > 0) return;
#pragma unroll
        for (int p = 1; p < KS; ++p)
#pragma unroll
            for (int d = 0; d < D; ++d) acc[d] += s_part[(p - 1) * HB + hb][d * 64 + lane];
    }
    if (!kok || i >= n) return;
    float z[D];
#pragma unroll
    for (int d = 0; d < D; ++d) z[d] = acc[d] * scale;
    float *zr = Z + (size_t)i * ldz + k * D;
    *reinterpret_cast<f32x4v *>(zr) = f32x4v{z[0], z[1], z[2], z[3]};
    *reinterpret_cast<f32x4v *>(zr + 4) = f32x4v{z[4], z[5], z[6], z[7]};
    if (a1) {
        float sg = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) sg = fmaf(z[d], a1[k * D + d], sg);
        sigma[(size_t)i * H + k] = sg;
    }
}

// ------------------------------------------ forward on bf16 limb MFMAs (round 5) ----
// D = 8 (the W2S projection): the VALU form above runs 8 fmac + 2 mask ops per (row,
// column, head).  Here the products run on v_mfma_f32_16x16x32_bf16, fp32-accurate as
// the FFN GEMMs (three RNE bf16 limbs per operand, six products).  A head's 8 outputs
// take half of the 16 MFMA columns (the other half repeats them), because each head
// masks the A rows with its own keep bits.
// Block = one 32-row tile (one mask word per (head, column)) x all heads, wave w =
// heads 2w, 2w + 1, the whole K.  Per 32-column step the block stages, double-buffered
// in LDS with the next step's global loads in flight in registers: X split ONCE into
// three limb planes (each thread splits one float4), the 8 heads' mask words, and the
// W limb planes' 32-column slice (hsg_wsplit planes [3][Np][Kp], rows = outputs).  Per
// head a wave then builds the 16-bit lane masks of its A fragments from the 8 words of
// its columns (shifted so rows r and r + 16 sit at bits 15 / 31; v_perm_b32's sign-byte
// selectors make a bf16 pair's mask in one instruction), ANDs them into the limbs and
// runs 2 tiles x 6 MFMAs.  One barrier per step.  Epilogue: scale, Z, and the optional
// source logits sigma[i, k] = <Z[i, 8k:8k+8], a1_k> (an 8-lane butterfly).
__global__ __launch_bounds__(256) void k_hproj_fwd_mf(int n, int in, int H, const float *__restrict__ X, int ldx,
                                                     const __bf16 *__restrict__ Wp, int Np, int Kp,
                                                     const uint32_t *__restrict__ bits, float scale,
                                                     float *__restrict__ Z, int ldz, const float *__restrict__ a1,
                                                     float *__restrict__ sigma) {
    constexpr int HM = 8;                                     // heads per block (max), 2 per wave
    __shared__ __attribute__((aligned(16))) __bf16 sA[2][3][32 * 32];     // X limbs [row][col]
    __shared__ __attribute__((aligned(16))) uint32_t sM[2][HM][32];       // keep words [head][col]
    __shared__ __attribute__((aligned(16))) __bf16 sW[2][3][HM * 8 * 32]; // W limbs [out][col]
    // LDS swizzles (bf16 rows of 32 columns = four 16-byte chunks): chunk j of X-limb row
    // rr sits at j ^ hx(rr >> 2), of W-limb row o at j ^ 2 ((o >> 2) & 1), so that each
    // 16-lane group of a ds_read_b128 fragment read ({0-3, 12-15, 20-27}, ... on gfx950)
    // lands on 16 distinct 4-bank slots
    auto ax = [](int rr, int j) { return rr * 32 + 8 * (j ^ ((0x78 >> (2 * ((rr >> 2) & 3))) & 3)); };
    auto aw = [](int o, int j) { return o * 32 + 8 * (j ^ (2 * ((o >> 2) & 1))); };
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int rt = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int nst = Kp / 32;
    const auto rX = rsrc(X, (long)n * ldx * 4);
    const auto rW = rsrc(Wp, (long)3 * Np * Kp * 2);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    // staging units: X float4 (row xr, columns 4 xq..), mask word (head mk, column mc),
    // W 16-byte pieces (limb, output row, 8 columns): HW * 3 per thread
    const int xr = tid >> 3, xq = tid & 7;
    const uint32_t xo = rt * 32 + xr < n ? (uint32_t)(rt * 32 + xr) * ldx * 4 : kOOB;
    const int mk = tid >> 5, mc = tid & 31;
    const uint32_t mo = mk < H ? (uint32_t)((mk * NWI + rt) * LDC) * 4 : kOOB;
    const uint32_t plane = (uint32_t)Np * Kp * 2;
    // two steps of global loads in flight (register sets R = 0, 1 for even / odd steps)
    u32x4v rxs[2], rws[2][3];
    uint32_t rms[2] = {0u, 0u};
    auto gload = [&](int s, u32x4v &rx, uint32_t &rm, u32x4v (&rw)[3]) {
        const int c = 32 * s + 4 * xq;
        rx = bld4(rX, (xo == kOOB || c >= in) ? kOOB : xo + 4u * c);
        const int cm = 32 * s + mc;
        rm = bldu(rM, (mo == kOOB || cm >= LDC) ? kOOB : mo + 4u * cm);
#pragma unroll
        for (int i = 0; i < 3; ++i) {                             // piece u: limb u / 256, output (u / 4) % 64, 8 columns
            const int u = tid + 256 * i, l = u >> 8, o = (u >> 2) & 63, q = u & 3;
            rw[i] = bld4(rW, o < H * 8 ? l * plane + (uint32_t)o * Kp * 2 + 2u * (32 * s + 8 * q) : kOOB);
        }
    };
    auto lstore = [&](int b, const u32x4v &rx, uint32_t rm, const u32x4v (&rw)[3]) {
        typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
        u32x2v w0, w1, w2;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            unsigned x0, x1, x2;
            hsg_split_rne_pair(__uint_as_float(rx[2 * p]), __uint_as_float(rx[2 * p + 1]), x0, x1, x2);
            w0[p] = x0; w1[p] = x1; w2[p] = x2;
        }
        const int xa = ax(xr, xq >> 1) + 4 * (xq & 1);
        *reinterpret_cast<u32x2v *>(&sA[b][0][xa]) = w0;
        *reinterpret_cast<u32x2v *>(&sA[b][1][xa]) = w1;
        *reinterpret_cast<u32x2v *>(&sA[b][2][xa]) = w2;
        sM[b][mk][mc] = rm;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int u = tid + 256 * i, l = u >> 8, o = (u >> 2) & 63, q = u & 3;
            *reinterpret_cast<u32x4v *>(&sW[b][l][aw(o, q)]) = rw[i];
        }
    };
    f32x4v acc[2][2];                                             // [row tile][head of the wave]
#pragma unroll
    for (int f = 0; f < 2; ++f) acc[f][0] = acc[f][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int sh = 15 - r;                                        // bit r -> 15, bit r + 16 -> 31
    gload(0, rxs[0], rms[0], rws[0]);
    if (nst > 1) gload(1, rxs[1], rms[1], rws[1]);
    auto step = [&](int s, int b) {                              // b = s & 1 (compile-time in the caller)
        lstore(b, rxs[b], rms[b], rws[b]);
        __syncthreads();
        if (s + 2 < nst) gload(s + 2, rxs[b], rms[b], rws[b]);
        hsg_bf16x8_t a[2][3];
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int l = 0; l < 3; ++l)
                a[f][l] = *reinterpret_cast<const hsg_bf16x8_t *>(&sA[b][l][ax(16 * f + r, g)]);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int k = 2 * w + h;
            if (k >= H) break;                                    // wave-uniform
            const u32x4v m0 = *reinterpret_cast<const u32x4v *>(&sM[b][k][8 * g]);
            const u32x4v m1 = *reinterpret_cast<const u32x4v *>(&sM[b][k][8 * g + 4]);
            hsg_bf16x8_t bb[3];
#pragma unroll
            for (int l = 0; l < 3; ++l)
                bb[l] = *reinterpret_cast<const hsg_bf16x8_t *>(&sW[b][l][aw(k * 8 + (r & 7), g)]);
            const uint32_t wd[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
            hsg_u32x4_t M[2];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t t0 = wd[2 * q] << sh, t1 = wd[2 * q + 1] << sh;
                M[0][q] = __builtin_amdgcn_perm(t1, t0, 0x0A0A0808u);    // row r:      sign bytes of bit 15
                M[1][q] = __builtin_amdgcn_perm(t1, t0, 0x0B0B0909u);    // row r + 16: sign bytes of bit 31
            }
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const hsg_bf16x8_t x0 = __builtin_bit_cast(hsg_bf16x8_t, __builtin_bit_cast(hsg_u32x4_t, a[f][0]) & M[f]);
                const hsg_bf16x8_t x1 = __builtin_bit_cast(hsg_bf16x8_t, __builtin_bit_cast(hsg_u32x4_t, a[f][1]) & M[f]);
                const hsg_bf16x8_t x2 = __builtin_bit_cast(hsg_bf16x8_t, __builtin_bit_cast(hsg_u32x4_t, a[f][2]) & M[f]);
                f32x4v c = acc[f][h];                             // smallest limb products first
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x2, bb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, bb[1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, bb[2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x1, bb[0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, bb[1], c, 0, 0, 0);
                acc[f][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x0, bb[0], c, 0, 0, 0);
            }
        }
    };
    for (int s = 0; s < nst; s += 2) {
        step(s, 0);
        if (s + 1 < nst) step(s + 1, 1);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int k = 2 * w + h;
        if (k >= H) break;
        const float av = a1 ? a1[k * 8 + (r & 7)] : 0.f;
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = rt * 32 + 16 * f + 4 * g + e;
                const float z = acc[f][h][e] * scale;
                if (r < 8 && i < n) Z[(size_t)i * ldz + k * 8 + r] = z;
                if (a1) {
                    float sg = z * av;                            // lanes r = 0..7: one head's 8 outputs
                    sg += __shfl_xor(sg, 1);
                    sg += __shfl_xor(sg, 2);
                    sg += __shfl_xor(sg, 4);
                    if (r == 0 && i < n) sigma[(size_t)i * H + k] = sg;
                }
            }
    }
}

// ------------------------------------------------------------------ dX ----
// v_mfma_f32_16x16x4_f32, no LDS.  One wave = 16 rows x (16*CT) input columns.
// Per head k the K = D product  t = dZ[i0.., kD..kD+D) W[kD.., c..]  runs on MFMA
// (lane (li, lk) supplies d = 4s + lk), then is added to the running total under
// the head's mask:  tot += bit(i, k, c) ? t : 0.  HF heads are in flight at once
// (independent accumulator chains); the loads of step s+1 are issued before the
// MFMAs of step s.  Rows/columns past the edge read clamped addresses and are
// never stored.
template <int CT, int HF>
__global__ __launch_bounds__(256) void k_hproj_dx(int n, int in, int H, int D, const float *__restrict__ dZ,
                                                  int ldz, const float *__restrict__ W,
                                                  const uint32_t *__restrict__ bits, float scale,
                                                  float *__restrict__ dX, int ldx, int accumulate) {
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int nct = (in + 16 * CT - 1) / (16 * CT);
    const int task = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int rt = task / nct, ctile = task - rt * nct;
    const int i0 = rt * 16;
    if (i0 >= n) return;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int cbase = ctile * 16 * CT;
    const auto rZ = rsrc(dZ, (long)n * ldz * 4);
    const auto rW = rsrc(W, (long)H * D * in * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    const int zi = i0 + li;
    const uint32_t zbase = zi < n ? (uint32_t)zi * ldz * 4 : kOOB;
    int cb[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) cb[t] = cbase + 16 * t + li;
    const int DS = (D + 3) / 4;
    f32x4v tot[CT];
#pragma unroll
    for (int t = 0; t < CT; ++t) tot[t] = f32x4v{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < H; kb += HF) {
        // mask words of this head group (used after the products)
        uint32_t mw[HF][CT];
#pragma unroll
        for (int f = 0; f < HF; ++f) {
            const uint32_t mrow = (uint32_t)(((kb + f) * NWI + i0 / 32) * LDC) * 4;
#pragma unroll
            for (int t = 0; t < CT; ++t) mw[f][t] = bldu(rM, (kb + f < H && cb[t] < in) ? mrow + cb[t] * 4 : kOOB);
        }
        f32x4v acc[HF][CT];
#pragma unroll
        for (int f = 0; f < HF; ++f)
#pragma unroll
            for (int t = 0; t < CT; ++t) acc[f][t] = f32x4v{0.f, 0.f, 0.f, 0.f};
        float av[HF], bv[HF][CT];
        auto fetch = [&](int s, float (&a)[HF], float (&b)[HF][CT]) {
            const int d = 4 * s + lk;
#pragma unroll
            for (int f = 0; f < HF; ++f) {
                const int k = kb + f;
                const bool ok = d < D && k < H;
                const int hd = k * D + d;
                a[f] = bld(rZ, (ok && zbase != kOOB) ? zbase + hd * 4 : kOOB);
#pragma unroll
                for (int t = 0; t < CT; ++t)
                    b[f][t] = bld(rW, (ok && cb[t] < in) ? (uint32_t)(hd * in + cb[t]) * 4 : kOOB);
            }
        };
        fetch(0, av, bv);
        for (int s = 0; s < DS; ++s) {
            float an[HF], bn[HF][CT];
            fetch(s + 1, an, bn);                    // past D: reads 0, never used
#pragma unroll
            for (int f = 0; f < HF; ++f)
#pragma unroll
                for (int t = 0; t < CT; ++t)
                    acc[f][t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[f], bv[f][t], acc[f][t], 0, 0, 0);
#pragma unroll
            for (int f = 0; f < HF; ++f) {
                av[f] = an[f];
#pragma unroll
                for (int t = 0; t < CT; ++t) bv[f][t] = bn[f][t];
            }
        }
        // C layout: col = li (input column), row = 4 lk + r
        const int sh = (i0 & 31) + 4 * lk;
#pragma unroll
        for (int f = 0; f < HF; ++f)
#pragma unroll
            for (int t = 0; t < CT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) tot[t][r] += ((mw[f][t] >> (sh + r)) & 1u) ? acc[f][t][r] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < CT; ++t) {
        const int gc = cbase + 16 * t + li;
        if (gc >= in) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int gi = i0 + 4 * lk + r;
            if (gi < n) {
                const long o = (long)gi * ldx + gc;
                dX[o] = accumulate ? dX[o] + tot[t][r] * scale : tot[t][r] * scale;
            }
        }
    }
}

// dX for narrow heads (D = 8, H <= 8: the W2S shape), every operand requested up
// front in 16-byte pieces.  Wave = 16 rows x 64 columns; the four 16-column MFMA
// tiles are interleaved (tile t, output column n <-> column cbase + 4n + t), so a lane's
// W quad W[hd, cbase+4li .. +3], keep-word quad and dX quad serve all four tiles, and
// the reduction index of head k's two 16x16x4 steps is hd = kD + 2 lk + s, so the
// lane's dZ pair is one 8-byte load: 8 + 16 + 8 vector loads per wave instead of the
// chained kernel's 112 dword loads.  Heads are added in head order.
// byte B of y as a float (v_cvt_f32_ubyteB); spelled out because the compiler, knowing
// each byte of the spread keep bits is 0 or 1, would rewrite (y >> 8B) & 0xff into a
// v_bfe_u32 + v_cvt_f32_ubyte0 pair
template <int B>
__device__ __forceinline__ float cvt_ubyte(uint32_t y) {
    float f;
    if constexpr (B == 0) asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(y));
    else if constexpr (B == 1) asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(y));
    else if constexpr (B == 2) asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(y));
    else asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(y));
    return f;
}

template <int HH, int HG, bool SPREAD = true>
__device__ __forceinline__ void hproj_dx_n8_tile(int task, int n, int in, int H, const float *__restrict__ dZ,
                                                 int ldz, const float *__restrict__ W,
                                                 const uint32_t *__restrict__ bits, float scale,
                                                 float *__restrict__ dX, int ldx, int accumulate) {
    constexpr int D = 8;
    typedef float f32x2v __attribute__((ext_vector_type(2)));
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int nct = (in + 63) / 64;
    const int rt = task / nct, ctile = task - rt * nct;
    const int i0 = rt * 16;
    if (i0 >= n) return;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int c = ctile * 64 + 4 * li;                     // this lane's column quad
    const bool cok = c < in;                               // in % 4 == 0: whole quads
    const auto rZ = rsrc(dZ, (long)n * ldz * 4);
    const auto rW = rsrc(W, (long)H * D * in * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    const int zi = i0 + li;
    const uint32_t zbase = zi < n ? (uint32_t)zi * ldz * 4 : kOOB;
    const int sh = (i0 & 31) + 4 * lk;
    f32x4v tot[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) tot[t] = f32x4v{0.f, 0.f, 0.f, 0.f};
    // heads in groups of HG: a group's operands are requested together, then used
#pragma unroll
    for (int k0 = 0; k0 < HH; k0 += HG) {
        f32x2v av[HG];
        f32x4v bv[HG][2];
        u32x4v mw[HG];
#pragma unroll
        for (int f = 0; f < HG; ++f) {
            const int k = k0 + f;
            const bool ok = k < H;
            const int hd = k * D + 2 * lk;
            const u32x4v z = bld4(rZ, (ok && zbase != kOOB) ? zbase + hd * 4 : kOOB);   // (hd, hd+1) used
            av[f] = f32x2v{__uint_as_float(z.x), __uint_as_float(z.y)};
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const u32x4v w = bld4(rW, (ok && cok) ? (uint32_t)((hd + s) * in + c) * 4 : kOOB);
                bv[f][s] = f32x4v{__uint_as_float(w.x), __uint_as_float(w.y), __uint_as_float(w.z), __uint_as_float(w.w)};
            }
            mw[f] = bld4(rM, (ok && cok) ? (uint32_t)(((k * NWI + i0 / 32) * LDC) + c) * 4 : kOOB);
        }
#pragma unroll
        for (int f = 0; f < HG; ++f) {
            f32x4v acc[4];
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[f][0], bv[f][0][t], f32x4v{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[f][1], bv[f][1][t], acc[t], 0, 0, 0);
            if (!SPREAD && k0 + f < H) {
#pragma unroll
                for (int t = 0; t < 4; ++t)
#pragma unroll
                    for (int r = 0; r < 4; ++r) tot[t][r] += ((mw[f][t] >> (sh + r)) & 1u) ? acc[t][r] : 0.f;
            }
            if (SPREAD && k0 + f < H) {
                // the tile's 4 keep bits (rows 4 lk .. +3) spread to bytes 0..3
                // (bit i -> bit 8i: x * 0x204081), each byte -> 0.0 / 1.0 by
                // v_cvt_f32_ubyteN, then one fma per value: 2.75 VALU per value
                // instead of select + add on a compare (+ the AGPR read)
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t y = (__builtin_amdgcn_ubfe(mw[f][t], sh, 4) * 0x204081u) & 0x01010101u;
                    tot[t][0] = __builtin_fmaf(cvt_ubyte<0>(y), acc[t][0], tot[t][0]);
                    tot[t][1] = __builtin_fmaf(cvt_ubyte<1>(y), acc[t][1], tot[t][1]);
                    tot[t][2] = __builtin_fmaf(cvt_ubyte<2>(y), acc[t][2], tot[t][2]);
                    tot[t][3] = __builtin_fmaf(cvt_ubyte<3>(y), acc[t][3], tot[t][3]);
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // C layout: col = li (tile t: column c + t), row = 4 lk + r
    if (!cok) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int gi = i0 + 4 * lk + r;
        if (gi >= n) continue;
        f32x4v *o = reinterpret_cast<f32x4v *>(dX + (long)gi * ldx + c);
        f32x4v v = f32x4v{tot[0][r], tot[1][r], tot[2][r], tot[3][r]} * scale;
        if (accumulate) v += *o;
        *o = v;
    }
}

template <int HH, int HG, bool SPREAD = true>
__global__ __launch_bounds__(256) void k_hproj_dx_n8(int n, int in, int H, const float *__restrict__ dZ, int ldz,
                                                     const float *__restrict__ W,
                                                     const uint32_t *__restrict__ bits, float scale,
                                                     float *__restrict__ dX, int ldx, int accumulate) {
    hproj_dx_n8_tile<HH, HG, SPREAD>((int)(blockIdx.x * 4 + (threadIdx.x >> 6)), n, in, H, dZ, ldz, W, bits, scale,
                                     dX, ldx, accumulate);
}

// dX with one wave per head (wide heads, e.g. S2W: H = 6, D = 50, few rows): block =
// H waves on one 16-row x 16-column tile.  Wave k requests its head's DS dZ values,
// DS W values and keep word up front, runs the DS-step MFMA chain, and leaves the
// masked product in LDS; the block then adds the heads in head order (the order of
// k_hproj_dx: bitwise equal results).  DSM = largest DS the instance holds.
// (the body as a device function of the block index: also the dX half of
// k_hproj_bwd_hw, whose 256-thread blocks run heads k, k + 4, ... per wave)
template <int DSM>
__device__ __forceinline__ void hproj_dx_hw_tile(int bid, int n, int in, int H, int D, const float *__restrict__ dZ,
                                                 int ldz, const float *__restrict__ W,
                                                 const uint32_t *__restrict__ bits, float scale,
                                                 float *__restrict__ dX, int ldx, int accumulate) {
    __shared__ float sP[16][4][64];                   // [head][r][lane]
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int nct = (in + 15) / 16;
    const int rt = bid / nct, ctile = bid - rt * nct;
    const int i0 = rt * 16;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int nw = (int)(blockDim.x >> 6);
    const int DS = (D + 3) / 4;
    const auto rZ = rsrc(dZ, (long)n * ldz * 4);
    const auto rW = rsrc(W, (long)H * D * in * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    const int zi = i0 + li, c = ctile * 16 + li;
    const uint32_t zbase = zi < n ? (uint32_t)zi * ldz * 4 : kOOB;
    const int sh = (i0 & 31) + 4 * lk;
    for (int k = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); k < H; k += nw) {
        float av[DSM], bv[DSM];
#pragma unroll
        for (int s = 0; s < DSM; ++s) {
            const int d = 4 * s + lk;
            const bool ok = s < DS && d < D;
            const int hd = k * D + d;
            av[s] = bld(rZ, (ok && zbase != kOOB) ? zbase + hd * 4 : kOOB);
            bv[s] = bld(rW, (ok && c < in) ? (uint32_t)(hd * in + c) * 4 : kOOB);
        }
        const uint32_t mw = bldu(rM, c < in ? (uint32_t)(((k * NWI + i0 / 32) * LDC) + c) * 4 : kOOB);
        f32x4v acc = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < DSM; ++s)
            if (s < DS) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) sP[k][r][lane] = ((mw >> (sh + r)) & 1u) ? acc[r] : 0.f;
    }
    __syncthreads();
    for (int o = threadIdx.x; o < 256; o += blockDim.x) {         // 16 x 16 outputs
        const int r = o >> 6, ln = o & 63;
        float tot = 0.f;
        for (int h = 0; h < H; ++h) tot += sP[h][r][ln];
        const int gi = i0 + 4 * (ln >> 4) + r, gc = ctile * 16 + (ln & 15);
        if (gi < n && gc < in) {
            const long ofs = (long)gi * ldx + gc;
            dX[ofs] = accumulate ? dX[ofs] + tot * scale : tot * scale;
        }
    }
}

template <int DSM>
__global__ __launch_bounds__(1024) void k_hproj_dx_hw(int n, int in, int H, int D, const float *__restrict__ dZ,
                                                      int ldz, const float *__restrict__ W,
                                                      const uint32_t *__restrict__ bits, float scale,
                                                      float *__restrict__ dX, int ldx, int accumulate) {
    hproj_dx_hw_tile<DSM>((int)blockIdx.x, n, in, H, D, dZ, ldz, W, bits, scale, dX, ldx, accumulate);
}

// ------------------------------------------------------------------ dW ----
// v_mfma_f32_16x16x4_f32, reduction over rows.  Block = 64 input columns (wave w:
// columns 16w..16w+15) x SL slots (slot = 16 outputs of one head) x one chunk of
// rows.  Per 32-row step, staged in LDS:
//   Xs[32][80]       X[r, c0 .. c0+63]
//   Zs[32][SL*16+16] dZ of the SL slots, zero-padded to 16 per slot
//   Ms[SL][64]       the slots' mask words for these 32 rows
// and MFMA A[c][r] = bit X[r, c], B[r][j] = dZ[r, kD+d0+j].  The next step's
// global loads are issued before this step's MFMAs.  Each block writes its own
// partial slab part[chunk][H*D][in]; k_sum_parts adds the chunks in order.
constexpr int kDwXs = 80;                         // row stride: 4 rows hit 4 disjoint bank quarters

struct DwGeom {
    int ctiles, sgroups, chunks, rows;            // rows per chunk (multiple of 32)
};

// 4 slots per block (twice the blocks of 8, half the accumulators per wave) and a
// 1,024-block target: cfg2 step 1.502 vs 1.526 ms (tools/ab.py; 1,536 / 2,048 blocks
// and the 8-slot, 512-block plan are slower)
int dw_slots() {
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_DWS")) return atoi(e) == 8 ? 8 : 4;        // dev A/B
    return 4;
}

DwGeom dw_geom(int n, int in, int H, int D) {
    DwGeom g;
    const int ns = H * ((D + 15) / 16);
    g.ctiles = (in + 63) / 64;
    g.sgroups = (ns + dw_slots() - 1) / dw_slots();
    const int steps = (n + 31) / 32 > 0 ? (n + 31) / 32 : 1;
    int target = dw_slots() == 4 ? 1024 : 512;          // blocks to aim for
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_DWB")) target = atoi(e);     // dev sweep
    int want = target / (g.ctiles * g.sgroups);
    if (want < 1) want = 1;
    if (want > steps) want = steps;
    const int per = (steps + want - 1) / want;    // 32-row steps per chunk
    g.rows = per * 32;
    g.chunks = (steps + per - 1) / per;
    return g;
}

// VEC (SL = 4, D = 8, in % 4 == 0, 16-byte rows): X and the four heads' dZ columns
// (32 contiguous floats per row) are staged with 16-byte loads -- 4 loads per thread
// per 32-row step instead of 17 dword loads; the padding columns of the dZ stage are
// zeroed once.  Same LDS image, same products (bitwise equal).
template <int SL, bool VEC = false>
__device__ __forceinline__ void hproj_dw_block(int bx, int by, int bz, int n, int in, int H, int D,
                                               int rows_per_chunk, const float *__restrict__ dZ, int ldz,
                                               const float *__restrict__ X, int ldx,
                                               const uint32_t *__restrict__ bits, float *__restrict__ part) {
    __shared__ __attribute__((aligned(16))) float Xs[32][kDwXs];
    constexpr int ZC = SL * 16, NZ = 32 * ZC / 256, NM = SL * 64 / 256;   // slot columns, per-thread loads
    // dZ stage: slot q at column ZS q.  VEC: slots 24 apart, so the eight 16-byte
    // stores of a row (slot halves at 24q + 4h) fall on distinct banks mod 32 (at 16
    // apart slots q and q + 2 collided: 2-way on every stage store), and rows 112 apart
    // (16 mod 32: the reads of rows rr and rr + 1 in one 32-lane group stay disjoint)
    constexpr int ZS = VEC ? 24 : 16, ZW = VEC ? 112 : ZC + 16;
    __shared__ __attribute__((aligned(16))) float Zs[32][ZW];
    __shared__ uint32_t Ms[SL][64];
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int SPH = (D + 15) / 16, NS = H * SPH;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int c0 = bx * 64;
    const int s0 = by * SL;
    const int rb = bz * rows_per_chunk;
    const int rend = min(rb + rows_per_chunk, n);
    // per-thread staging: X 2 x 4 columns, dZ 16 values, 2 mask words.  The
    // column parts of every offset are fixed per thread; buffer loads with kOOB
    // offsets for the edges keep all 26 loads unconditional and in flight together.
    const auto rX = rsrc(X, (long)n * ldx * 4);
    const auto rZ = rsrc(dZ, (long)n * ldz * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    static_assert(!VEC || SL == 4, "vector staging: 4 slots of D = 8");
    float xr[8], zr[NZ];
    f32x4v xq[2], zq;
    uint32_t mr[NM];
    int xcol[2], zcol[NZ];
    uint32_t moff[NM];
#pragma unroll
    for (int u = 0; u < 2; ++u) xcol[u] = c0 + ((tid + 256 * u) & 15) * 4;   // 32 rows x 16 column quads
#pragma unroll
    for (int u = 0; u < NZ; ++u) {
        const int a = (tid + 256 * u) % ZC;           // 32 rows x ZC slot columns
        const int v = s0 + (a >> 4);
        const int k = min(v, NS - 1) / SPH, d = (min(v, NS - 1) - k * SPH) * 16 + (a & 15);
        zcol[u] = (v < NS && d < D) ? k * D + d : -1;
    }
#pragma unroll
    for (int u = 0; u < NM; ++u) {
        const int e = tid + 256 * u;                  // SL slots x 64 columns
        const int v = s0 + (e >> 6), gc = c0 + (e & 63);
        moff[u] = (v < NS && gc < LDC) ? (uint32_t)((v / SPH) * NWI * LDC + gc) * 4 : kOOB;
    }
    auto fetch = [&](int r0) {
        if constexpr (VEC) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int gi = r0 + ((tid + 256 * u) >> 4);
                const u32x4v v = bld4(rX, (gi < rend && xcol[u] < in) ? (uint32_t)(gi * ldx + xcol[u]) * 4 : kOOB);
                xq[u] = f32x4v{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
            }
            const int gi = r0 + (tid >> 3), q = tid & 7, v = s0 + (q >> 1);
            const u32x4v z = bld4(rZ, (gi < rend && v < NS) ? (uint32_t)(gi * ldz + v * 8 + (q & 1) * 4) * 4 : kOOB);
            zq = f32x4v{__uint_as_float(z.x), __uint_as_float(z.y), __uint_as_float(z.z), __uint_as_float(z.w)};
        } else {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int gi = r0 + ((tid + 256 * u) >> 4);
            const bool rok = gi < rend;
#pragma unroll
            for (int v = 0; v < 4; ++v)
                xr[u * 4 + v] = bld(rX, (rok && xcol[u] + v < in) ? (uint32_t)(gi * ldx + xcol[u] + v) * 4 : kOOB);
        }
#pragma unroll
        for (int u = 0; u < NZ; ++u) {
            const int gi = r0 + (tid + 256 * u) / ZC;
            zr[u] = bld(rZ, (gi < rend && zcol[u] >= 0) ? (uint32_t)(gi * ldz + zcol[u]) * 4 : kOOB);
        }
        }
        const uint32_t roff = (uint32_t)(r0 / 32) * LDC * 4;
#pragma unroll
        for (int u = 0; u < NM; ++u) mr[u] = bldu(rM, moff[u] != kOOB ? moff[u] + roff : kOOB);
    };
    auto stash = [&]() {
        if constexpr (VEC) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = tid + 256 * u;
                *reinterpret_cast<f32x4v *>(&Xs[e >> 4][(e & 15) * 4]) = xq[u];
            }
            const int q = tid & 7;
            *reinterpret_cast<f32x4v *>(&Zs[tid >> 3][(q >> 1) * ZS + (q & 1) * 4]) = zq;
        } else {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + 256 * u;
            const int rr = e >> 4, cq = (e & 15) * 4;
            *reinterpret_cast<f32x4v *>(&Xs[rr][cq]) = f32x4v{xr[u * 4], xr[u * 4 + 1], xr[u * 4 + 2], xr[u * 4 + 3]};
        }
#pragma unroll
        for (int u = 0; u < NZ; ++u) {
            const int e = tid + 256 * u;
            Zs[e / ZC][e % ZC] = zr[u];
        }
        }
#pragma unroll
        for (int u = 0; u < NM; ++u) {
            const int e = tid + 256 * u;
            Ms[e >> 6][e & 63] = mr[u];
        }
    };
    if constexpr (VEC)                                    // dZ stage columns 8..15 of each slot: zero
        *reinterpret_cast<f32x4v *>(&Zs[tid >> 3][((tid >> 1) & 3) * ZS + 8 + (tid & 1) * 4]) =
            f32x4v{0.f, 0.f, 0.f, 0.f};
    f32x4v acc[SL];
#pragma unroll
    for (int q = 0; q < SL; ++q) acc[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int col = wv * 16 + li;
    if (rb < rend) fetch(rb);
    for (int r0 = rb; r0 < rend; r0 += 32) {
        __syncthreads();
        stash();
        __syncthreads();
        if (r0 + 32 < rend) fetch(r0 + 32);
        // the step's mask words in registers; the keep bit of row rr is one v_bfe_i32
        // (0 or -1) and a v_and on the X value -- the select form cost a shift, an and,
        // a compare and a v_cndmask per MFMA (plus s_nop pads before the MFMA reading it)
        uint32_t mq[SL];
#pragma unroll
        for (int q = 0; q < SL; ++q) mq[q] = Ms[q][col];
#pragma unroll
        for (int s4 = 0; s4 < 32; s4 += 4) {
            const int rr = s4 + lk;
            const uint32_t xv = __float_as_uint(Xs[rr][col]);
            // slots past NS were staged as zeros: no branch around the MFMAs (a
            // conditional MFMA makes the compiler shuffle accumulators)
            float a[SL], b[SL];
#pragma unroll
            for (int q = 0; q < SL; ++q) {
                a[q] = __uint_as_float(xv & (uint32_t)__builtin_amdgcn_sbfe((int)mq[q], rr, 1));
                b[q] = Zs[rr][q * ZS + li];
            }
#pragma unroll
            for (int q = 0; q < SL; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q], b[q], acc[q], 0, 0, 0);
        }
    }
    // D: col = lane & 15 -> slot output j, row = (lane >> 4) * 4 + r -> input column
    const long base = (long)bz * H * D * in;
#pragma unroll
    for (int q = 0; q < SL; ++q) {
        const int v = s0 + q;
        if (v >= NS) continue;
        const int k = v / SPH, j = (v - k * SPH) * 16 + li;
        if (j >= D) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int gc = c0 + wv * 16 + lk * 4 + r;
            if (gc < in) part[base + (long)(k * D + j) * in + gc] = acc[q][r];
        }
    }
}

template <int SL, bool VEC = false>
__global__ __launch_bounds__(256) void k_hproj_dw(int n, int in, int H, int D, int rows_per_chunk,
                                                  const float *__restrict__ dZ, int ldz,
                                                  const float *__restrict__ X, int ldx,
                                                  const uint32_t *__restrict__ bits, float *__restrict__ part) {
    hproj_dw_block<SL, VEC>((int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, n, in, H, D, rows_per_chunk, dZ, ldz,
                            X, ldx, bits, part);
}

// The wide-head (S2W) backward of one projection in ONE launch: blocks [0, dx_blocks)
// are k_hproj_dx_hw tiles (4 waves per block, heads k, k + 4, ... per wave: the same
// products and the same head-order sums, so dX is bitwise the two-launch one), the rest
// k_hproj_dw<4> blocks (the same row chunks and partial slabs).  The two halves only
// share dZ; each was a latency-bound launch of a few hundred blocks (7.3 + 6.6 us).
template <int DSM>
__global__ __launch_bounds__(256) void k_hproj_bwd_hw(int n, int in, int H, int D, const float *__restrict__ dZ,
                                                      int ldz, const float *__restrict__ W,
                                                      const uint32_t *__restrict__ bits, float scale,
                                                      float *__restrict__ dX, int ldxo, int accumulate,
                                                      const float *__restrict__ X, int ldx, int rows_per_chunk,
                                                      float *__restrict__ part, int dx_blocks, int cx, int cy) {
    const int b = (int)blockIdx.x;
    if (b < dx_blocks) {
        hproj_dx_hw_tile<DSM>(b, n, in, H, D, dZ, ldz, W, bits, scale, dX, ldxo, accumulate);
        return;
    }
    const int e = b - dx_blocks;
    hproj_dw_block<4, false>(e % cx, (e / cx) % cy, e / (cx * cy), n, in, H, D, rows_per_chunk, dZ, ldz, X, ldx, bits,
                             part);
}

// ---------------------------------------------- dW on bf16 limb MFMAs (round 5) ----
// D = 8, H <= 8 (the W2S projection).  k_hproj_dw pads each 8-wide head to a 16-wide
// slot of v_mfma_f32_16x16x4_f32 (half its exact-f32 MFMA work is zeros) and was 53 %
// issue-stalled.  Here  dW_k = dZ_k^T (M_k o X)  runs on v_mfma_f32_16x16x32_bf16 with
// the K axis = 32 rows, fp32-accurate (three RNE bf16 limbs per operand, six products):
// C[m][c] += A[m][i] B[i][c], A = dZ^T of head k (rows m = its 8 outputs, repeated in
// m = 8..15 and discarded), B = the keep-masked X.  The keep bits of 32 rows at one
// column are ONE mask word -- the MFMA's K axis is the word's axis -- so a lane's 8 rows
// are one byte of it, turned into the four 16-bit lane masks of its bf16 pairs by two
// shifts and a v_perm_b32 with sign-byte selectors per pair (a 256-entry LDS table
// instead: 2.3e6 bank-conflict cycles per launch, its rows are random).
// Block = 64 columns (wave w: columns 16w .. 16w + 15) x all heads x one chunk of rows
// (the 16x16x4 kernel's chunking, so the partial slabs part[chunk][H*8][in] are the
// same), the chunks XCD-local (their dZ rows, re-read by every column tile, stay in
// one L2); per 32-row step the block stages, double-buffered in LDS with two steps of
// global loads in flight in registers (22.1 -> 20.2 us against one): X and dZ split ONCE
// into limb images stored column-major (thread = (column, 8 rows): 8 coalesced dword
// loads, three ds_write_b128), and the step's mask words.  A wave then reads its B
// fragments once, and per head its A fragments and mask word, masks B (12 + 12 VALU)
// and runs 6 MFMAs.
// kDwMfP: image row pitch (bf16).  40 (80 B): fragment reads 2-way, staging writes
// conflict-free; 48 (96 B): reads conflict-free, writes 2-way (tools/lds_banks.py-style
// check over gfx950's ds_read_b128 lane groups).  32 (round 6, the default): unpadded
// 64-B rows of four 16-B slots (8 rows of K each), slot s of row r stored at s ^ ((r >> 1)
// & 3): the staging ds_write_b128 (8 contiguous lanes = 8 rows, one slot: banks mod 32)
// and both fragment reads (ds_read_b128 lane groups of 4 + 4 + 8 lanes = 8 rows x 2
// slots: banks mod 64) all land on distinct 4-bank groups (tools/lds_banks.py dwmf)
template <int kDwMfP>
__device__ __forceinline__ int dwmf_off(int r, int slot) {
    if constexpr (kDwMfP == 32) return r * 32 + 8 * (slot ^ ((r >> 1) & 3));
    else return r * kDwMfP + 8 * slot;
}

// NB: LDS image buffers (2: double-buffered, the launch of its own; 1: the merged W2S
// backward k_hproj_bwd_n8, whose dX blocks need the CU's LDS for occupancy -- one more
// barrier per step, 26.6 instead of 53 KB).  bl / ctiles / chunks: the logical block
// and grid (the merged kernel's dW blocks follow its dX blocks).
template <int kDwMfP, int NB = 2>
__device__ __forceinline__ void hproj_dw_mf_block(int bl, int ctiles, int chunks, int n, int in, int H,
                                                  int rows_per_chunk, const float *__restrict__ dZ, int ldz,
                                                  const float *__restrict__ X, int ldx,
                                                  const uint32_t *__restrict__ bits, float *__restrict__ part) {
    constexpr int HM = 8;
    __shared__ __attribute__((aligned(16))) __bf16 sX[NB][3][64 * kDwMfP];   // X limbs [column][row]
    __shared__ __attribute__((aligned(16))) __bf16 sZ[NB][3][64 * kDwMfP];   // dZ limbs [output][row]
    __shared__ uint32_t sM[NB][HM][64];                                      // keep words [head][column]
    const int NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // XCD-aware order: workgroup b runs on XCD b % 8, so logical block L = xcd_order(b)
    // puts the column tiles of one row chunk on one XCD and their dZ rows (re-read by
    // every column tile) come from its L2 instead of HBM
    const int total = ctiles * chunks;
    const int L = (bl & 7) * (total >> 3) + min(bl & 7, total & 7) + (bl >> 3);     // a bijection
    const int chunk = L / ctiles;
    const int c0 = (L % ctiles) * 64;
    const int rb = chunk * rows_per_chunk;
    const int rend = min(rb + rows_per_chunk, n);
    const auto rX = rsrc(X, (long)n * ldx * 4);
    const auto rZ = rsrc(dZ, (long)n * ldz * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    // staging: thread = (column sc, rows 8 sr .. 8 sr + 7) of X and of dZ; mask words
    // (head tid / 64 and 4 + tid / 64, column tid % 64)
    const int sc = tid & 63, sr = tid >> 6;
    const int gx = c0 + sc;
    const bool xok = gx < in, zok = sc < H * 8;
    // two steps of global loads in flight: register sets 0 / 1 for even / odd steps
    float vxs[2][8], vzs[2][8];
    uint32_t vms[2][2];
    auto gload = [&](int r0, float (&vx)[8], float (&vz)[8], uint32_t (&vm)[2]) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int r = r0 + 8 * sr + j;
            const bool rok = r < rend;
            vx[j] = __uint_as_float(bldu(rX, rok && xok ? (uint32_t)(r * ldx + gx) * 4 : kOOB));
            vz[j] = __uint_as_float(bldu(rZ, rok && zok ? (uint32_t)(r * ldz + sc) * 4 : kOOB));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = sr + 4 * u;
            vm[u] = bldu(rM, k < H && gx < LDC ? (uint32_t)((k * NWI + r0 / 32) * LDC + gx) * 4 : kOOB);
        }
    };
    auto lstore = [&](int b, const float (&vx)[8], const float (&vz)[8], const uint32_t (&vm)[2]) {
        hsg_u32x4_t x0, x1, x2, z0, z1, z2;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            unsigned a, bb, c;
            hsg_split_rne_pair(vx[2 * q], vx[2 * q + 1], a, bb, c);
            x0[q] = a; x1[q] = bb; x2[q] = c;
            hsg_split_rne_pair(vz[2 * q], vz[2 * q + 1], a, bb, c);
            z0[q] = a; z1[q] = bb; z2[q] = c;
        }
        const int o = dwmf_off<kDwMfP>(sc, sr);
        *reinterpret_cast<hsg_u32x4_t *>(&sX[b][0][o]) = x0;
        *reinterpret_cast<hsg_u32x4_t *>(&sX[b][1][o]) = x1;
        *reinterpret_cast<hsg_u32x4_t *>(&sX[b][2][o]) = x2;
        *reinterpret_cast<hsg_u32x4_t *>(&sZ[b][0][o]) = z0;
        *reinterpret_cast<hsg_u32x4_t *>(&sZ[b][1][o]) = z1;
        *reinterpret_cast<hsg_u32x4_t *>(&sZ[b][2][o]) = z2;
        sM[b][sr][sc] = vm[0];
        sM[b][sr + 4][sc] = vm[1];
    };
    f32x4v acc[HM];
#pragma unroll
    for (int k = 0; k < HM; ++k) acc[k] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int cl = lane & 15, ig = lane >> 4;
    const int xo = dwmf_off<kDwMfP>(16 * w + cl, ig);             // B fragment: column 16w + cl, rows 8 ig ..
    const int zo = dwmf_off<kDwMfP>(cl & 7, ig);                  // A fragment: output k*8 + (cl & 7)
    if (rb < rend) gload(rb, vxs[0], vzs[0], vms[0]);
    if (rb + 32 < rend) gload(rb + 32, vxs[1], vzs[1], vms[1]);
    auto step = [&](int r0, int b) {                             // b = step parity (compile-time below)
        constexpr int ib = 0;                                     // (NB == 1: the one image)
        const int bi = NB == 1 ? ib : b;
        if constexpr (NB == 1) {
            if (r0 != rb) __syncthreads();                        // every wave done with the last step's image
        }
        lstore(bi, vxs[b], vzs[b], vms[b]);
        __syncthreads();
        if (r0 + 64 < rend) gload(r0 + 64, vxs[b], vzs[b], vms[b]);
        hsg_u32x4_t bx[3];
#pragma unroll
        for (int l = 0; l < 3; ++l) bx[l] = *reinterpret_cast<const hsg_u32x4_t *>(&sX[bi][l][xo]);
#pragma unroll
        for (int k = 0; k < HM; ++k) {
            if (k >= H) break;                                    // wave-uniform
            // the lane's 8 rows are bits 8 ig .. 8 ig + 7 of the word: pair q's mask from
            // bits 2q / 2q + 1 shifted to 15 / 31 and v_perm_b32's sign-byte selectors (a
            // 256-entry LDS table here cost 2.3e6 bank-conflict cycles per launch: random rows)
            const uint32_t x = sM[bi][k][16 * w + cl] >> (8 * ig);
            hsg_u32x4_t M;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                M[q] = __builtin_amdgcn_perm(x << (30 - 2 * q), x << (15 - 2 * q), 0x0B0B0808u);
            hsg_bf16x8_t az[3];
#pragma unroll
            for (int l = 0; l < 3; ++l)
                az[l] = *reinterpret_cast<const hsg_bf16x8_t *>(&sZ[bi][l][k * 8 * kDwMfP + zo]);  // (r >> 1) & 3 of
                                                                  // row k*8 + c: that of c
            const hsg_bf16x8_t b0 = __builtin_bit_cast(hsg_bf16x8_t, bx[0] & M);
            const hsg_bf16x8_t b1 = __builtin_bit_cast(hsg_bf16x8_t, bx[1] & M);
            const hsg_bf16x8_t b2 = __builtin_bit_cast(hsg_bf16x8_t, bx[2] & M);
            f32x4v c = acc[k];                                    // smallest limb products first
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az[2], b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az[1], b1, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az[0], b2, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az[1], b0, c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az[0], b1, c, 0, 0, 0);
            acc[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(az[0], b0, c, 0, 0, 0);
        }
    };
    for (int r0 = rb; r0 < rend; r0 += 64) {
        step(r0, 0);
        if (r0 + 32 < rend) step(r0 + 32, 1);
    }
    // C: lane holds column 16w + cl, outputs 4 ig + e (ig < 2: the head's 8 outputs)
    const int gc = c0 + 16 * w + cl;
    if (ig < 2 && gc < in) {
        float *dst = part + (size_t)chunk * H * 8 * in + gc;
#pragma unroll
        for (int k = 0; k < HM; ++k) {
            if (k >= H) break;
#pragma unroll
            for (int e = 0; e < 4; ++e) dst[(size_t)(k * 8 + 4 * ig + e) * in] = acc[k][e];
        }
    }
}

template <int kDwMfP>
__global__ __launch_bounds__(256, 2) void k_hproj_dw_mf(int n, int in, int H, int rows_per_chunk,
                                                       const float *__restrict__ dZ, int ldz,
                                                       const float *__restrict__ X, int ldx,
                                                       const uint32_t *__restrict__ bits, float *__restrict__ part) {
    hproj_dw_mf_block<kDwMfP>((int)(blockIdx.y * gridDim.x + blockIdx.x), (int)gridDim.x, (int)gridDim.y, n, in, H,
                              rows_per_chunk, dZ, ldz, X, ldx, bits, part);
}

// The narrow-head (W2S) backward of one projection in ONE launch (round 6): blocks [0,
// dx_blocks) are k_hproj_dx_n8 tiles (4 waves = 4 tasks each), the rest k_hproj_dw_mf
// blocks on a single LDS image (NB = 1), the same row chunks and partial slabs -- dX
// and the slabs are bitwise those of the two launches.  The dX tiles (~1,500 blocks of
// short chains) and the dW blocks (500 blocks of six 32-row steps) were two latency-bound
// launches back to back; here the dW blocks run beside the dX tiles.
__global__ __launch_bounds__(256) void k_hproj_bwd_n8(int n, int in, int H, const float *__restrict__ dZ, int ldz,
                                                     const float *__restrict__ W, const uint32_t *__restrict__ bits,
                                                     float scale, float *__restrict__ dX, int ldxo, int accumulate,
                                                     const float *__restrict__ X, int ldx, int rows_per_chunk,
                                                     float *__restrict__ part, int dx_blocks, int ctiles, int chunks) {
    const int b = (int)blockIdx.x;
    if (b < dx_blocks) {
        hproj_dx_n8_tile<8, 2>(b * 4 + (int)(threadIdx.x >> 6), n, in, H, dZ, ldz, W, bits, scale, dX, ldxo,
                               accumulate);
        return;
    }
    hproj_dw_mf_block<32, 1>(b - dx_blocks, ctiles, chunks, n, in, H, rows_per_chunk, dZ, ldz, X, ldx, bits, part);
}

// ------------------------------------------------- dW, narrow heads, 4x4x1 ----
// (round 5) Heads of D % 4 == 0 with H * D <= 64 (the W2S projection: 8 heads x 8) on
// v_mfma_f32_4x4x1_16b_f32: 16 independent 4 x 4 outer products per instruction, K = 1
// row.  Block b of the instruction is the output quad (W rows 4b .. 4b + 3, i.e. one
// head k_b = 4b / D, columns c .. c + 3): A[i] at lane 4b + i = keep(r, k_b, c + i) *
// X[r, c + i], B[j] at lane 4b + j = dZ[r, 4b + j] = dZ[r, lane], so one instruction
// is 64 W rows x 4 columns x 1 row with nothing padded -- the 16x16x4 kernel above
// pads each 8-wide head to a 16-wide slot (half its MFMA work is zeros) and spends
// three VALU + two s_nop per MFMA on the mask.  Here the keep bit is one v_bfe_i32 +
// v_and per MFMA lane value.  D[i][j] lands in register i of lane 4b + j: lane l
// accumulates W row l, four columns per quad -> one 16-byte store per quad.
// Per wave M4Q column quads; per block M4W waves (M4W * M4Q * 4 columns) and a chunk of
// rows in 32-row steps (the keep-mask word granularity).  Per step the block stages
// X[32 rows][block columns] transposed (Xt[column][row], 4-row groups XOR-swizzled by
// the column quad so the transposing dword stores spread over the banks; a lane's
// 4-row A values are one ds_read_b128) and dZ[32][64] (zero past H * D); the next
// step's global loads are issued before this step's MFMAs.  The chunk's partial slab
// part[chunk][H*D][in] is the contract of k_hproj_dw (hsg_slab_reduce / k_sum_parts).
constexpr int M4Q = 5, M4W = 5;                   // 5 waves x 5 quads = 100 columns per block
constexpr int M4C = M4W * M4Q * 4, M4XS = 36;     // block columns; Xt column stride (floats)

struct DwM4Geom {
    int ctiles, chunks, rows;
};

// measured slower than the 16x16x4 kernel (36.1 vs 25.2 us per cfg2 W2S launch in the
// step): with the keep bit on the A value, each 4x4x1 MFMA (11 cycles alone) costs 27
// cycles per wave (tools/census/mfma_rate_probe.hip), i.e. the two mask VALU per 256
// MACs outweigh the padding the 16x16x4 form wastes.  Dev opt-in (HSG_HPROJ_DWM4=1).
// the bf16 limb MFMA dW (k_hproj_dw_mf): D = 8, H <= 8 (dev A/B: HSG_HPROJ_DWMF=0 restores
// the 16x16x4 kernel)
bool dw_mf_shape(int in, int H, int D) {
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_DWMF")) if (atoi(e) == 0) return false;
    return D == 8 && H >= 1 && H <= 8 && in >= 1;
}

bool dw_m4_shape(int in, int H, int D) {
    const char *e = HSG_DEV_ENV("HSG_HPROJ_DWM4");
    return e && atoi(e) == 1 && D % 4 == 0 && H * D <= 64 && in % 4 == 0;
}

DwM4Geom dw_m4_geom(int n, int in) {
    DwM4Geom g;
    g.ctiles = (in + M4C - 1) / M4C;
    int per = 4;                                          // 32-row steps per chunk (128 rows)
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_DWM4_STEPS")) per = atoi(e) > 0 ? atoi(e) : per;   // dev sweep
    const int steps = (n + 31) / 32 > 0 ? (n + 31) / 32 : 1;
    if (per > steps) per = steps;
    g.rows = per * 32;
    g.chunks = (steps + per - 1) / per;
    return g;
}

__global__ __launch_bounds__(64 * M4W) void k_hproj_dw_m4(int n, int in, int H, int D, int rows_per_chunk,
                                                        const float *__restrict__ dZ, int ldz,
                                                        const float *__restrict__ X, int ldx,
                                                        const uint32_t *__restrict__ bits, float *__restrict__ part) {
    constexpr int NT = 64 * M4W;
    constexpr int XQ = M4C / 4;                           // column quads per block row
    constexpr int NXL = (32 * XQ + NT - 1) / NT;          // X float4 loads per thread per step
    constexpr int NZL = (32 * 16 + NT - 1) / NT;          // dZ float4 loads per thread per step
    __shared__ __attribute__((aligned(16))) float Xt[M4C][M4XS];
    __shared__ __attribute__((aligned(16))) float Zs[32][64];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int HD = H * D, NWI = (n + 31) / 32, LDC = mask_ldc(in);
    const int cb = blockIdx.x * M4C, cw = wv * M4Q * 4;  // block / wave column offsets
    const int rb = blockIdx.y * rows_per_chunk;
    const int rend = min(rb + rows_per_chunk, n);
    const auto rX = rsrc(X, (long)n * ldx * 4);
    const auto rZ = rsrc(dZ, (long)n * ldz * 4);
    const auto rM = rsrc(bits, (long)H * NWI * LDC * 4);
    const int i4 = lane & 3, kb = min(lane & ~3, HD - 1) / D;   // A index, head of the lane's block
    u32x4v xg[NXL], zg[NZL];
    uint32_t mw[M4Q], mn[M4Q];
    auto fetch = [&](int r0) {
#pragma unroll
        for (int v = 0; v < NXL; ++v) {
            const int u = tid + NT * v, row = u / XQ, cq = u % XQ, col = cb + 4 * cq;
            const bool ok = u < 32 * XQ && r0 + row < rend && col < in;
            xg[v] = bld4(rX, ok ? (uint32_t)((r0 + row) * ldx + col) * 4 : kOOB);
        }
#pragma unroll
        for (int v = 0; v < NZL; ++v) {
            const int u = tid + NT * v, row = u >> 4, c4 = (u & 15) * 4;
            const bool ok = u < 32 * 16 && r0 + row < rend && c4 < HD;
            zg[v] = bld4(rZ, ok ? (uint32_t)((r0 + row) * ldz + c4) * 4 : kOOB);
        }
#pragma unroll
        for (int q = 0; q < M4Q; ++q) {
            const int col = cb + cw + 4 * q + i4;
            mn[q] = bldu(rM, col < in ? (uint32_t)((kb * NWI + r0 / 32) * LDC + col) * 4 : kOOB);
        }
    };
    auto stash = [&]() {
#pragma unroll
        for (int v = 0; v < NXL; ++v) {
            const int u = tid + NT * v, row = u / XQ, cq = u % XQ;
            if (u < 32 * XQ) {
                const int pos = (((row >> 2) ^ (cq & 7)) << 2) | (row & 3);
#pragma unroll
                for (int e = 0; e < 4; ++e) Xt[4 * cq + e][pos] = __uint_as_float(xg[v][e]);
            }
        }
#pragma unroll
        for (int v = 0; v < NZL; ++v) {
            const int u = tid + NT * v;
            if (u < 32 * 16) *reinterpret_cast<u32x4v *>(&Zs[u >> 4][(u & 15) * 4]) = zg[v];
        }
    };
    f32x4v acc[M4Q];
#pragma unroll
    for (int q = 0; q < M4Q; ++q) acc[q] = f32x4v{0.f, 0.f, 0.f, 0.f};
    if (rb < rend) fetch(rb);
    for (int r0 = rb; r0 < rend; r0 += 32) {
        __syncthreads();                                   // every wave is done with the last step
        stash();
#pragma unroll
        for (int q = 0; q < M4Q; ++q) mw[q] = mn[q];
        __syncthreads();
        if (r0 + 32 < rend) fetch(r0 + 32);
#pragma unroll
        for (int g = 0; g < 8; ++g) {                      // 4-row groups
            f32x4v xq[M4Q];
#pragma unroll
            for (int q = 0; q < M4Q; ++q) {
                const int cl = cw + 4 * q + i4, cq = (cw >> 2) + q;
                xq[q] = *reinterpret_cast<const f32x4v *>(&Xt[cl][(g ^ (cq & 7)) << 2]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int rr = 4 * g + e;
                const float bz = Zs[rr][lane];
#pragma unroll
                for (int q = 0; q < M4Q; ++q) {
                    const int keep = __builtin_amdgcn_sbfe((int)mw[q], rr, 1);   // 0 or -1
                    const float a = __uint_as_float(__float_as_uint(xq[q][e]) & (uint32_t)keep);
                    acc[q] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, bz, acc[q], 0, 0, 0);
                }
            }
        }
    }
    if (lane < HD) {
        float *dst = part + (long)blockIdx.y * HD * in + (long)lane * in;
#pragma unroll
        for (int q = 0; q < M4Q; ++q) {
            const int col = cb + cw + 4 * q;
            if (col < in) *reinterpret_cast<f32x4v *>(dst + col) = acc[q];
        }
    }
}

__global__ __launch_bounds__(256) void k_sum_parts(long total, int chunks, float scale, const float *__restrict__ part,
                                                   float *__restrict__ out, int accumulate) {
    for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
        float s = 0.f;
#pragma unroll 8
        for (int z = 0; z < chunks; ++z) s += part[(long)z * total + e];
        out[e] = accumulate ? out[e] + s * scale : s * scale;
    }
}

int status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

float drop_scale(float p) {
    const float t = p * 65536.f;
    const float thr = (float)(uint32_t)(t >= 65535.f ? 65535.f : t);
    return 1.f / (1.f - thr / 65536.f);
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// buffer descriptors address < 2 GiB per operand (kOOB is the first bad offset)
bool fits_buffers(int n, int in, int H, int D, int ld_rows) {
    const long lim = (long)kOOB;
    return (long)n * ld_rows * 4 < lim && (long)H * D * in * 4 < lim &&
           (long)H * ((n + 31) / 32) * mask_ldc(in) * 4 < lim;
}

}  // namespace

extern "C" {

int hsg_dropmask_words(int n, int in, int H) { return H * ((n + 31) / 32) * mask_ldc(in); }

float hsg_dropmask_scale(float p) { return drop_scale(p); }

int hsg_dropmask(int n, int in, int H, float p, const int64_t *seed, uint32_t offset, uint32_t *bits,
                 void *stream) {
    if (n < 0 || in < 1 || H < 1 || p < 0.f || p >= 1.f || !seed || !bits) return HSG_EINVAL;
    if ((long)n * in * ((H + 1) / 2) >= (1L << 32)) return HSG_EINVAL;   // 32-bit hash counter
    if (n == 0) return 0;
    const long total = (long)((H + 1) / 2) * ((n + 31) / 32) * mask_ldc(in);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_dropmask, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, in, H, p, seed, offset,
                       bits);
    return status();
}

int hsg_seed_advance(int64_t *seed, int64_t *snap, void *stream) {
    if (!seed || !snap) return HSG_EINVAL;
    hipLaunchKernelGGL(k_seed_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, seed, snap);
    return status();
}

int hsg_dropmask_multi(int njobs, const int *n, const int *in, const int *H, const float *p, const int64_t *seed,
                       const uint32_t *offset, uint32_t *const *bits, void *stream) {
    return hsg_dropmask_multi_wt(njobs, n, in, H, p, seed, offset, bits, 0, 0, 0, nullptr, nullptr, stream);
}

int hsg_dropmask_multi_wt(int njobs, const int *n, const int *in, const int *H, const float *p, const int64_t *seed,
                          const uint32_t *offset, uint32_t *const *bits, int wH, int wD, int wIn, const float *W,
                          float *Wt, void *stream) {
    return hsg_step_prologue(njobs, n, in, H, p, seed, offset, bits, wH, wD, wIn, W, Wt, 0, nullptr, nullptr,
                             nullptr, nullptr, nullptr, nullptr, stream);
}

int hsg_step_prologue(int njobs, const int *n, const int *in, const int *H, const float *p, const int64_t *seed,
                      const uint32_t *offset, uint32_t *const *bits, int wH, int wD, int wIn, const float *W,
                      float *Wt, int nsplit, const float *const *sW, const int *sN, const int *sK, const int *sldw,
                      const int *strans, void *const *splanes, void *stream) {
    if (njobs < 1 || njobs > 8 || !seed) return HSG_EINVAL;
    if (nsplit < 0 || nsplit > 4 || (nsplit > 0 && (!sW || !sN || !sK || !sldw || !strans || !splanes)))
        return HSG_EINVAL;
    if (W && (wH < 1 || wD < 1 || wIn < 1 || !Wt)) return HSG_EINVAL;
    DropJobs j{};
    j.W = W;
    j.Wt = Wt;
    j.wH = wH;
    j.wD = wD;
    j.wIn = wIn;
    j.njobs = njobs;
    j.start[0] = 0;
    // 2 units per thread: 26.1 -> 24.4 us per cfg2 prologue (4: 24.6, 8: 27.1;
    // profiles/r05/ab_dropmask_upt/)
    j.upt = 2;
    if (const char *e = HSG_DEV_ENV("HSG_DROPMASK_UPT")) j.upt = max(1, min(16, atoi(e)));    // dev A/B
    for (int q = 0; q < njobs; ++q) {
        if (n[q] < 0 || in[q] < 1 || H[q] < 1 || p[q] < 0.f || p[q] >= 1.f || !bits[q]) return HSG_EINVAL;
        if ((long)n[q] * in[q] * ((H[q] + 1) / 2) >= (1L << 32)) return HSG_EINVAL;
        j.n[q] = n[q]; j.in[q] = in[q]; j.H[q] = H[q]; j.p[q] = p[q]; j.offset[q] = offset[q]; j.bits[q] = bits[q];
        const long total = (long)((H[q] + 1) / 2) * ((n[q] + 31) / 32) * mask_ldc(in[q]);
        j.start[q + 1] = j.start[q] + (int)((total + 256L * j.upt - 1) / (256L * j.upt));
    }
    const int wblocks = W ? (wIn + 63) / 64 * wH : 0;
    j.ws_first = j.start[njobs] + wblocks;
    if (nsplit > 0 && hsg_wsplit_setup(j.ws, nsplit, sW, sN, sK, sldw, strans, splanes)) return HSG_EINVAL;
    const int total = j.ws_first + (nsplit > 0 ? j.ws.start[nsplit] : 0);
    if (total == 0) return 0;
    hipLaunchKernelGGL(k_dropmask_multi, dim3(total), dim3(256), 0, (hipStream_t)stream, j, seed);
    return status();
}

int hsg_hproj_fwd(int n, int in, int H, int D, const float *X, int ldx, const float *W, const uint32_t *bits,
                  float p, float *Z, int ldz, void *stream) {
    return hsg_hproj_fwd_logits(n, in, H, D, X, ldx, W, bits, p, Z, ldz, nullptr, nullptr, stream);
}

int hsg_hproj_fwd_logits_supported(int H, int D) {
    const int sph = (D + 15) / 16;
    return H >= 1 && D >= 1 && 4 % sph == 0 ? 1 : 0;                // the slot group holds whole heads
}

int hsg_hproj_fwd_logits(int n, int in, int H, int D, const float *X, int ldx, const float *W, const uint32_t *bits,
                         float p, float *Z, int ldz, const float *a1, float *sigma, void *stream) {
    if (n < 0 || in < 1 || H < 1 || D < 1 || ldx < in || !fits_buffers(n, in, H, D, ldx)) return HSG_EINVAL;
    if ((a1 == nullptr) != (sigma == nullptr)) return HSG_EINVAL;
    if (a1 && !hsg_hproj_fwd_logits_supported(H, D)) return HSG_EINVAL;
    if (n == 0) return 0;
    const int sph = (D + 15) / 16;
    const int ns = H * sph;
    const bool vec = in % 4 == 0 && ldx % 4 == 0 && aligned16(X) && aligned16(W);
    // slot-group size: 2 when a head has at most 2 slots (W2S, D = 8: 28.6 us against
    // 32.1 us at SG = 4, rocprofv3 kernel trace), else 4 (whole heads per wave)
    int sg = sph <= 2 ? 2 : 4;
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_SG")) {                     // dev A/B
        const int v = atoi(e);
        sg = (v == 1 && sph == 1) ? 1 : (v == 2 && sph <= 2) ? 2 : 4;
    }
    int pf = 1;                                                                       // register ring depth (2, 4: no gain, tools/ab.py)
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_PF")) pf = atoi(e);                         // dev A/B (1, 2, 4)
    // one wave per block: the small S2W grid (420 waves at cfg2) spreads over more CUs
    // (8.84 -> 8.34 us per launch in the trace; step -3 us and +-0 us in two A/Bs)
    int wpb = 1;
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_WPB")) wpb = atoi(e) == 4 ? 4 : (atoi(e) == 2 ? 2 : 1);   // dev A/B
#define HSG_HF(SG_)                                                                                              \
    {                                                                                                            \
        const long tasks = (long)((n + 15) / 16) * ((ns + SG_ - 1) / SG_);                                       \
        const dim3 grid((unsigned)((tasks + wpb - 1) / wpb)), blk(64 * wpb);                                     \
        if (HSG_PF_DEV && vec && pf == 4)                                                                        \
            hipLaunchKernelGGL((k_hproj_fwd<SG_, true, HSG_PF_DEV ? 4 : 1>), grid, blk, 0, (hipStream_t)stream, n, \
                               in, H, D, X, ldx, W, bits, drop_scale(p), Z, ldz, a1, sigma);                     \
        else if (HSG_PF_DEV && vec && pf == 2)                                                                   \
            hipLaunchKernelGGL((k_hproj_fwd<SG_, true, HSG_PF_DEV ? 2 : 1>), grid, blk, 0, (hipStream_t)stream, n, \
                               in, H, D, X, ldx, W, bits, drop_scale(p), Z, ldz, a1, sigma);                     \
        else if (vec)                                                                                            \
            hipLaunchKernelGGL((k_hproj_fwd<SG_, true>), grid, blk, 0, (hipStream_t)stream, n, in, H, D, X,       \
                               ldx, W, bits, drop_scale(p), Z, ldz, a1, sigma);                                  \
        else                                                                                                     \
            hipLaunchKernelGGL((k_hproj_fwd<SG_, false>), grid, blk, 0, (hipStream_t)stream, n, in, H, D, X,      \
                               ldx, W, bits, drop_scale(p), Z, ldz, a1, sigma);                                  \
    }
#ifdef HSG_DEV
    if (sg == 1) HSG_HF(1) else
#endif
    if (sg == 2) HSG_HF(2) else HSG_HF(4)
#undef HSG_HF
    return status();
}

int hsg_hproj_wt(int H, int D, int in, const float *W, float *Wt, void *stream) {
    if (H < 1 || D < 1 || in < 1 || !W || !Wt) return HSG_EINVAL;
    hipLaunchKernelGGL(k_hproj_wt, dim3((unsigned)((in + 63) / 64), (unsigned)H), dim3(256), 0, (hipStream_t)stream, H,
                       D, in, W, Wt);
    return status();
}

int hsg_hproj_fwd_t8_supported(int in, int H, int D) {
    return D == 8 && H >= 1 && in >= 4 && in % 4 == 0 ? 1 : 0;
}

int hsg_hproj_fwd_t8(int n, int in, int H, const float *X, int ldx, const float *Wt, const uint32_t *bits, float p,
                     float *Z, int ldz, const float *a1, float *sigma, void *stream) {
    if (n < 0 || !hsg_hproj_fwd_t8_supported(in, H, 8) || ldx < in || ldx % 4 != 0 || ldz < H * 8 ||
        ldz % 4 != 0 || !X || !Wt || !bits || !Z || !aligned16(X) || !aligned16(Z) || !fits_buffers(n, in, H, 8, ldx))
        return HSG_EINVAL;
    if ((a1 == nullptr) != (sigma == nullptr)) return HSG_EINVAL;
    if (n == 0) return 0;
    // block = HB heads x KS K parts (HSG_HPROJ_FWD_PLAN = HB*10 + KS for A/B)
    hipStream_t st = (hipStream_t)stream;
    const float s = drop_scale(p);
    const int nrt = (n + 63) / 64;
#ifdef HSG_DEV
    int plan = 22;
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_FWD_PLAN")) plan = atoi(e);
#define HSG_T8(HB_, KS_)                                                                                          \
    if (plan == HB_ * 10 + KS_) {                                                                                 \
        const int bpr = (H + HB_ - 1) / HB_;                                                                      \
        hipLaunchKernelGGL((k_hproj_fwd_v8<HB_, KS_>), dim3((unsigned)((nrt + 7) / 8 * 8 * bpr)),                 \
                           dim3(64 * HB_ * KS_), 0, st, n, in, H, X, ldx, Wt, bits, s, Z, ldz, a1, sigma);       \
        return status();                                                                                          \
    }
    HSG_T8(4, 2) HSG_T8(8, 1) HSG_T8(4, 1) HSG_T8(2, 4) HSG_T8(1, 4)
#undef HSG_T8
#endif
    const int bpr = (H + 1) / 2;
    hipLaunchKernelGGL((k_hproj_fwd_v8<2, 2>), dim3((unsigned)((nrt + 7) / 8 * 8 * bpr)), dim3(256), 0, st, n, in, H,
                       X, ldx, Wt, bits, s, Z, ldz, a1, sigma);
    return status();
}

// D = 8 on bf16 limb MFMAs (k_hproj_fwd_mf): W as hsg_wsplit planes [3][Np][Kp] of
// W [H*8][in] (rows = outputs)
int hsg_hproj_fwd_mf_supported(int in, int H, int D) {
    return D == 8 && H >= 1 && H <= 8 && in >= 4 && in % 4 == 0 ? 1 : 0;
}
int hsg_hproj_fwd_mf(int n, int in, int H, const float *X, int ldx, const void *planes, int Np, int Kp,
                     const uint32_t *bits, float p, float *Z, int ldz, const float *a1, float *sigma, void *stream) {
    if (n < 0 || !hsg_hproj_fwd_mf_supported(in, H, 8) || ldx < in || ldx % 4 != 0 || ldz < H * 8 || !X ||
        !planes || !bits || !Z || !aligned16(X) || !aligned16(planes) || Np < H * 8 || Kp < in || Kp % 32 != 0 ||
        !fits_buffers(n, in, H, 8, ldx) || (long)3 * Np * Kp * 2 >= (long)kOOB)
        return HSG_EINVAL;
    if ((a1 == nullptr) != (sigma == nullptr)) return HSG_EINVAL;
    if (n == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const float s = drop_scale(p);
    const dim3 grid((unsigned)((n + 31) / 32));
    hipLaunchKernelGGL(k_hproj_fwd_mf, grid, dim3(256), 0, st, n, in, H, X, ldx,
                       reinterpret_cast<const __bf16 *>(planes), Np, Kp, bits, s, Z, ldz, a1, sigma);
    return status();
}

int hsg_hproj_dx(int n, int in, int H, int D, const float *dZ, int ldz, const float *W, const uint32_t *bits,
                 float p, float *dX, int ldx, int accumulate, void *stream) {
    if (n < 0 || in < 1 || H < 1 || D < 1 || ldz < H * D || !fits_buffers(n, in, H, D, ldz)) return HSG_EINVAL;
    if (n == 0) return 0;
    const float s = drop_scale(p);
    hipStream_t st = (hipStream_t)stream;
    const long rtiles = (n + 15) / 16;
    // wide wave tiles (16 x 64) when that still gives >= 2048 waves, else 16 x 16
    const long wide = rtiles * ((in + 63) / 64);
#ifdef HSG_DEV
    if (const char *e = HSG_DEV_ENV("HSG_HPROJ_DX")) {                     // dev sweep: CT*10 + HF
        const int v = atoi(e), ct = v / 10, hf = v % 10;
        const long tiles = rtiles * ((in + 16 * ct - 1) / (16 * ct));
        const dim3 g((unsigned)((tiles + 3) / 4));
#define HSG_DXV(CT_, HF_)                                                                                       \
    if (ct == CT_ && hf == HF_) {                                                                               \
        hipLaunchKernelGGL((k_hproj_dx<CT_, HF_>), g, dim3(256), 0, st, n, in, H, D, dZ, ldz, W, bits, s, dX, ldx, \
                           accumulate);                                                                         \
        return status();                                                                                        \
    }
        HSG_DXV(4, 1) HSG_DXV(4, 4) HSG_DXV(2, 2)
#undef HSG_DXV
    }
#endif
    // dev A/B (HSG_HPROJ_DXPRE): 0 = the chained kernels only; 1 (default) = one wave
    // per head when the grid is small, k_hproj_dx_n8 for narrow heads; 2 = one wave per
    // head for every small-D shape that is not narrow
    // (an up-front-operand form of k_hproj_dx<4, 1> with dword loads: 35.7 us, slower)
    const char *pe = HSG_DEV_ENV("HSG_HPROJ_DXPRE");
    const int mode = pe ? atoi(pe) : 1;
    if (mode != 0 && wide >= 2048 && H <= 8 && D == 8 && in % 4 == 0 && ldx % 4 == 0 && ldz % 2 == 0 &&
        aligned16(dX) && ((uintptr_t)dZ & 7) == 0 && aligned16(W)) {
        // narrow heads: 16-byte operand pieces, all requested up front (W2S)
        // two heads' operands at a time (22.4 us cold; 4 / 8 at a time: 23.2 / 23.1 us)
        // dev A/B: HSG_HPROJ_DX_SEL=1 restores the compare + select masking
        const char *se = HSG_DEV_ENV("HSG_HPROJ_DX_SEL");
        if (se && atoi(se) == 1)
            hipLaunchKernelGGL((k_hproj_dx_n8<8, 2, false>), dim3((unsigned)((wide + 3) / 4)), dim3(256), 0, st, n, in,
                               H, dZ, ldz, W, bits, s, dX, ldx, accumulate);
        else
            hipLaunchKernelGGL((k_hproj_dx_n8<8, 2>), dim3((unsigned)((wide + 3) / 4)), dim3(256), 0, st, n, in, H, dZ,
                               ldz, W, bits, s, dX, ldx, accumulate);
        return status();
    }
    if (mode != 0 && (wide < 2048 || mode == 2) && H <= 16 && D <= 64) {
        // few rows, wide heads: one wave per head (S2W: 6.4 us against 17.7 us for the
        // chained kernel, cold cache)
        const unsigned blocks = (unsigned)(rtiles * ((in + 15) / 16));
        if (D <= 32)
            hipLaunchKernelGGL((k_hproj_dx_hw<8>), dim3(blocks), dim3(64 * H), 0, st, n, in, H, D, dZ, ldz, W, bits, s,
                               dX, ldx, accumulate);
        else
            hipLaunchKernelGGL((k_hproj_dx_hw<16>), dim3(blocks), dim3(64 * H), 0, st, n, in, H, D, dZ, ldz, W, bits,
                               s, dX, ldx, accumulate);
        return status();
    }
    if (wide >= 2048) {                  // HF = 1: 26.9 us vs 28.0 (HF = 2) on the W2S shape
        hipLaunchKernelGGL((k_hproj_dx<4, 1>), dim3((unsigned)((wide + 3) / 4)), dim3(256), 0, st, n, in, H, D, dZ,
                           ldz, W, bits, s, dX, ldx, accumulate);
    } else {
        const long narrow = rtiles * ((in + 15) / 16);
        hipLaunchKernelGGL((k_hproj_dx<1, 4>), dim3((unsigned)((narrow + 3) / 4)), dim3(256), 0, st, n, in, H, D,
                           dZ, ldz, W, bits, s, dX, ldx, accumulate);
    }
    return status();
}

int hsg_hproj_bwd(int n, int in, int H, int D, const float *dZ, int ldz, const float *W, const float *X, int ldx,
                  const uint32_t *bits, float p, float *dX, int ldxo, int accumulate, float *part, void *stream) {
    if (n < 0 || in < 1 || H < 1 || D < 1 || !dZ || !W || !X || !bits || !dX || !part || ldx < in || ldxo < in ||
        ldz < H * D || !fits_buffers(n, in, H, D, ldx > ldz ? ldx : ldz) || !fits_buffers(n, in, H, D, ldxo))
        return HSG_EINVAL;
    if (n == 0) return 0;
    // the merged launch where the two-launch path would run k_hproj_dx_hw and the
    // dword-staged k_hproj_dw<4> (the S2W shape); dev A/B: HSG_HPROJ_BWD_MERGE=0
    const long rtiles = (n + 15) / 16, wide = rtiles * ((in + 63) / 64);
    const char *me = HSG_DEV_ENV("HSG_HPROJ_BWD_MERGE");
    const char *pe = HSG_DEV_ENV("HSG_HPROJ_DXPRE");
    const bool vec = dw_slots() == 4 && D == 8 && in % 4 == 0 && ldx % 4 == 0 && ldz % 4 == 0 && aligned16(X) &&
                     aligned16(dZ);
    const bool merge = (!me || atoi(me) != 0) && (!pe || atoi(pe) == 1) && wide < 2048 && H <= 16 && D <= 64 &&
                       !dw_mf_shape(in, H, D) && !dw_m4_shape(in, H, D) && dw_slots() == 4 && !vec;
    // the narrow-head (W2S) pair in one launch (round 6): where the two-launch path would
    // run k_hproj_dx_n8 and k_hproj_dw_mf; dev A/B: HSG_HPROJ_BWD_N8=0
    const char *ne = HSG_DEV_ENV("HSG_HPROJ_BWD_N8");
    const bool merge_n8 = (!ne || atoi(ne) != 0) && (!me || atoi(me) != 0) && (!pe || atoi(pe) == 1) &&
                          wide >= 2048 && H <= 8 && D == 8 && in % 4 == 0 && ldxo % 4 == 0 && ldz % 2 == 0 &&
                          aligned16(dX) && ((uintptr_t)dZ & 7) == 0 && aligned16(W) && dw_mf_shape(in, H, D) &&
                          !HSG_DEV_ENV("HSG_HPROJ_DX_SEL") && !HSG_DEV_ENV("HSG_HPROJ_DWMF_P");
    if (merge_n8) {
        const DwGeom g = dw_geom(n, in, H, D);
        const int ctiles = (in + 63) / 64, dx_blocks = (int)((wide + 3) / 4);
        const unsigned total = (unsigned)(dx_blocks + ctiles * g.chunks);
        hipLaunchKernelGGL(k_hproj_bwd_n8, dim3(total), dim3(256), 0, (hipStream_t)stream, n, in, H, dZ, ldz, W, bits,
                           drop_scale(p), dX, ldxo, accumulate, X, ldx, g.rows, part, dx_blocks, ctiles, g.chunks);
        return status();
    }
    if (!merge) {
        int rc = hsg_hproj_dx(n, in, H, D, dZ, ldz, W, bits, p, dX, ldxo, accumulate, stream);
        if (rc) return rc;
        return hsg_hproj_dw(n, in, H, D, dZ, ldz, X, ldx, bits, p, part, nullptr, 0, stream);
    }
    const DwGeom g = dw_geom(n, in, H, D);
    const int dx_blocks = (int)(rtiles * ((in + 15) / 16));
    const unsigned total = (unsigned)(dx_blocks + g.ctiles * g.sgroups * g.chunks);
    if (D <= 32)
        hipLaunchKernelGGL(k_hproj_bwd_hw<8>, dim3(total), dim3(256), 0, (hipStream_t)stream, n, in, H, D, dZ, ldz, W,
                           bits, drop_scale(p), dX, ldxo, accumulate, X, ldx, g.rows, part, dx_blocks, g.ctiles,
                           g.sgroups);
    else
        hipLaunchKernelGGL(k_hproj_bwd_hw<16>, dim3(total), dim3(256), 0, (hipStream_t)stream, n, in, H, D, dZ, ldz, W,
                           bits, drop_scale(p), dX, ldxo, accumulate, X, ldx, g.rows, part, dx_blocks, g.ctiles,
                           g.sgroups);
    return status();
}

int hsg_hproj_dw_chunks(int n, int in, int H, int D) {
    if (n < 0 || in < 1 || H < 1 || D < 1) return 0;
    if (dw_mf_shape(in, H, D)) return dw_geom(n, in, H, D).chunks;
    return dw_m4_shape(in, H, D) ? dw_m4_geom(n, in).chunks : dw_geom(n, in, H, D).chunks;
}

int hsg_hproj_dw(int n, int in, int H, int D, const float *dZ, int ldz, const float *X, int ldx,
                 const uint32_t *bits, float p, float *part, float *dW, int accumulate, void *stream) {
    if (n < 0 || in < 1 || H < 1 || D < 1 || !part || ldx < in || ldz < H * D ||
        !fits_buffers(n, in, H, D, ldx > ldz ? ldx : ldz))
        return HSG_EINVAL;
    hipStream_t st = (hipStream_t)stream;
    DwGeom g = dw_geom(n, in, H, D);
    const long total = (long)H * D * in;
    if (dw_mf_shape(in, H, D) && n > 0) {
        // D = 8 on bf16 limb MFMAs, on the 16x16x4 kernel's row chunks (same slabs)
#ifdef HSG_DEV
        // dev A/B: pitch 48 (conflict-free fragment reads): 22.05 / 22.21 vs 22.53 / 22.17 us
        // with pitch 40 back to back -- the 2-way reads do not bound it
        const char *pe = HSG_DEV_ENV("HSG_HPROJ_DWMF_P");
        if (pe && atoi(pe) == 48)
            hipLaunchKernelGGL(k_hproj_dw_mf<48>, dim3((in + 63) / 64, g.chunks), dim3(256), 0, st, n, in, H, g.rows, dZ,
                               ldz, X, ldx, bits, part);
        else if (pe && atoi(pe) == 40)
            hipLaunchKernelGGL(k_hproj_dw_mf<40>, dim3((in + 63) / 64, g.chunks), dim3(256), 0, st, n, in, H, g.rows, dZ,
                               ldz, X, ldx, bits, part);
        else
#endif
            hipLaunchKernelGGL(k_hproj_dw_mf<32>, dim3((in + 63) / 64, g.chunks), dim3(256), 0, st, n, in, H, g.rows, dZ,
                               ldz, X, ldx, bits, part);
        if (int rc = status()) return rc;
        if (!dW) return 0;
        int blocks = (int)((total + 255) / 256);
        if (blocks > 2048) blocks = 2048;
        hipLaunchKernelGGL(k_sum_parts, dim3(blocks), dim3(256), 0, st, total, g.chunks, drop_scale(p), part, dW,
                           accumulate);
        return status();
    }
    if (dw_m4_shape(in, H, D)) {
        // the chunking is the 4x4x1 kernel's (hsg_hproj_dw_chunks); operands it cannot
        // take as 16-byte rows go to the 16x16x4 kernel on the same row chunks
        const DwM4Geom m = dw_m4_geom(n, in);
        if (n > 0 && ldx % 4 == 0 && ldz % 4 == 0 && aligned16(X) && aligned16(dZ)) {
            hipLaunchKernelGGL(k_hproj_dw_m4, dim3(m.ctiles, m.chunks), dim3(64 * M4W), 0, st, n, in, H, D, m.rows,
                               dZ, ldz, X, ldx, bits, part);
            if (int rc = status()) return rc;
            if (!dW) return 0;
            int blocks = (int)((total + 255) / 256);
            if (blocks > 2048) blocks = 2048;
            hipLaunchKernelGGL(k_sum_parts, dim3(blocks), dim3(256), 0, st, total, m.chunks, drop_scale(p), part, dW,
                               accumulate);
            return status();
        }
        g.rows = m.rows;
        g.chunks = m.chunks;
    }
    if (n > 0) {
        const char *ve = HSG_DEV_ENV("HSG_HPROJ_DWVEC");                   // dev A/B: 0 = dword staging
        const bool vec = (!ve || atoi(ve) != 0) && dw_slots() == 4 && D == 8 && in % 4 == 0 && ldx % 4 == 0 &&
                         ldz % 4 == 0 && aligned16(X) && aligned16(dZ);
        if (vec)
            hipLaunchKernelGGL((k_hproj_dw<4, true>), dim3(g.ctiles, g.sgroups, g.chunks), dim3(256), 0, st, n, in, H,
                               D, g.rows, dZ, ldz, X, ldx, bits, part);
#ifdef HSG_DEV
        else if (dw_slots() == 8)
            hipLaunchKernelGGL(k_hproj_dw<8>, dim3(g.ctiles, g.sgroups, g.chunks), dim3(256), 0, st, n, in, H, D,
                               g.rows, dZ, ldz, X, ldx, bits, part);
#endif
        else
            hipLaunchKernelGGL(k_hproj_dw<4>, dim3(g.ctiles, g.sgroups, g.chunks), dim3(256), 0, st, n, in, H, D,
                               g.rows, dZ, ldz, X, ldx, bits, part);
        int rc = status();
        if (rc) return rc;
    }
    if (!dW) return n > 0 ? 0 : HSG_EINVAL;            // partial slabs only (hsg_slab_reduce sums them)
    int blocks = (int)((total + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(k_sum_parts, dim3(blocks), dim3(256), 0, st, total, n > 0 ? g.chunks : 0, drop_scale(p),
                       part, dW, accumulate);
    return status();
}

}  // extern "C"
