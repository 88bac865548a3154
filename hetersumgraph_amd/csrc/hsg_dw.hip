// hsg_dw.hip -- the FFN weight gradients of one WSWGAT layer, BOTH in ONE launch (gfx950).
//
// Replaces the two deferred split-K GEMMs of the fused stack's backward
// (PositionwiseFeedForward, module/GATLayer.py:35-44: dW2 = dY^T H and dW1 = dH^T X
// over every application's rows, K = applications x rows = 38,400 at cfg2 for S2W).
// Both operands are M/N-contiguous ([K][M] and [K][N] row-major: the activations as the
// forward wrote them), the products fp32-accurate (three bf16 limbs per operand, six
// products on v_mfma_f32_16x16x32_bf16, as k_gemm3; NL = 1: the bf16 mode's one
// product), and the K slices are written as partial slabs [splits][M][N] that
// hsg_slab_reduce sums in a fixed order (deterministic, no atomics).
//
// Why a kernel of its own (round 4): k_gemm3's 64x64 tiles move (64 + 64) x 4 B of
// operand per K row for 4,096 outputs; at cfg2 the two S2W weight gradients pulled
// 1.57 GB through L2 per step (99 + 98 us, L2->CU bound).  Here a
// block owns 160 x 128 outputs (2 x 2 waves of 80 x 64, 16x16x32 MFMAs), so the
// same work moves 0.71 GB, and both GEMMs of a layer share one grid of exactly two
// blocks per CU (16 tiles x 32 K slices at cfg2): half the slab bytes of 64 slices.
//
// Pipeline (k_gemm3's): global -> registers (float4 along M/N), split into limbs,
// ds_write_b64 into k-major limb images, two barriers per 32-deep K tile, the next
// tile's global loads in flight during the MFMAs.  Fragments come back k-contiguous
// through the hardware transpose read ds_read_b64_tr_b16 (two per fragment), on image
// layouts chosen so that every such read is bank-conflict-free (Img below).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "../../include/hsg.h"
#include "hsg_dev.h"
#include "hsg_wsplit.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short v4s16 __attribute__((ext_vector_type(4)));
typedef short v8s16 __attribute__((ext_vector_type(8)));

constexpr int kBK = 32;            // K rows per tile = one 16x16x32 MFMA step
constexpr int kNT = 256;           // 4 waves, 2 x 2 over the output tile

// k-major limb image of one operand's K tile: 32 rows (k) x ROWS columns (m or n), bf16.
// A fragment read (16x16x32 operand: lane l takes column c0 + (l & 15), k = 8 (l >> 4)
// + 0..7) touches, per 32-lane half, 8 image rows x 16 columns = 8 windows of 8 dwords;
// the layout puts those 8 windows on 8 distinct 8-bank groups:
//   ROWS % 128 == 0: a row is a multiple of 64 dwords (every row starts at bank 0), and
//     16-column group j of row r sits at group j ^ f(r), f(r) = (r & 3) | ((r >> 3) & 1) << 2;
//   ROWS = 160 (80 dwords = 16 mod 64 per row): 16 bf16 of padding after every 8 rows,
//     so rows r and r + 8 start 8 dwords apart.
template <int ROWS>
struct Img {
    static_assert(ROWS % 128 == 0 || ROWS == 160, "image layout");
    static constexpr bool XOR = ROWS % 128 == 0;
    static constexpr int SIZE = XOR ? kBK * ROWS : kBK * ROWS + 16 * (kBK / 8);   // bf16 per limb plane
    __device__ __forceinline__ static int off(int r, int c) {     // c % 4 == 0
        if constexpr (XOR) {
            const int f = (r & 3) | (((r >> 3) & 1) << 2);
            return r * ROWS + (((c >> 4) ^ f) << 4) + (c & 15);
        } else {
            return r * ROWS + 16 * (r >> 3) + c;
        }
    }
};

// One operand's K tile in registers: thread t of NT covers (k row, 4 consecutive
// columns) units t, t + NT, ...; rows past the K slice and columns past M/N load
// zeros; units past the tile (NT not dividing it) are idle.
template <int ROWS, int NL, int NT = kNT, bool BF = false>
struct Stage {
    static constexpr int UNITS = kBK * ROWS / 4;
    static constexpr int NU = (UNITS + NT - 1) / NT;
    // BF (the bf16 mode's bf16 activations, round 5): the operand is bf16 rows, read as
    // 8-byte quads and kept as they are until the image store -- converting them in
    // load() made every prefetch wait at once (k_dw 140 vs 58 us at cfg5); the image then
    // holds the same values the fp32 path's RNE conversion would put there
    typedef typename std::conditional<BF, bf16x4, f32x4>::type Unit;
    typedef typename std::conditional<BF, __bf16, float>::type Elem;
    Unit v[NU];

    __device__ __forceinline__ void load(const void *__restrict__ g, int ld, int c0, int nc, int k0, int k1) {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int idx = threadIdx.x + NT * i;
            const int kk = idx / (ROWS / 4), c = c0 + 4 * (idx % (ROWS / 4));
            Unit x;
            if constexpr (BF) x = bf16x4{(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
            else x = f32x4{0.f, 0.f, 0.f, 0.f};
            if ((UNITS % NT == 0 || idx < UNITS) && k0 + kk < k1 && c < nc)
                x = *reinterpret_cast<const Unit *>(reinterpret_cast<const Elem *>(g) + (size_t)(k0 + kk) * ld + c);
            v[i] = x;                                  // nc % 4 == 0 (host-checked): whole quads
        }
    }

    __device__ __forceinline__ void store(__bf16 *img) const {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int idx = threadIdx.x + NT * i;
            if (UNITS % NT != 0 && idx >= UNITS) continue;
            const int o = Img<ROWS>::off(idx / (ROWS / 4), 4 * (idx % (ROWS / 4)));
            if constexpr (BF) {
                static_assert(NL == 1, "bf16 operands: the bf16 mode's one product");
                *reinterpret_cast<bf16x4 *>(&img[o]) = v[i];
            } else {
                bf16x4 x0, x1, x2;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if constexpr (NL == 3) {
                        __bf16 a, b, c;
                        hsg_split3(v[i][e], a, b, c);
                        x0[e] = a; x1[e] = b; x2[e] = c;
                    } else {
                        x0[e] = (__bf16)v[i][e];             // RNE: the bf16 mode's operand
                    }
                }
                *reinterpret_cast<bf16x4 *>(&img[o]) = x0;
                if constexpr (NL == 3) {
                    *reinterpret_cast<bf16x4 *>(&img[Img<ROWS>::SIZE + o]) = x1;
                    *reinterpret_cast<bf16x4 *>(&img[2 * Img<ROWS>::SIZE + o]) = x2;
                }
            }
        }
    }
};

// 16x16x32 operand fragment of image columns [c0, c0 + 16): lane l receives column
// c0 + (l & 15), k = 8 (l >> 4) + 0..7.  ds_read_b64_tr_b16 per 16-lane group: lane
// 4q + p addresses image row q of a 4 x 16 block at columns 4p..4p+3, and lane i of
// the group receives column i, rows 0..3 -- two reads (k 0..3, 4..7) per fragment.
template <int ROWS>
__device__ __forceinline__ bf16x8 frag(const __bf16 *plane, int c0, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, kb = 8 * (lane >> 4);
    typedef __attribute__((address_space(3))) v4s16 lds_v4s16;
    const v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4s16 *)(const_cast<__bf16 *>(&plane[Img<ROWS>::off(kb + q, c0 + 4 * p)])));
    const v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_v4s16 *)(const_cast<__bf16 *>(&plane[Img<ROWS>::off(kb + 4 + q, c0 + 4 * p)])));
    const v8s16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, r);          // whole-vector reinterpretation
}

struct DwJob {
    const void *A, *B;        // [K][M] (lda), [K][N] (ldb): fp32, or bf16 per abf / bbf
    int abf, bbf;
    float *ws;                // [splits][M][N]
    int M, N, lda, ldb;
    int cfg;                  // tile: 0 = 160 x 128, 1 = 128 x 160, 2 = 128 x 128
    int tiles_m, tiles_n;
    int start;                // first logical block of the job
};
struct DwJobs {
    DwJob j[2];
    int nj, K, splits, ktps, total;
};

// Workgroup b runs on XCD b % 8 (for locality only): logical block xcd_order(b) gives
// each XCD a contiguous run of (job, K slice, tile), so the tiles that share a slice's
// operand rows meet in one L2.  A bijection on [0, total).
__device__ __forceinline__ int xcd_order(int b, int total) {
    const int x = b & 7, j = b >> 3, per = total >> 3, rem = total & 7;
    return x * per + min(x, rem) + j;
}

template <int BM, int BN, int NL, bool ABF = false, bool BBF = false>
__device__ __forceinline__ void dw_tile(const DwJob &jb, int tz, int t, const DwJobs &J, __bf16 *sA, __bf16 *sB) {
    constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 16, TN = WN / 16;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int ty = t / jb.tiles_n, tx = t % jb.tiles_n;
    const int m0 = ty * BM, n0 = tx * BN;
    const int kt_total = (J.K + kBK - 1) / kBK;
    const int kt0 = tz * J.ktps, kt1 = min(kt_total, kt0 + J.ktps);

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    Stage<BM, NL, kNT, ABF> ra;
    Stage<BN, NL, kNT, BBF> rb;
    if (kt0 < kt1) {
        ra.load(jb.A, jb.lda, m0, jb.M, kt0 * kBK, J.K);
        rb.load(jb.B, jb.ldb, n0, jb.N, kt0 * kBK, J.K);
    }
    for (int kt = kt0; kt < kt1; ++kt) {
        __syncthreads();                          // every wave is done with the previous tile
        ra.store(sA);
        rb.store(sB);
        __syncthreads();
        if (kt + 1 < kt1) {                       // the next tile's loads overlap this tile's MFMAs
            ra.load(jb.A, jb.lda, m0, jb.M, (kt + 1) * kBK, J.K);
            rb.load(jb.B, jb.ldb, n0, jb.N, (kt + 1) * kBK, J.K);
        }
        bf16x8 a[NL][TM];
#pragma unroll
        for (int l = 0; l < NL; ++l)
#pragma unroll
            for (int i = 0; i < TM; ++i) a[l][i] = frag<BM>(sA + l * Img<BM>::SIZE, wm * WM + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            bf16x8 b[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l) b[l] = frag<BN>(sB + l * Img<BN>::SIZE, wn * WN + 16 * j, lane);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if constexpr (NL == 3) {              // smallest limb products first, a0 b0 last
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1], acc[i][j], 0, 0, 0);
                }
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0], acc[i][j], 0, 0, 0);
            }
        }
        __builtin_amdgcn_iglp_opt(0);
    }

    // the K slice's partial product: lane holds column (lane & 15), rows 4 (lane >> 4) + e
    float *ws = jb.ws + (size_t)tz * jb.M * jb.N;
    const int c = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WN + 16 * j + c;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int m = m0 + wm * WM + 16 * i + rq + e;
                if (m < jb.M && n < jb.N) ws[(size_t)m * jb.N + n] = acc[i][j][e];
            }
        }
}

template <int NL>
__global__ __launch_bounds__(kNT, 2) void k_dw(DwJobs J) {
    __shared__ __attribute__((aligned(16))) __bf16 sA[NL * Img<160>::SIZE];
    __shared__ __attribute__((aligned(16))) __bf16 sB[NL * Img<160>::SIZE];
    const int L = xcd_order((int)blockIdx.x, J.total);
    const int q = (J.nj > 1 && L >= J.j[1].start) ? 1 : 0;
    const DwJob &jb = J.j[q];
    const int loc = L - jb.start, tiles = jb.tiles_m * jb.tiles_n;
    const int tz = loc / tiles, t = loc - tz * tiles;            // K slices outer: a slice's tiles adjacent
    if constexpr (NL == 1) {              // the bf16 mode: operands fp32 or bf16 per job
        const int f = jb.abf | (jb.bbf << 1);
#define HSG_DWT(BM_, BN_)                                                                   \
        if (f == 0) dw_tile<BM_, BN_, 1>(jb, tz, t, J, sA, sB);                             \
        else if (f == 1) dw_tile<BM_, BN_, 1, true, false>(jb, tz, t, J, sA, sB);           \
        else if (f == 2) dw_tile<BM_, BN_, 1, false, true>(jb, tz, t, J, sA, sB);           \
        else dw_tile<BM_, BN_, 1, true, true>(jb, tz, t, J, sA, sB);
        if (jb.cfg == 0) { HSG_DWT(160, 128) }
        else if (jb.cfg == 1) { HSG_DWT(128, 160) }
        else { HSG_DWT(128, 128) }
#undef HSG_DWT
        return;
    }
    if (jb.cfg == 0) dw_tile<160, 128, NL>(jb, tz, t, J, sA, sB);
    else if (jb.cfg == 1) dw_tile<128, 160, NL>(jb, tz, t, J, sA, sB);
    else dw_tile<128, 128, NL>(jb, tz, t, J, sA, sB);
}

// ---------------------------------------------------------------------------------
// k_dw2: the same contract on one block of 8 waves per CU with a DOUBLE-buffered limb
// image and register-staged loads two K tiles ahead: tile k+1 is split and stored
// while tile k is multiplied (one barrier per K tile), the global loads of tile k+3
// are in flight meanwhile.  k_dw (two blocks of 4 waves per CU, one image each) pays
// two barriers and the store phase per K tile, and keeps one tile of loads in flight.
// Waves: 2 x 4 over 160 x 128 (80 x 32 each), 4 x 2 over 128 x 160 (32 x 80), 2 x 4
// over 128 x 128 (64 x 32).
// ---------------------------------------------------------------------------------
constexpr int kNT2 = 512;

template <int BM, int BN, int WGM, int NL>
__device__ __forceinline__ void dw2_tile(const DwJob &jb, int tz, int t, const DwJobs &J, __bf16 *lds) {
    constexpr int WGN = 8 / WGM;
    constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
    constexpr int IA = NL * Img<BM>::SIZE, IB = NL * Img<BN>::SIZE, IMG = IA + IB;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / WGN, wn = wid % WGN;
    const int ty = t / jb.tiles_n, tx = t % jb.tiles_n;
    const int m0 = ty * BM, n0 = tx * BN;
    const int kt_total = (J.K + kBK - 1) / kBK;
    const int kt0 = tz * J.ktps, kt1 = min(kt_total, kt0 + J.ktps);

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    Stage<BM, NL, kNT2> ra[2];
    Stage<BN, NL, kNT2> rb[2];
    auto load = [&](int s, int kt) {
        if (kt < kt1) {
            ra[s].load(jb.A, jb.lda, m0, jb.M, kt * kBK, J.K);          // fp32 operands (dev kernel)
            rb[s].load(jb.B, jb.ldb, n0, jb.N, kt * kBK, J.K);
        }
    };
    auto store = [&](int s, int buf) {
        ra[s].store(lds + buf * IMG);
        rb[s].store(lds + buf * IMG + IA);
    };
    auto mma = [&](int buf) {
        const __bf16 *sA = lds + buf * IMG, *sB = lds + buf * IMG + IA;
        bf16x8 a[NL][TM];
#pragma unroll
        for (int l = 0; l < NL; ++l)
#pragma unroll
            for (int i = 0; i < TM; ++i) a[l][i] = frag<BM>(sA + l * Img<BM>::SIZE, wm * WM + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            bf16x8 b[NL];
#pragma unroll
            for (int l = 0; l < NL; ++l) b[l] = frag<BN>(sB + l * Img<BN>::SIZE, wn * WN + 16 * j, lane);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if constexpr (NL == 3) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1], acc[i][j], 0, 0, 0);
                }
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0], acc[i][j], 0, 0, 0);
            }
        }
    };
    // prologue: tile kt0 in image 0, tiles kt0 + 1 / kt0 + 2 in registers
    load(0, kt0);
    load(1, kt0 + 1);
    store(0, 0);
    load(0, kt0 + 2);
    // K tile kt (image (kt - kt0) & 1) is multiplied while tile kt + 1 (register set
    // (kt - kt0 + 1) & 1) goes into the other image; that set then loads tile kt + 3.
    // Unrolled by two so the register sets stay compile-time.
    for (int kt = kt0; kt < kt1; kt += 2) {
        __syncthreads();
        if (kt + 1 < kt1) store(1, 1);
        load(1, kt + 3);
        mma(0);
        __builtin_amdgcn_iglp_opt(0);
        if (kt + 1 >= kt1) break;
        __syncthreads();
        if (kt + 2 < kt1) store(0, 0);
        load(0, kt + 4);
        mma(1);
        __builtin_amdgcn_iglp_opt(0);
    }

    float *ws = jb.ws + (size_t)tz * jb.M * jb.N;
    const int c = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WN + 16 * j + c;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int m = m0 + wm * WM + 16 * i + rq + e;
                if (m < jb.M && n < jb.N) ws[(size_t)m * jb.N + n] = acc[i][j][e];
            }
        }
}

template <int NL>
__global__ __launch_bounds__(kNT2, 1) void k_dw2(DwJobs J) {
    __shared__ __attribute__((aligned(16))) __bf16 lds[2 * NL * (Img<160>::SIZE + Img<128>::SIZE)];
    const int L = xcd_order((int)blockIdx.x, J.total);
    const int q = (J.nj > 1 && L >= J.j[1].start) ? 1 : 0;
    const DwJob &jb = J.j[q];
    const int loc = L - jb.start, tiles = jb.tiles_m * jb.tiles_n;
    const int tz = loc / tiles, t = loc - tz * tiles;
    if (jb.cfg == 0) dw2_tile<160, 128, 2, NL>(jb, tz, t, J, lds);
    else if (jb.cfg == 1) dw2_tile<128, 160, 4, NL>(jb, tz, t, J, lds);
    else dw2_tile<128, 128, 2, NL>(jb, tz, t, J, lds);
}

constexpr int kTileM[3] = {160, 128, 128}, kTileN[3] = {128, 160, 128};

// the tile with the least padded output area (ties: the first)
int pick_cfg(int M, int N) {
    int best = 0;
    long area = -1;
    for (int c = 0; c < 3; ++c) {
        const long a = (long)((M + kTileM[c] - 1) / kTileM[c]) * kTileM[c] * ((N + kTileN[c] - 1) / kTileN[c]) * kTileN[c];
        if (area < 0 || a < area) { area = a; best = c; }
    }
    return best;
}

bool al16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// k_dw2 (HSG_DW_V2=1, dev A/B until measured)
bool dw_v2() {
    const char *e = HSG_DEV_ENV("HSG_DW_V2");
    return e && atoi(e) == 1;
}

}  // namespace

extern "C" {

int hsg_gemm_dw_tiles(int M, int N) {
    const int c = pick_cfg(M, N);
    return ((M + kTileM[c] - 1) / kTileM[c]) * ((N + kTileN[c] - 1) / kTileN[c]);
}

static int dw_slabs(int njobs, const int *M, const int *N, int K, const void *const *A, const int *lda,
                    const void *const *B, const int *ldb, const int *io, int splits, int bf16, float *const *ws,
                    void *stream) {
    if (njobs < 1 || njobs > 2 || K < 1 || splits < 1 || !M || !N || !A || !B || !lda || !ldb || !ws)
        return HSG_EINVAL;
    DwJobs J{};
    J.nj = njobs;
    J.K = K;
    const int kt_total = (K + kBK - 1) / kBK;
    if (splits > kt_total) return HSG_EINVAL;
    J.ktps = (kt_total + splits - 1) / splits;
    J.splits = (kt_total + J.ktps - 1) / J.ktps;          // every slice non-empty
    if (J.splits != splits) return HSG_EINVAL;             // the caller sized ws for `splits` slabs
    int start = 0;
    for (int q = 0; q < njobs; ++q) {
        DwJob &jb = J.j[q];
        if (M[q] < 1 || N[q] < 1 || (M[q] & 3) || (N[q] & 3) || lda[q] < M[q] || ldb[q] < N[q] || (lda[q] & 3) ||
            (ldb[q] & 3) || !A[q] || !B[q] || !ws[q] || !al16(A[q]) || !al16(B[q]))
            return HSG_EINVAL;
        const int iq = io ? io[q] : 0;
        if (iq && (!bf16 || (iq & ~3))) return HSG_EINVAL;      // bf16 operands: the bf16 mode only
        jb.A = A[q]; jb.B = B[q]; jb.ws = ws[q];
        jb.abf = iq & 1;
        jb.bbf = (iq >> 1) & 1;
        jb.M = M[q]; jb.N = N[q]; jb.lda = lda[q]; jb.ldb = ldb[q];
        jb.cfg = pick_cfg(M[q], N[q]);
        jb.tiles_m = (M[q] + kTileM[jb.cfg] - 1) / kTileM[jb.cfg];
        jb.tiles_n = (N[q] + kTileN[jb.cfg] - 1) / kTileN[jb.cfg];
        jb.start = start;
        start += jb.tiles_m * jb.tiles_n * splits;
    }
    J.total = start;
    hipStream_t st = (hipStream_t)stream;
    if (dw_v2() && !(J.j[0].abf | J.j[0].bbf | (njobs > 1 ? J.j[1].abf | J.j[1].bbf : 0))) {
        if (bf16) hipLaunchKernelGGL(k_dw2<1>, dim3((unsigned)J.total), dim3(kNT2), 0, st, J);
        else hipLaunchKernelGGL(k_dw2<3>, dim3((unsigned)J.total), dim3(kNT2), 0, st, J);
    } else if (bf16) hipLaunchKernelGGL(k_dw<1>, dim3((unsigned)J.total), dim3(kNT), 0, st, J);
    else hipLaunchKernelGGL(k_dw<3>, dim3((unsigned)J.total), dim3(kNT), 0, st, J);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int hsg_gemm_dw_slabs(int njobs, const int *M, const int *N, int K, const float *const *A, const int *lda,
                      const float *const *B, const int *ldb, int splits, int bf16, float *const *ws, void *stream) {
    return dw_slabs(njobs, M, N, K, reinterpret_cast<const void *const *>(A), lda,
                    reinterpret_cast<const void *const *>(B), ldb, nullptr, splits, bf16, ws, stream);
}

int hsg_gemm_dw_slabs_io(int njobs, const int *M, const int *N, int K, const void *const *A, const int *lda,
                         const void *const *B, const int *ldb, const int *io, int splits, float *const *ws,
                         void *stream) {
    return dw_slabs(njobs, M, N, K, A, lda, B, ldb, io, splits, 1, ws, stream);
}

}  // extern "C"
