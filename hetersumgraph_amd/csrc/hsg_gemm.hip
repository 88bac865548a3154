// hsg_gemm.hip -- fp32 MFMA GEMM with fused epilogues for gfx950 (MI355X).
//
// The dense parts of one WSWGAT application are fp32 GEMMs: the head
// projection fc (GATLayer.py:110/146), and the position-wise FFN
// W2 relu(W1 x + b1) + b2 (GATLayer.py:39) with its backward.  gfx950 has no
// xf32 path, but v_mfma_f32_32x32x2_f32 computes an exact f32 fmaf chain at the
// f32 vector peak while leaving the VALU free for the epilogue.
//
//   C[m][n] = epi( sum_k A(m,k) * B(k,n) )
//     A(m,k) = a_kc ? A[m*lda + k] : A[k*lda + m]      (K-contiguous or M-contiguous)
//     B(k,n) = b_kc ? B[n*ldb + k] : B[k*ldb + n]      (K-contiguous or N-contiguous)
//   epi: STORE  v (+bias[n]) (relu if requested)
//        RELU_BWD v * (aux[m][n] > 0)            -- relu' applied to dH
//        ADD    v (+bias[n]) + aux[m][n]         -- accumulate (aux may alias C)
//
// Block = 256 threads (2x2 waves), tile BM x BN x 32, register-staged double
// buffer in LDS, one barrier per K tile.  LDS images:
//   K-contiguous operands: [rows][32+4] floats, read with ds_read_b128 (4 MFMA
//     k-steps per read; the +4 pad makes the 16-lane b128 groups conflict-free);
//   M/N-contiguous operands: [32][BM+4], read with ds_read_b32 (lanes on
//     consecutive columns -> conflict-free).
// K of one MFMA k-step s (0..15) is s for lanes 0-31 and 16+s for lanes 32-63,
// identically for A and B, so the sum over a 32-deep tile is exact.
// BF = true (hsg_gemm_bf16): the same tiles, operands rounded to bf16 (RNE) when the
// fragments are read from LDS, v_mfma_f32_32x32x16_bf16 with fp32 accumulation.
// Split-K (grid.z > 1) writes fp32 partial slabs, reduced (with the epilogue) by
// k_splitk_reduce in split order -> deterministic.
//
// k_gemm3 (hsg_gemm_f32's default path): fp32 operands, fp32-ACCURATE products on the
// bf16 matrix cores.  Each operand element is split into three bf16 limbs,
// x = x0 + x1 + x2 (x0 = RNE(x), x1 = RNE(x - x0), x2 = RNE(x - x0 - x1); both
// differences are exact in fp32), when its tile is staged into LDS, and
// sum_k a*b is accumulated in fp32 from the six limb products whose order is
// <= 2^-16 relative (a0b0, a0b1, a1b0, a0b2, a1b1, a2b0; bf16 x bf16 products are
// exact in fp32).  The dropped terms (a1b2, a2b1, a2b2, and the limb residual) are
// <= ~3 * 2^-24 of |a b|: the error class of an fp32 fmaf chain (measured against
// fp64 in tests/test_gpu_gemm.py).  Six v_mfma_f32_32x32x16_bf16 (32 cycles each)
// replace eight v_mfma_f32_32x32x2_f32 (64 cycles) per 16-deep k step: a 2.67x
// higher MFMA ceiling than the exact-f32 instruction (gfx950 has no xf32).
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>

#include "../../include/hsg.h"
#include "hsg_dev.h"
#include "hsg_wave.h"
#include "hsg_rng.h"
#include "hsg_wsplit.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kBK = 32;
constexpr int kPad = 4;

struct GemmArgs {
    int M, N, K;
    const float *A;
    int lda;
    const float *B;
    int ldb;
    float *C;
    int ldc;
    const float *bias;
    const float *aux;
    int ldaux;
    int epi;
    int relu;
    int k_tiles_per_split;
    float *ws;            // split-K partials [splits][M][N]
    float *colpart;       // optional: per-block-row column sums of C, [ceil(M/BM)][N]
    int splits;           // K slices (tile ids run over splits x tiles_m x tiles_n)
    int xcd;              // 1: XCD-aware tile order (see xcd_tile)
    // HSG_EPI_ADD_ELUG only (epi_rows): C2 = C * elu'(h) with e = aux2 - aux3 (ld: ldaux)
    const float *aux2 = nullptr;
    const float *aux3 = nullptr;
    float *C2 = nullptr;
    // optional with HSG_EPI_ADD_ELUG: rho partials of the edge backward, rho[m][g][s] =
    // sum over the columns c of 64-column group g in head c / rho_d = 64 g / rho_d + s
    // of C2 * h with h = elu^-1(e) (hsg_gemm_psw_elug_rho)
    float *rho = nullptr;
    int rho_d = 0;
    // k_gemm11's LayerNorm epilogue only (hsg_gemm_*_psw_ln): C = the pre-dropout FFN
    // output y, lnout = LN(dropout(y) + aux) with gamma / beta, per-row mean / rstd
    const float *gamma = nullptr, *beta = nullptr;
    float *lnout = nullptr, *mean = nullptr, *rstd = nullptr;
    const int64_t *seed = nullptr;
    float eps = 0.f, p_drop = 0.f;
    uint32_t offset = 0;
    // HSG_EPI_ADD_ELUG with a bf16 x (aux2; k_gemm7 IO bit 4, round 6): its row pitch
    int ldx = 0;
};

// Workgroup b is dispatched to XCD b % 8, and so is tile t (the persistent grid is a
// multiple of 8).  xcd_tile gives each XCD one contiguous range of the logical
// (split, row-tile, col-tile) order, so the column tiles that share an A row band
// (and the tiles of one K slice) meet in the same 4 MB L2 instead of streaming the
// band through all eight.  A bijection on [0, total) for any total.
__device__ __forceinline__ int xcd_tile(int t, int total) {
    const int x = t & 7, j = t >> 3, per = total >> 3, rem = total & 7;
    return x * per + min(x, rem) + j;
}

__device__ __forceinline__ float epi_apply(float v, int m, int n, const GemmArgs &p) {
    if (p.epi == HSG_EPI_RELU_BWD) return p.aux[(size_t)m * p.ldaux + n] > 0.f ? v : 0.f;
    if (p.bias) v += p.bias[n];
    if (p.epi == HSG_EPI_ADD) v += p.aux[(size_t)m * p.ldaux + n];
    if (p.relu) v = fmaxf(v, 0.f);
    return v;
}

template <bool KC, int ROWS, int BK>
struct Stage {
    // one operand tile: KC -> [ROWS x 32] from rows of a K-contiguous matrix;
    // !KC -> [32 x ROWS] from 32 rows of a ROWS-contiguous matrix
    static constexpr int LD = KC ? (BK + kPad) : (ROWS + kPad);
    static constexpr int NV = ROWS * BK / 4 / 256;   // float4 per thread
    f32x4 v[NV];

    __device__ __forceinline__ void load(const float *__restrict__ g, int ld, int r0, int nr, int k0, int nk) {
        const bool full = KC ? (r0 + ROWS <= nr && k0 + BK <= nk) : (k0 + BK <= nk && r0 + ROWS <= nr);
        if (full) {
#pragma unroll
            for (int i = 0; i < NV; ++i) {
                const int idx = threadIdx.x + 256 * i;
                int row, col;
                if constexpr (KC) { row = idx / (BK / 4); col = (idx % (BK / 4)) * 4; }
                else { row = idx / (ROWS / 4); col = (idx % (ROWS / 4)) * 4; }
                const int gr = KC ? r0 + row : k0 + row;
                const int gc = KC ? k0 + col : r0 + col;
                v[i] = *reinterpret_cast<const f32x4 *>(g + (size_t)gr * ld + gc);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int idx = threadIdx.x + 256 * i;
            int row, col;   // row in the "major" dimension of global memory, col contiguous
            if constexpr (KC) { row = idx / (BK / 4); col = (idx % (BK / 4)) * 4; }
            else { row = idx / (ROWS / 4); col = (idx % (ROWS / 4)) * 4; }
            const int gr = KC ? r0 + row : k0 + row;          // global row
            const int gc = KC ? k0 + col : r0 + col;          // global col
            const int lim_r = KC ? nr : nk, lim_c = KC ? nk : nr;
            f32x4 x = {0.f, 0.f, 0.f, 0.f};
            if (gr < lim_r) {
                const float *src = g + (size_t)gr * ld + gc;
                if (gc + 3 < lim_c) {
                    x = *reinterpret_cast<const f32x4 *>(src);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gc + e < lim_c) x[e] = src[e];
                }
            }
            v[i] = x;
        }
    }

    __device__ __forceinline__ void store(float *s) const {
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int idx = threadIdx.x + 256 * i;
            int row, col;
            if constexpr (KC) { row = idx / (BK / 4); col = (idx % (BK / 4)) * 4; }
            else { row = idx / (ROWS / 4); col = (idx % (ROWS / 4)) * 4; }
            *reinterpret_cast<f32x4 *>(s + row * LD + col) = v[i];
        }
    }
};

// NBUF = 2: register-staged double buffer in LDS, one barrier per K tile.
// NBUF = 1: one LDS buffer (half the LDS, twice the resident blocks), the next
// tile still prefetched into registers, two barriers per K tile.
#ifdef HSG_GEMM_CENSUS
__device__ unsigned long long g_census[16384 * 4];
#endif

template <int BM, int BN, bool AK, bool BKC, int NBUF, int BK, bool BF = false>
__global__ __launch_bounds__(256, 2) void k_gemm(GemmArgs p) {
#ifdef HSG_GEMM_CENSUS
    const unsigned long long c_t0 = __builtin_readcyclecounter();
#endif
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int TM = WM / 32, TN = WN / 32;
    using SA = Stage<AK, BM, BK>;
    using SB = Stage<BKC, BN, BK>;
    __shared__ __attribute__((aligned(16))) float sA[NBUF][AK ? BM * SA::LD : BK * SA::LD];
    __shared__ __attribute__((aligned(16))) float sB[NBUF][BKC ? BN * SB::LD : BK * SB::LD];

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int li = lane & 31, h = lane >> 5;
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int tiles_mn = tiles_n * tiles_m;
    const int kt_total = (p.K + BK - 1) / BK;
    const int total = tiles_mn * p.splits;
    SA ra;
    SB rb;
    // first K slice of tile t into registers (single-buffer kernels prefetch the next
    // tile's first slice during the current tile's last K step)
    auto load_first = [&](int t) {
        if (p.xcd) t = xcd_tile(t, total);
        const int tx_ = t % tiles_n, ty_ = (t / tiles_n) % tiles_m, tz_ = t / tiles_mn;
        const int k0 = tz_ * p.k_tiles_per_split * BK;
        ra.load(p.A, p.lda, ty_ * BM, p.M, k0, p.K);
        rb.load(p.B, p.ldb, tx_ * BN, p.N, k0, p.K);
    };
    if (NBUF == 1 && (int)blockIdx.x < total) load_first(blockIdx.x);
    // persistent over output tiles (grid may be smaller than the tile count)
    for (int t = blockIdx.x; t < total; t += gridDim.x) {
    const int lt = p.xcd ? xcd_tile(t, total) : t;
    const int tx = lt % tiles_n, ty = (lt / tiles_n) % tiles_m, tz = lt / tiles_mn;
    const int m0 = ty * BM, n0 = tx * BN;
    const int kt0 = tz * p.k_tiles_per_split;
    const int kt1 = min(kt_total, kt0 + p.k_tiles_per_split);
    const int tn = t + gridDim.x;
    bool prefetched = false;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    int cur = 0;
    if constexpr (NBUF == 1) {
        ra.store(sA[0]);                  // registers hold this tile's first slice
        rb.store(sB[0]);
    } else if (kt0 < kt1) {
        ra.load(p.A, p.lda, m0, p.M, kt0 * BK, p.K);
        rb.load(p.B, p.ldb, n0, p.N, kt0 * BK, p.K);
        ra.store(sA[0]);
        rb.store(sB[0]);
    }
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
        const bool more = kt + 1 < kt1;
        if (more) {
            ra.load(p.A, p.lda, m0, p.M, (kt + 1) * BK, p.K);
            rb.load(p.B, p.ldb, n0, p.N, (kt + 1) * BK, p.K);
        } else if (NBUF == 1 && tn < total) {
            load_first(tn);               // overlaps this step's MFMAs and the epilogue
            prefetched = true;
        }
        const float *a_s = sA[NBUF == 2 ? cur : 0];
        const float *b_s = sB[NBUF == 2 ? cur : 0];
        // double-buffered fragments (the scheduler folds them onto one register set,
        // trading an LDS round trip per group for occupancy; pinning the order with
        // sched_group_barrier measured slower at 111 VGPRs / 4 waves per SIMD)
        f32x4 af[2][TM], bf[2][TN];
        auto frag = [&](f32x4 (&fa)[TM], f32x4 (&fb)[TN], int s4) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm * WM + i * 32 + li;
                if constexpr (AK) {
                    fa[i] = *reinterpret_cast<const f32x4 *>(a_s + row * SA::LD + h * (BK / 2) + s4);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) fa[i][q] = a_s[(h * (BK / 2) + s4 + q) * SA::LD + row];
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int col = wn * WN + j * 32 + li;
                if constexpr (BKC) {
                    fb[j] = *reinterpret_cast<const f32x4 *>(b_s + col * SB::LD + h * (BK / 2) + s4);
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) fb[j][q] = b_s[(h * (BK / 2) + s4 + q) * SB::LD + col];
                }
            }
        };
        if constexpr (BF) {
            // bf16 operands (RNE from the fp32 LDS image), fp32 accumulate:
            // v_mfma_f32_32x32x16_bf16, lane (li, h) element j <-> k = h*BK/2 + 8s + j
#pragma unroll
            for (int s8 = 0; s8 < BK / 16; ++s8) {
                bf16x8 xa[TM], xb[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int row = wm * WM + i * 32 + li;
                    if constexpr (AK) {
                        const float *q = a_s + row * SA::LD + h * (BK / 2) + 8 * s8;
                        const f32x4 lo = *reinterpret_cast<const f32x4 *>(q);
                        const f32x4 hi = *reinterpret_cast<const f32x4 *>(q + 4);
#pragma unroll
                        for (int e = 0; e < 4; ++e) { xa[i][e] = (__bf16)lo[e]; xa[i][4 + e] = (__bf16)hi[e]; }
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) xa[i][e] = (__bf16)a_s[(h * (BK / 2) + 8 * s8 + e) * SA::LD + row];
                    }
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int col = wn * WN + j * 32 + li;
                    if constexpr (BKC) {
                        const float *q = b_s + col * SB::LD + h * (BK / 2) + 8 * s8;
                        const f32x4 lo = *reinterpret_cast<const f32x4 *>(q);
                        const f32x4 hi = *reinterpret_cast<const f32x4 *>(q + 4);
#pragma unroll
                        for (int e = 0; e < 4; ++e) { xb[j][e] = (__bf16)lo[e]; xb[j][4 + e] = (__bf16)hi[e]; }
                    } else {
#pragma unroll
                        for (int e = 0; e < 8; ++e) xb[j][e] = (__bf16)b_s[(h * (BK / 2) + 8 * s8 + e) * SB::LD + col];
                    }
                }
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[i], xb[j], acc[i][j], 0, 0, 0);
            }
        } else {
        frag(af[0], bf[0], 0);
#pragma unroll
        for (int g = 0; g < BK / 8; ++g) {
            if (g + 1 < BK / 8) frag(af[(g + 1) & 1], bf[(g + 1) & 1], 4 * (g + 1));
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[g & 1][i][q], bf[g & 1][j][q],
                                                                          acc[i][j], 0, 0, 0);
        }
        }
        if constexpr (NBUF == 2) {
            if (more) {
                ra.store(sA[cur ^ 1]);
                rb.store(sB[cur ^ 1]);
            }
            __syncthreads();
            cur ^= 1;
        } else {
            __syncthreads();                  // every wave is done reading the tile
            if (more) {
                ra.store(sA[0]);
                rb.store(sB[0]);
            }
            __syncthreads();
        }
    }

    if (NBUF == 1 && !prefetched && tn < total) load_first(tn);   // empty K range
    // epilogue: lane holds rows (r&3)+8*(r>>2)+4*h, column li of each 32x32 tile
    const bool split = p.splits > 1;
    float csum[TN];                       // column sums of this wave's stored values (colpart)
#pragma unroll
    for (int j = 0; j < TN; ++j) csum[j] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WN + j * 32 + li;
            if (n >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= p.M) continue;
                if (split) {
                    p.ws[((size_t)tz * p.M + m) * p.N + n] = acc[i][j][r];
                } else {
                    const float v = epi_apply(acc[i][j][r], m, n, p);
                    p.C[(size_t)m * p.ldc + n] = v;
                    csum[j] += v;
                }
            }
        }
    if (p.colpart && !split) {           // block-uniform: fixed-order block partial per column
        // lanes li and li+32 hold the two row halves of the same column
#pragma unroll
        for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32);
        __syncthreads();                  // the tiles in LDS are no longer read
        float *red = sA[0];
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) red[wm * BN + wn * WN + j * 32 + li] = csum[j];
        }
        __syncthreads();
        for (int c = threadIdx.x; c < BN; c += 256) {
            const int n = n0 + c;
            if (n < p.N) p.colpart[(size_t)ty * p.N + n] = red[c] + red[BN + c];
        }
    }
    __syncthreads();                      // LDS is refilled by the next tile's prologue
    }
#ifdef HSG_GEMM_CENSUS
    if (threadIdx.x == 0 && blockIdx.x < 16384) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_census[blockIdx.x * 4 + 0] = hw;
        g_census[blockIdx.x * 4 + 1] = xcc;
        g_census[blockIdx.x * 4 + 2] = c_t0;
        g_census[blockIdx.x * 4 + 3] = __builtin_readcyclecounter();
    }
#endif
}

// ------------------------------------------------- 3-limb bf16 split (k_gemm3) --
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short v4s16 __attribute__((ext_vector_type(4)));

// bf16 per LDS row of a limb plane: BK k + 8 pad (row stride 16 B mod 64: the 16-lane
// ds_read_b128 groups hit 64 distinct banks)
template <int BK> struct Ldh { static constexpr int v = BK + 8; };

__device__ __forceinline__ void split3(float x, __bf16 &x0, __bf16 &x1, __bf16 &x2) { hsg_split3(x, x0, x1, x2); }

// One operand tile for k_gemm3: ROWS (M or N) x BK (K) from global into registers,
// then into NL bf16 limb planes in LDS, in the operand's own global orientation:
//   KC:  [ROWS][BK + 8] (k-contiguous rows): a thread covers (row, 4 consecutive k)
//        -> NL x ds_write_b64; fragments are single ds_read_b128s;
//   !KC: [BK][ROWS + 8] (k-major, as the M/N-contiguous operand sits in memory): a
//        thread covers (k, 4 consecutive rows) -> NL x ds_write_b64, and fragments
//        come back k-contiguous through the hardware transpose read
//        ds_read_b64_tr_b16 (two per fragment) -- no in-register transpose.
template <bool KC, int ROWS, int BK, int NL, int NT = 256>
struct Stage3 {
    static constexpr int LD = KC ? Ldh<BK>::v : ROWS + 8;     // bf16 per image row
    static constexpr int IMG = KC ? ROWS * LD : BK * LD;      // bf16 per limb plane
    static constexpr int NU = ROWS * BK / (4 * NT);           // float4 units per thread
    static_assert(NU * 4 * NT == ROWS * BK, "tile must split evenly over the block");
    f32x4 v[NU];

    __device__ __forceinline__ static f32x4 ld4(const float *__restrict__ g, int ld, int gr, int gc, int lim_r,
                                                int lim_c) {
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (gr < lim_r) {
            const float *src = g + (size_t)gr * ld + gc;
            if (gc + 3 < lim_c) {
                x = *reinterpret_cast<const f32x4 *>(src);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (gc + e < lim_c) x[e] = src[e];
            }
        }
        return x;
    }

    __device__ __forceinline__ void load(const float *__restrict__ g, int ld, int r0, int nr, int k0, int nk) {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int idx = threadIdx.x + NT * i;
            if constexpr (KC) {
                const int row = idx / (BK / 4), col = (idx % (BK / 4)) * 4;
                v[i] = ld4(g, ld, r0 + row, k0 + col, nr, nk);
            } else {
                const int kk = idx / (ROWS / 4), mq = idx % (ROWS / 4);
                v[i] = ld4(g, ld, k0 + kk, r0 + 4 * mq, nk, nr);
            }
        }
    }

    __device__ __forceinline__ void store(__bf16 (*s)[IMG]) const {
#pragma unroll
        for (int i = 0; i < NU; ++i) {
            const int idx = threadIdx.x + NT * i;
            const int o = KC ? (idx / (BK / 4)) * LD + (idx % (BK / 4)) * 4
                             : (idx / (ROWS / 4)) * LD + (idx % (ROWS / 4)) * 4;
            bf16x4 x0, x1, x2;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if constexpr (NL == 3) {
                    __bf16 a, b, c;
                    split3(v[i][e], a, b, c);
                    x0[e] = a; x1[e] = b; x2[e] = c;
                } else {
                    x0[e] = (__bf16)v[i][e];
                }
            }
            *reinterpret_cast<bf16x4 *>(&s[0][o]) = x0;
            if constexpr (NL == 3) {
                *reinterpret_cast<bf16x4 *>(&s[1][o]) = x1;
                *reinterpret_cast<bf16x4 *>(&s[2][o]) = x2;
            }
        }
    }

    // MFMA 32x32x16 operand fragment of rows [row0, row0 + 32), k step s16: lane
    // (li = lane & 31, h = lane >> 5) gets rows row0 + li, k = 16 s16 + 8h + 0..7
    __device__ __forceinline__ static bf16x8 frag(const __bf16 *plane, int row0, int s16, int lane) {
        if constexpr (KC) {
            return *reinterpret_cast<const bf16x8 *>(&plane[(row0 + (lane & 31)) * LD + 16 * s16 + 8 * (lane >> 5)]);
        } else {
            // 16-lane group: lane 4q + p addresses image row (k) q, columns 4p..4p+3
            // of its 4 x 16 block; lane i of the group receives column i, rows 0..3
            const int i = lane & 15, q = i >> 2, p = i & 3;
            const int kb = 16 * s16 + 8 * (lane >> 5);
            const int col = row0 + 16 * ((lane >> 4) & 1) + 4 * p;
            typedef __attribute__((address_space(3))) v4s16 lds_v4s16;
            const v4s16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_v4s16 *)(const_cast<__bf16 *>(&plane[(kb + q) * LD + col])));
            const v4s16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (lds_v4s16 *)(const_cast<__bf16 *>(&plane[(kb + 4 + q) * LD + col])));
            // whole-vector reinterpretation (element-wise short -> __bf16 casts were
            // lowered to wrong lane selects)
            typedef short v8s16 __attribute__((ext_vector_type(8)));
            const v8s16 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
            return __builtin_bit_cast(bf16x8, r);
        }
    }
};

// Block = NT threads (2 x NT/128 waves), tile BM x BN x BK, one LDS buffer of limb planes;
// the next PF K tiles are prefetched into registers (PF = 2: the loads of tile kt+2
// are issued while tile kt is multiplied, two tiles of MFMA work to hide their
// latency).  Two barriers per K tile.  NL = 1 is a bf16-operand probe of the same
// pipeline (dev only).  The epilogue (and split-K / column partials) is k_gemm's.
// 64x64 transpose-read tiles (the weight gradients): 5 waves per SIMD (102 -> 96 VGPRs,
// no spill), so the weight-gradient
// grid (2,560 blocks at cfg2) runs in exactly two rounds of resident blocks instead of
// 2.5 at 4 per CU
template <int BM, int BN, bool AK, bool BKC, int BK, int PF, int NL, int IGLP = -1, int NT = 256>
__global__ __launch_bounds__(NT, NT == 256 ? (BM * BN == 64 * 64 && !AK && !BKC ? 5 : 2) : 1) void k_gemm3(GemmArgs p) {
    constexpr int WGN = NT / 128;                          // waves along N (2 along M)
    constexpr int WM = BM / 2, WN = BN / WGN;
    constexpr int TM = WM / 32, TN = WN / 32;
    using SA = Stage3<AK, BM, BK, NL, NT>;
    using SB = Stage3<BKC, BN, BK, NL, NT>;
    __shared__ __attribute__((aligned(16))) __bf16 sA[NL][SA::IMG];
    __shared__ __attribute__((aligned(16))) __bf16 sB[NL][SB::IMG];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid / WGN, wn = wid % WGN;
    const int li = lane & 31, h = lane >> 5;
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int tiles_mn = tiles_n * tiles_m;
    const int kt_total = (p.K + BK - 1) / BK;
    const int total = tiles_mn * p.splits;
    SA ra[PF];
    SB rb[PF];
    for (int t = blockIdx.x; t < total; t += gridDim.x) {
    const int lt = p.xcd ? xcd_tile(t, total) : t;
    const int tx = lt % tiles_n, ty = (lt / tiles_n) % tiles_m, tz = lt / tiles_mn;
    const int m0 = ty * BM, n0 = tx * BN;
    const int kt0 = tz * p.k_tiles_per_split;
    const int kt1 = min(kt_total, kt0 + p.k_tiles_per_split);

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
    for (int q = 0; q < PF; ++q)
        if (kt0 + q < kt1) {
            ra[q].load(p.A, p.lda, m0, p.M, (kt0 + q) * BK, p.K);
            rb[q].load(p.B, p.ldb, n0, p.N, (kt0 + q) * BK, p.K);
        }
    for (int kt = kt0; kt < kt1; kt += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
        const int k = kt + q;
        if (k >= kt1) break;
        __syncthreads();                      // every wave is done with the previous tile
        ra[q].store(sA);
        rb[q].store(sB);
        __syncthreads();
        if (k + PF < kt1) {                   // tile k+PF's loads overlap the next PF tiles' MFMAs
            ra[q].load(p.A, p.lda, m0, p.M, (k + PF) * BK, p.K);
            rb[q].load(p.B, p.ldb, n0, p.N, (k + PF) * BK, p.K);
        }
#pragma unroll
        for (int s16 = 0; s16 < BK / 16; ++s16) {
            bf16x8 a[NL][TM], b[NL][TN];
#pragma unroll
            for (int l = 0; l < NL; ++l) {
#pragma unroll
                for (int i = 0; i < TM; ++i) a[l][i] = SA::frag(sA[l], wm * WM + i * 32, s16, lane);
#pragma unroll
                for (int j = 0; j < TN; ++j) b[l][j] = SB::frag(sB[l], wn * WN + j * 32, s16, lane);
            }
            // smallest limb products first, a0*b0 last
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (NL == 3) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
                    }
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
                }
        }
        if constexpr (IGLP >= 0) __builtin_amdgcn_iglp_opt(IGLP);
    }
    }

    // epilogue: lane holds rows (r&3)+8*(r>>2)+4*h, column li of each 32x32 tile
    const bool split = p.splits > 1;
    float csum[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) csum[j] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WN + j * 32 + li;
            if (n >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= p.M) continue;
                if (split) {
                    p.ws[((size_t)tz * p.M + m) * p.N + n] = acc[i][j][r];
                } else {
                    const float v = epi_apply(acc[i][j][r], m, n, p);
                    p.C[(size_t)m * p.ldc + n] = v;
                    csum[j] += v;
                }
            }
        }
    if (p.colpart && !split) {
#pragma unroll
        for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32);
        __syncthreads();
        float *red = reinterpret_cast<float *>(&sA[0][0]);
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) red[wm * BN + wn * WN + j * 32 + li] = csum[j];
        }
        __syncthreads();
        for (int c = threadIdx.x; c < BN; c += NT) {
            const int n = n0 + c;
            if (n < p.N) p.colpart[(size_t)ty * p.N + n] = red[c] + red[BN + c];
        }
    }
    __syncthreads();                          // LDS is refilled by the next tile
    }
}

// ---------------------------------------------------------------------------------
// k_gemm4: the 3-limb split GEMM for two K-contiguous operands with an LDS-DMA
// pipeline.  The fp32 K tiles (32 floats = 128 B per row) go global -> LDS by
// global_load_lds_dwordx4 (1 KB = 8 rows per wave-instruction, no VGPRs), S stages
// deep, one raw barrier per K tile with a counted vmcnt so S-2 tiles stay in flight
// across it.  The limbs are split at fragment-read time (fp32 fragments by
// ds_read_b128, split3 in registers beside the MFMAs), so LDS holds 4 B per element
// instead of three 2-B planes and there is no split-and-store phase between barriers.
// Chunk q (16 B) of tile row r sits at position q ^ swz(r): every 16-lane group of a
// fragment read then covers 16 distinct 16-B bank slots (conflict-free); the swizzle
// is applied on the global SOURCE address since the DMA's LDS image is lane-linear.
// K-tail chunks (k >= K; K % 4 == 0) read a zeroed 16-B global word; rows past M/N
// are clamped (their outputs are never stored).
// ---------------------------------------------------------------------------------
__device__ __attribute__((aligned(16))) float g_zero16[4];

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// The 16x16x32 fragment map (lane = 16 kb + row, kb the 8-deep k block) meets the
// ds_read_b128 lane groups of gfx950 -- {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and
// the same +32 (MI355X_MICROARCH.md, LDS) -- not contiguous 16-lane groups: one group
// reads rows {0-3, 12-15} at k block kb and rows 4-11 at kb + 1.  Rows of the same
// parity share a 32-dword half of the banks, so per parity the chunk positions
// (2 kb) ^ f(r) of the 8 rows must be distinct: f(r) = (r >> 1) & 5 puts rows 0-3 /
// 12-15 and rows 4-11 on the same four positions {0, 1, 4, 5}, and the + 2 of the next
// k block moves the latter onto {2, 3, 6, 7}.  (swz, built for contiguous groups,
// gave every k_gemm7 A read a 2-way conflict: SQ_LDS_BANK_CONFLICT 3.2e6 per launch.)
// The weight planes' 64-B rows: row r's chunk kb sits at kb ^ bswz16(r); per row
// residue r & 3 the group's four rows {t, 12 + t} (kb) and {4 + t, 8 + t} (kb + 1) then
// land on four distinct chunks.  tools/lds_banks.py checks both maps.
__device__ __forceinline__ int swz16(int r) { return (r >> 1) & 5; }
__device__ __forceinline__ int bswz16(int r) { return (r >> 2) & 2; }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int ROWS, bool M16 = false>    // M16: the 16x16x32 image (swz16)
__device__ __forceinline__ void glds_tile(float *img, const float *__restrict__ g, int ld, int r0, int nr, int k0,
                                          int K, int wid, int lane) {
#pragma unroll
    for (int pc = 0; pc < ROWS / 32; ++pc) {              // ROWS/8 pieces of 8 rows over 4 waves
        const int piece = pc * 4 + wid;
        const int r = piece * 8 + (lane >> 3);
        const int q = (lane & 7) ^ (M16 ? swz16(r) : swz(r));
        const int k = k0 + 4 * q;
        const int gr = min(r0 + r, nr - 1);
        const float *src = k < K ? g + (size_t)gr * ld + k : g_zero16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(img + piece * 256), 16, 0, 0);
    }
}

// Truncation split of 8 fp32 values into three bf16 limb vectors, exact for normal
// numbers: l0 = the top 16 bits of x (bf16 truncation), r = x - l0 is exact and has
// at most 16 significant bits, l1 = its top 16 bits, s = r - l1 is exact with at most
// 8 significant bits, so l2 = s exactly and x = l0 + l1 + l2.  Per pair of values:
// 3 v_perm_b32 (the high halves of two registers packed into one) + 4 v_and_b32 +
// 4 v_sub_f32, no conversions.  The subtractions are pinned to scalar v_sub_f32 (inline
// asm): SLP-packed v_pk_add_f32 beside MFMAs is an anti-lever on gfx950
// (MI355X_MICROARCH.md, price of one filler; k_gemm7 -1..-2 us per launch).  With
// RNE-split weights (k_wsplit) the dropped limb products stay <= 2^-22 |ab|.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void split_trunc8(const f32x4 x, const f32x4 y, bf16x8 &l0, bf16x8 &l1, bf16x8 &l2) {
    const float v[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    u32x4 w0, w1, w2;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const unsigned a = __float_as_uint(v[2 * p]), b = __float_as_uint(v[2 * p + 1]);
        w0[p] = __builtin_amdgcn_perm(b, a, 0x07060302u);
        float ra, rb, sa, sb;
        asm("v_sub_f32 %0, %1, %2" : "=v"(ra) : "v"(v[2 * p]), "v"(__uint_as_float(a & 0xFFFF0000u)));
        asm("v_sub_f32 %0, %1, %2" : "=v"(rb) : "v"(v[2 * p + 1]), "v"(__uint_as_float(b & 0xFFFF0000u)));
        const unsigned ua = __float_as_uint(ra), ub = __float_as_uint(rb);
        w1[p] = __builtin_amdgcn_perm(ub, ua, 0x07060302u);
        asm("v_sub_f32 %0, %1, %2" : "=v"(sa) : "v"(ra), "v"(__uint_as_float(ua & 0xFFFF0000u)));
        asm("v_sub_f32 %0, %1, %2" : "=v"(sb) : "v"(rb), "v"(__uint_as_float(ub & 0xFFFF0000u)));
        w2[p] = __builtin_amdgcn_perm(__float_as_uint(sb), __float_as_uint(sa), 0x07060302u);
    }
    l0 = __builtin_bit_cast(bf16x8, w0);
    l1 = __builtin_bit_cast(bf16x8, w1);
    l2 = __builtin_bit_cast(bf16x8, w2);
}

// RNE split of 8 fp32 values, x = l0 + l1 + l2 exactly (hsg_split_rne8, hsg_wsplit.h)
__device__ __forceinline__ void split_rne8(const f32x4 x, const f32x4 y, bf16x8 &l0, bf16x8 &l1, bf16x8 &l2) {
    hsg_u32x4_t w0, w1, w2;
    hsg_split_rne8(x, y, w0, w1, w2);
    l0 = __builtin_bit_cast(bf16x8, w0);
    l1 = __builtin_bit_cast(bf16x8, w1);
    l2 = __builtin_bit_cast(bf16x8, w2);
}

__device__ __forceinline__ void frag_split(const float *img, int r, int s16, int h, bf16x8 &l0, bf16x8 &l1,
                                           bf16x8 &l2) {
    const int q0 = 4 * s16 + 2 * h, sw = swz(r);
    const f32x4 x = *reinterpret_cast<const f32x4 *>(&img[r * 32 + 4 * (q0 ^ sw)]);
    const f32x4 y = *reinterpret_cast<const f32x4 *>(&img[r * 32 + 4 * ((q0 + 1) ^ sw)]);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        __bf16 a, b, c;
        split3(e < 4 ? x[e] : y[e - 4], a, b, c);
        l0[e] = a; l1[e] = b; l2[e] = c;
    }
}

template <int BM, int BN, int S>
__global__ __launch_bounds__(256, 2) void k_gemm4(GemmArgs p) {
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int TM = WM / 32, TN = WN / 32;
    constexpr int STAGE = (BM + BN) * 32;                  // floats per stage
    constexpr int NLD = (BM + BN) / 32;                    // DMA instructions per wave per K tile
    __shared__ __attribute__((aligned(16))) float lds[S * STAGE];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int li = lane & 31, h = lane >> 5;
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int tiles_mn = tiles_n * tiles_m;
    const int kt_total = (p.K + 31) / 32;
    const int total = tiles_mn * p.splits;
    const int t = blockIdx.x;
    const int lt = p.xcd ? xcd_tile(t, total) : t;
    const int tx = lt % tiles_n, ty = (lt / tiles_n) % tiles_m, tz = lt / tiles_mn;
    const int m0 = ty * BM, n0 = tx * BN;
    const int kt0 = tz * p.k_tiles_per_split;
    const int nt = min(kt_total, kt0 + p.k_tiles_per_split) - kt0;

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto issue = [&](int i) {
        float *st = lds + (i % S) * STAGE;
        const int k0 = (kt0 + i) * 32;
        glds_tile<BM>(st, p.A, p.lda, m0, p.M, k0, p.K, wid, lane);
        glds_tile<BN>(st + BM * 32, p.B, p.ldb, n0, p.N, k0, p.K, wid, lane);
    };
#pragma unroll
    for (int i = 0; i < S - 1; ++i)
        if (i < nt) issue(i);
    for (int i = 0; i < nt; ++i) {
        // this wave's DMAs of tile i have landed once at most the newer tiles' are pending
        const int ahead = min(S - 2, nt - 1 - i);
        if (ahead >= 2) wait_vmcnt<2 * NLD>();
        else if (ahead == 1) wait_vmcnt<NLD>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();                      // every wave's DMAs of tile i landed;
        asm volatile("" ::: "memory");                     // every wave is done reading tile i-1
        if (i + S - 1 < nt) issue(i + S - 1);              // into tile i-1's stage
        const float *sa = lds + (i % S) * STAGE, *sb = sa + BM * 32;
#pragma unroll
        for (int s16 = 0; s16 < 2; ++s16) {
            bf16x8 a[3][TM], b[3][TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) frag_split(sb, wn * WN + j * 32 + li, s16, h, b[0][j], b[1][j], b[2][j]);
#pragma unroll
            for (int i2 = 0; i2 < TM; ++i2) frag_split(sa, wm * WM + i2 * 32 + li, s16, h, a[0][i2], a[1][i2], a[2][i2]);
#pragma unroll
            for (int i2 = 0; i2 < TM; ++i2)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    acc[i2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i2], b[0][j], acc[i2][j], 0, 0, 0);
                    acc[i2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i2], b[1][j], acc[i2][j], 0, 0, 0);
                    acc[i2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i2], b[2][j], acc[i2][j], 0, 0, 0);
                    acc[i2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i2], b[0][j], acc[i2][j], 0, 0, 0);
                    acc[i2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i2], b[1][j], acc[i2][j], 0, 0, 0);
                    acc[i2][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i2], b[0][j], acc[i2][j], 0, 0, 0);
                }
        }
    }

    // epilogue (as k_gemm3): lane holds rows (r&3)+8*(r>>2)+4*h, column li of each 32x32 tile
    const bool split = p.splits > 1;
    float csum[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) csum[j] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * WN + j * 32 + li;
            if (n >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m >= p.M) continue;
                if (split) {
                    p.ws[((size_t)tz * p.M + m) * p.N + n] = acc[i][j][r];
                } else {
                    const float v = epi_apply(acc[i][j][r], m, n, p);
                    p.C[(size_t)m * p.ldc + n] = v;
                    csum[j] += v;
                }
            }
        }
    if (p.colpart && !split) {
#pragma unroll
        for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32);
        __syncthreads();                                   // no DMA is pending here
        float *red = lds;
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) red[wm * BN + wn * WN + j * 32 + li] = csum[j];
        }
        __syncthreads();
        for (int c = threadIdx.x; c < BN; c += 256) {
            const int n = n0 + c;
            if (n < p.N) p.colpart[(size_t)ty * p.N + n] = red[c] + red[BN + c];
        }
    }
}

// ---------------------------------------------------------------------------------
// k_gemm5: C = A B^T with fp32 A (K-contiguous) and a PRE-SPLIT weight B: its three
// bf16 limb planes [3][Np][Kp] are made once per step by k_wsplit (hsg_wsplit), so
// only A is split in the GEMM, at fragment-read time.  Block = 128 rows x BN columns,
// 4 waves stacked along M (each wave splits its own 32 A rows once and multiplies
// them into all BN columns: 6·BN/32 MFMAs per 8-element split).  Both operands go
// global -> LDS by global_load_lds_dwordx4, S stages deep (as k_gemm4).  Limb plane
// tile rows are 64 B; chunk c (16 B) of row r sits at c ^ ((r >> 2) & 3), which
// makes the ds_read_b128 fragment reads conflict-free.
// ---------------------------------------------------------------------------------
// one launch splits up to four weights (hsg_wsplit.h)
__global__ __launch_bounds__(256) void k_wsplit(HsgWSplitJobs j) { hsg_wsplit_block(j, (int)blockIdx.x); }

// Epilogue of one wave's TN 32x32 accumulator tiles (lane: rows row0 + (r&3) + 8(r>>2)
// + 4h, column col0 + 32j + li), epi_apply's semantics.  The aux operand (relu' mask
// or addend) is loaded for all of the lane's elements FIRST, unconditionally from
// clamped indices, so the 16·TN loads are in flight together instead of each one
// waiting behind its own bounds branch; the stores stay guarded.
template <int TN>
__device__ __forceinline__ void epi_store(const f32x16 (&acc)[TN], int row0, int col0, int li, int h,
                                          const GemmArgs &p, float (&csum)[TN]) {
    float aux[TN][16];
    if (p.epi != HSG_EPI_STORE) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int nc = min(col0 + 32 * j + li, p.N - 1);
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int mc = min(row0 + (r & 3) + 8 * (r >> 2) + 4 * h, p.M - 1);
                aux[j][r] = p.aux[(size_t)mc * p.ldaux + nc];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = col0 + 32 * j + li;
        const float bn = p.bias ? p.bias[min(n, p.N - 1)] : 0.f;
        csum[j] = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = acc[j][r];
            if (p.epi == HSG_EPI_RELU_BWD) {
                v = aux[j][r] > 0.f ? v : 0.f;
            } else {
                v += bn;
                if (p.epi == HSG_EPI_ADD) v += aux[j][r];
                if (p.relu) v = fmaxf(v, 0.f);
            }
            if (m < p.M && n < p.N) {
                p.C[(size_t)m * p.ldc + n] = v;
                csum[j] += v;
            }
        }
    }
}

// LDS-staged epilogue: each wave writes its 32 x BN accumulator tile row-major into
// the (drained) stage area, then reads it back as float4 row quads, so the aux loads,
// the C stores (and the column sums) move 16 B per lane with consecutive lanes on
// consecutive quads of a row -- 4x fewer store instructions than the per-element
// epilogues, whose dword stores left the tail store-issue-bound (cfg2 S2W FFN GEMMs
// -4..-9 us per launch).  Lane -> (row step, quad): QPR quads per row, RPS = 64 / QPR
// rows per step; lanes past RPS * QPR idle.  Each lane keeps one quad, so its column
// sums are per-lane partials over its rows.
// sum over each aligned 16-lane row of the wave, in every lane (DPP, hsg_wave.h):
// __shfl_xor lowers to a chain of ds_bpermute round trips through the LDS path
__device__ __forceinline__ float row16_sum(float x) { return hsg_group_sum<16>(x); }

typedef float f32x4v7 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4v7 __attribute__((ext_vector_type(4)));

// CBF / AUXBF (the bf16 mode's bf16 activations, round 5): C is stored and the aux
// operand (the relu' mask H) read as bf16 quads (8 B) at the same element offsets
// GBF: the ELU-gate epilogue's G rows stored as bf16 (the bf16 mode; rho is summed from
// the fp32 G before the rounding)
// Lane map: a row's QPR quads on QS = 16 / 32 / 64 lanes (the power of two >= QPR), RPS
// rows per step.  rho groups (HSG_EPI_ADD_ELUG): 64 columns for tiles of a multiple of 64
// (16 lanes), the whole tile row for other widths (GW = BN: 112-wide tiles, 32 lanes).
template <int BN>
struct EpiMap {
    static constexpr int QPR = BN / 4, QS = QPR <= 16 ? 16 : QPR <= 32 ? 32 : 64, RPS = 64 / QS;
    static constexpr int GW = BN % 64 == 0 ? 64 : BN;
};
// XBF (round 6): the ELU gate's x (aux2) as bf16 rows of pitch p.ldx -- the bf16 mode's
// bf16 edge-layer output (hsg_gat_fwd_ws16)
template <int BN, bool CBF = false, bool AUXBF = false, bool GBF = false, bool XBF = false>
struct EpiRows {
    static constexpr int LDW = BN + 4, QPR = EpiMap<BN>::QPR, QS = EpiMap<BN>::QS, RPS = EpiMap<BN>::RPS;
    static constexpr int GW = EpiMap<BN>::GW;
    static constexpr int STEPS = (32 + RPS - 1) / RPS;
    f32x4 bn, aux[STEPS], ex[STEPS];
    bf16x4v7 auxb[AUXBF ? STEPS : 1];

    // the epilogue's global operands (bias, aux, and for HSG_EPI_ADD_ELUG x - origin),
    // requested together; k_gemm7 issues this before its last K tile's MFMAs so the
    // round trip overlaps them
    __device__ __forceinline__ void load(const GemmArgs &p, int row0, int col0, int lane) {
        const int q = min(lane % QS, QPR - 1), rs = lane / QS;
        const int n = col0 + 4 * q;
        const int nc = min(n, p.N - 4);                    // N % 4 == 0 (host-checked): whole quads
        bn = f32x4{0.f, 0.f, 0.f, 0.f};
        if (p.bias) bn = *reinterpret_cast<const f32x4 *>(p.bias + nc);
        if (p.epi != HSG_EPI_STORE) {
#pragma unroll
            for (int t = 0; t < STEPS; ++t) {
                const int m = min(row0 + min(t * RPS + rs, 31), p.M - 1);
                if constexpr (AUXBF) {      // kept raw until finish(): a conversion here would wait
                    auxb[t] = *reinterpret_cast<const bf16x4v7 *>(      // for the load at once
                        reinterpret_cast<const __bf16 *>(p.aux) + (size_t)m * p.ldaux + nc);
                } else {
                    aux[t] = *reinterpret_cast<const f32x4 *>(p.aux + (size_t)m * p.ldaux + nc);
                }
            }
        }
        if (p.epi == HSG_EPI_ADD_ELUG) {                   // e = x - origin = elu(h)
#pragma unroll
            for (int t = 0; t < STEPS; ++t) {
                const int m = min(row0 + min(t * RPS + rs, 31), p.M - 1);
                const size_t o = (size_t)m * p.ldaux + nc;
                if constexpr (XBF) {
                    const bf16x4v7 xb = *reinterpret_cast<const bf16x4v7 *>(
                        reinterpret_cast<const __bf16 *>(p.aux2) + (size_t)m * p.ldx + nc);
                    ex[t] = f32x4{(float)xb[0], (float)xb[1], (float)xb[2], (float)xb[3]} -
                            *reinterpret_cast<const f32x4 *>(p.aux3 + o);
                } else {
                    ex[t] = *reinterpret_cast<const f32x4 *>(p.aux2 + o) - *reinterpret_cast<const f32x4 *>(p.aux3 + o);
                }
            }
        }
    }

    template <bool NS = false>    // NS: dev diagnostic, no C store (tools/gemm5_sweep.py plan 34)
    __device__ __forceinline__ void finish(const float *wl, int row0, int col0, int lane, const GemmArgs &p,
                                           f32x4 &csum) {
        __builtin_amdgcn_s_waitcnt(0xc07f);                 // lgkmcnt(0): the wave's own LDS writes
        __builtin_amdgcn_wave_barrier();
        const int q = lane % QS, rs = lane / QS;
        const int n = col0 + 4 * q;
        const bool qok = q < QPR && rs < RPS && n < p.N;
        // rho partials per GW-column group (the GW / 4 lanes of a group are consecutive
        // lanes of one row step): head slot of each of the lane's 4 columns
        const bool rho = p.epi == HSG_EPI_ADD_ELUG && p.rho;
        int slot[4] = {3, 3, 3, 3};
        if (rho) {
            const int hb = (n / GW * GW) / p.rho_d;
#pragma unroll
            for (int e = 0; e < 4; ++e) slot[e] = n + e < p.N ? (n + e) / p.rho_d - hb : 3;
        }
        csum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < STEPS; ++t) {
            const int r = t * RPS + rs, m = row0 + r;
            const bool rok = r < 32 && m < p.M;
            float c[3] = {0.f, 0.f, 0.f};
            if (qok && rok) {
                f32x4 v = *reinterpret_cast<const f32x4 *>(&wl[r * LDW + 4 * q]);
                if (p.epi == HSG_EPI_RELU_BWD) {
                    if constexpr (AUXBF) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = (float)auxb[t][e] > 0.f ? v[e] : 0.f;
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = aux[t][e] > 0.f ? v[e] : 0.f;
                    }
                } else {
                    v += bn;
                    if (p.epi == HSG_EPI_ADD || p.epi == HSG_EPI_ADD_ELUG) v += aux[t];
                    if (p.relu) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                    }
                }
                if constexpr (CBF) {
                    *reinterpret_cast<bf16x4v7 *>(reinterpret_cast<__bf16 *>(p.C) + (size_t)m * p.ldc + n) =
                        bf16x4v7{(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};   // RNE
                } else if (!NS || v[0] == 1234.5f) {
                    *reinterpret_cast<f32x4 *>(p.C + (size_t)m * p.ldc + n) = v;
                }
                if (p.epi == HSG_EPI_ADD_ELUG) {
                    // G = dOut * elu'(h): 1 for e = elu(h) > 0, else e + 1 = exp(h) (continuous at 0)
                    f32x4 g;
#pragma unroll
                    for (int e = 0; e < 4; ++e) g[e] = ex[t][e] > 0.f ? v[e] : v[e] * (ex[t][e] + 1.f);
                    if constexpr (GBF)
                        *reinterpret_cast<bf16x4v7 *>(reinterpret_cast<__bf16 *>(p.C2) + (size_t)m * p.ldaux + n) =
                            bf16x4v7{(__bf16)g[0], (__bf16)g[1], (__bf16)g[2], (__bf16)g[3]};
                    else
                        *reinterpret_cast<f32x4 *>(p.C2 + (size_t)m * p.ldaux + n) = g;
                    if (rho) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            // e <= 0: G h = v u log(u), u = 1 + e rounded: d(u log u)/du =
                            // log u + 1, so the rounding of u moves G h by <= |v| ulp(1) -- no
                            // log1p needed.  u <= 0: the rounded e reached -1 (exp(h) below
                            // ulp(origin)), G h -> 0 there
                            const float x = ex[t][e], u = 1.f + x;
                            const float gh = x > 0.f ? g[e] * x : (u > 0.f ? g[e] * __logf(u) : 0.f);
                            c[0] += slot[e] == 0 ? gh : 0.f;
                            c[1] += slot[e] == 1 ? gh : 0.f;
                            c[2] += slot[e] == 2 ? gh : 0.f;
                        }
                    }
                }
                csum += v;
            }
            if (rho) {                                      // wave-uniform: sums over the group
#pragma unroll
                for (int s = 0; s < 3; ++s) c[s] = hsg_group_sum<GW == 64 ? 16 : QS>(c[s]);
                if (q % (GW / 4) == 0 && qok && rok) {
                    float *dst = p.rho + ((size_t)m * ((p.N + GW - 1) / GW) + n / GW) * 3;
                    dst[0] = c[0];
                    dst[1] = c[1];
                    dst[2] = c[2];
                }
            }
        }
    }
};

template <int BN>
__device__ __forceinline__ void epi_rows(const float *wl, int row0, int col0, int lane, const GemmArgs &p,
                                         f32x4 &csum) {
    EpiRows<BN> e;
    e.load(p, row0, col0, lane);
    e.finish(wl, row0, col0, lane, p, csum);
}

// 64-row column partials (hsg_gemm_row_tiles) from epi_rows' per-lane sums: waves
// 0-1 are slab 2 ty, waves 2-3 slab 2 ty + 1.  Needs 4 * RPS * BN floats of LDS.
template <int BN>
__device__ __forceinline__ void epi_rows_colpart(float *red, const f32x4 &cs, int wid, int lane, int ty, int n0,
                                                 const GemmArgs &p) {
    constexpr int QPR = EpiMap<BN>::QPR, QS = EpiMap<BN>::QS, RPS = EpiMap<BN>::RPS;
    const int q = lane % QS, rs = lane / QS;
    __syncthreads();
    if (q < QPR && rs < RPS) *reinterpret_cast<f32x4 *>(&red[(wid * RPS + rs) * BN + 4 * q]) = cs;
    __syncthreads();
    const int rows64 = (p.M + 63) / 64;
    for (int cc = threadIdx.x; cc < 2 * BN; cc += 256) {
        const int half = cc / BN, col = cc % BN, n = n0 + col, slab = 2 * ty + half;
        float v = 0.f;
        for (int w = 2 * half; w < 2 * half + 2; ++w)
            for (int r = 0; r < RPS; ++r) v += red[(w * RPS + r) * BN + col];
        if (n < p.N && slab < rows64) p.colpart[(size_t)slab * p.N + n] = v;
    }
}

bool epi_rows_ok(const GemmArgs &p) {
    const auto al = [](const void *q) { return (((uintptr_t)q) & 15) == 0; };
    if ((p.N & 3) || (p.ldc & 3) || !al(p.C) || (p.bias && !al(p.bias)) ||
        (p.aux && ((p.ldaux & 3) || !al(p.aux))))
        return false;
    return p.epi != HSG_EPI_ADD_ELUG || (al(p.aux2) && al(p.aux3) && al(p.C2));
}

template <int BN, int S, int IGLP = -1, bool ELDS = false, bool HOIST = false>
__global__ __launch_bounds__(256, 2) void k_gemm5(GemmArgs p, const __bf16 *__restrict__ planes, int Np, int Kp) {
    constexpr int BM = 128, TN = BN / 32;
    constexpr int A_FL = BM * 32;                          // floats of the A tile
    constexpr int B_BF = BN * 32;                          // bf16 per limb-plane tile
    constexpr int STAGE_FL = A_FL + 3 * B_BF / 2;          // stage size in floats
    constexpr int BPC = BN / 16;                           // 1-KB pieces per limb plane tile
    constexpr int NLD = (BM / 8 + 3 * BPC) / 4;            // DMA instructions per wave per K tile
    static_assert((3 * BPC) % 4 == 0, "B pieces must split evenly over 4 waves");
    __shared__ __attribute__((aligned(16))) float lds[S * STAGE_FL];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int li = lane & 31, h = lane >> 5;
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int total = tiles_n * tiles_m;
    const int lt = p.xcd ? xcd_tile(blockIdx.x, total) : (int)blockIdx.x;
    const int tx = lt % tiles_n, ty = lt / tiles_n;
    const int m0 = ty * BM, n0 = tx * BN;
    const int nt = Kp / 32;

    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    // HOIST: the per-lane DMA source addresses of tile 0, computed once (row clamps,
    // swizzles, limb offsets); tile i adds i * 32 k, and only a tile reaching past K
    // (the last one, K % 32 != 0) takes the per-chunk zero-page select
    const float *abase[BM / 32];
    const __bf16 *bbase[3 * BPC / 4];
    if constexpr (HOIST) {
#pragma unroll
        for (int pc = 0; pc < BM / 32; ++pc) {
            const int r = (pc * 4 + wid) * 8 + (lane >> 3);
            abase[pc] = p.A + (size_t)min(m0 + r, p.M - 1) * p.lda + 4 * ((lane & 7) ^ swz(r));
        }
#pragma unroll
        for (int pc = 0; pc < 3 * BPC / 4; ++pc) {
            const int piece = pc * 4 + wid;
            const int limb = piece / BPC, prow = (piece % BPC) * 16;
            const int r = prow + (lane >> 2);
            bbase[pc] = planes + ((size_t)(limb * Np + n0 + r) * Kp + 8 * ((lane & 3) ^ ((r >> 2) & 3)));
        }
    }
    auto issue = [&](int i) {
        float *st = lds + (i % S) * STAGE_FL;
        const int k0 = i * 32;
        __bf16 *sb = reinterpret_cast<__bf16 *>(st + A_FL);
        if constexpr (HOIST) {
            const bool tail = k0 + 32 > p.K;                // wave-uniform
#pragma unroll
            for (int pc = 0; pc < BM / 32; ++pc) {
                const float *src = abase[pc] + k0;
                if (tail && k0 + 4 * ((lane & 7) ^ swz((pc * 4 + wid) * 8 + (lane >> 3))) >= p.K) src = g_zero16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(st + (pc * 4 + wid) * 256),
                                                 16, 0, 0);
            }
#pragma unroll
            for (int pc = 0; pc < 3 * BPC / 4; ++pc) {
                const int piece = pc * 4 + wid;
                const int limb = piece / BPC, prow = (piece % BPC) * 16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(bbase[pc] + k0),
                                                 (__attribute__((address_space(3))) void *)(sb + limb * B_BF + prow * 32),
                                                 16, 0, 0);
            }
            return;
        }
        glds_tile<BM>(st, p.A, p.lda, m0, p.M, k0, p.K, wid, lane);
#pragma unroll
        for (int pc = 0; pc < 3 * BPC / 4; ++pc) {
            const int piece = pc * 4 + wid;
            const int limb = piece / BPC, prow = (piece % BPC) * 16;
            const int r = prow + (lane >> 2);
            const int c = (lane & 3) ^ ((r >> 2) & 3);
            const __bf16 *src = planes + ((size_t)(limb * Np + n0 + r) * Kp + k0 + 8 * c);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(sb + limb * B_BF + prow * 32),
                                             16, 0, 0);
        }
    };
#pragma unroll
    for (int i = 0; i < S - 1; ++i)
        if (i < nt) issue(i);
    for (int i = 0; i < nt; ++i) {
        const int ahead = min(S - 2, nt - 1 - i);
        if (ahead >= 2) wait_vmcnt<2 * NLD>();
        else if (ahead == 1) wait_vmcnt<NLD>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (i + S - 1 < nt) issue(i + S - 1);
        const float *sa = lds + (i % S) * STAGE_FL;
        const __bf16 *sb = reinterpret_cast<const __bf16 *>(sa + A_FL);
#pragma unroll
        for (int s16 = 0; s16 < 2; ++s16) {
            bf16x8 a0, a1, a2;
            frag_split(sa, wid * 32 + li, s16, h, a0, a1, a2);
            bf16x8 b[3][TN];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int r = j * 32 + li, c = 2 * s16 + h;
                const int off = r * 32 + 8 * (c ^ ((r >> 2) & 3));
#pragma unroll
                for (int l = 0; l < 3; ++l) b[l][j] = *reinterpret_cast<const bf16x8 *>(&sb[l * B_BF + off]);
            }
            // the TN accumulator chains interleaved product by product
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b[0][j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[1][j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[2][j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b[0][j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[1][j], acc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b[0][j], acc[j], 0, 0, 0);
        }
        if constexpr (IGLP == 0 || IGLP == 1) __builtin_amdgcn_iglp_opt(IGLP);
    }

    if constexpr (ELDS) {                                   // LDS-staged epilogue (epi_rows)
        __syncthreads();                                    // every wave is done with the stages
        float *wl = lds + wid * 32 * (BN + 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) wl[((r & 3) + 8 * (r >> 2) + 4 * h) * (BN + 4) + 32 * j + li] = acc[j][r];
        f32x4 cs;
        epi_rows<BN>(wl, m0 + wid * 32, n0, lane, p, cs);
        if (p.colpart) epi_rows_colpart<BN>(lds, cs, wid, lane, ty, n0, p);
        return;
    }
    float csum[TN];
    epi_store<TN>(acc, m0 + wid * 32, n0, li, h, p, csum);
    if (p.colpart) {                                        // 64-row partials, as hsg_gemm_row_tiles
#pragma unroll
        for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32);
        __syncthreads();                                   // no DMA is pending here
        float *red = lds;
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) red[wid * BN + j * 32 + li] = csum[j];
        }
        __syncthreads();
        const int rows64 = (p.M + 63) / 64;
        for (int c = threadIdx.x; c < 2 * BN; c += 256) {
            const int half = c / BN, n = n0 + c % BN, slab = 2 * ty + half;
            if (n < p.N && slab < rows64)
                p.colpart[(size_t)slab * p.N + n] = red[(2 * half) * BN + c % BN] + red[(2 * half + 1) * BN + c % BN];
        }
    }
}

// ---------------------------------------------------------------------------------
// k_gemm7: k_gemm5's contract (fp32 A split in-kernel, pre-split weight planes) on
// v_mfma_f32_16x16x32_bf16 with WIDE wave tiles: block = 128 rows x BN columns, 4
// waves stacked along M, each wave 32 rows x BN (TN = BN/16 column subtiles).  One
// split of a wave's A fragment (8 k-values of 2 x 16 rows per 32-deep step, 9 VALU
// per pair: split_trunc8) feeds 2 * TN * 6 MFMAs, so the split costs <= 1 VALU per
// MFMA at BN >= 80 (k_gemm5: 4.5 per 32x32x16 MFMA, which left its issue port, not
// the matrix core, the limit).  16x16x32 also lets N = 300 run as 4 tiles of 80
// (6.7 % padding) instead of 5 of 64 or 3 of 128.  Operands go global -> LDS by
// global_load_lds_dwordx4 through S stages of 32-deep tiles (k_gemm5's images, with
// the swizzles swz16 / bswz16 that make both fragment reads conflict-free for the
// 16x16x32 lane map under gfx950's ds_read_b128 lane groups; round 4's k_gemm5
// swizzles cost 2-way conflicts on every read).
// The epilogue goes through LDS (epi_rows: float4 aux loads and C stores).  Measured
// (tools/gemm5_sweep.py, 5 interleaved rounds): BN = 64 is the fastest tile on all
// four cfg2 S2W FFN shapes; the wide tiles (80 | 128) were not faster.
// ---------------------------------------------------------------------------------

// PM: 0 = fp32-accurate (RNE 3-limb split, six products), 1 = the same with the
// truncation split (dev), 2 = bf16 mode (hsg_gemm_bf16 semantics: A and the weight
// rounded to bf16 RNE, ONE product: only limb plane 0 of the weight is staged)
// SA: the DMA sources as a wave-uniform base pointer (advanced by 32 k per tile, SGPRs)
// plus per-lane 32-bit byte offsets computed once (row clamps, swizzles, limb rows), so
// the K loop issues the saddr form of global_load_lds with no per-tile address VALU;
// only a tile reaching past K takes the per-chunk zero-page select.
// IO (round 5, bf16 mode only, PM = 2): bit 0 -- A is bf16 (the FFN's bf16 H / dY /
// dH rows: lda % 8 == 0, 16-byte rows, columns K .. ceil8(K) - 1 zero): the A tile is
// staged as bf16 rows of 64 B (the weight planes' image and swizzle, bswz16) and a
// fragment is one ds_read_b128, no conversion; bit 1 -- C is stored as bf16; bit 2 --
// the aux operand (relu' mask) is bf16.  The products are those of the fp32-A path
// (which rounds A to bf16 at fragment read): the bf16 mode's numbers are unchanged, its
// bytes halved.
template <int BN, int S, int PM = 0, int OCC = 2, bool SA = false, int IO = 0>
__global__ __launch_bounds__(256, OCC) void k_gemm7(GemmArgs p, const __bf16 *__restrict__ planes, int Np, int Kp) {
    constexpr int BM = 128, TN = BN / 16;
    constexpr bool ABF = (IO & 1) != 0, CBF = (IO & 2) != 0, AUXBF = (IO & 4) != 0, GBF = (IO & 8) != 0;
    constexpr bool XBF = (IO & 16) != 0;
    static_assert(!ABF || (PM == 2 && !SA), "bf16 A: the bf16 mode's one-product path");
    constexpr int A_FL = ABF ? BM * 16 : BM * 32;          // floats of the A tile
    constexpr int B_BF = BN * 32;                          // bf16 per limb-plane tile
    constexpr int NL = PM == 2 ? 1 : 3;                    // weight limb planes staged
    constexpr bool NOMFMA = PM >= 5;                       // dev diagnostics (plans 34-38)
    constexpr bool NOSPLIT = PM >= 6, NOB = PM == 7, NOA = PM == 8;
    constexpr int STAGE_FL = A_FL + NL * B_BF / 2;         // stage size in floats
    constexpr int BPC = BN / 16;                           // 1-KB pieces (16 rows) per limb plane tile
    constexpr int NBP = (NL * BPC + 3) / 4;                // B DMA instructions per wave per K tile
    constexpr int NLA = ABF ? BM / 64 : BM / 32;           // A DMA instructions per wave per K tile
    constexpr int NLD = NLA + NBP;                         // all DMA instructions per wave per K tile
    constexpr int EPI_FL = BM * (BN + 4);                  // the epilogue's row images reuse the stages
    static_assert(BN % 16 == 0, "BN must be a multiple of 16");
    __shared__ __attribute__((aligned(16))) float lds[S * STAGE_FL > EPI_FL ? S * STAGE_FL : EPI_FL];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int total = tiles_n * tiles_m;
    const int lt = p.xcd ? xcd_tile(blockIdx.x, total) : (int)blockIdx.x;
    const int tx = lt % tiles_n, ty = lt / tiles_n;
    const int m0 = ty * BM, n0 = tx * BN;
    const int nt = Kp / 32;

    f32x4v7 acc[2][TN];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4v7{0.f, 0.f, 0.f, 0.f};
    EpiRows<BN, CBF, AUXBF, GBF, XBF> ep;

    uint32_t aoff[BM / 32], boff[NBP];
    if constexpr (SA) {
#pragma unroll
        for (int pc = 0; pc < BM / 32; ++pc) {
            const int r = (pc * 4 + wid) * 8 + (lane >> 3);
            aoff[pc] = ((uint32_t)min(m0 + r, p.M - 1) * (uint32_t)p.lda + 4u * ((lane & 7) ^ swz16(r))) * 4u;
        }
#pragma unroll
        for (int pc = 0; pc < NBP; ++pc) {
            const int piece = min(pc * 4 + wid, NL * BPC - 1);
            const int limb = piece / BPC, r = (piece % BPC) * 16 + (lane >> 2);
            boff[pc] = ((uint32_t)(limb * Np + n0 + r) * (uint32_t)Kp + 8u * ((lane & 3) ^ bswz16(r))) * 2u;
        }
    }
    auto issue = [&](int it) {
        float *st = lds + (it % S) * STAGE_FL;
        const int k0 = it * 32;
        if constexpr (SA) {
            const char *ab = reinterpret_cast<const char *>(p.A) + (size_t)k0 * 4;
            const char *bb = reinterpret_cast<const char *>(planes) + (size_t)k0 * 2;
            __bf16 *sb = reinterpret_cast<__bf16 *>(st + A_FL);
            if (k0 + 32 <= p.K) {                                 // wave-uniform: no K-tail chunk
#pragma unroll
                for (int pc = 0; pc < BM / 32; ++pc)
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(ab + aoff[pc]),
                                                     (__attribute__((address_space(3))) void *)(st + (pc * 4 + wid) * 256),
                                                     16, 0, 0);
            } else {
#pragma unroll
                for (int pc = 0; pc < BM / 32; ++pc) {
                    const int r = (pc * 4 + wid) * 8 + (lane >> 3);
                    const bool in = k0 + 4 * ((lane & 7) ^ swz16(r)) < p.K;
                    const void *src = in ? (const void *)(ab + aoff[pc]) : (const void *)g_zero16;
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                     (__attribute__((address_space(3))) void *)(st + (pc * 4 + wid) * 256),
                                                     16, 0, 0);
                }
            }
#pragma unroll
            for (int pc = 0; pc < NBP; ++pc) {
                const int piece = min(pc * 4 + wid, NL * BPC - 1);
                const int limb = piece / BPC, prow = (piece % BPC) * 16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(bb + boff[pc]),
                                                 (__attribute__((address_space(3))) void *)(sb + limb * B_BF + prow * 32),
                                                 16, 0, 0);
            }
            return;
        }
        if constexpr (ABF) {
            // 16 rows of 64 B per 1-KB piece, BM / 16 pieces over 4 waves
            const __bf16 *Ab = reinterpret_cast<const __bf16 *>(p.A);
#pragma unroll
            for (int pc = 0; pc < NLA; ++pc) {
                const int piece = pc * 4 + wid;
                const int r = piece * 16 + (lane >> 2);
                const int c = (lane & 3) ^ bswz16(r);
                const int k = k0 + 8 * c;
                const void *src = k < p.K ? (const void *)(Ab + (size_t)min(m0 + r, p.M - 1) * p.lda + k)
                                          : (const void *)g_zero16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(st + piece * 256), 16, 0, 0);
            }
        } else if constexpr (!NOA) {
            glds_tile<BM, true>(st, p.A, p.lda, m0, p.M, k0, p.K, wid, lane);
        }
        __bf16 *sb = reinterpret_cast<__bf16 *>(st + A_FL);
#pragma unroll
        for (int pc = 0; pc < (NOB ? 0 : NBP); ++pc) {
            // NL * BPC pieces over 4 waves; a wave short of pieces repeats the last one
            // (the same bytes to the same LDS address), so every wave issues NBP DMAs
            // and one vmcnt count serves all of them
            const int piece = min(pc * 4 + wid, NL * BPC - 1);
            const int limb = piece / BPC, prow = (piece % BPC) * 16;
            const int r = prow + (lane >> 2);
            const int c = (lane & 3) ^ bswz16(r);
            const __bf16 *src = planes + ((size_t)(limb * Np + n0 + r) * Kp + k0 + 8 * c);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                             (__attribute__((address_space(3))) void *)(sb + limb * B_BF + prow * 32),
                                             16, 0, 0);
        }
    };
#pragma unroll
    for (int i = 0; i < S - 1; ++i)
        if (i < nt) issue(i);
    const int li = lane & 15, kb = lane >> 4;
    for (int it = 0; it < nt; ++it) {
        const int ahead = min(S - 2, nt - 1 - it);
        if (ahead >= 2) wait_vmcnt<2 * NLD>();
        else if (ahead == 1) wait_vmcnt<NLD>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (it + S - 1 < nt) issue(it + S - 1);
        if (it == nt - 1) ep.load(p, m0 + wid * 32, n0, lane);   // overlaps the last tile's MFMAs
        (void)NOSPLIT;
        const float *sa = lds + (it % S) * STAGE_FL;
        const __bf16 *sb = reinterpret_cast<const __bf16 *>(sa + A_FL);
        bf16x8 a[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if constexpr (ABF) {
                const int r = wid * 32 + 16 * i + li;
                a[i][0] = *reinterpret_cast<const bf16x8 *>(reinterpret_cast<const __bf16 *>(sa) + r * 32 +
                                                            8 * (kb ^ bswz16(r)));
                continue;
            }
            const int r = wid * 32 + 16 * i + li, sw = swz16(r);
            const f32x4 x = *reinterpret_cast<const f32x4 *>(&sa[r * 32 + 4 * ((2 * kb) ^ sw)]);
            const f32x4 y = *reinterpret_cast<const f32x4 *>(&sa[r * 32 + 4 * ((2 * kb + 1) ^ sw)]);
            if constexpr (NOSPLIT) {
                a[i][0] = __builtin_bit_cast(bf16x8, x);
                a[i][1] = __builtin_bit_cast(bf16x8, y);
                a[i][2] = a[i][0];
            } else if constexpr (PM == 0 || PM == 4 || PM == 5) {
                split_rne8(x, y, a[i][0], a[i][1], a[i][2]);
            } else if constexpr (PM == 1) {
                split_trunc8(x, y, a[i][0], a[i][1], a[i][2]);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) a[i][0][e] = (__bf16)(e < 4 ? x[e] : y[e - 4]);   // RNE
            }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int r = 16 * j + li;
            const int off = r * 32 + 8 * (kb ^ bswz16(r));
            bf16x8 b[3];
#pragma unroll
            for (int l = 0; l < NL; ++l) b[l] = *reinterpret_cast<const bf16x8 *>(&sb[l * B_BF + off]);
            if constexpr (NOMFMA) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int l = 0; l < 3; ++l)
                        acc[i][j][l] += __builtin_bit_cast(float, __builtin_bit_cast(u32x4, a[i][l])[0] ^
                                                                      __builtin_bit_cast(u32x4, b[l])[1]);
            } else if constexpr (PM == 2) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[0], acc[i][j], 0, 0, 0);
            } else {
#pragma unroll
                for (int i = 0; i < 2; ++i) {   // small products first
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[2], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[0], acc[i][j], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_iglp_opt(0);
    }

    // LDS-staged epilogue (epi_rows): float4 aux loads, C stores and column sums
    __syncthreads();                                        // every wave is done with the stages
    float *wl = lds + wid * 32 * (BN + 4);
    const int c = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) wl[(16 * i + rq + e) * (BN + 4) + 16 * j + c] = acc[i][j][e];
    f32x4 cs;
    if (nt == 0) ep.load(p, m0 + wid * 32, n0, lane);
    ep.template finish<PM == 4>(wl, m0 + wid * 32, n0, lane, p, cs);
    if (p.colpart) epi_rows_colpart<BN>(lds, cs, wid, lane, ty, n0, p);
}

template <int BN, int S, int PM = 0, int OCC = 2, bool SA = false, int IO = 0>
int launch7(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    p.splits = 1;
    p.k_tiles_per_split = Kp / 32;
    if ((p.N + BN - 1) / BN * BN > Np) return HSG_EINVAL;   // B tile rows must exist in the planes
    if (!epi_rows_ok(p)) return HSG_EINVAL;                 // the float4 epilogue needs whole aligned quads
    const long g = (long)((p.N + BN - 1) / BN) * ((p.M + 127) / 128);
    if (SA && ((long)p.M * p.lda * 4 >= (1L << 32) || (long)3 * Np * Kp * 2 >= (1L << 32))) return HSG_EINVAL;
    hipLaunchKernelGGL((k_gemm7<BN, S, PM, OCC, SA, IO>), dim3((unsigned)g), dim3(256), 0, st, p, planes, Np, Kp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// ---------------------------------------------------------------------------------
// k_gemm12 (round 6): k_gemm7's products with the weight tile RESIDENT in LDS and no
// barrier in the K loop.  The k_gemm7 diagnostics (tools/gemm5_sweep.py plans 35-38,
// profiles/r06/g7diag/) put its floor in the per-K-step barrier + one-stage DMA
// prefetch: with B loads alone (no A, no MFMA) it still takes 31 of its 47 us.  Here a
// block (4 waves, one per SIMD, one block per CU) keeps the whole 64-column B tile of
// its column range (3 limb planes x Kp, K <= 320: 120 KB) in LDS, loaded ONCE; the A
// rows a wave multiplies are private to it, so they go global -> registers, two K steps
// ahead, with no LDS and no barrier.  A wave's task is a 32-row band x 64 columns over
// the full K (k_gemm7's wave tile, same fragments, same product order: C is bitwise
// k_gemm7's).  XCD x (blockIdx % 8) owns the contiguous x-th eighth of the row bands
// and all column tiles, so A is fetched from HBM once per XCD L2 and reused by the
// column tiles there.  Column partials (colpart) are per 32-row band.
// MEASURED SLOWER (dev opt-in HSG_GEMM12=1; profiles/r06/g12/): C bitwise k_gemm7's,
// but 59-71 us against k_gemm7's 47 us on ffn1 / dH at cfg2 whatever the A prefetch
// depth (1-6 steps), the iglp / sched_group_barrier interleave, or an explicit
// software pipeline of the split and the B reads: one wave per SIMD has no partner to
// fill its LDS-read, split and epilogue latencies, and the LDS a resident B tile takes
// leaves no room for a second block.
// ---------------------------------------------------------------------------------
#ifdef HSG_DEV
constexpr int kG12BN = 64;
constexpr int kG12MaxKp = 320;

__host__ __device__ constexpr size_t g12_lds_bytes(int nt) {
    return (size_t)nt * 3 * kG12BN * 32 * 2 + (size_t)4 * 32 * (kG12BN + 4) * 4;
}

template <bool IGLP>
__global__ __launch_bounds__(256, 1) void k_gemm12(GemmArgs p, const __bf16 *__restrict__ planes, int Np, int Kp,
                                                   int tiles_n, int q) {
    constexpr int BN = kG12BN, TN = BN / 16, BPC = BN / 16, B_BF = BN * 32;
    extern __shared__ __attribute__((aligned(16))) float g12_lds[];
    const int nt = Kp / 32;
    __bf16 *sB = reinterpret_cast<__bf16 *>(g12_lds);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float *wl = g12_lds + nt * 3 * B_BF / 2 + wid * 32 * (BN + 4);
    const int xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
    const int ct = local % tiles_n, sub = local / tiles_n;
    const int n0 = ct * BN;
    const int nbands = (p.M + 31) / 32;
    const int bb = xcd * nbands / 8, be = (xcd + 1) * nbands / 8;
    const int S = 4 * q, s = 4 * sub + wid;

    // the block's B tile: nt K tiles x 3 limbs x BPC 1-KB pieces, k_gemm7's image per tile
    for (int pc = wid; pc < nt * 3 * BPC; pc += 4) {
        const int kt = pc / (3 * BPC), rem = pc % (3 * BPC);
        const int limb = rem / BPC, prow = (rem % BPC) * 16;
        const int r = prow + (lane >> 2);
        const int c = (lane & 3) ^ bswz16(r);
        const __bf16 *src = planes + ((size_t)(limb * Np + n0 + r) * Kp + kt * 32 + 8 * c);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(sB + (kt * 3 + limb) * B_BF +
                                                                                    prow * 32),
                                         16, 0, 0);
    }
    wait_vmcnt<0>();
    __syncthreads();

    const int ntask = s < be - bb ? (be - bb - s + S - 1) / S : 0;
    const int nsteps = ntask * nt;
    const int li = lane & 15, kb = lane >> 4;
    f32x4v7 acc[2][TN];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4v7{0.f, 0.f, 0.f, 0.f};
    EpiRows<BN> ep;

    // A fragments of flattened step st (task st / nt, K tile st % nt): rows 16 i + li,
    // k = 8 kb .. 8 kb + 7 of the tile as two float4 (K % 4 == 0: whole quads)
    auto load_step = [&](int st, f32x4 (&R)[4]) {
        if (st >= nsteps) return;
        const int band = bb + s + (st / nt) * S, k = (st % nt) * 32 + 8 * kb;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = min(band * 32 + 16 * i + li, p.M - 1);
            const float *a = p.A + (size_t)m * p.lda + k;
            R[2 * i] = k < p.K ? *reinterpret_cast<const f32x4 *>(a) : f32x4{0.f, 0.f, 0.f, 0.f};
            R[2 * i + 1] = k + 4 < p.K ? *reinterpret_cast<const f32x4 *>(a + 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    };
    // software pipeline (one wave per SIMD has no partner to hide its latencies): step
    // st's MFMAs run on fragments made during step st - 1 -- the split limbs of its A
    // rows and its B fragments read from LDS -- while that step's VALU split and
    // ds_reads for st + 1 are interleaved between them (sched_group_barrier)
    auto split_a = [&](const f32x4 (&R)[4], bf16x8 (&a)[2][3]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) split_rne8(R[2 * i], R[2 * i + 1], a[i][0], a[i][1], a[i][2]);
    };
    auto read_b = [&](int kt, bf16x8 (&b)[TN][3]) {
        const __bf16 *sb = sB + kt * 3 * B_BF;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int r = 16 * j + li;
            const int off = r * 32 + 8 * (kb ^ bswz16(r));
#pragma unroll
            for (int l = 0; l < 3; ++l) b[j][l] = *reinterpret_cast<const bf16x8 *>(&sb[l * B_BF + off]);
        }
    };
    auto mfmas = [&](const bf16x8 (&a)[2][3], const bf16x8 (&b)[TN][3]) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i) {   // k_gemm7's order: small products first
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][2], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][0], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][1], acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][0], acc[i][j], 0, 0, 0);
            }
    };
    // two register sets, even / odd steps (nt is even: a band starts on the even set)
    f32x4 R[2][4];
    bf16x8 A0[2][3], A1[2][3], B0[TN][3], B1[TN][3];
    load_step(0, R[0]);
    load_step(1, R[1]);
    if (nsteps > 0) {
        split_a(R[0], A0);
        read_b(0, B0);
    }
    auto step = [&](int st, int kt, f32x4 (&Rn)[4], const bf16x8 (&Ac)[2][3], const bf16x8 (&Bc)[TN][3],
                    bf16x8 (&An)[2][3], bf16x8 (&Bn)[TN][3], f32x4 (&Rl)[4]) {
        // Rn holds step st + 1's A rows; Rl (= step st's ring slot, consumed) gets st + 2's
        if (st + 1 < nsteps) {
            read_b(kt + 1 == nt ? 0 : kt + 1, Bn);
            split_a(Rn, An);
        }
        load_step(st + 2, Rl);
        mfmas(Ac, Bc);
        if constexpr (IGLP) {
#pragma unroll
            for (int g = 0; g < 12; ++g) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // 4 MFMA
                __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // 1 ds_read
                __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);   // 6 VALU
            }
        }
    };
    for (int task = 0; task < ntask; ++task) {
        const int row0 = (bb + s + task * S) * 32;
        for (int kt = 0; kt < nt; kt += 2) {
            const int st = task * nt + kt;
            if (kt + 2 >= nt) ep.load(p, row0, n0, lane);       // overlaps the last steps' MFMAs
            step(st, kt, R[1], A0, B0, A1, B1, R[0]);
            step(st + 1, kt + 1, R[0], A1, B1, A0, B0, R[1]);
        }
        // the band's epilogue through the wave's private LDS rows (k_gemm7's EpiRows)
        const int c = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) {
#pragma unroll
                for (int e = 0; e < 4; ++e) wl[(16 * i + rq + e) * (BN + 4) + 16 * j + c] = acc[i][j][e];
                acc[i][j] = f32x4v7{0.f, 0.f, 0.f, 0.f};
            }
        f32x4 cs;
        ep.finish(wl, row0, n0, lane, p, cs);
        if (p.colpart) {
            // 32-row partial of this band: the lane sums over its rows (rs = lane / 16)
            // added in rs order, then one float4 per column quad
            constexpr int QS = EpiMap<BN>::QS;
            static_assert(QS == 16, "BN = 64: 16 quads per row step");
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float v1 = __shfl(cs[e], (lane & 15) + 16), v2 = __shfl(cs[e], (lane & 15) + 32),
                            v3 = __shfl(cs[e], (lane & 15) + 48);
                cs[e] = ((cs[e] + v1) + v2) + v3;
            }
            const int n = n0 + 4 * c;
            if (lane < 16 && n < p.N) *reinterpret_cast<f32x4 *>(p.colpart + (size_t)(row0 / 32) * p.N + n) = cs;
        }
    }
}

// k_gemm12's plan: fp32-accurate products, wide FFN shapes (N > 320) with the whole
// K in one resident B tile, and rows enough for every wave of the grid
bool plan12(int M, int N, int K) {
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    const char *f = HSG_DEV_ENV("HSG_GEMM12");               // dev opt-in: 1 = k_gemm12
    if (!f || atoi(f) != 1) return false;
    return N > 320 && Kp <= kG12MaxKp && (Kp / 32) % 5 == 0 && (K & 3) == 0 && M >= 8 * 32 * 32 &&
           (N + kG12BN - 1) / kG12BN <= 32;
}

int launch12(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    const int tiles_n = (p.N + kG12BN - 1) / kG12BN;
    if (tiles_n * kG12BN > Np || !epi_rows_ok(p) || p.epi == HSG_EPI_ADD_ELUG) return HSG_EINVAL;
    if ((p.lda & 3) || (((uintptr_t)p.A) & 15)) return HSG_EINVAL;
    const int q = max(1, 32 / tiles_n);
    int ig = 0;                                               // dev: sched_group_barrier interleave
    if (const char *f = HSG_DEV_ENV("HSG_GEMM12_IGLP")) ig = atoi(f);
    const auto go = [&](auto kern) {
        static bool attr = false;
        if (!attr) {
            if (hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)g12_lds_bytes(kG12MaxKp / 32)) != hipSuccess)
                return (int)HSG_EINVAL;
            attr = true;
        }
        hipLaunchKernelGGL(kern, dim3(8 * tiles_n * q), dim3(256), g12_lds_bytes(Kp / 32), st, p, planes, Np, Kp,
                           tiles_n, q);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : (int)e;
    };
    return ig ? go(k_gemm12<true>) : go(k_gemm12<false>);
}
#endif  // HSG_DEV

// ---------------------------------------------------------------------------------
// k_gemm11 (round 4): the pre-split-weight FFN GEMM on ONE round of big tiles.
// k_gemm7's 128 x 64 blocks (two per CU) move (128 x 4 + 64 x 6) B of operand per K
// for 8,192 outputs; at cfg2 its loads alone took 36 of its ~48 us per S2W FFN GEMM
// (DESIGN §3), and 1,200 / 750 tiles ran in 2.3 / 1.5 rounds of the 512 resident
// slots.  Here one block per CU (8 waves, 2 per SIMD) owns BM x BN outputs, with the
// tile sized so the whole GEMM is ONE round of at most one block per CU:
//   N > 320 (ffn1 H = x W1^T, dH = dy W2):  160 x 256, waves 2 x 4 of 80 x 64
//   N <= 320 (ffn2 y = H W2^T, dx += dH W1): 192 x 160, waves 4 x 2 of 48 x 80
// (cfg2: 240 / 200 tiles on 256 CUs), i.e. 2176 / 1728 B per K for 40,960 / 30,720
// outputs -- 2.1x / 1.9x fewer operand bytes per output than k_gemm7.  Same staging as
// k_gemm7 (global_load_lds_dwordx4 into two stages of 32-deep K tiles, swizzled
// images, one barrier per K tile), fragments by ds_read_b128, the fp32 operand split
// into three RNE bf16 limbs at fragment read (split_rne8), six products on
// v_mfma_f32_16x16x32_bf16; PM = 2: the bf16 mode (one product, limb plane 0 only).
// Epilogue through LDS (float4 bias / aux loads and C stores, as epi_rows), in two
// passes of half the waves when the images of all eight do not fit; column partials
// (colpart) are written per wave row band of WM rows (hsg_gemm_psw_row_tiles).
// ---------------------------------------------------------------------------------
template <int BM, int BN, int WGM, int WGN, int PM, int S = 2>
struct Cfg11 {
    static constexpr int NW = WGM * WGN, NT = 64 * NW;
    static constexpr int WM = BM / WGM, WN = BN / WGN, TM = WM / 16, TN = WN / 16;
    static constexpr int NL = PM == 2 ? 1 : 3;
    static constexpr int A_FL = BM * 32;                   // floats of the A tile
    static constexpr int B_BF = BN * 32;                   // bf16 per limb-plane tile
    static constexpr int STAGE_FL = A_FL + NL * B_BF / 2;
    static constexpr int APC = BM / 8, BPC = BN / 16;      // 1-KB DMA pieces: A (8 rows), B (16 rows / limb)
    static constexpr int NPC = APC + NL * BPC;
    static constexpr int NLD = (NPC + NW - 1) / NW;        // DMA instructions per wave per K tile
    static constexpr int LDW = WN + 4;                     // epilogue image row (floats)
    static constexpr int EPW = WM * LDW;                   // floats per wave image
    static constexpr int EPASS = S * STAGE_FL >= NW * EPW ? 1 : 2;
    static constexpr int LDS_FL = S * STAGE_FL > NW * EPW / EPASS ? S * STAGE_FL : NW * EPW / EPASS;
    // epilogue: float4 quads per row, rows per step (lanes past RPS * QPR idle)
    static constexpr int QPR = WN / 4, RPS = 64 / QPR;
    static constexpr int STEPS = (WM + RPS - 1) / RPS;
    // steps whose global operands are in flight together: the largest divisor of STEPS <= 10
    static constexpr int CH = STEPS % 10 == 0 ? 10 : STEPS % 8 == 0 ? 8 : STEPS % 6 == 0 ? 6 : STEPS % 5 == 0 ? 5
                            : STEPS % 4 == 0 ? 4 : STEPS;
    static_assert(WM % 16 == 0 && WN % 16 == 0 && QPR <= 64, "tile shape");
    static_assert(LDS_FL * 4 <= 163840, "LDS");
};

// S: LDS stages (2: the next K tile's DMA overlaps this tile's MFMAs; 1: one stage,
// several blocks per CU overlap each other instead), OCC: blocks per CU (launch bounds)
template <int BM, int BN, int WGM, int WGN, int PM, bool LN = false, int S = 2, int OCC = 1>
__global__ __launch_bounds__(64 * WGM * WGN, OCC) void k_gemm11(GemmArgs p, const __bf16 *__restrict__ planes,
                                                                int Np, int Kp) {
    static_assert(S == 1 || S == 2, "stages");
    using C = Cfg11<BM, BN, WGM, WGN, PM, S>;
    constexpr int NW = C::NW, WM = C::WM, WN = C::WN, TM = C::TM, TN = C::TN, NL = C::NL;
    constexpr int LDT = BN - 12;                               // LN epilogue: the tile's image, N <= BN - 16 columns
    constexpr int LDS_ALL = LN && BM * LDT > C::LDS_FL ? BM * LDT : C::LDS_FL;
    static_assert(LDS_ALL * 4 <= 163840, "LDS");
    __shared__ __attribute__((aligned(16))) float lds[LDS_ALL];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid / WGN, wn = wid % WGN;
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int total = tiles_n * tiles_m;
    const int lt = p.xcd ? xcd_tile(blockIdx.x, total) : (int)blockIdx.x;
    const int tx = lt % tiles_n, ty = lt / tiles_n;
    const int m0 = ty * BM, n0 = tx * BN;
    const int nt = Kp / 32;

    f32x4v7 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4v7{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int it) {
        float *st = lds + (S == 2 ? (it & 1) : 0) * C::STAGE_FL;
        __bf16 *sb = reinterpret_cast<__bf16 *>(st + C::A_FL);
        const int k0 = it * 32;
#pragma unroll
        for (int i = 0; i < C::NLD; ++i) {
            // NPC pieces over NW waves; a wave short of pieces repeats the last one (the
            // same bytes to the same LDS address), so every wave issues NLD DMAs and one
            // vmcnt count serves all of them
            const int piece = min(i * NW + wid, C::NPC - 1);          // wave-uniform
            if (piece < C::APC) {
                const int r = piece * 8 + (lane >> 3);
                const int q = (lane & 7) ^ swz16(r);
                const int k = k0 + 4 * q;
                const int gr = min(m0 + r, p.M - 1);
                const float *src = k < p.K ? p.A + (size_t)gr * p.lda + k : g_zero16;
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(st + piece * 256), 16, 0, 0);
            } else {
                const int bp = piece - C::APC;
                const int limb = bp / C::BPC, prow = (bp % C::BPC) * 16;
                const int r = prow + (lane >> 2);
                const int c = (lane & 3) ^ bswz16(r);
                const __bf16 *src = planes + ((size_t)(limb * Np + n0 + r) * Kp + k0 + 8 * c);
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                                 (__attribute__((address_space(3))) void *)(sb + limb * C::B_BF + prow * 32),
                                                 16, 0, 0);
            }
        }
    };
    if (S == 2 && nt > 0) issue(0);
    const int li = lane & 15, kb = lane >> 4;
    for (int it = 0; it < nt; ++it) {
        if constexpr (S == 1) {
            if (it > 0) __syncthreads();                        // every wave is done with the stage
            issue(it);
        }
        wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (S == 2 && it + 1 < nt) issue(it + 1);           // lands while this tile is multiplied
        const float *sa = lds + (S == 2 ? (it & 1) : 0) * C::STAGE_FL;
        const __bf16 *sb = reinterpret_cast<const __bf16 *>(sa + C::A_FL);
        bf16x8 a[TM][3];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int r = wm * WM + 16 * i + li, sw = swz16(r);
            const f32x4 x = *reinterpret_cast<const f32x4 *>(&sa[r * 32 + 4 * ((2 * kb) ^ sw)]);
            const f32x4 y = *reinterpret_cast<const f32x4 *>(&sa[r * 32 + 4 * ((2 * kb + 1) ^ sw)]);
            if constexpr (PM == 2) {
#pragma unroll
                for (int e = 0; e < 8; ++e) a[i][0][e] = (__bf16)(e < 4 ? x[e] : y[e - 4]);   // RNE
            } else {
                split_rne8(x, y, a[i][0], a[i][1], a[i][2]);
            }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int r = wn * WN + 16 * j + li;
            const int off = r * 32 + 8 * (kb ^ bswz16(r));
            bf16x8 b[3];
#pragma unroll
            for (int l = 0; l < NL; ++l) b[l] = *reinterpret_cast<const bf16x8 *>(&sb[l * C::B_BF + off]);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if constexpr (PM == 2) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[0], acc[i][j], 0, 0, 0);
                } else {                                    // small products first
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[2], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[0], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[0], acc[i][j], 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_iglp_opt(0);
    }

    if constexpr (LN) {
        // y = acc + b2 (stored: the backward's LN reads it), out = LN(dropout(y) + x):
        // the whole BM x BN tile (BN >= N: full rows) imaged in LDS, then wave w takes
        // rows w, w + NW, ...; lane = float4 quads 4 lane + 256 i of the row, the
        // arithmetic (and dropout index r * N + c) of k_ln_fwd4, so the result is that
        // kernel's on the same y
        static_assert(BN <= 512, "two quads per lane per row");
        __syncthreads();                                       // every wave is done with the stages
        {
            const int c = lane & 15, rq = 4 * (lane >> 4);
            float *img = lds + (wm * WM) * LDT + wn * WN;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    if (wn * WN + 16 * j < p.N)                // subtiles past N (padding) are not imaged
#pragma unroll
                        for (int e = 0; e < 4; ++e) img[(16 * i + rq + e) * LDT + 16 * j + c] = acc[i][j][e];
        }
        constexpr int RW = BM / NW;                            // rows per wave
        static_assert(BM % NW == 0, "rows per wave");
        // the residual rows and the per-column operands, requested before the barrier
        f32x4 xr[RW][2], bq[2], gq[2], tq[2];
        int rowv = wid;
        asm volatile("" : "+v"(rowv));                         // after the image writes
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int c = min(4 * lane + 256 * i, p.N - 4);
            bq[i] = *reinterpret_cast<const f32x4 *>(p.bias + c);
            gq[i] = *reinterpret_cast<const f32x4 *>(p.gamma + c);
            tq[i] = *reinterpret_cast<const f32x4 *>(p.beta + c);
        }
#pragma unroll
        for (int t = 0; t < RW; ++t) {
            const int m = min(m0 + rowv + NW * t, p.M - 1);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = min(4 * lane + 256 * i, p.N - 4);
                xr[t][i] = *reinterpret_cast<const f32x4 *>(p.aux + (size_t)m * p.ldaux + c);
            }
        }
        __syncthreads();
        const uint32_t dkey = p.p_drop > 0.f ? hsg_drop_key((uint64_t)p.seed[0], p.offset) : 0u;
        const uint32_t thr = hsg_drop_threshold(p.p_drop);
        const float scale = p.p_drop > 0.f ? 1.f / (1.f - p.p_drop) : 1.f;
#pragma unroll
        for (int t = 0; t < RW; ++t) {
            const int r = rowv + NW * t, m = m0 + r;
            if (m >= p.M) break;                               // wave-uniform
            f32x4 sv[2];
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = 4 * lane + 256 * i;
                sv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
                if (c < p.N) {
                    f32x4 v = *reinterpret_cast<const f32x4 *>(&lds[r * LDT + c]) + bq[i];
                    const size_t o = (size_t)m * p.N + c;
                    *reinterpret_cast<f32x4 *>(p.C + (size_t)m * p.ldc + c) = v;
                    if (p.p_drop > 0.f) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = hsg_keep32(dkey, (uint32_t)(o + e), thr) ? v[e] * scale : 0.f;
                    }
                    sv[i] = v + xr[t][i];
                    sum += (sv[i][0] + sv[i][1]) + (sv[i][2] + sv[i][3]);
                }
            }
            for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
            const float mu = sum / p.N;
            float var = 0.f;
#pragma unroll
            for (int i = 0; i < 2; ++i)
                if (4 * lane + 256 * i < p.N)
#pragma unroll
                    for (int e = 0; e < 4; ++e) { const float d = sv[i][e] - mu; var = fmaf(d, d, var); }
            for (int o = 32; o >= 1; o >>= 1) var += __shfl_xor(var, o);
            const float rsd = rsqrtf(var / p.N + p.eps);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = 4 * lane + 256 * i;
                if (c < p.N) *reinterpret_cast<f32x4 *>(p.lnout + (size_t)m * p.N + c) = (sv[i] - mu) * rsd * gq[i] + tq[i];
            }
            if (lane == 0) { p.mean[m] = mu; p.rstd[m] = rsd; }
        }
        return;
    }

    // epilogue: each wave's WM x WN tile through LDS, float4 quads (lane: quad q of
    // row rs of each RPS-row step), in EPASS passes of NW / EPASS waves
    int q = lane % C::QPR, rs = lane / C::QPR;
    // opaque to the scheduler: nothing of the epilogue (its operand addresses) is
    // computed before the K loop ends, where it would hold registers across it
    asm volatile("" : "+v"(q), "+v"(rs));
    const int row0 = m0 + wm * WM, n = n0 + wn * WN + 4 * q;
    const bool nok = n < p.N && rs < C::RPS;                   // N % 4 == 0: whole quads
    const int nc = min(n, p.N - 4);
    f32x4 bn = f32x4{0.f, 0.f, 0.f, 0.f};
    if (p.bias) bn = *reinterpret_cast<const f32x4 *>(p.bias + nc);
    f32x4 csum = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int pass = 0; pass < C::EPASS; ++pass) {
        __syncthreads();                                       // stages (or the previous pass) consumed
        const bool mine = C::EPASS == 1 || (wid / (NW / C::EPASS)) == pass;
        float *wl = lds + (wid % (NW / C::EPASS)) * C::EPW;
        if (mine) {
            const int c = lane & 15, rq = 4 * (lane >> 4);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) wl[(16 * i + rq + e) * C::LDW + 16 * j + c] = acc[i][j][e];
            __builtin_amdgcn_s_waitcnt(0xc07f);                // lgkmcnt(0): the wave's own LDS writes
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");                     // no epilogue load above the image writes
            // CH steps of global operands in flight at a time
            constexpr int CH = C::CH;
#pragma unroll 1
            for (int s0 = 0; s0 < C::STEPS; s0 += CH) {       // (unrolled, the chunks' loads pile up: spills)
                asm volatile("" ::: "memory");                 // one chunk's loads in flight at a time
                f32x4 aux[CH], ex[CH];
#pragma unroll
                for (int t = 0; t < CH; ++t) {
                    const int m = min(row0 + min((s0 + t) * C::RPS + rs, WM - 1), p.M - 1);
                    if (p.epi != HSG_EPI_STORE) aux[t] = *reinterpret_cast<const f32x4 *>(p.aux + (size_t)m * p.ldaux + nc);
                    if (p.epi == HSG_EPI_ADD_ELUG) {
                        const size_t o = (size_t)m * p.ldaux + nc;
                        ex[t] = *reinterpret_cast<const f32x4 *>(p.aux2 + o) - *reinterpret_cast<const f32x4 *>(p.aux3 + o);
                    }
                }
#pragma unroll
                for (int t = 0; t < CH; ++t) {
                    const int r = (s0 + t) * C::RPS + rs, m = row0 + r;
                    if (!nok || r >= WM || m >= p.M) continue;
                    f32x4 v = *reinterpret_cast<const f32x4 *>(&wl[r * C::LDW + 4 * q]);
                    if (p.epi == HSG_EPI_RELU_BWD) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = aux[t][e] > 0.f ? v[e] : 0.f;
                    } else {
                        v += bn;
                        if (p.epi == HSG_EPI_ADD || p.epi == HSG_EPI_ADD_ELUG) v += aux[t];
                        if (p.relu) {
#pragma unroll
                            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
                        }
                    }
                    *reinterpret_cast<f32x4 *>(p.C + (size_t)m * p.ldc + n) = v;
                    if (p.epi == HSG_EPI_ADD_ELUG) {
                        f32x4 g;                            // G = dOut * elu'(h), e = elu(h) = x - origin
#pragma unroll
                        for (int e = 0; e < 4; ++e) g[e] = ex[t][e] > 0.f ? v[e] : v[e] * (ex[t][e] + 1.f);
                        *reinterpret_cast<f32x4 *>(p.C2 + (size_t)m * p.ldaux + n) = g;
                    }
                    csum += v;
                }
            }
        }
    }
    if (p.colpart) {                  // one partial row per wave row band (WM rows), fixed order
        f32x4 t = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < C::RPS; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] += __shfl(csum[e], k * C::QPR + q);
        if (rs == 0 && n < p.N) *reinterpret_cast<f32x4 *>(p.colpart + (size_t)(ty * WGM + wm) * p.N + n) = t;
    }
}

// dev opt-in (HSG_GEMM11=1): k_gemm11 measured slower than k_gemm7 on every cfg2 FFN
// shape (57.5 vs ~49 us: the one round of big tiles leaves the operand loads and the C
// stores of all CUs unoverlapped at its two ends)
bool gemm11_on() {
    const char *e = HSG_DEV_ENV("HSG_GEMM11");
    return e && atoi(e) >= 1;
}

// cfg2-class shapes only: the two big-tile plans, picked when they run the GEMM in ONE
// round of at most one block per CU at >= 75 % of the CUs; 0 = not applicable
int plan11(int M, int N, int cus) {
    if (N > 512) return 0;
    const int BM = N > 320 ? 160 : 192, BN = N > 320 ? 256 : 160;
    const long tiles = (long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > cus || 4 * tiles < 3L * cus) return 0;
    return N > 320 ? 1 : 2;
}

int device_cus() {
    static std::atomic<int> cached{-1};
    int c = cached.load(std::memory_order_relaxed);
    if (c < 0) {
        int dev = 0;
        c = 0;
        if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            c = 0;
        cached.store(c, std::memory_order_relaxed);
    }
    return c;
}

// 112- against 64-wide k_gemm7 tiles for N <= 320 (two blocks per CU resident, 128-row
// tiles): a tile's time grows with its width, so the cost is rounds x width -- cfg2
// (150 row tiles): 450 tiles in ONE round x 112 against 750 in two x 64, so 112 (40.0
// vs 45.6 us); cfg4 / cfg5 (175 / 225 row tiles): 525 / 675 tiles take two rounds x 112
// against two / three x 64 (84.5 / 91.8 us on 112-wide tiles against ~57 / ~70)
bool wide112_pays(int M, int N) {
    const int cus = device_cus() > 0 ? device_cus() : 256;
    const long slots = 2L * cus, mt = (M + 127) / 128;
    const long r112 = (mt * ((N + 111) / 112) + slots - 1) / slots, r64 = (mt * ((N + 63) / 64) + slots - 1) / slots;
    return r112 * 112 < r64 * 64;
}

template <int BM, int BN, int WGM, int WGN, int PM, int S = 2, int OCC = 1>
int launch11(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    p.splits = 1;
    p.k_tiles_per_split = Kp / 32;
    if ((p.N + BN - 1) / BN * BN > Np) return HSG_EINVAL;   // B tile rows must exist in the planes
    if (!epi_rows_ok(p)) return HSG_EINVAL;
    const long g = (long)((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM);
    hipLaunchKernelGGL((k_gemm11<BM, BN, WGM, WGN, PM, false, S, OCC>), dim3((unsigned)g), dim3(64 * WGM * WGN), 0, st, p, planes, Np,
                       Kp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// the LayerNorm-epilogue plan (full rows: BN = 320 >= N), ONE round at >= 60 % of the
// CUs: 96-row tiles (waves 2 x 4 of 48 x 80), else 128-row (64 x 80); 0 = none
int plan11ln(int M, int N, int cus) {
    if (N > 304 || N % 4) return 0;                         // the image holds 308 columns
    const long t96 = (M + 95) / 96, t128 = (M + 127) / 128;
    if (t96 <= cus && 5 * t96 >= 3L * cus) return 96;
    if (t128 <= cus && 5 * t128 >= 3L * cus) return 128;
    return 0;
}

template <int PM>
int try11ln(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    const int bm = plan11ln(p.M, p.N, device_cus());
    p.splits = 1;
    p.k_tiles_per_split = Kp / 32;
    if (!bm || 320 > Np) return HSG_EINVAL;
    const unsigned g = (unsigned)((p.M + bm - 1) / bm);
    if (bm == 96)
        hipLaunchKernelGGL((k_gemm11<96, 320, 2, 4, PM, true>), dim3(g), dim3(512), 0, st, p, planes, Np, Kp);
    else
        hipLaunchKernelGGL((k_gemm11<128, 320, 2, 4, PM, true>), dim3(g), dim3(512), 0, st, p, planes, Np, Kp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// the big-tile plan of this shape, or HSG_EINVAL when it does not apply
template <int PM>
int try11(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    // HSG_GEMM11=2 / 3: 128 x 128 tiles of 4 waves (2 x 2 of 64 x 64; 64-row column-partial
    // bands, as k_gemm7) for N > 320 only, one stage at 3 blocks per CU / two stages at 2
    // k_gemm11's epilogue writes C and G but no rho partials: the rho GEMM
    // always runs on k_gemm7, whose column tiles are multiples of 64
    if (p.rho) return HSG_EINVAL;
    const char *e = HSG_DEV_ENV("HSG_GEMM11");
    const int v = e ? atoi(e) : 0;
    if (v == 2 || v == 3) {
        if (p.N <= 320) return HSG_EINVAL;
        return v == 2 ? launch11<128, 128, 2, 2, PM, 1, 3>(p, planes, Np, Kp, st)
                      : launch11<128, 128, 2, 2, PM, 2, 2>(p, planes, Np, Kp, st);
    }
    const int pl = plan11(p.M, p.N, device_cus());
    if (pl == 1) return launch11<160, 256, 2, 4, PM>(p, planes, Np, Kp, st);
    if (pl == 2) return launch11<192, 160, 4, 2, PM>(p, planes, Np, Kp, st);
    return HSG_EINVAL;
}

// ---------------------------------------------------------------------------------
// k_gemm6: k_gemm5's contract (fp32 A, pre-split weight planes) with A never staged
// through LDS: each wave owns 32 A rows that no other wave reads, so every lane loads
// its own fragment (row li, 8 consecutive k per 16-k step: 2 x dwordx4) straight
// into registers, two K tiles ahead, and splits it there.  Only the weight limbs go
// through LDS (register-staged, double-buffered, one barrier per K tile); all loads
// are ordinary VGPR loads, so the compiler's counted vmcnt waits stay exact.
// ---------------------------------------------------------------------------------
template <int BN>
__global__ __launch_bounds__(256, 2) void k_gemm6(GemmArgs p, const __bf16 *__restrict__ planes, int Np, int Kp) {
    constexpr int BM = 128, TN = BN / 32;
    constexpr int B_BF = BN * 32;                          // bf16 per limb-plane tile
    constexpr int B_BUF = 3 * B_BF;                        // bf16 per buffer
    constexpr int BU = 3 * BN * 4 / 256;                   // 16-B B units per thread per K tile
    __shared__ __attribute__((aligned(16))) __bf16 sb[2 * B_BUF];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int li = lane & 31, h = lane >> 5;
    const int tiles_n = (p.N + BN - 1) / BN, tiles_m = (p.M + BM - 1) / BM;
    const int total = tiles_n * tiles_m;
    const int lt = p.xcd ? xcd_tile(blockIdx.x, total) : (int)blockIdx.x;
    const int tx = lt % tiles_n, ty = lt / tiles_n;
    const int m0 = ty * BM, n0 = tx * BN;
    const int nt = Kp / 32;
    const float *arow = p.A + (size_t)min(m0 + wid * 32 + li, p.M - 1) * p.lda;

    f32x16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    // A fragment quads of K tile kt: u = 2*s16 + e -> k = 32 kt + 16 s16 + 8 h + 4 e
    auto load_a = [&](f32x4 (&r)[4], int kt) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = kt * 32 + 16 * (u >> 1) + 8 * h + 4 * (u & 1);
            const float *src = k < p.K ? arow + k : g_zero16;
            r[u] = *reinterpret_cast<const f32x4 *>(src);
        }
    };
    auto load_b = [&](uint4 (&r)[BU], int kt) {
#pragma unroll
        for (int v = 0; v < BU; ++v) {
            const int u = threadIdx.x + 256 * v;
            const int limb = u / (BN * 4), rr = (u >> 2) % BN, c = u & 3;
            r[v] = *reinterpret_cast<const uint4 *>(planes + ((size_t)(limb * Np + n0 + rr) * Kp + kt * 32 + 8 * c));
        }
    };
    auto store_b = [&](int buf, const uint4 (&r)[BU]) {
#pragma unroll
        for (int v = 0; v < BU; ++v) {
            const int u = threadIdx.x + 256 * v;
            const int limb = u / (BN * 4), rr = (u >> 2) % BN, c = u & 3;
            *reinterpret_cast<uint4 *>(&sb[buf * B_BUF + limb * B_BF + rr * 32 + 8 * (c ^ ((rr >> 2) & 3))]) = r[v];
        }
    };
    auto compute = [&](int buf, const f32x4 (&a)[4]) {
        const __bf16 *b = sb + buf * B_BUF;
#pragma unroll
        for (int s16 = 0; s16 < 2; ++s16) {
            bf16x8 a0, a1, a2;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                __bf16 x0, x1, x2;
                split3(a[2 * s16 + (e >> 2)][e & 3], x0, x1, x2);
                a0[e] = x0; a1[e] = x1; a2[e] = x2;
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int r = j * 32 + li, c = 2 * s16 + h;
                const int off = r * 32 + 8 * (c ^ ((r >> 2) & 3));
                const bf16x8 b0 = *reinterpret_cast<const bf16x8 *>(&b[off]);
                const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(&b[B_BF + off]);
                const bf16x8 b2 = *reinterpret_cast<const bf16x8 *>(&b[2 * B_BF + off]);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, b0, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b2, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b0, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b1, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0, acc[j], 0, 0, 0);
            }
        }
    };

    f32x4 aA[4], aB[4];
    uint4 braw[BU];
    load_a(aA, 0);
    load_b(braw, 0);
    store_b(0, braw);
    if (nt > 1) {
        load_a(aB, 1);
        load_b(braw, 1);
    }
    __syncthreads();
    // one K tile per step; the two A register sets alternate (steps unrolled in pairs)
    auto step = [&](int i, f32x4 (&acur)[4], f32x4 (&anext2)[4]) {
        compute(i & 1, acur);
        if (i + 1 < nt) store_b((i + 1) & 1, braw);        // tile i+1's limbs, loaded a step ago
        if (i + 2 < nt) {
            load_a(anext2, i + 2);
            load_b(braw, i + 2);
        }
        __syncthreads();
    };
    int i = 0;
    for (; i + 1 < nt; i += 2) {
        step(i, aA, aA);
        step(i + 1, aB, aB);
    }
    if (i < nt) step(i, aA, aA);

    float csum[TN];
    epi_store<TN>(acc, m0 + wid * 32, n0, li, h, p, csum);
    if (p.colpart) {
#pragma unroll
        for (int j = 0; j < TN; ++j) csum[j] += __shfl_xor(csum[j], 32);
        float *red = reinterpret_cast<float *>(sb);         // the last step ended in a barrier
        if (h == 0) {
#pragma unroll
            for (int j = 0; j < TN; ++j) red[wid * BN + j * 32 + li] = csum[j];
        }
        __syncthreads();
        const int rows64 = (p.M + 63) / 64;
        for (int c = threadIdx.x; c < 2 * BN; c += 256) {
            const int half = c / BN, n = n0 + c % BN, slab = 2 * ty + half;
            if (n < p.N && slab < rows64)
                p.colpart[(size_t)slab * p.N + n] = red[(2 * half) * BN + c % BN] + red[(2 * half + 1) * BN + c % BN];
        }
    }
}

// Sums the split slabs in split order (deterministic).  The slab loads are issued 8
// at a time ahead of the adds, so a thread has 8 independent loads in flight instead
// of one dependent load per split; the addition order is unchanged.
__global__ __launch_bounds__(256) void k_splitk_reduce(GemmArgs p, int splits) {
    const size_t total = (size_t)p.M * p.N;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        float v = 0.f;
        const float *w = p.ws + idx;
        int z = 0;
        for (; z + 8 <= splits; z += 8) {
            float t[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) t[q] = w[(size_t)(z + q) * total];
#pragma unroll
            for (int q = 0; q < 8; ++q) v += t[q];
        }
        for (; z < splits; ++z) v += w[(size_t)z * total];
        const int m = (int)(idx / p.N), n = (int)(idx % p.N);
        p.C[(size_t)m * p.ldc + n] = epi_apply(v, m, n, p);
    }
}

// resident 256-thread blocks of a kernel on the whole device (occupancy API x CUs);
// the per-kernel blocks-per-CU answer is cached (it depends on the code object only)
template <class F>
long resident_blocks(bool a, int b, F kernel_of) {
    static std::atomic<int> per_cu[4] = {{-1}, {-1}, {-1}, {-1}};
    const int slot = (a ? 2 : 0) + (b ? 1 : 0);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    int per = per_cu[slot].load(std::memory_order_relaxed);
    if (per < 0) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel_of(a ? 1 : 0, b), 256, 0) != hipSuccess)
            return 0;
        per_cu[slot].store(per, std::memory_order_relaxed);
    }
    return (long)cus * per;
}

template <int BM, int BN, int NBUF = 2, int BK = kBK, bool BF = false>
int launch_tiles(GemmArgs p, bool ak, bool bk, int splits, hipStream_t st) {
    const int kt_total = (p.K + BK - 1) / BK;
    p.k_tiles_per_split = (kt_total + splits - 1) / splits;
    p.splits = splits;
    const long tiles = (long)((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM) * splits;
    // persistent grid: the resident block count (occupancy API x CUs), so tile
    // phases desynchronise and each block overlaps a tile's epilogue with the next
    // tile's first loads
    long g = tiles;
    if (NBUF == 1) {
        const long cap = resident_blocks(ak, bk ? 1 : 0, [&](int a, int b) -> const void * {
            if (a && b) return (const void *)k_gemm<BM, BN, true, true, NBUF, BK, BF>;
            if (a) return (const void *)k_gemm<BM, BN, true, false, NBUF, BK, BF>;
            if (b) return (const void *)k_gemm<BM, BN, false, true, NBUF, BK, BF>;
            return (const void *)k_gemm<BM, BN, false, false, NBUF, BK, BF>;
        });
        if (cap > 0 && cap < g) g = cap;
    }
    if (const char *e = HSG_DEV_ENV("HSG_GEMM_GRID")) g = atol(e) < g ? atol(e) : g;   // dev sweep
    dim3 grid((unsigned)g);
    if (ak && bk) hipLaunchKernelGGL((k_gemm<BM, BN, true, true, NBUF, BK, BF>), grid, dim3(256), 0, st, p);
    else if (ak && !bk) hipLaunchKernelGGL((k_gemm<BM, BN, true, false, NBUF, BK, BF>), grid, dim3(256), 0, st, p);
    else if (!ak && bk) hipLaunchKernelGGL((k_gemm<BM, BN, false, true, NBUF, BK, BF>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((k_gemm<BM, BN, false, false, NBUF, BK, BF>), grid, dim3(256), 0, st, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int BM, int BN, int BK = 32, int PF = 1, int NL = 3, int IGLP = -1, int NT = 256>
int launch3(GemmArgs p, bool ak, bool bk, int splits, hipStream_t st) {
    const int kt_total = (p.K + BK - 1) / BK;
    p.k_tiles_per_split = (kt_total + splits - 1) / splits;
    p.splits = splits;
    long g = (long)((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM) * splits;
    if (const char *e = HSG_DEV_ENV("HSG_GEMM_GRID")) g = atol(e) < g ? atol(e) : g;   // dev sweep
    dim3 grid((unsigned)g);
    if (ak && bk) hipLaunchKernelGGL((k_gemm3<BM, BN, true, true, BK, PF, NL, IGLP, NT>), grid, dim3(NT), 0, st, p);
    else if (ak && !bk) hipLaunchKernelGGL((k_gemm3<BM, BN, true, false, BK, PF, NL, IGLP, NT>), grid, dim3(NT), 0, st, p);
    else if (!ak && bk) hipLaunchKernelGGL((k_gemm3<BM, BN, false, true, BK, PF, NL, IGLP, NT>), grid, dim3(NT), 0, st, p);
    else hipLaunchKernelGGL((k_gemm3<BM, BN, false, false, BK, PF, NL, IGLP, NT>), grid, dim3(NT), 0, st, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int BM, int BN, int S>
int launch4(GemmArgs p, int splits, hipStream_t st) {
    const int kt_total = (p.K + 31) / 32;
    p.k_tiles_per_split = (kt_total + splits - 1) / splits;
    p.splits = splits;
    const long g = (long)((p.N + BN - 1) / BN) * ((p.M + BM - 1) / BM) * splits;
    hipLaunchKernelGGL((k_gemm4<BM, BN, S>), dim3((unsigned)g), dim3(256), 0, st, p);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int BN>
int launch6(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    p.splits = 1;
    p.k_tiles_per_split = Kp / 32;
    const long g = (long)((p.N + BN - 1) / BN) * ((p.M + 127) / 128);
    hipLaunchKernelGGL((k_gemm6<BN>), dim3((unsigned)g), dim3(256), 0, st, p, planes, Np, Kp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

template <int BN, int S, int IGLP = -1, bool ELDS = false, bool HOIST = false>
int launch5(GemmArgs p, const __bf16 *planes, int Np, int Kp, hipStream_t st) {
    p.splits = 1;
    p.k_tiles_per_split = Kp / 32;
    if (ELDS && !epi_rows_ok(p)) return HSG_EINVAL;
    const long g = (long)((p.N + BN - 1) / BN) * ((p.M + 127) / 128);
    hipLaunchKernelGGL((k_gemm5<BN, S, IGLP, ELDS, HOIST>), dim3((unsigned)g), dim3(256), 0, st, p, planes, Np, Kp);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

// k_gemm3 tile plan: 0 = 64x64, 1 = 128x64, 2 = 64x128, 3 = 128x128 (measured on the
// WSWGAT shapes, tools/gemm3_sweep.py: 64x64 for narrow outputs and for N-aligned
// K-contiguous weights, 128x64 otherwise; the wide tiles never won).  GEMMs that emit
// column partials use 64-row tiles in every mode (hsg_gemm_row_tiles).
int plan3(int M, int N, int K, int splits, bool colpart, bool bk) {
    (void)M; (void)K; (void)splits;
    if (colpart) return 0;
    if (N <= 64 || (bk && N % 128 == 0)) return 0;
    return 1;
}

// Plan: 64x64 tiles with a single LDS buffer (up to 8 resident blocks per CU)
// measured fastest on the WSWGAT shapes except long-K tall GEMMs, where 128x64
// single-buffer tiles amortise their prologue better (tools/gemm_tiles.py).
// Split-K when the output has too few 64x64 tiles to fill the GPU (~1280 blocks).
int plan_splits(int M, int N, int K) {
    const int kt = (K + kBK - 1) / kBK;
    const long tiles = (long)((M + 63) / 64) * ((N + 63) / 64);
    int sp = 1;
    if (tiles < 512 && kt >= 8) {
        sp = (int)((1280 + tiles - 1) / tiles);
        if (sp > kt / 4) sp = kt / 4;
        if (sp < 1) sp = 1;
    }
    return sp;
}

int plan_tile(int M, int N, int K, int splits) {
    const int kt = (K + kBK - 1) / kBK;
    const long big = (long)((M + 127) / 128) * ((N + 63) / 64) * splits;
    if (splits == 1 && kt >= 16 && big >= 512) return 4;
    return 5;
}

}  // namespace

extern "C" {

int hsg_gemm_auto_splits(int M, int N, int K) { return plan_splits(M, N, K); }

size_t hsg_gemm_workspace_floats(int M, int N, int K, int splits) {
    if (splits == 0) splits = plan_splits(M, N, K);
    return splits > 1 ? (size_t)splits * M * N : 0;
}

int hsg_gemm_row_tiles(int M, int N, int K, int splits) {
    (void)N; (void)K; (void)splits;
    return (M + 63) / 64;            // GEMMs with column partials run 64-row tiles in every mode
}

}  // extern "C"

namespace {

enum { MODE_F32_MFMA = 0, MODE_BF16 = 1, MODE_F32_SPLIT = 2 };

int gemm_impl(int mode, int M, int N, int K, const float *A, int lda, int a_kcontig, const float *B, int ldb,
              int b_kcontig, float *C, int ldc, const float *bias, const float *aux, int ldaux, int epi,
              int relu, int splits, float *workspace, float *colsum_part, void *stream, bool slabs_only = false) {
    if (M < 0 || N < 0 || K < 0 || !C) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && epi != HSG_EPI_RELU_BWD && epi != HSG_EPI_ADD) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && !aux) return HSG_EINVAL;
    // float4 staging needs 16-byte aligned rows
    if ((lda & 3) || (ldb & 3) || (((uintptr_t)A) & 15) || (((uintptr_t)B) & 15)) return HSG_EINVAL;
    if (M == 0 || N == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    const int kt_total = (K + kBK - 1) / kBK;
    if (splits == 0) splits = plan_splits(M, N, K);
    if (splits < 1) splits = 1;
    if (splits > kt_total) splits = kt_total > 0 ? kt_total : 1;
    if (splits > 1 && !workspace) return HSG_EINVAL;
    if (splits > 1 && colsum_part) return HSG_EINVAL;     // column partials need the unsplit epilogue
    GemmArgs p{M, N, K, A, lda, B, ldb, C, ldc, bias, aux, ldaux, epi, relu,
               (kt_total + splits - 1) / splits, workspace, colsum_part, splits, 1};
    if (const char *x = HSG_DEV_ENV("HSG_GEMM_XCD")) p.xcd = atoi(x);        // dev A/B switch
    const bool ak = a_kcontig != 0, bk = b_kcontig != 0;
    int best = colsum_part ? 5 : plan_tile(M, N, K, splits);     // column partials: 64-row tiles
    if (const char *f = HSG_DEV_ENV("HSG_GEMM_TILE"))      // dev override (tools/gemm_tiles.py)
        if (!colsum_part) best = atoi(f);
    int rc;
    // both operands M/N-contiguous (the weight gradients dW = dY^T X): the split path
    // with transpose-read staging, 64x64 tiles and the iglp_opt(0) interleave
    // (tools/gemm_dw3.py: 108-114 us against 129-142 us for the exact-f32 MFMA on the
    // cfg2 S2W shapes); HSG_GEMM3_DW=0 selects the exact-f32 MFMA (dev A/B)
    bool dw3 = false;
    if (mode == MODE_F32_SPLIT && !ak && !bk && !HSG_DEV_ENV("HSG_GEMM3_TILE")) {
        const char *e = HSG_DEV_ENV("HSG_GEMM3_DW");
        if (e && e[0] == '0') mode = MODE_F32_MFMA;
        else dw3 = true;
    }
    // bf16 mode: the split kernel's plans with ONE limb (the RNE bf16 rounding of each
    // operand, one product) -- the same staging, tiles and transpose reads as the f32
    // mode; HSG_GEMM_BF16_OLD=1 keeps the register-staged k_gemm<..., BF> tiles (dev A/B)
    if (mode == MODE_BF16 && !HSG_DEV_ENV("HSG_GEMM_BF16_OLD")) {
        int t3 = plan3(M, N, K, splits, colsum_part != nullptr, bk);
        if (!ak && !bk) rc = launch3<64, 64, 32, 1, 1, 0>(p, ak, bk, splits, st);
        else if (t3 == 1) rc = launch3<128, 64, 32, 1, 1>(p, ak, bk, splits, st);
        else rc = launch3<64, 64, 32, 1, 1>(p, ak, bk, splits, st);
        if (rc || splits == 1 || slabs_only) return rc;
        const size_t total = (size_t)M * N;
        int blocks = (int)((total + 255) / 256);
        if (blocks > 2048) blocks = 2048;
        hipLaunchKernelGGL(k_splitk_reduce, dim3(blocks), dim3(256), 0, st, p, splits);
        hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : (int)e;
    }
#ifdef HSG_DEV
    int g4 = 0;                                             // dev switch: k_gemm4 plans
    if (const char *f = HSG_DEV_ENV("HSG_GEMM4")) g4 = atoi(f);
    if (mode == MODE_F32_SPLIT && ak && bk && (K & 3) == 0 && g4 > 0) {
        if (colsum_part || g4 == 1) rc = launch4<64, 64, 3>(p, splits, st);
        else if (g4 == 2) rc = launch4<128, 64, 3>(p, splits, st);
        else if (g4 == 3) rc = launch4<64, 64, 4>(p, splits, st);
        else if (g4 == 4) rc = launch4<128, 64, 2>(p, splits, st);
        else if (g4 == 5) rc = launch4<64, 64, 2>(p, splits, st);
        else rc = launch4<128, 128, 2>(p, splits, st);
    } else
#endif
    if (mode == MODE_F32_SPLIT) {
        int t3 = plan3(M, N, K, splits, colsum_part != nullptr, bk);
        if (const char *f = HSG_DEV_ENV("HSG_GEMM3_TILE"))      // dev override
            if (!colsum_part) t3 = atoi(f);
        int var = dw3 ? 5 : 0;                              // dev variants (tools/gemm3_sweep.py)
        if (dw3) t3 = 0;
        if (const char *f = HSG_DEV_ENV("HSG_GEMM3_VAR")) var = atoi(f);
        if (var == 5) {                                     // iglp_opt(0) interleave (the dW default)
            if (t3 == 1) rc = launch3<128, 64, 32, 1, 3, 0>(p, ak, bk, splits, st);
#ifdef HSG_DEV
            else if (t3 == 3) rc = launch3<128, 128, 32, 1, 3, 0>(p, ak, bk, splits, st);
#endif
            else rc = launch3<64, 64, 32, 1, 3, 0>(p, ak, bk, splits, st);
        }
#ifdef HSG_DEV
        else if (var == 1) {                                // 2-deep register prefetch
            if (t3 == 1) rc = launch3<128, 64, 32, 2>(p, ak, bk, splits, st);
            else rc = launch3<64, 64, 32, 2>(p, ak, bk, splits, st);
        } else if (var == 2) {                              // BK = 64
            if (t3 == 1) rc = launch3<128, 64, 64, 1>(p, ak, bk, splits, st);
            else rc = launch3<64, 64, 64, 1>(p, ak, bk, splits, st);
        } else if (var == 3) {                              // one limb (bf16 probe, not f32-accurate)
            if (t3 == 1) rc = launch3<128, 64, 32, 1, 1>(p, ak, bk, splits, st);
            else rc = launch3<64, 64, 32, 1, 1>(p, ak, bk, splits, st);
        } else if (var == 4) {                              // one limb, 2-deep prefetch
            if (t3 == 1) rc = launch3<128, 64, 32, 2, 1>(p, ak, bk, splits, st);
            else rc = launch3<64, 64, 32, 2, 1>(p, ak, bk, splits, st);
        } else if (var == 6) {                              // 8 waves (2 x 4), iglp_opt(0)
            if (t3 == 1) rc = launch3<64, 256, 32, 1, 3, 0, 512>(p, ak, bk, splits, st);
            else if (t3 == 3) rc = launch3<128, 256, 32, 1, 3, 0, 512>(p, ak, bk, splits, st);
            else rc = launch3<64, 128, 32, 1, 3, 0, 512>(p, ak, bk, splits, st);
        } else if (t3 == 3) rc = launch3<128, 128>(p, ak, bk, splits, st);
        else if (t3 == 2) rc = launch3<64, 128>(p, ak, bk, splits, st);
#endif
        else if (t3 == 1) rc = launch3<128, 64>(p, ak, bk, splits, st);
        else rc = launch3<64, 64>(p, ak, bk, splits, st);
    }
#ifdef HSG_DEV
    else if (mode == MODE_BF16) {
        // bf16 operands: the register-staged single-buffer plans (dev A/B)
        if (best == 4) rc = launch_tiles<128, 64, 1, kBK, true>(p, ak, bk, splits, st);
        else rc = launch_tiles<64, 64, 1, kBK, true>(p, ak, bk, splits, st);
    } else if (best == 0) rc = launch_tiles<128, 128>(p, ak, bk, splits, st);
    else if (best == 1) rc = launch_tiles<128, 64>(p, ak, bk, splits, st);
    else if (best == 2) rc = launch_tiles<64, 64>(p, ak, bk, splits, st);
    else if (best == 3) rc = launch_tiles<128, 128, 1>(p, ak, bk, splits, st);
    else if (best == 6) rc = launch_tiles<64, 64, 1, 64>(p, ak, bk, splits, st);
    else if (best == 7) rc = launch_tiles<128, 64, 1, 64>(p, ak, bk, splits, st);
    else if (best == 8) rc = launch_tiles<64, 64, 2, 64>(p, ak, bk, splits, st);
    else if (best == 10) rc = launch_tiles<64, 128, 1>(p, ak, bk, splits, st);
    else if (best == 11) rc = launch_tiles<64, 128, 2>(p, ak, bk, splits, st);
    else if (best == 12) rc = launch_tiles<128, 128, 1, 64>(p, ak, bk, splits, st);
#endif
    // the exact-f32 MFMA (hsg_gemm_f32_mfma): plan_tile's two single-buffer tiles
    else if (best == 4) rc = launch_tiles<128, 64, 1>(p, ak, bk, splits, st);
    else rc = launch_tiles<64, 64, 1>(p, ak, bk, splits, st);
    if (rc || splits == 1 || slabs_only) return rc;
    const size_t total = (size_t)M * N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(k_splitk_reduce, dim3(blocks), dim3(256), 0, st, p, splits);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

int hsg_gemm_f32(int M, int N, int K, const float *A, int lda, int a_kcontig, const float *B, int ldb,
                 int b_kcontig, float *C, int ldc, const float *bias, const float *aux, int ldaux, int epi,
                 int relu, int splits, float *workspace, float *colsum_part, void *stream) {
    int mode = MODE_F32_SPLIT;
    if (const char *e = HSG_DEV_ENV("HSG_GEMM_F32"))          // dev A/B: "mfma" = exact-f32 instruction
        if (e[0] == 'm') mode = MODE_F32_MFMA;
    return gemm_impl(mode, M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, bias, aux, ldaux, epi, relu,
                     splits, workspace, colsum_part, stream);
}

int hsg_gemm_bf16_slabs(int M, int N, int K, const float *A, int lda, int a_kcontig, const float *B, int ldb,
                        int b_kcontig, int splits, float *workspace, void *stream) {
    const int kt_total = (K + kBK - 1) / kBK;
    if (splits < 2 || splits > kt_total || !workspace) return HSG_EINVAL;
    float dummy_c;
    return gemm_impl(MODE_BF16, M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, &dummy_c, N, nullptr, nullptr, 0,
                     HSG_EPI_STORE, 0, splits, workspace, nullptr, stream, true);
}

int hsg_gemm_f32_slabs(int M, int N, int K, const float *A, int lda, int a_kcontig, const float *B, int ldb,
                       int b_kcontig, int splits, float *workspace, void *stream) {
    const int kt_total = (K + kBK - 1) / kBK;
    if (splits < 2 || splits > kt_total || !workspace) return HSG_EINVAL;
    float dummy_c;
    return gemm_impl(MODE_F32_SPLIT, M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, &dummy_c, N, nullptr, nullptr, 0,
                     HSG_EPI_STORE, 0, splits, workspace, nullptr, stream, true);
}

// ---------------------------------------------------------------------------------
// Deferred column sums: many outputs in one launch.  Job q: for c < cols[q] and
// output row b < out_rows[q],
//   out[q][b][c] = (accumulate[q] ? out : 0) + scale[q] * sum_s sum_{r in range_b(s)} part_s[r*pitch + coff + c]
// over its segments s (in order); range_b(s) is the b-th of out_rows[q] equal row
// ranges of segment s (out_rows > 1: a staged partial for tall, narrow slabs).
// 8 row groups per column, group sums added in order: deterministic.  Block = 32
// columns x 8 row groups of one output row; job q owns blocks [start[q], start[q+1]).
// ---------------------------------------------------------------------------------
constexpr int kRedJobs = 24, kRedSegs = 4;
struct RedJobs {
    float *out[kRedJobs];
    const float *seg[kRedJobs][kRedSegs];
    int rows[kRedJobs][kRedSegs];
    int nseg[kRedJobs], cols[kRedJobs], pitch[kRedJobs], coff[kRedJobs], acc[kRedJobs], orows[kRedJobs];
    int vec[kRedJobs];                                    // 4: float4 columns (aligned), else 1
    float scale[kRedJobs];
    int start[kRedJobs + 1];
    int njobs;
};

// Block = 32 lanes along the columns x 8 row groups.  Thread (g, cl) sums rows
// r = g (mod 8) of every segment (four interleaved partial sums, rows added to each
// in row order, up to 16 rows in flight), then the
// 8 groups are added in group order: a fixed order per column, the same for the
// scalar (V = 1: 32 columns per block) and the float4 (V = 4: 128 columns per block,
// 512-B row pieces) form, so both give bitwise equal sums.
extern "C++" {
template <int V, bool PRED = false>
__device__ __forceinline__ void slab_reduce_job(const RedJobs &j, int q, int blk) {
    typedef float vec_t __attribute__((ext_vector_type(V)));
    __shared__ __attribute__((aligned(16))) float red[8][32 * V];
    const int cl = threadIdx.x & 31, g = threadIdx.x >> 5;
    const int nbc = (j.cols[q] + 32 * V - 1) / (32 * V);
    const int ob = blk / nbc;                              // output row (row range of every segment)
    const int c = (blk - ob * nbc) * 32 * V + V * cl;
    const int pitch = j.pitch[q], coff = j.coff[q], orows = j.orows[q];
    vec_t s[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] = vec_t(0.f);
    if (c < j.cols[q]) {
        for (int sg = 0; sg < j.nseg[q]; ++sg) {
            const float *P = j.seg[q][sg] + coff + c;
            const int rows = j.rows[q][sg], per = (rows + orows - 1) / orows;
            const int r1 = min(rows, (ob + 1) * per);
            // up to 16 rows in flight per thread, ALL requested before any is added (PRED,
            // the default: rows past the range are not loaded and add 0; 25.2 -> 23.4 us per
            // cfg2 step, profiles/r04_dev/slab_pred/; dev HSG_SLAB_PRED=0: they load a
            // clamped valid row, as before), so a segment of <= 128
            // rows is one round trip (the ragged 4-row / 1-row tail loops made the 100-row
            // head-projection segments ~4 dependent round trips each); rows go into the
            // four partial sums in row order
            for (int r = ob * per + g; r < r1; r += 128) {
                vec_t v[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    if constexpr (PRED) {       // rows past the range not loaded at all (round 4)
                        v[u] = vec_t(0.f);
                        if (r + 8 * u < r1) v[u] = *reinterpret_cast<const vec_t *>(P + (size_t)(r + 8 * u) * pitch);
                    } else {
                        v[u] = *reinterpret_cast<const vec_t *>(P + (size_t)min(r + 8 * u, r1 - 1) * pitch);
                    }
                }
#pragma unroll
                for (int u = 0; u < 16; ++u) s[u & 3] += r + 8 * u < r1 ? v[u] : vec_t(0.f);
            }
        }
    }
    const vec_t t = (s[0] + s[1]) + (s[2] + s[3]);
    *reinterpret_cast<vec_t *>(&red[g][V * cl]) = t;
    __syncthreads();
    if (g == 0 && c < j.cols[q]) {
        vec_t a = vec_t(0.f);
#pragma unroll
        for (int u = 0; u < 8; ++u) a += *reinterpret_cast<const vec_t *>(&red[u][V * cl]);
        vec_t *o = reinterpret_cast<vec_t *>(j.out[q] + (size_t)ob * j.cols[q] + c);
        *o = j.acc[q] ? *o + j.scale[q] * a : j.scale[q] * a;
    }
}

template <bool PRED = false>
__global__ __launch_bounds__(256) void k_slab_reduce(RedJobs j) {
    int q = 0;
    while (q + 1 < j.njobs && (int)blockIdx.x >= j.start[q + 1]) ++q;
    const int blk = (int)blockIdx.x - j.start[q];
    if (j.vec[q] == 4) slab_reduce_job<4, PRED>(j, q, blk);
    else slab_reduce_job<1, PRED>(j, q, blk);
}
}  // extern "C++"

int hsg_slab_reduce(int njobs, float *const *out, const int *cols, const int *out_rows, const int *pitch,
                    const int *coff, const float *scale, const int *accumulate, const int *nseg,
                    const float *const *seg, const int *seg_rows, void *stream) {
    if (njobs < 1 || njobs > kRedJobs) return HSG_EINVAL;
    RedJobs j{};
    j.njobs = njobs;
    j.start[0] = 0;
    int si = 0;
    for (int q = 0; q < njobs; ++q) {
        if (!out[q] || cols[q] < 0 || nseg[q] < 1 || nseg[q] > kRedSegs || coff[q] < 0 ||
            pitch[q] < coff[q] + cols[q] || out_rows[q] < 1)
            return HSG_EINVAL;
        j.orows[q] = out_rows[q];
        j.out[q] = out[q];
        j.cols[q] = cols[q]; j.pitch[q] = pitch[q]; j.coff[q] = coff[q];
        j.scale[q] = scale[q]; j.acc[q] = accumulate[q] != 0; j.nseg[q] = nseg[q];
        for (int sg = 0; sg < nseg[q]; ++sg, ++si) {
            if (seg_rows[si] < 0 || (seg_rows[si] > 0 && !seg[si])) return HSG_EINVAL;
            j.seg[q][sg] = seg[si];
            j.rows[q][sg] = seg_rows[si];
        }
        // float4 columns when every segment, the output and the column geometry allow
        bool v4 = cols[q] % 4 == 0 && pitch[q] % 4 == 0 && coff[q] % 4 == 0 && ((uintptr_t)out[q] & 15) == 0;
        for (int sg = 0; sg < nseg[q]; ++sg) v4 = v4 && ((uintptr_t)j.seg[q][sg] & 15) == 0;
        if (const char *e = HSG_DEV_ENV("HSG_SLAB_VEC")) v4 = v4 && atoi(e) != 1;                // dev A/B
        j.vec[q] = v4 ? 4 : 1;
        j.start[q + 1] = j.start[q] + (cols[q] + 32 * j.vec[q] - 1) / (32 * j.vec[q]) * out_rows[q];
    }
    if (j.start[njobs] == 0) return 0;
#ifdef HSG_DEV
    if (const char *e = HSG_DEV_ENV("HSG_SLAB_PRED"); e && atoi(e) == 0) {
        hipLaunchKernelGGL(k_slab_reduce<false>, dim3(j.start[njobs]), dim3(256), 0, (hipStream_t)stream, j);
        return hipGetLastError() == hipSuccess ? 0 : HSG_EINVAL;
    }
#endif
    hipLaunchKernelGGL(k_slab_reduce<true>, dim3(j.start[njobs]), dim3(256), 0, (hipStream_t)stream, j);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int hsg_gemm_f32_mfma(int M, int N, int K, const float *A, int lda, int a_kcontig, const float *B, int ldb,
                      int b_kcontig, float *C, int ldc, const float *bias, const float *aux, int ldaux, int epi,
                      int relu, int splits, float *workspace, float *colsum_part, void *stream) {
    return gemm_impl(MODE_F32_MFMA, M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, bias, aux, ldaux, epi,
                     relu, splits, workspace, colsum_part, stream);
}

int hsg_gemm_bf16(int M, int N, int K, const float *A, int lda, int a_kcontig, const float *B, int ldb,
                  int b_kcontig, float *C, int ldc, const float *bias, const float *aux, int ldaux, int epi,
                  int relu, int splits, float *workspace, float *colsum_part, void *stream) {
    return gemm_impl(MODE_BF16, M, N, K, A, lda, a_kcontig, B, ldb, b_kcontig, C, ldc, bias, aux, ldaux, epi, relu,
                     splits, workspace, colsum_part, stream);
}

void hsg_wsplit_dims(int N, int K, int *Np, int *Kp) {
    *Np = (N + 127) / 128 * 128;
    *Kp = (K + 31) / 32 * 32;
}

int hsg_wsplit(int njobs, const float *const *W, const int *N, const int *K, const int *ldw, const int *trans,
               void *const *planes, void *stream) {
    if (njobs < 1 || njobs > 4) return HSG_EINVAL;
    HsgWSplitJobs j{};
    if (hsg_wsplit_setup(j, njobs, W, N, K, ldw, trans, planes)) return HSG_EINVAL;
    hipLaunchKernelGGL(k_wsplit, dim3(j.start[njobs]), dim3(256), 0, (hipStream_t)stream, j);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int hsg_gemm_f32_psw(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                     const float *bias, const float *aux, int ldaux, int epi, int relu, float *colsum_part,
                     void *stream) {
    if (M < 0 || N < 0 || K < 0 || !C || !planes || !A) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && epi != HSG_EPI_RELU_BWD && epi != HSG_EPI_ADD) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && !aux) return HSG_EINVAL;
    if ((lda & 3) || (K & 3) || (((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K) return HSG_EINVAL;
    if (M == 0 || N == 0) return 0;
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, A, lda, nullptr, 0, C, ldc, bias, aux, ldaux, epi, relu, Kp / 32, nullptr, colsum_part, 1, 1};
    if (const char *x = HSG_DEV_ENV("HSG_GEMM_XCD")) p.xcd = atoi(x);
    // k_gemm7 64-wide, LDS-staged float4 epilogue, RNE split with scalar subtractions:
    // cfg2 S2W FFN GEMMs 51.0 / 44.0 / 48.5 / 44.7 us against 55.6 / 48.0 / 53.4 / 47.9
    // for k_gemm5 (plan 7), medians of 5 interleaved rounds in one process
    // (tools/gemm5_sweep.py).  The truncation split (plan 28) is 1-2 us faster but its
    // larger limbs (|a1| < 2^-7 |a|) double the dropped-product bound, and a reference
    // golden's gradient gate-flip row left its tolerance with it.
    const __bf16 *pl = reinterpret_cast<const __bf16 *>(planes);
    hipStream_t st = (hipStream_t)stream;
#ifdef HSG_DEV
    int plan = 27;
    if (const char *f = HSG_DEV_ENV("HSG_GEMM5")) plan = atoi(f);
    if (plan == 2) return launch5<128, 2>(p, pl, Np, Kp, st);
    if (plan == 3) return launch5<64, 3>(p, pl, Np, Kp, st);
    if (plan == 4) return launch5<128, 3>(p, pl, Np, Kp, st);
    if (plan == 5) return launch6<64>(p, pl, Np, Kp, st);
    if (plan == 6) return launch6<128>(p, pl, Np, Kp, st);
    if (plan == 7) return launch5<64, 2, 0>(p, pl, Np, Kp, st);
    if (plan == 8) return launch5<64, 2, 1>(p, pl, Np, Kp, st);
    if (plan == 24) return launch5<64, 2, 0, true>(p, pl, Np, Kp, st);
    if (plan == 25) return launch5<64, 2, 0, true, true>(p, pl, Np, Kp, st);
    if (plan == 26) return launch5<128, 2, 0, true, true>(p, pl, Np, Kp, st);
    // (the plan-specific lines come before the unaligned fallback)
    if (plan == 28 && epi_rows_ok(p)) return launch7<64, 2, 1>(p, pl, Np, Kp, st);   // truncation split
    if (plan == 30 && epi_rows_ok(p)) return N <= 320 ? launch7<80, 2>(p, pl, Np, Kp, st) : launch7<128, 2>(p, pl, Np, Kp, st);
    if (plan == 34 && epi_rows_ok(p)) return launch7<64, 2, 4>(p, pl, Np, Kp, st);   // dev: no C store
    if (plan == 35 && epi_rows_ok(p)) return launch7<64, 2, 5>(p, pl, Np, Kp, st);   // dev: no MFMA
    if (plan == 36 && epi_rows_ok(p)) return launch7<64, 2, 6>(p, pl, Np, Kp, st);   // dev: loads only
    if (plan == 37 && epi_rows_ok(p)) return launch7<64, 2, 7>(p, pl, Np, Kp, st);   // dev: A loads only
    if (plan == 38 && epi_rows_ok(p)) return launch7<64, 2, 8>(p, pl, Np, Kp, st);   // dev: B loads only
    if (plan == 40 && epi_rows_ok(p)) return launch7<64, 2, 0, 2, true>(p, pl, Np, Kp, st);   // hoisted DMA offsets
    if (plan == 41 && epi_rows_ok(p))                       // + 80-wide tiles for N <= 320
        return N <= 320 ? launch7<80, 2, 0, 2, true>(p, pl, Np, Kp, st) : launch7<64, 2, 0, 2, true>(p, pl, Np, Kp, st);
    if (plan == 43 && epi_rows_ok(p))                       // + hoisted DMA offsets
        return N <= 320 && (N + 111) / 112 * 112 <= Np ? launch7<112, 2, 0, 2, true>(p, pl, Np, Kp, st)
                                                       : launch7<64, 2, 0, 2, true>(p, pl, Np, Kp, st);
    if (plan == 44 && epi_rows_ok(p)) return launch7<64, 2>(p, pl, Np, Kp, st);     // round-4 default: 64-wide
    if (plan != 27) return launch5<64, 2>(p, pl, Np, Kp, st);
    if (gemm11_on()) {
        // one round of big tiles (k_gemm11, dev opt-in: measured slower)
        // where the shape allows; its column partials are per WM-row band
        // (hsg_gemm_psw_row_tiles), so with colsum_part it never falls back
        const int rc = try11<0>(p, pl, Np, Kp, st);
        if (rc != HSG_EINVAL || (colsum_part && atoi(HSG_DEV_ENV("HSG_GEMM11")) == 1 && plan11(M, N, device_cus())))
            return rc;
    }
#endif
    // dev opt-in: the resident-B kernel for N > 320 with K <= 320 (measured slower).  Its
    // column partials are per 32-row band (hsg_gemm_psw_row_tiles), so a call it refuses
    // with colsum_part is refused, not handed to k_gemm7's 64-row partials
#ifdef HSG_DEV
    if (plan12(M, N, K)) {
        const int rc = launch12(p, pl, Np, Kp, st);
        if (rc != HSG_EINVAL || colsum_part) return rc;
    }
#endif
    // N <= 320 (ffn2 y = H W2^T at N = 300): 112-wide tiles, 3 per row band instead of 5
    // of 64 -- 450 tiles at cfg2, ONE round of the 512 resident blocks instead of 1.46 --
    // and each wave's A split feeds 7 instead of 4 column subtiles: 44.1 -> 39.1 us back
    // to back (tools/gemm5_sweep.py, plan 42 against 27; same products, bitwise)
    // (where the planes' padded rows cover the 112-wide tiles; else 64)
    if (epi_rows_ok(p))
        return N <= 320 && (N + 111) / 112 * 112 <= Np && wide112_pays(M, N) ? launch7<112, 2>(p, pl, Np, Kp, st)
                                                                             : launch7<64, 2>(p, pl, Np, Kp, st);
    return launch5<64, 2, 0>(p, pl, Np, Kp, st);             // unaligned / ragged quads
}

// bf16-mode k_gemm7 (one product per tile): dev plans for the tile / depth / occupancy sweep
// the bf16 mode with bf16 activations (io: HSG_IO_* bits): the FFN's four GEMMs take
// io 2 (x W1^T -> H), 1 (H W2^T), 7 (dY W2 with the H mask -> dH) and 1 (dH W1, ELU
// gate); tiles as launch7b's default
extern "C++" {
template <int IO>
static int launch7io_narrow(GemmArgs p, const __bf16 *pl, int Np, int Kp, hipStream_t st) {
#ifdef HSG_DEV
    if (const char *e = HSG_DEV_ENV("HSG_GEMM7IO")) {         // dev sweep of the N <= 320 tile
        const int v = atoi(e);
        if (v == 1) return launch7<128, 2, 2, 2, false, IO>(p, pl, Np, Kp, st);
        if (v == 3) return launch7<64, 2, 2, 3, false, IO>(p, pl, Np, Kp, st);
        if (v == 4) return launch7<64, 2, 2, 2, false, IO>(p, pl, Np, Kp, st);
    }
#endif
    // cfg5 in-step (profiles/r05/): 3 stages at 3 blocks per CU 42.7 us against 45.0
    // (2 stages, 2 blocks), 44.9 (2 stages, 3 blocks) and 58.2 (128-wide tiles)
    return launch7<64, 3, 2, 3, false, IO>(p, pl, Np, Kp, st);
}
}  // extern "C++"

static int launch7io(GemmArgs p, const __bf16 *pl, int Np, int Kp, int io, hipStream_t st) {
    const bool wide = p.N > 320;
    switch (io) {
    case 0: return wide ? launch7<128, 2, 2>(p, pl, Np, Kp, st) : launch7<64, 2, 2>(p, pl, Np, Kp, st);
    case 1: return wide ? launch7<128, 2, 2, 2, false, 1>(p, pl, Np, Kp, st) : launch7io_narrow<1>(p, pl, Np, Kp, st);
    case 2: return wide ? launch7<128, 2, 2, 2, false, 2>(p, pl, Np, Kp, st) : launch7io_narrow<2>(p, pl, Np, Kp, st);
    case 7: return wide ? launch7<128, 2, 2, 2, false, 7>(p, pl, Np, Kp, st) : launch7io_narrow<7>(p, pl, Np, Kp, st);
    case 3: return wide ? launch7<128, 2, 2, 2, false, 3>(p, pl, Np, Kp, st) : launch7io_narrow<3>(p, pl, Np, Kp, st);
    case 9: return wide ? launch7<128, 2, 2, 2, false, 9>(p, pl, Np, Kp, st) : launch7io_narrow<9>(p, pl, Np, Kp, st);
    case 25: return wide ? launch7<128, 2, 2, 2, false, 25>(p, pl, Np, Kp, st) : launch7io_narrow<25>(p, pl, Np, Kp, st);
    default: return HSG_EINVAL;
    }
}

static int launch7b(GemmArgs p, const __bf16 *pl, int Np, int Kp, hipStream_t st) {
    int plan = 0;
#ifdef HSG_DEV
    if (gemm11_on()) {
        const int rc = try11<2>(p, pl, Np, Kp, st);        // one round of big tiles where it applies
        if (rc != HSG_EINVAL || (p.colpart && atoi(HSG_DEV_ENV("HSG_GEMM11")) == 1 && plan11(p.M, p.N, device_cus())))
            return rc;
    }
    if (const char *f = HSG_DEV_ENV("HSG_GEMM7B")) plan = atoi(f);
#endif
    switch (plan) {
#ifdef HSG_DEV
    case 1: return launch7<64, 3, 2>(p, pl, Np, Kp, st);
    case 2: return launch7<64, 4, 2>(p, pl, Np, Kp, st);
    case 3: return launch7<128, 2, 2>(p, pl, Np, Kp, st);
    case 4: return launch7<128, 3, 2>(p, pl, Np, Kp, st);
    case 5: return (p.N + 255) / 256 * 256 <= Np ? launch7<256, 2, 2>(p, pl, Np, Kp, st)
                                                 : launch7<128, 2, 2>(p, pl, Np, Kp, st);
    case 6: return launch7<64, 2, 2, 4>(p, pl, Np, Kp, st);
    case 7: return launch7<64, 3, 2, 3>(p, pl, Np, Kp, st);
    case 8: return launch7<128, 2, 2, 3>(p, pl, Np, Kp, st);
    case 9: return launch7<64, 2, 2>(p, pl, Np, Kp, st);
#endif
    default:
        // tools/gemm5_sweep.py BF16=1 at cfg5's 28800 word rows (3 interleaved rounds):
        // N = 512 runs 31.1 us on 128-wide tiles against 37.8 on 64 (half the A re-reads);
        // N = 300 is 29.1 us on 64 and 31.0 on 128 (384-wide padding)
        return p.N > 320 ? launch7<128, 2, 2>(p, pl, Np, Kp, st) : launch7<64, 2, 2>(p, pl, Np, Kp, st);
    }
}

int hsg_gemm_bf16_psw(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                      const float *bias, const float *aux, int ldaux, int epi, int relu, float *colsum_part,
                      void *stream) {
    if (M < 0 || N < 0 || K < 0 || !C || !planes || !A) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && epi != HSG_EPI_RELU_BWD && epi != HSG_EPI_ADD) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && !aux) return HSG_EINVAL;
    if ((lda & 3) || (K & 3) || (((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K) return HSG_EINVAL;
    if (M == 0 || N == 0) return 0;
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, A, lda, nullptr, 0, C, ldc, bias, aux, ldaux, epi, relu, Kp / 32, nullptr, colsum_part, 1, 1};
    if (!epi_rows_ok(p)) return HSG_EINVAL;      // the caller keeps hsg_gemm_bf16 on the unsplit weight
    return launch7b(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, (hipStream_t)stream);
}

int hsg_gemm_psw_ln(int M, int N, int K, const float *A, int lda, const void *planes, const float *bias, float *y,
                    const float *x, const float *gamma, const float *beta, float eps, float p_drop, const int64_t *seed,
                    uint32_t offset, float *out, float *mean, float *rstd, int bf16, void *stream) {
    if (M < 0 || N < 4 || K < 0 || !A || !planes || !bias || !y || !x || !gamma || !beta || !out || !mean || !rstd)
        return HSG_EINVAL;
    if ((lda & 3) || (K & 3) || (((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K) return HSG_EINVAL;
    if (p_drop < 0.f || p_drop >= 1.f || (p_drop > 0.f && (!seed || (long)M * N >= (1L << 32)))) return HSG_EINVAL;
    const auto al = [](const void *q) { return (((uintptr_t)q) & 15) == 0; };
    if (!al(bias) || !al(gamma) || !al(beta) || !al(out) || !al(x) || !al(y)) return HSG_EINVAL;
    if (M == 0) return 0;
#ifndef HSG_DEV
    // measured break-even against hsg_gemm_f32_psw + hsg_ln_fwd: the
    // product library declines, the caller runs the two launches
    (void)eps; (void)offset;
    return HSG_EINVAL;
#else
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, A, lda, nullptr, 0, y, N, bias, x, N, HSG_EPI_STORE, 0, Kp / 32, nullptr, nullptr, 1, 1};
    p.gamma = gamma; p.beta = beta; p.lnout = out; p.mean = mean; p.rstd = rstd;
    p.seed = seed; p.eps = eps; p.p_drop = p_drop; p.offset = offset;
    const __bf16 *pl = reinterpret_cast<const __bf16 *>(planes);
    return bf16 ? try11ln<2>(p, pl, Np, Kp, (hipStream_t)stream) : try11ln<0>(p, pl, Np, Kp, (hipStream_t)stream);
#endif
}

// bf16-mode GEMM on bf16 activations (round 5): A / C / aux given as bf16 rows per
// io (HSG_IO_A_BF16 | HSG_IO_C_BF16 | HSG_IO_AUX_BF16; element strides lda / ldc /
// ldaux).  bf16 A: lda % 8 == 0, 16-byte aligned, columns K .. ceil8(K) - 1 zero.
int hsg_gemm_bf16_psw_io(int M, int N, int K, const void *A, int lda, const void *planes, void *C, int ldc,
                         const float *bias, const void *aux, int ldaux, int epi, int relu, float *colsum_part,
                         int io, void *stream) {
    if (M < 0 || N < 0 || K < 0 || !C || !planes || !A) return HSG_EINVAL;
    if (io != 0 && io != 1 && io != 2 && io != 3 && io != 7) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && epi != HSG_EPI_RELU_BWD && epi != HSG_EPI_ADD) return HSG_EINVAL;
    if (epi != HSG_EPI_STORE && !aux) return HSG_EINVAL;
    if ((io & 4) && epi != HSG_EPI_RELU_BWD) return HSG_EINVAL;           // a bf16 aux is a relu' mask
    if ((io & 2) && epi == HSG_EPI_ADD) return HSG_EINVAL;                 // accumulate: fp32 C
    const bool abf = io & 1;
    if ((((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K || (abf ? (lda & 7) : ((lda & 3) || (K & 3))))
        return HSG_EINVAL;
    if (M == 0 || N == 0) return 0;
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, reinterpret_cast<const float *>(A), lda, nullptr, 0, reinterpret_cast<float *>(C), ldc, bias,
               reinterpret_cast<const float *>(aux), ldaux, epi, relu, Kp / 32, nullptr, colsum_part, 1, 1};
    if (!epi_rows_ok(p)) return HSG_EINVAL;
    return launch7io(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, io, (hipStream_t)stream);
}

// the dx GEMM with the ELU gate (fp32 mode): 112-wide tiles for N <= 320, as the plain
// GEMM, where the weight planes cover them and every 112-column rho group meets at most
// three heads (the edge backward reads three slots per group); else 64.  112 only where
// its group count differs from 64's: hsg_gat_bwd_src_g_io tells the two layouts apart by
// the count alone, and for N in 113..128 both would give 2 groups
static int elug_gw(int M, int N, int K, int head_dim) {
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    if (N > 320 || (N + 111) / 112 * 112 > Np || !wide112_pays(M, N)) return 64;
    if ((N + 111) / 112 == (N + 63) / 64) return 64;
#ifdef HSG_DEV
    if (const char *e = HSG_DEV_ENV("HSG_ELUG_GW")) if (atoi(e) == 64) return 64;     // dev A/B
#endif
    if (head_dim > 0) {
        if (head_dim > 112) return 64;
        for (int g0 = 0; g0 < N; g0 += 112)
            if ((min(g0 + 112, N) - 1) / head_dim - g0 / head_dim > 2) return 64;
    }
    return 112;
}

int hsg_gemm_psw_row_tiles(int M, int N, int K, int bf16) {
    (void)K; (void)bf16;
    if (M < 0 || N < 1) return 0;
#ifdef HSG_DEV
    const int pl = gemm11_on() && atoi(HSG_DEV_ENV("HSG_GEMM11")) == 1 ? plan11(M, N, device_cus()) : 0;
    if (pl == 1) return (M + 159) / 160 * 2;               // k_gemm11<160, 256, 2, 4>: 80-row bands
    if (pl == 2) return (M + 191) / 192 * 4;               // k_gemm11<192, 160, 4, 2>: 48-row bands
    if (!bf16 && plan12(M, N, K)) return (M + 31) / 32;    // k_gemm12: 32-row bands
#endif
    return (M + 63) / 64;
}

int hsg_gemm_psw_elug_rho(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                          const float *aux, const float *x, const float *origin, float *G, int ld, float *rho,
                          int head_dim, int bf16, void *stream) {
    if (M < 0 || N < 0 || K < 0 || !C || !planes || !A || !aux || !x || !origin || !G) return HSG_EINVAL;
    if ((lda & 3) || (K & 3) || (((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K || ld < N)
        return HSG_EINVAL;
    if (rho && (head_dim < 32 || N % head_dim)) return HSG_EINVAL;   // <= 3 heads per 64-column group
    if (M == 0 || N == 0) return 0;
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, A, lda, nullptr, 0, C, ldc, nullptr, aux, ld, HSG_EPI_ADD_ELUG, 0, Kp / 32, nullptr, nullptr,
               1, 1, x, origin, G};
    p.rho = rho;
    p.rho_d = head_dim;
    if (!epi_rows_ok(p)) return HSG_EINVAL;
    // rho groups: 64 columns, or the 112-wide tile (elug_gw); the dev library's k_gemm11
    // declines a rho GEMM (try11), so it falls through to k_gemm7
    if (bf16) return launch7b(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, (hipStream_t)stream);
    if (elug_gw(M, N, K, head_dim) == 112)
        return launch7<112, 2>(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, (hipStream_t)stream);
    return launch7<64, 2>(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, (hipStream_t)stream);
}

int hsg_gemm_psw_elug_rho_gw(int M, int N, int K, int head_dim, int bf16) {
    return bf16 ? 64 : elug_gw(M, N, K, head_dim);
}

// hsg_gemm_psw_elug_rho in the bf16 mode on a bf16 A (the FFN's bf16 dH rows; lda %
// 8 == 0, 16-byte aligned, columns K .. ceil8(K) - 1 zero)
int hsg_gemm_bf16_psw_elug_rho_a16(int M, int N, int K, const void *A, int lda, const void *planes, float *C,
                                   int ldc, const float *aux, const float *x, const float *origin, void *G, int ld,
                                   float *rho, int head_dim, int g_bf16, void *stream) {
    if (M < 0 || N < 0 || K < 0 || !C || !planes || !A || !aux || !x || !origin || !G) return HSG_EINVAL;
    if ((lda & 7) || (((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K || ld < N) return HSG_EINVAL;
    if (rho && (head_dim < 32 || N % head_dim)) return HSG_EINVAL;
    if (M == 0 || N == 0) return 0;
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, reinterpret_cast<const float *>(A), lda, nullptr, 0, C, ldc, nullptr, aux, ld,
               HSG_EPI_ADD_ELUG, 0, Kp / 32, nullptr, nullptr, 1, 1, x, origin, reinterpret_cast<float *>(G)};
    p.rho = rho;
    p.rho_d = head_dim;
    if (!epi_rows_ok(p)) return HSG_EINVAL;
    return launch7io(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, g_bf16 ? 9 : 1, (hipStream_t)stream);
}

// ... with x given as bf16 rows of pitch ldx (x_bf16: the bf16 mode's bf16 edge-layer
// output, hsg_gat_fwd_ws16; ldx % 8 == 0, 16-byte aligned), round 6.  x_bf16 == 0 is
// hsg_gemm_bf16_psw_elug_rho_a16.
int hsg_gemm_bf16_psw_elug_rho_x16(int M, int N, int K, const void *A, int lda, const void *planes, float *C,
                                   int ldc, const float *aux, const void *x, int ldx, int x_bf16, const float *origin,
                                   void *G, int ld, float *rho, int head_dim, int g_bf16, void *stream) {
    if (!x_bf16)
        return hsg_gemm_bf16_psw_elug_rho_a16(M, N, K, A, lda, planes, C, ldc, aux, reinterpret_cast<const float *>(x),
                                              origin, G, ld, rho, head_dim, g_bf16, stream);
    if (M < 0 || N < 0 || K < 0 || !C || !planes || !A || !aux || !x || !origin || !G || !g_bf16) return HSG_EINVAL;
    if ((lda & 7) || (((uintptr_t)A) & 15) || (((uintptr_t)planes) & 15) || lda < K || ld < N) return HSG_EINVAL;
    if ((ldx & 7) || ldx < N) return HSG_EINVAL;
    if (rho && (head_dim < 32 || N % head_dim)) return HSG_EINVAL;
    if (M == 0 || N == 0) return 0;
    int Np, Kp;
    hsg_wsplit_dims(N, K, &Np, &Kp);
    GemmArgs p{M, N, K, reinterpret_cast<const float *>(A), lda, nullptr, 0, C, ldc, nullptr, aux, ld,
               HSG_EPI_ADD_ELUG, 0, Kp / 32, nullptr, nullptr, 1, 1, reinterpret_cast<const float *>(x), origin,
               reinterpret_cast<float *>(G)};
    p.rho = rho;
    p.rho_d = head_dim;
    p.ldx = ldx;
    if (!epi_rows_ok(p)) return HSG_EINVAL;
    return launch7io(p, reinterpret_cast<const __bf16 *>(planes), Np, Kp, 25, (hipStream_t)stream);
}

int hsg_gemm_f32_psw_elug(int M, int N, int K, const float *A, int lda, const void *planes, float *C, int ldc,
                          const float *aux, const float *x, const float *origin, float *G, int ld, int bf16,
                          void *stream) {
    return hsg_gemm_psw_elug_rho(M, N, K, A, lda, planes, C, ldc, aux, x, origin, G, ld, nullptr, 0, bf16, stream);
}

#ifdef HSG_GEMM_CENSUS
int hsg_gemm_census_read(unsigned long long *host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_census), sizeof(unsigned long long) * 4 * n);
}
#endif

}  // extern "C"
