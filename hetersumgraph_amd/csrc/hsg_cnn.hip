// hsg_cnn.hip -- the sentence CNN encoder (module/Encoder.py:56-76) for gfx950.
//
// Reference: x = embed(ids) + pos_embed(pos) over the whole padded sentence
// (L = sent_max_len rows), six Conv2d(1, 50, (h, D)) for h = 2..7, ReLU, max-pool
// over time, concat -> [n, 300].  As written that is sum_h 2*(L-h+1)*50*h*D flops
// per sentence (~81 MFLOP at L=100, D=300), most of it on padding.
//
// Here the convolution is restated as ONE GEMM plus a shifted sum:
//   Y = X Wall^T,  Wall [(tap(h,i))*50 + c][d] = W_h[c][0][i][d]  (27 taps x 50)
//   conv_h[t][c] = b_h[c] + sum_{i<h} Y[t+i][tap(h,i)*50 + c]
// and X holds only the rows the windows can see: the len_s non-pad rows of each
// sentence plus ONE pad row (embed[0] + pos_embed[0], the value of every padded
// position since the reference's padding is trailing), so the GEMM runs over
// sum_s (len_s + 1) rows instead of n*L.  Every window that lies entirely in the
// padding has the same value (its rows are all the pad row), so the max-pool
// evaluates it once, at t = len_s, which is also where the reference's first-max
// scan would meet it.  The GEMM is hsg_gemm_f32 (MFMA f32); this file holds the
// row gather, the shifted-sum/ReLU/max-pool epilogue with argmax, and the
// backward's scatter of dY (the weight gradient is then dY^T X, another GEMM).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hsg.h"

namespace {

constexpr int kGroups = 6;      // kernel heights 2..7
constexpr int kCh = 50;         // channels per height
constexpr int kTaps = 27;       // 2 + 3 + ... + 7

__host__ __device__ constexpr int tap_base(int g) { return g * (g + 3) / 2; }   // sum_{j<g} (j+2)

// X[rowoff[s] + t] = embed[ids[s][t]] + pos[t+1] for t < len_s; X[rowoff[s] + len_s] =
// embed[0] + pos[0] (the pad row).  One wave per row.
__global__ __launch_bounds__(256) void k_cnn_gather(int n, int L, int D, const int64_t *__restrict__ ids,
                                                    const float *__restrict__ E, const float *__restrict__ P,
                                                    const int32_t *__restrict__ rowoff, float *__restrict__ X) {
    const int lane = threadIdx.x & 63;
    const long total = rowoff[n];
    for (long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6); r < total; r += (long)gridDim.x * 4) {
        // sentence of row r: binary search over rowoff
        int lo = 0, hi = n - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (rowoff[mid] <= r) lo = mid;
            else hi = mid - 1;
        }
        const int s = lo;
        const int t = (int)(r - rowoff[s]);
        const int len = rowoff[s + 1] - rowoff[s] - 1;
        const int64_t w = t < len ? ids[(long)s * L + t] : 0;
        const int p = t < len ? t + 1 : 0;
        const float *er = E + w * D, *pr = P + (long)p * D;
        float *xr = X + r * D;
        for (int d = lane; d < D; d += 64) xr[d] = er[d] + pr[d];
    }
}

struct Bias {
    const float *b[kGroups];
};

// feat[s][g*50 + c] = relu(max_t conv_g[t][c]), arg[s][g*50+c] = first t of the max.
// One thread per (s, g, c); consecutive threads = consecutive c (coalesced Y reads).
__global__ __launch_bounds__(256) void k_cnn_pool(int n, int L, const int32_t *__restrict__ rowoff,
                                                  const float *__restrict__ Y, int ldy, Bias bias,
                                                  float *__restrict__ feat, int32_t *__restrict__ arg) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)n * kGroups * kCh) return;
    const int s = (int)(idx / (kGroups * kCh));
    const int gc = (int)(idx - (long)s * kGroups * kCh);
    const int g = gc / kCh, c = gc - g * kCh, h = g + 2;
    const int T = L - h + 1;                       // windows of the padded sentence
    const long r0 = rowoff[s];
    const int len = rowoff[s + 1] - rowoff[s] - 1;
    const float *Yp = Y + (r0 + len) * ldy;        // this sentence's pad row
    const float b = bias.b[g][c];
    const int col0 = tap_base(g) * kCh + c;
    float best = -INFINITY;
    int bt = 0;
    const int tv = len < T ? len : T;
    for (int t = 0; t < tv; ++t) {
        float v = b;
        for (int i = 0; i < h; ++i) {
            const int r = t + i;
            const float *yr = r < len ? Y + (r0 + r) * ldy : Yp;
            v += yr[col0 + i * kCh];
        }
        if (v > best) { best = v; bt = t; }
    }
    if (len < T) {                                 // the all-padding windows (identical): t = len
        float v = b;
        for (int i = 0; i < h; ++i) v += Yp[col0 + i * kCh];
        if (v > best) { best = v; bt = len; }
    }
    feat[idx] = best > 0.f ? best : 0.f;
    arg[idx] = bt;
}

// dY (zero-filled by the caller): for each (s, g, c) with feat > 0, route dfeat to
// the h rows of its max window (rows past len_s are the sentence's pad row).  All
// (s, g, c, i) targets are distinct, so plain stores: deterministic.
__global__ __launch_bounds__(256) void k_cnn_pool_bwd(int n, const int32_t *__restrict__ rowoff,
                                                      const float *__restrict__ feat, const int32_t *__restrict__ arg,
                                                      const float *__restrict__ dfeat, float *__restrict__ dY,
                                                      int lddy) {
    const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long)n * kGroups * kCh) return;
    if (!(feat[idx] > 0.f)) return;                // ReLU'
    const int s = (int)(idx / (kGroups * kCh));
    const int gc = (int)(idx - (long)s * kGroups * kCh);
    const int g = gc / kCh, c = gc - g * kCh, h = g + 2;
    const long r0 = rowoff[s];
    const int len = rowoff[s + 1] - rowoff[s] - 1;
    const float gv = dfeat[idx];
    const int t = arg[idx];
    const int col0 = tap_base(g) * kCh + c;
    for (int i = 0; i < h; ++i) {
        const int r = t + i;
        const long row = r < len ? r0 + r : r0 + len;
        dY[row * lddy + col0 + i * kCh] += gv;     // pad-row targets of one (s,g,c) differ in i -> distinct
    }
}

int status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

int hsg_cnn_taps(void) { return kTaps * kCh; }

int hsg_cnn_gather(int n, int L, int D, const int64_t *ids, const float *embed, const float *pos,
                   const int32_t *rowoff, long rows, float *X, void *stream) {
    if (n < 0 || L < 1 || D < 1 || rows < n || !rowoff || !X || (n && (!ids || !embed || !pos))) return HSG_EINVAL;
    if (rows == 0) return 0;
    long blocks = (rows + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(k_cnn_gather, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, n, L, D, ids, embed,
                       pos, rowoff, X);
    return status();
}

int hsg_cnn_pool(int n, int L, const int32_t *rowoff, const float *Y, int ldy, const float *const *bias,
                 float *feat, int32_t *arg, void *stream) {
    if (n < 0 || L < 7 || !rowoff || !bias || ldy < kTaps * kCh) return HSG_EINVAL;
    if (n == 0) return 0;
    Bias b;
    for (int g = 0; g < kGroups; ++g) {
        if (!bias[g]) return HSG_EINVAL;
        b.b[g] = bias[g];
    }
    const long total = (long)n * kGroups * kCh;
    hipLaunchKernelGGL(k_cnn_pool, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n, L,
                       rowoff, Y, ldy, b, feat, arg);
    return status();
}

int hsg_cnn_pool_bwd(int n, const int32_t *rowoff, const float *feat, const int32_t *arg, const float *dfeat,
                     float *dY, int lddy, void *stream) {
    if (n < 0 || !rowoff || lddy < kTaps * kCh || (n && (!feat || !arg || !dfeat || !dY))) return HSG_EINVAL;
    if (n == 0) return 0;
    const long total = (long)n * kGroups * kCh;
    hipLaunchKernelGGL(k_cnn_pool_bwd, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                       rowoff, feat, arg, dfeat, dY, lddy);
    return status();
}

}  // extern "C"
