// hsg_relbuild.hip -- device construction of a typed relation (struct hsg_rel).
//
// Replaces, once per batch instead of per head and layer call, what DGL 0.4 does
// inside every WSGATLayer/SWGATLayer call:
//   filter_nodes(unit == a) / filter_nodes(unit == b)   GATLayer.py:105-106, 143-144
//   filter_edges(src.unit == a & dst.unit == b)         GATLayer.py:107, 145
//   the in-edge set of g.pull(dst, ...)                 GATLayer.py:113, 149
// and the tf-idf box lookup of HSumGraph.set_wnfeature (HiGraph.py:146-151).
//
// Output (all int32 unless noted, sized by the caller with the upper bounds n, E):
//   CSR by destination rank, edges inside a segment in edge-id order (DGL's mailbox
//   order), the source rank and tau row (tf-idf box, 10 = never written) per CSR
//   edge, the phantom count per destination (untyped in-edges), the CSC mirror by
//   source rank (stable: CSR position order) with its permutation, and the node
//   lists.  Everything is deterministic: counts come from atomics (order free),
//   orders from rocprim's stable LSD radix sort.
//
// Steps (9 launches + 2 radix sorts + 3 scans, all on `stream`):
//   1 k_node_flags   flag source / destination nodes                    [n]
//   2 scan           node ranks within the source / destination sets
//   3 k_edge_keys    per edge: in-degree, typed flag, key = dst rank     [E]
//   4 sort           (key, edge id) stable by key -> CSR order
//   5 scan           indptr
//   6 k_csr_fill     src rank, tau row, eid, CSC key per CSR edge
//   7 sort           (src rank, CSR position) stable -> CSC order
//   8 scan           cindptr; k_csc_fill: cdst
//   9 k_node_fill    src/dst node lists, phantom, counts
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstdio>
#include <cstdlib>

#include "hsg.h"

namespace {

constexpr int kThreads = 256;
constexpr int kZeroRow = 10;   // tau row of typed edges that never got a tfidfembed
constexpr int kBoxes = 10;     // nn.Embedding(10, F), HiGraph.py:52

inline int blocks_for(long long n) { return (int)((n + kThreads - 1) / kThreads); }

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

int key_bits(int n) {  // keys are in [0, n]; n is the "not typed" sentinel
    int b = 1;
    while ((1ll << b) <= n) ++b;
    return b;
}

// Workspace carve-up; identical in the size query and the build.
struct Work {
    int32_t *fs, *fd;          // [n+1] source / destination node flags
    int32_t *rs, *rd;          // [n+1] exclusive scans of the flags (ranks)
    int32_t *indeg;            // [n]   in-degree over all edges
    int32_t *tcnt;             // [n+1] typed in-degree per destination rank
    int32_t *scnt;             // [n+1] typed out-degree per source rank
    int32_t *key, *val;        // [E]   sort input
    int32_t *key2, *val2;      // [E]   sort output (CSR order: dst rank, edge id)
    int32_t *ckey, *cval;      // [E]   CSC sort input
    int32_t *ckey2;            // [E]   CSC sort keys out
    void *tmp;
    size_t tmp_bytes;
};

size_t carve(Work *w, char *base, int n, int E, size_t tmp_bytes) {
    size_t off = 0;
    auto take = [&](int32_t **p, size_t count) {
        if (w) *p = reinterpret_cast<int32_t *>(base + off);
        off += align_up(count * sizeof(int32_t));
    };
    Work dummy;
    Work *t = w ? w : &dummy;
    take(&t->fs, n + 1); take(&t->fd, n + 1);
    take(&t->rs, n + 1); take(&t->rd, n + 1);
    take(&t->indeg, n);  take(&t->tcnt, n + 1); take(&t->scnt, n + 1);
    take(&t->key, E); take(&t->val, E); take(&t->key2, E); take(&t->val2, E);
    take(&t->ckey, E); take(&t->cval, E); take(&t->ckey2, E);
    if (w) { w->tmp = base + off; w->tmp_bytes = tmp_bytes; }
    return off + align_up(tmp_bytes);
}

hipError_t temp_bytes(int n, int E, size_t *out, hipStream_t s) {
    size_t a = 0, b = 0;
    hipError_t e = rocprim::radix_sort_pairs(nullptr, a, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (int32_t *)nullptr, (int32_t *)nullptr,
                                             (unsigned)(E > 0 ? E : 1), 0, key_bits(n), s);
    if (e != hipSuccess) return e;
    e = rocprim::exclusive_scan(nullptr, b, (int32_t *)nullptr, (int32_t *)nullptr, 0,
                                (size_t)n + 1, rocprim::plus<int32_t>(), s);
    if (e != hipSuccess) return e;
    *out = a > b ? a : b;
    return hipSuccess;
}

__global__ void k_node_flags(int n, const float *__restrict__ unit, float su, float du,
                             int32_t *__restrict__ fs, int32_t *__restrict__ fd) {
    int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) {
        float u = unit[i];
        fs[i] = u == su;
        fd[i] = u == du;
    } else if (i == n) {  // sentinel slot: the scan writes the set size here
        fs[i] = 0;
        fd[i] = 0;
    }
}

__global__ void k_edge_keys(int n, int E, const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                            const int32_t *__restrict__ fs, const int32_t *__restrict__ fd,
                            const int32_t *__restrict__ rd, int32_t *__restrict__ indeg,
                            int32_t *__restrict__ tcnt, int32_t *__restrict__ key,
                            int32_t *__restrict__ val, int32_t *__restrict__ counts) {
    int e = blockIdx.x * kThreads + threadIdx.x;
    if (e >= E) return;
    int64_t u = src[e], v = dst[e];
    int k = n;
    if (u < 0 || u >= n || v < 0 || v >= n) {
        atomicAdd(&counts[4], 1);   // bad node id: the host raises
    } else {
        atomicAdd(&indeg[v], 1);
        if (fs[u] && fd[v]) {
            k = rd[v];
            atomicAdd(&tcnt[k], 1);
        }
    }
    key[e] = k;
    val[e] = e;
}

// i: CSR position (or an untyped edge past n_typed, key == n)
__global__ void k_csr_fill(int n, int E, const int32_t *__restrict__ key2, const int32_t *__restrict__ val2,
                           const int64_t *__restrict__ src, const int32_t *__restrict__ rs,
                           const int64_t *__restrict__ tffrac, const float *__restrict__ edtype,
                           int32_t *__restrict__ esrc, uint8_t *__restrict__ tf, int64_t *__restrict__ eid,
                           int32_t *__restrict__ scnt, int32_t *__restrict__ ckey,
                           int32_t *__restrict__ cval, int32_t *__restrict__ counts) {
    int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= E) return;
    int k = key2[i];
    cval[i] = i;
    if (k >= n) {
        ckey[i] = n;
        return;
    }
    int e = val2[i];
    int r = rs[src[e]];
    esrc[i] = r;
    eid[i] = e;
    atomicAdd(&scnt[r], 1);
    ckey[i] = r;
    int row = kZeroRow;
    if (tffrac && (!edtype || edtype[e] == 0.f)) {
        int64_t b = tffrac[e];
        if (b < 0 || b >= kBoxes) atomicAdd(&counts[3], 1);   // nn.Embedding would raise
        else row = (int)b;
    }
    tf[i] = (uint8_t)row;
}

__global__ void k_csc_fill(int n_typed_max, const int32_t *__restrict__ ckey2, const int32_t *__restrict__ cperm,
                           const int32_t *__restrict__ key2, int32_t *__restrict__ cdst, int n) {
    int j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= n_typed_max || ckey2[j] >= n) return;
    cdst[j] = key2[cperm[j]];
}

__global__ void k_node_fill(int n, const int32_t *__restrict__ fs, const int32_t *__restrict__ fd,
                            const int32_t *__restrict__ rs, const int32_t *__restrict__ rd,
                            const int32_t *__restrict__ indeg, const int32_t *__restrict__ tcnt,
                            const int32_t *__restrict__ indptr, int64_t *__restrict__ src_nodes,
                            int64_t *__restrict__ dst_nodes, int32_t *__restrict__ phantom,
                            int32_t *__restrict__ counts) {
    int i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) {
        if (fs[i]) src_nodes[rs[i]] = i;
        if (fd[i]) {
            int r = rd[i];
            dst_nodes[r] = i;
            phantom[r] = indeg[i] - tcnt[r];
        }
    }
    if (i == 0) {
        counts[0] = rs[n];
        counts[1] = rd[n];
        counts[2] = indptr[n];
    }
}

// Work list of one CSR / CSC (hsg_rel_work, round 6).  One block of kWorkThreads walks
// the nodes in tiles: per node k(v) = deg > P ? ceil(deg / P) : 1 items, an exclusive
// block scan of k over the tile (+ the running offset) places them, and the pieces of
// a long node split its segment into k near-equal runs.  Items are 4 int32 (node code,
// beg, end, first item of the node); after the n items come n zeroed arrival counters
// (the pieces' in-kernel merge).  *count = items, or 0 when no node is long (nothing to
// balance: the kernels then walk the nodes).
constexpr int kWorkThreads = 1024;

__global__ __launch_bounds__(kWorkThreads) void k_rel_work(int n, const int32_t *__restrict__ indptr, int min_len,
                                                            int mult, int32_t *__restrict__ work, int max_items,
                                                            int32_t *__restrict__ count) {
    __shared__ int s_scan[kWorkThreads];
    __shared__ int s_any;
    const int t = threadIdx.x;
    const int E = indptr[n];
    const int mean = (E + n - 1) / n;                       // ceil(E / n), n >= 1
    const int P = max(min_len, mult * mean);
    if (t == 0) s_any = 0;
    __syncthreads();
    int base = 0;
    for (int v0 = 0; v0 < n; v0 += kWorkThreads) {
        const int v = v0 + t;
        int beg = 0, deg = 0, k = 0;
        if (v < n) {
            beg = indptr[v];
            deg = indptr[v + 1] - beg;
            k = deg > P ? (deg + P - 1) / P : 1;
        }
        if (k > 1) s_any = 1;                              // benign race: every writer stores 1
        // inclusive Hillis-Steele scan of k over the tile
        s_scan[t] = k;
        __syncthreads();
        for (int o = 1; o < kWorkThreads; o <<= 1) {
            const int x = t >= o ? s_scan[t - o] : 0;
            __syncthreads();
            s_scan[t] += x;
            __syncthreads();
        }
        const int first = base + s_scan[t] - k;
        if (v < n) {
            for (int p = 0; p < k; ++p) {                  // near-equal runs: the first deg % k one longer
                const int q = deg / k, r = deg % k;
                const int b = beg + p * q + min(p, r), e = b + q + (p < r ? 1 : 0);
                if (first + p < max_items) {
                    int32_t *w = work + 4 * (first + p);
                    w[0] = k == 1 ? v : -(v + 1);
                    w[1] = b;
                    w[2] = e;
                    w[3] = first;
                }
            }
        }
        base += s_scan[kWorkThreads - 1];
        __syncthreads();                                 // s_scan reused by the next tile
    }
    const bool ok = s_any && base <= max_items;
    if (ok)
        for (int i = t; i < base; i += kWorkThreads) work[4 * base + i] = 0;   // arrival counters
    if (t == 0) *count = ok ? base : 0;
}

}  // namespace

extern "C" int hsg_rel_work(int n, const int32_t *indptr, int min_len, int mult, int32_t *work, int max_items,
                            int32_t *count, void *stream) {
    if (n < 0 || !count || mult < 0 || (n > 0 && (!indptr || !work || max_items < n))) return HSG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (n == 0 || min_len <= 0) return (int)hipMemsetAsync(count, 0, sizeof(int32_t), s);
    k_rel_work<<<1, kWorkThreads, 0, s>>>(n, indptr, min_len, mult, work, max_items, count);
    return (int)hipGetLastError();
}

extern "C" size_t hsg_rel_build_workspace_bytes(int n_nodes, int n_edges) {
    if (n_nodes < 0 || n_edges < 0) return 0;
    size_t tb = 0;
    if (temp_bytes(n_nodes, n_edges, &tb, nullptr) != hipSuccess) return 0;
    return carve(nullptr, nullptr, n_nodes, n_edges, tb);
}

extern "C" int hsg_rel_build(float src_unit, float dst_unit, int n, int E,
                             const int64_t *src, const int64_t *dst, const float *unit,
                             const int64_t *tffrac, const float *edtype, int32_t *counts,
                             int32_t *indptr, int32_t *esrc, uint8_t *tf, int64_t *eid,
                             int32_t *phantom, int32_t *cindptr, int32_t *cdst, int32_t *cperm,
                             int64_t *src_nodes, int64_t *dst_nodes, void *workspace,
                             size_t workspace_bytes, void *stream) {
    if (n < 0 || E < 0 || !counts || !indptr || !cindptr || (n > 0 && !unit) || (E > 0 && (!src || !dst)))
        return HSG_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    size_t tb = 0;
    hipError_t err = temp_bytes(n, E, &tb, s);
    if (err != hipSuccess) {
        if (getenv("HSG_DEBUG")) fprintf(stderr, "hsg_rel_build: temp size query -> %s\n", hipGetErrorString(err));
        return err;
    }
    Work w;
    if (carve(nullptr, nullptr, n, E, tb) > workspace_bytes || !workspace) return HSG_EINVAL;
    carve(&w, static_cast<char *>(workspace), n, E, tb);
    // rocprim takes the temp size by reference: hand each call its own copy
    auto scan = [&](const int32_t *in, int32_t *out) {
        size_t b = tb;
        return rocprim::exclusive_scan(w.tmp, b, in, out, 0, (size_t)n + 1, rocprim::plus<int32_t>(), s);
    };
    auto sort = [&](int32_t *k_in, int32_t *k_out, int32_t *v_in, int32_t *v_out, int bits) {
        size_t b = tb;
        return rocprim::radix_sort_pairs(w.tmp, b, reinterpret_cast<uint32_t *>(k_in),
                                         reinterpret_cast<uint32_t *>(k_out), v_in, v_out, (unsigned)E, 0,
                                         bits, s);
    };
#define HSG_TRY(x)                                                                    \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            if (getenv("HSG_DEBUG"))                                                  \
                fprintf(stderr, "hsg_rel_build: %s -> %s\n", #x, hipGetErrorString(e_)); \
            return e_;                                                                \
        }                                                                             \
    } while (0)
    HSG_TRY(hipMemsetAsync(counts, 0, 5 * sizeof(int32_t), s));
    HSG_TRY(hipMemsetAsync(w.indeg, 0, (size_t)(n > 0 ? n : 1) * sizeof(int32_t), s));
    HSG_TRY(hipMemsetAsync(w.tcnt, 0, (size_t)(n + 1) * sizeof(int32_t), s));
    HSG_TRY(hipMemsetAsync(w.scnt, 0, (size_t)(n + 1) * sizeof(int32_t), s));

    k_node_flags<<<blocks_for(n + 1), kThreads, 0, s>>>(n, unit, src_unit, dst_unit, w.fs, w.fd);
    HSG_TRY(hipGetLastError());
    HSG_TRY(scan(w.fs, w.rs));
    HSG_TRY(scan(w.fd, w.rd));
    const int bits = key_bits(n);
    if (E > 0) {
        k_edge_keys<<<blocks_for(E), kThreads, 0, s>>>(n, E, src, dst, w.fs, w.fd, w.rd, w.indeg, w.tcnt,
                                                        w.key, w.val, counts);
        HSG_TRY(hipGetLastError());
        HSG_TRY(sort(w.key, w.key2, w.val, w.val2, bits));
    }
    HSG_TRY(scan(w.tcnt, indptr));
    if (E > 0) {
        k_csr_fill<<<blocks_for(E), kThreads, 0, s>>>(n, E, w.key2, w.val2, src, w.rs, tffrac, edtype, esrc, tf,
                                                       eid, w.scnt, w.ckey, w.cval, counts);
        HSG_TRY(hipGetLastError());
        HSG_TRY(sort(w.ckey, w.ckey2, w.cval, cperm, bits));
        k_csc_fill<<<blocks_for(E), kThreads, 0, s>>>(E, w.ckey2, cperm, w.key2, cdst, n);
        HSG_TRY(hipGetLastError());
    }
    HSG_TRY(scan(w.scnt, cindptr));
    k_node_fill<<<blocks_for(n > 0 ? n : 1), kThreads, 0, s>>>(n, w.fs, w.fd, w.rs, w.rd, w.indeg, w.tcnt, indptr,
                                                               src_nodes, dst_nodes, phantom, counts);
    HSG_TRY(hipGetLastError());
#undef HSG_TRY
    return 0;
}
