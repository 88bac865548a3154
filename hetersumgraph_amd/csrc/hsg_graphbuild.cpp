// hsg_graphbuild.cpp -- native document-graph builder (host C++, libhsg_host.so).
//
// The reference builds every document graph in Python, one add_edges call per
// edge, inside 32 DataLoader workers (module/dataloader.py:222-268, 328-406;
// train.py:354).  This file does the same construction over flat id arrays:
// one pass per document discovers the word nodes, a second emits the edges in the
// reference's order, and documents run on a small thread pool.  The edge order,
// node order and tf-idf boxes are exactly the reference's (include/hsg_graph.h);
// the oracle is oracle/create_graph.py, pinned to graphs made by the reference's
// own CreateGraph (tests/golden/make_graph_golden.py).
#include <cmath>
#include <cstdint>
#include <algorithm>
#include <atomic>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/hsg_graph.h"

namespace {

struct DocView {
    int nsent = 0, nart = 0;
    int64_t sent0 = 0, art0 = 0;   // first sentence / document index in the flat arrays
};

// prefix sums of the per-document sentence and document counts
std::vector<DocView> doc_views(const hsg_docs *d) {
    std::vector<DocView> v(d->n_docs);
    int64_t s = 0, a = 0;
    for (int i = 0; i < d->n_docs; ++i) {
        v[i].nsent = d->doc_nsent[i];
        v[i].nart = d->doc_narticle ? d->doc_narticle[i] : 0;
        v[i].sent0 = s;
        v[i].art0 = a;
        s += v[i].nsent;
        a += v[i].nart;
    }
    return v;
}

// np.round(tfidf * 9): float64 product, round half to even (the default rounding
// mode, which nearbyint honours)
inline int64_t tf_box(double tfidf) { return (int64_t)std::nearbyint(tfidf * 9.0); }

struct Sink {
    // counting (all pointers null) or writing one document at (node0, edge0)
    int64_t node0 = 0, e = 0;
    int64_t *src = nullptr, *dst = nullptr, *tf = nullptr;
    float *et = nullptr;
    bool write = false;
    inline void edge(int64_t u, int64_t v, int64_t t, float type) {
        if (write) {
            src[e] = node0 + u;
            dst[e] = node0 + v;
            tf[e] = t;
            et[e] = type;
        }
        ++e;
    }
};

// Per-document construction; returns the node count and emits edges into `sink`.
int64_t build_doc(const hsg_docs *d, const DocView &dv, const std::unordered_set<int64_t> &filt, Sink &sink,
                  float *unit, float *ndtype, int64_t *wid, int64_t *sent_node) {
    const int L = d->sent_max_len;
    const int64_t *ids = d->sent_ids + dv.sent0 * L;
    // AddWordNode (dataloader.py:198-211): first occurrence over sentences, then words
    std::unordered_map<int64_t, int64_t> wid2nid;
    std::vector<int64_t> nid2wid;
    wid2nid.reserve((size_t)dv.nsent * L);
    for (int64_t k = 0; k < (int64_t)dv.nsent * L; ++k) {
        const int64_t w = ids[k];
        if (filt.count(w) || wid2nid.count(w)) continue;
        wid2nid.emplace(w, (int64_t)nid2wid.size());
        nid2wid.push_back(w);
    }
    const int64_t nw = (int64_t)nid2wid.size();
    const int64_t N = dv.nsent;
    const bool multi = d->doc_narticle != nullptr;
    const int64_t n_nodes = nw + N + (multi ? dv.nart : 0);
    if (sink.write) {
        const int64_t o = sink.node0;
        for (int64_t i = 0; i < nw; ++i) { unit[o + i] = 0.f; ndtype[o + i] = 0.f; wid[o + i] = nid2wid[i]; }
        for (int64_t i = 0; i < N; ++i) {
            unit[o + nw + i] = 1.f;
            ndtype[o + nw + i] = 1.f;
            wid[o + nw + i] = 0;
            sent_node[dv.sent0 + i] = o + nw + i;
        }
        if (multi)
            for (int64_t i = 0; i < dv.nart; ++i) {
                unit[o + nw + N + i] = 1.f;
                ndtype[o + nw + N + i] = 2.f;
                wid[o + nw + N + i] = 0;
            }
    }
    std::unordered_map<int64_t, double> tfw;
    std::unordered_set<int64_t> seen;
    // word <-> node edges for one word sequence (Counter first-occurrence order)
    auto word_edges = [&](const int64_t *seq, int64_t len, int64_t node, const int64_t *tp, const int64_t *tw,
                          const double *tv) {
        tfw.clear();
        for (int64_t p = tp[0]; p < tp[1]; ++p) tfw[tw[p]] = tv[p];
        seen.clear();
        for (int64_t j = 0; j < len; ++j) {
            const int64_t w = seq[j];
            if (!seen.insert(w).second) continue;
            auto it = wid2nid.find(w);
            if (it == wid2nid.end()) continue;
            auto t = tfw.find(w);
            if (t == tfw.end()) continue;
            const int64_t box = tf_box(t->second);
            sink.edge(it->second, node, box, 0.f);
            sink.edge(node, it->second, box, 0.f);
        }
    };
    for (int64_t i = 0; i < N; ++i) {
        const int64_t s = dv.sent0 + i;
        word_edges(ids + i * L, L, nw + i, d->sent_tf_ptr + s, d->sent_tf_wid, d->sent_tf_val);
        if (!multi) {
            for (int64_t j = 0; j < N; ++j) sink.edge(nw + i, nw + j, 0, 1.f);   // sentence -> all
            for (int64_t j = 0; j < N; ++j) sink.edge(nw + j, nw + i, 0, 1.f);   // all -> sentence
        } else {
            sink.edge(nw + i, nw + N + d->sent_article[s], 0, 2.f);             // sentence -> document
        }
    }
    if (multi) {
        for (int64_t a = 0; a < dv.nart; ++a) {
            const int64_t ga = dv.art0 + a;
            const int64_t *seq = d->art_word_ids + d->art_word_ptr[ga];
            word_edges(seq, d->art_word_ptr[ga + 1] - d->art_word_ptr[ga], nw + N + a, d->art_tf_ptr + ga,
                       d->art_tf_wid, d->art_tf_val);
        }
    }
    return n_nodes;
}

bool docs_ok(const hsg_docs *d) {
    if (!d || d->n_docs < 0 || d->sent_max_len < 0) return false;
    if (d->n_docs && (!d->doc_nsent || !d->sent_tf_ptr)) return false;
    int64_t ns = 0, na = 0;
    for (int i = 0; i < d->n_docs; ++i) {
        if (d->doc_nsent[i] < 0) return false;
        ns += d->doc_nsent[i];
        if (d->doc_narticle) {
            if (d->doc_narticle[i] < 0) return false;
            na += d->doc_narticle[i];
        }
    }
    if (ns && (!d->sent_ids || !d->sent_tf_wid || !d->sent_tf_val)) return false;
    if (d->doc_narticle) {
        if (ns && !d->sent_article) return false;
        if (!d->art_word_ptr || !d->art_tf_ptr) return false;
        for (int i = 0, s = 0; i < d->n_docs; s += d->doc_nsent[i], ++i)
            for (int j = 0; j < d->doc_nsent[i]; ++j)
                if (d->sent_article[s + j] < 0 || d->sent_article[s + j] >= d->doc_narticle[i]) return false;
        (void)na;
    }
    return true;
}

template <class F>
void parallel_docs(int n, int threads, F fn) {
    int t = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
    t = std::max(1, std::min({t, 16, n}));
    if (t <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<int> next{0};
    std::vector<std::thread> pool;
    for (int k = 0; k < t; ++k)
        pool.emplace_back([&] {
            for (int i = next++; i < n; i = next++) fn(i);
        });
    for (auto &th : pool) th.join();
}

}  // namespace

extern "C" {

int hsg_graph_count(const hsg_docs *docs, int64_t n_filter, const int64_t *filter_ids, int64_t *n_nodes,
                    int64_t *n_edges, int threads) {
    if (!docs_ok(docs) || n_filter < 0 || (n_filter && !filter_ids) || !n_nodes || !n_edges) return HSG_GRAPH_EINVAL;
    const std::unordered_set<int64_t> filt(filter_ids, filter_ids + n_filter);
    const auto views = doc_views(docs);
    parallel_docs(docs->n_docs, threads, [&](int i) {
        Sink s;
        n_nodes[i] = build_doc(docs, views[i], filt, s, nullptr, nullptr, nullptr, nullptr);
        n_edges[i] = s.e;
    });
    return 0;
}

int hsg_graph_fill(const hsg_docs *docs, int64_t n_filter, const int64_t *filter_ids, const int64_t *node_off,
                   const int64_t *edge_off, float *unit, float *ndtype, int64_t *wid, int64_t *src, int64_t *dst,
                   int64_t *tffrac, float *edtype, int64_t *sent_node, int threads) {
    if (!docs_ok(docs) || n_filter < 0 || (n_filter && !filter_ids) || !node_off || !edge_off || !unit || !ndtype ||
        !wid || !src || !dst || !tffrac || !edtype || !sent_node)
        return HSG_GRAPH_EINVAL;
    const std::unordered_set<int64_t> filt(filter_ids, filter_ids + n_filter);
    const auto views = doc_views(docs);
    parallel_docs(docs->n_docs, threads, [&](int i) {
        Sink s;
        s.write = true;
        s.node0 = node_off[i];
        s.src = src + edge_off[i];
        s.dst = dst + edge_off[i];
        s.tf = tffrac + edge_off[i];
        s.et = edtype + edge_off[i];
        build_doc(docs, views[i], filt, s, unit, ndtype, wid, sent_node);
    });
    return 0;
}

}  // extern "C"
