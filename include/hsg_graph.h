/*
 * hsg_graph.h -- C ABI of the native document-graph builder (libhsg_host.so, host only).
 *
 * Replaces the per-edge Python construction of the reference's graph builders,
 *   ExampleSet.CreateGraph       module/dataloader.py:222-268  (HSG: words, sentences)
 *   MultiExampleSet.CreateGraph  module/dataloader.py:328-406  (HDSG: + document nodes)
 * and, through the offsets it is given, the node/edge renumbering of dgl.batch in
 * graph_collate_fn (dataloader.py:472-481).  Tokenisation (Example / Example2,
 * dataloader.py:56-137) and the JSON tf-idf tables stay on the Python side, which
 * hands over word ids and (word id, tf-idf) pairs; this library does the graph:
 *
 *   word nodes  = distinct non-filtered ids of the (truncated, padded) sentences, in
 *                 first-occurrence order (AddWordNode, dataloader.py:198-211)
 *   per sentence i, per distinct id in first-occurrence order (Counter order) that
 *   is a word node and has a tf-idf entry for i:
 *       word -> sentence and sentence -> word, tffrac = np.round(tfidf * 9)
 *       (round half to even), dtype 0                     (dataloader.py:248-257)
 *   HSG:  then sentence i -> every sentence, every sentence -> sentence i, dtype 1
 *                                                          (dataloader.py:262-263)
 *   HDSG: then sentence i -> its document node, dtype 2   (dataloader.py:385-386)
 *         and after all sentences, per document: word <-> document edges from the
 *         document's word list and tf-idf pairs, dtype 0  (dataloader.py:389-400)
 *   nodes: words (unit 0, dtype 0, id = vocab id), sentences (unit 1, dtype 1,
 *          id 0), documents (unit 1, dtype 2, id 0).
 *
 * Conventions: all pointers are host memory owned by the caller; return 0 or
 * HSG_GRAPH_EINVAL.  Documents are independent and built by `threads` worker
 * threads (0: hardware concurrency, at most 16); results do not depend on it.
 */
#ifndef HSG_GRAPH_H_
#define HSG_GRAPH_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HSG_GRAPH_EINVAL 2001

typedef struct hsg_docs {
    int32_t n_docs;
    int32_t sent_max_len;          /* L: padded sentence length                              */
    const int32_t *doc_nsent;      /* [n_docs] sentences per document (after truncation)     */
    const int64_t *sent_ids;       /* [sum nsent][L] padded word ids, documents concatenated  */
    const int64_t *sent_tf_ptr;    /* [sum nsent + 1] CSR over sentences of tf-idf pairs     */
    const int64_t *sent_tf_wid;    /*   word id of each pair                                  */
    const double *sent_tf_val;     /*   tf-idf value of each pair                             */
    /* multi-document graphs (HDSG); all NULL for HSG */
    const int32_t *doc_narticle;   /* [n_docs] document nodes per graph                       */
    const int32_t *sent_article;   /* [sum nsent] local document node of each sentence        */
    const int64_t *art_word_ptr;   /* [sum narticle + 1] CSR of each document's word ids      */
    const int64_t *art_word_ids;
    const int64_t *art_tf_ptr;     /* [sum narticle + 1] CSR of each document's tf-idf pairs  */
    const int64_t *art_tf_wid;
    const double *art_tf_val;
} hsg_docs;

/* Sizes of every document graph: n_nodes[d], n_edges[d].  filter_ids: the ids
 * that never become word nodes (stop words, punctuation, [PAD], low tf-idf words;
 * ExampleSet.__init__ dataloader.py:166-179), any order. */
int hsg_graph_count(const hsg_docs *docs, int64_t n_filter, const int64_t *filter_ids, int64_t *n_nodes,
                    int64_t *n_edges, int threads);

/* Writes every document graph into batched arrays: document d's nodes at
 * node_off[d] .. + n_nodes[d], its edges at edge_off[d] .. + n_edges[d], node ids
 * in src/dst already offset by node_off[d] (the dgl.batch numbering when the
 * offsets are the prefix sums in batch order).  sent_node[s] receives the global
 * node id of sentence s (documents concatenated in input order). */
int hsg_graph_fill(const hsg_docs *docs, int64_t n_filter, const int64_t *filter_ids, const int64_t *node_off,
                   const int64_t *edge_off, float *unit, float *ndtype, int64_t *wid, int64_t *src, int64_t *dst,
                   int64_t *tffrac, float *edtype, int64_t *sent_node, int threads);

#ifdef __cplusplus
}
#endif
#endif /* HSG_GRAPH_H_ */
