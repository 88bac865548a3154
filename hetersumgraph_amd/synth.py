"""Synthetic CNN/DM-, Multi-News- and NYT50-shaped document graphs.

The generator reproduces the node/edge *order and schema* that the reference's
graph builders emit, without their text pipeline (nltk, vocab files, tf-idf JSONL):

* HSG (single document), ``ExampleSet.CreateGraph`` module/dataloader.py:222-268:
  word nodes first (unit 0, dtype 0, ``id`` = vocab id), then N sentence nodes
  (unit 1, dtype 1).  For every sentence i, in word order, a word->sentence and a
  sentence->word edge are added in alternation (dataloader.py:254-257, ``tffrac`` =
  ``np.round(tfidf*9)``, dtype 0); then N sentence->all-sentence edges and N
  all-sentence->sentence edges (dtype 1, dataloader.py:262-263).
* HDSG (multi document), ``MultiExampleSet.CreateGraph`` dataloader.py:328-406:
  words, sentences, then doc nodes (unit 1, dtype 2).  Per sentence: w<->s edges
  then one s->doc edge (dtype 2); after all sentences, per doc: w<->d edges.

Sentence node columns ``words`` [N, sent_max_len], ``position`` [N,1] and ``label``
[N, doc_max_timesteps] follow dataloader.py:264-266 / 402-404.

Everything is drawn from ``numpy.random.default_rng(seed)`` (BASELINE.md
"Input distributions"): vocab ids distinct per doc in [4, vocab), sentence word
sets uniform without replacement from the doc's words, ``tfidf ~ U(0.05, 0.6)``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class DocArrays:
    """One document graph as flat arrays (node ids are local to the doc)."""

    n_nodes: int
    unit: np.ndarray          # float32 [n]
    ndtype: np.ndarray        # float32 [n]
    wid: np.ndarray           # int64 [n]  vocab id for word nodes, 0 otherwise
    src: np.ndarray           # int64 [E]
    dst: np.ndarray           # int64 [E]
    tffrac: np.ndarray        # int64 [E]  0 on non dtype-0 edges
    edtype: np.ndarray        # float32 [E]
    sent_nodes: np.ndarray    # int64 [N]
    words: np.ndarray         # int64 [N, sent_max_len]
    position: np.ndarray      # int64 [N, 1]
    label: np.ndarray         # int64 [N, doc_max_timesteps]
    extra: dict = field(default_factory=dict)


def _tf_box(rng, n, tf_range=(0.05, 0.6)):
    # dataloader.py:253 -- np.round is half-to-even, like the reference.
    return np.round(rng.uniform(tf_range[0], tf_range[1], size=n) * 9).astype(np.int64)


def _sentence_tokens(rng, word_vocab_ids, sent_max_len, vocab_size):
    """Token ids of one sentence: its linked words (first occurrence order) plus a
    few unlinked filler tokens, truncated/padded with PAD=0 (Example._pad_encoder_input,
    dataloader.py:97-109)."""
    n_fill = int(rng.integers(0, 4))
    fill = rng.integers(1, max(2, vocab_size), size=n_fill)
    toks = np.concatenate([word_vocab_ids, fill])[:sent_max_len]
    out = np.zeros(sent_max_len, dtype=np.int64)
    out[: len(toks)] = toks
    return out


def _labels(rng, N, doc_max_timesteps, n_pick=3):
    # Example.label_matrix (dataloader.py:90-95) padded by pad_label_m (201-207).
    lab = np.zeros((N, doc_max_timesteps), dtype=np.int64)
    picks = rng.choice(N, size=min(n_pick, N, doc_max_timesteps), replace=False)
    for j, i in enumerate(picks):
        lab[i, j] = 1
    return lab


def make_hsg_doc(rng, N, W, k, *, vocab_size=50000, sent_max_len=100,
                 doc_max_timesteps=50, k_jitter=0, isolated_words=0, tf_range=(0.05, 0.6)):
    """One HSG document graph (ExampleSet.CreateGraph order).

    ``k_jitter`` varies the words-per-sentence count in [k-j, k+j] (clipped to
    [0, W]); ``isolated_words`` forces that many word nodes to have no edges (words
    without a tf-idf entry)."""
    vocab_ids = rng.choice(np.arange(4, vocab_size), size=W, replace=False).astype(np.int64)
    n = W + N
    unit = np.zeros(n, np.float32)
    unit[W:] = 1.0
    ndtype = unit.copy()
    wid = np.zeros(n, np.int64)
    wid[:W] = vocab_ids
    usable = np.arange(W - isolated_words)
    src, dst, tf, et = [], [], [], []
    words = np.zeros((N, sent_max_len), np.int64)
    sent_ids = np.arange(W, W + N, dtype=np.int64)
    for i in range(N):
        ki = k if k_jitter == 0 else int(rng.integers(max(0, k - k_jitter), k + k_jitter + 1))
        ki = min(ki, len(usable))
        ws = rng.choice(usable, size=ki, replace=False).astype(np.int64)
        boxes = _tf_box(rng, ki, tf_range)
        s = W + i
        # alternating w->s, s->w (dataloader.py:254-257)
        pair_src = np.empty(2 * ki, np.int64)
        pair_dst = np.empty(2 * ki, np.int64)
        pair_src[0::2], pair_dst[0::2] = ws, s
        pair_src[1::2], pair_dst[1::2] = s, ws
        src.append(pair_src)
        dst.append(pair_dst)
        tf.append(np.repeat(boxes, 2))
        et.append(np.zeros(2 * ki, np.float32))
        # s -> all sentences, all sentences -> s (dataloader.py:262-263)
        src.append(np.full(N, s, np.int64))
        dst.append(sent_ids)
        src.append(sent_ids)
        dst.append(np.full(N, s, np.int64))
        tf.append(np.zeros(2 * N, np.int64))
        et.append(np.ones(2 * N, np.float32))
        words[i] = _sentence_tokens(rng, vocab_ids[ws], sent_max_len, vocab_size)
    return DocArrays(
        n_nodes=n, unit=unit, ndtype=ndtype, wid=wid,
        src=np.concatenate(src), dst=np.concatenate(dst),
        tffrac=np.concatenate(tf), edtype=np.concatenate(et),
        sent_nodes=sent_ids, words=words,
        position=np.arange(1, N + 1, dtype=np.int64).reshape(-1, 1),
        label=_labels(rng, N, doc_max_timesteps),
    )


def make_hdsg_example(rng, doc_sents, W, k, doc_words, *, vocab_size=50000,
                      sent_max_len=100, doc_max_timesteps=50, tf_range=(0.05, 0.6)):
    """One HDSG multi-document example (MultiExampleSet.CreateGraph order).

    ``doc_sents``: sentences per source document; ``doc_words``: tf-idf linked
    words per document node."""
    N = int(sum(doc_sents))
    D = len(doc_sents)
    vocab_ids = rng.choice(np.arange(4, vocab_size), size=W, replace=False).astype(np.int64)
    n = W + N + D
    unit = np.zeros(n, np.float32)
    unit[W:] = 1.0
    ndtype = np.zeros(n, np.float32)
    ndtype[W:W + N] = 1.0
    ndtype[W + N:] = 2.0
    wid = np.zeros(n, np.int64)
    wid[:W] = vocab_ids
    sent2doc = np.repeat(np.arange(D), doc_sents)
    src, dst, tf, et = [], [], [], []
    words = np.zeros((N, sent_max_len), np.int64)
    for i in range(N):
        ws = rng.choice(W, size=min(k, W), replace=False).astype(np.int64)
        boxes = _tf_box(rng, len(ws), tf_range)
        s = W + i
        ps = np.empty(2 * len(ws), np.int64)
        pd = np.empty(2 * len(ws), np.int64)
        ps[0::2], pd[0::2] = ws, s
        ps[1::2], pd[1::2] = s, ws
        src += [ps, np.array([s])]
        dst += [pd, np.array([W + N + sent2doc[i]])]
        tf += [np.repeat(boxes, 2), np.zeros(1, np.int64)]
        et += [np.zeros(2 * len(ws), np.float32), np.full(1, 2.0, np.float32)]
        words[i] = _sentence_tokens(rng, vocab_ids[ws], sent_max_len, vocab_size)
    for d in range(D):
        ws = rng.choice(W, size=min(doc_words, W), replace=False).astype(np.int64)
        boxes = _tf_box(rng, len(ws), tf_range)
        dn = W + N + d
        ps = np.empty(2 * len(ws), np.int64)
        pd = np.empty(2 * len(ws), np.int64)
        ps[0::2], pd[0::2] = ws, dn
        ps[1::2], pd[1::2] = dn, ws
        src.append(ps)
        dst.append(pd)
        tf.append(np.repeat(boxes, 2))
        et.append(np.zeros(2 * len(ws), np.float32))
    return DocArrays(
        n_nodes=n, unit=unit, ndtype=ndtype, wid=wid,
        src=np.concatenate(src), dst=np.concatenate(dst),
        tffrac=np.concatenate(tf), edtype=np.concatenate(et),
        sent_nodes=np.arange(W, W + N, dtype=np.int64), words=words,
        position=np.arange(1, N + 1, dtype=np.int64).reshape(-1, 1),
        label=_labels(rng, N, doc_max_timesteps),
        extra={"sent2doc": sent2doc, "n_docs": D},
    )


def to_graph(doc: DocArrays, graph_cls):
    """Build a graph through the DGL-0.4 construction API (bulk form of the
    reference's add_nodes/add_edges calls).  ``graph_cls`` is any class with that
    API: ``hetersumgraph_amd.graph.DGLGraph`` or the test-only shim."""
    import torch
    from .graph import zero_initializer

    g = graph_cls()
    g.add_nodes(doc.n_nodes)
    g.set_n_initializer(zero_initializer)
    g.set_e_initializer(zero_initializer)
    g.ndata["unit"] = torch.from_numpy(doc.unit.copy())
    g.ndata["dtype"] = torch.from_numpy(doc.ndtype.copy())
    g.ndata["id"] = torch.from_numpy(doc.wid.copy())
    g.add_edges(torch.from_numpy(doc.src.copy()), torch.from_numpy(doc.dst.copy()),
                data={"tffrac": torch.from_numpy(doc.tffrac.copy()),
                      "dtype": torch.from_numpy(doc.edtype.copy())})
    sn = torch.from_numpy(doc.sent_nodes.copy())
    g.nodes[sn].data["words"] = torch.from_numpy(doc.words.copy())
    g.nodes[sn].data["position"] = torch.from_numpy(doc.position.copy())
    g.nodes[sn].data["label"] = torch.from_numpy(doc.label.copy())
    return g


# --- canonical benchmark configurations -----------------------

CONFIGS = {
    # name: (kind, docs per batch, per-doc params)
    "cfg1": ("hsg", 4, dict(N=30, W=400, k=20)),
    "cfg2": ("hsg", 32, dict(N=35, W=600, k=36)),
    "cfg3": ("hsg", 32, dict(N=35, W=600, k=36)),      # per GPU, 8 GPUs
    "cfg4": ("hdsg", 32, dict(doc_sents=(15, 15, 15), W=700, k=20, doc_words=250)),
    "cfg5": ("hsg", 32, dict(N=80, W=900, k=14)),      # per GPU, doc_max_timesteps=80
}


def make_batch_docs(config, seed=0, n_docs=None, **over):
    kind, B, params = CONFIGS[config]
    params = dict(params, **over)
    rng = np.random.default_rng(seed)
    B = B if n_docs is None else n_docs
    dmt = 80 if config == "cfg5" else 50
    if kind == "hsg":
        return [make_hsg_doc(rng, doc_max_timesteps=dmt, **params) for _ in range(B)]
    return [make_hdsg_example(rng, doc_max_timesteps=dmt, **params) for _ in range(B)]
