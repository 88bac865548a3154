"""The native document-graph builder (libhsg_host.so through
hetersumgraph_amd.module.dataloader / datapipe) against

* graphs the reference's own ExampleSet / MultiExampleSet.CreateGraph built
  (tests/golden/graphs_ref.npz, tests/golden/make_graph_golden.py), and
* the Python restatement oracle/create_graph.py, itself pinned to the same
  golden graphs, on more and larger seeded datasets.

Bit-exact: node order and columns, edge order, tf-idf boxes (half-to-even),
edge types, sentence rows, labels.  CPU only (host library).
"""
import os

import numpy as np
import pytest
import torch

from graph_data import STOPWORDS, MinVocab, make_files  # noqa: F401

SENT_MAX_LEN, DOC_MAX = 12, 7
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "graphs_ref.npz")


@pytest.fixture(scope="module", autouse=True)
def host_lib():
    from hetersumgraph_amd import build
    build.build_host(verbose=False)


def _dataset(tmp_path, kind, seed, n=6, threads=1):
    from hetersumgraph_amd.module.dataloader import ExampleSet, MultiExampleSet
    d = str(tmp_path / f"{kind}{seed}")
    vocab = make_files(d, seed=seed, n_examples=n, multi=kind == "hdsg")
    args = [os.path.join(d, "data.jsonl"), vocab, DOC_MAX, SENT_MAX_LEN, os.path.join(d, "filter_word.txt"),
            os.path.join(d, "w2s.jsonl")]
    if kind == "hdsg":
        return MultiExampleSet(*args, os.path.join(d, "w2d.jsonl"), stopwords=STOPWORDS, threads=threads), vocab, d
    return ExampleSet(*args, stopwords=STOPWORDS, threads=threads), vocab, d


def _graph_arrays(G):
    nd, ed = G.ndata, G.edata
    src, dst = G.all_edges()
    return dict(n=G.number_of_nodes(), unit=nd["unit"].numpy(), dtype=nd["dtype"].numpy(), id=nd["id"].numpy(),
                words=nd["words"].numpy(), position=nd["position"].numpy(), label=nd["label"].numpy(),
                src=src.numpy(), dst=dst.numpy(), tffrac=ed["tffrac"].numpy(), edtype=ed["dtype"].numpy())


def _assert_same(got, want, where):
    assert int(got["n"]) == int(want["n"]), where
    for k in ("unit", "dtype", "id", "words", "position", "label", "src", "dst", "tffrac", "edtype"):
        a, b = np.asarray(got[k]), np.asarray(want[k])
        assert a.shape == b.shape, (where, k, a.shape, b.shape)
        assert np.array_equal(a.astype(np.float64), b.astype(np.float64)), (where, k)


@pytest.mark.parametrize("kind,seed", [("hsg", 7), ("hdsg", 11)])
def test_native_builder_matches_reference_graphs(tmp_path, kind, seed):
    """Golden seeds: the graphs the reference's CreateGraph produced."""
    z = np.load(GOLD)
    ds, _, _ = _dataset(tmp_path, kind, seed)
    assert sorted(set(ds.filterids)) == z[f"{kind}.filterids"].tolist()
    assert len(ds) == int(z[f"{kind}.n"])
    for i in range(len(ds)):
        G, idx = ds[i]
        assert idx == i
        want = {k: z[f"{kind}.{i}.{k}"] for k in ("n", "unit", "dtype", "id", "words", "position", "label", "src",
                                                  "dst", "tffrac", "edtype")}
        _assert_same(_graph_arrays(G), want, (kind, i))


def _oracle_arrays(ds, i, kind, vocab):
    from oracle import create_graph as cg
    e = ds.example_list[i]
    enc, pad, lab, art_len, doc_in = cg.example_arrays(e["text"], e["label"], vocab, SENT_MAX_LEN,
                                                       multi=kind == "hdsg")
    pad = pad[:DOC_MAX]
    label = cg.pad_label_m(lab, DOC_MAX)
    filt = set(ds.filterids)
    if kind == "hsg":
        g = cg.hsg_graph(pad, ds.w2s_tfidf[i], vocab, filt)
    else:
        g = cg.hdsg_graph(art_len, pad, doc_in, ds.w2s_tfidf[i], ds.w2d_tfidf[i], vocab, filt)
    n = len(g["unit"])
    words = np.zeros((n, SENT_MAX_LEN), np.int64)
    position = np.zeros((n, 1), np.int64)
    lab_full = np.zeros((n, DOC_MAX), np.int64)
    sn = g["sent_nodes"]
    words[sn] = np.asarray(pad, np.int64)
    position[sn, 0] = np.arange(1, len(sn) + 1)
    lab_full[sn] = np.asarray(label, np.int64)
    return dict(n=n, unit=g["unit"], dtype=g["ndtype"], id=g["wid"], words=words, position=position,
                label=lab_full, src=g["src"], dst=g["dst"], tffrac=g["tffrac"], edtype=g["edtype"])


@pytest.mark.parametrize("kind,seed", [("hsg", 7), ("hdsg", 11)])
def test_oracle_matches_reference_graphs(tmp_path, kind, seed):
    """Pins the restatement (oracle/create_graph.py) to the reference's graphs."""
    z = np.load(GOLD)
    ds, vocab, _ = _dataset(tmp_path, kind, seed)
    for i in range(len(ds)):
        want = {k: z[f"{kind}.{i}.{k}"] for k in ("n", "unit", "dtype", "id", "words", "position", "label", "src",
                                                  "dst", "tffrac", "edtype")}
        _assert_same(_oracle_arrays(ds, i, kind, vocab), want, (kind, i))


@pytest.mark.parametrize("kind", ["hsg", "hdsg"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_native_builder_matches_oracle(tmp_path, kind, seed):
    ds, vocab, _ = _dataset(tmp_path, kind, seed, n=12, threads=4)
    arrs = ds.graph_arrays(list(range(len(ds))))          # one native call, 4 threads
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd.synth import to_graph
    for i, a in enumerate(arrs):
        _assert_same(_graph_arrays(to_graph(a, hg.DGLGraph)), _oracle_arrays(ds, i, kind, vocab), (kind, seed, i))


def test_thread_count_does_not_change_graphs(tmp_path):
    ds, _, _ = _dataset(tmp_path, "hdsg", 5, n=10)
    idx = list(range(len(ds)))
    ds.threads = 1
    a = ds.graph_arrays(idx)
    ds.threads = 8
    b = ds.graph_arrays(idx)
    for x, y in zip(a, b):
        for k in ("unit", "ndtype", "wid", "src", "dst", "tffrac", "edtype", "sent_nodes"):
            assert np.array_equal(getattr(x, k), getattr(y, k))


def test_graph_collate_fn_batches_in_reference_order(tmp_path):
    """graph_collate_fn (dataloader.py:472-481): sentence-count-descending order
    via torch.sort, node ids renumbered as dgl.batch does."""
    from hetersumgraph_amd.module.dataloader import graph_collate_fn
    ds, _, _ = _dataset(tmp_path, "hsg", 7)
    samples = [ds[i] for i in range(len(ds))]
    G, order = graph_collate_fn(samples)
    counts = [int((s[0].ndata["dtype"] == 1).sum()) for s in samples]
    _, want = torch.sort(torch.LongTensor(counts), dim=0, descending=True)
    assert order == [int(i) for i in want]
    src, dst = G.all_edges()
    off = 0
    eo = 0
    for i in order:
        g = samples[i][0]
        s, d = g.all_edges()
        ne = len(s)
        assert torch.equal(src[eo:eo + ne], s + off) and torch.equal(dst[eo:eo + ne], d + off)
        off += g.number_of_nodes()
        eo += ne
    assert G.batch_num_nodes == [samples[i][0].number_of_nodes() for i in order]


def test_invalid_document_arrays_raise():
    from hetersumgraph_amd.datapipe import build_doc_arrays
    doc = dict(sent_pad=[[5, 6, 0]], label=[[1]], sent_tf=[(np.array([5], np.int64), np.array([0.3]))],
               sent2doc=[3], n_art=1, art_words=[[5]], art_tf=[(np.zeros(0, np.int64), np.zeros(0))])
    with pytest.raises(ValueError):
        build_doc_arrays([doc], 3, [0], multi=True)          # sentence -> document 3 of 1
