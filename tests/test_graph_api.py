"""The rest of the DGL-0.4 surface the reference touches, on CPU:

* generic ``apply_edges`` / ``pull`` UDF execution (GATLayer.py:74-75, 112-113,
  148-149) -- the reference's own WSGATLayer UDFs (edge attention, message, softmax
  reduce) run through this build's graph object and through the test-only DGL 0.4
  shim (tests/golden/dgl_shim.py, the semantics the golden vectors were made with)
  give identical node features;
* ``predecessors`` (HiGraph.py:237) in edge-id order;
* ``dgl.batch`` / ``dgl.unbatch`` round trip (HiGraph.py:248, Tester.py:106);
* ``save_graphs`` / ``load_graphs`` (this build's on-disk format, not DGL's binary
  one: INTEGRATION.md) and ``LoadHiExampleSet`` (dataloader.py:426-440);
* graphs pickled through ``DataLoader(num_workers=2, collate_fn=graph_collate_fn)``
  (train.py:354) batch to the same graph as in-process collation.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import dgl_shim


def _docs(seed=3):
    from hetersumgraph_amd import synth
    rng = np.random.default_rng(seed)
    return [synth.make_hsg_doc(rng, N=n, W=w, k=k, k_jitter=2, isolated_words=1, tf_range=(0.0, 1.0))
            for n, w, k in ((4, 15, 4), (6, 20, 5), (3, 9, 3))]


def _graphs(docs, cls):
    from hetersumgraph_amd import synth
    return [synth.to_graph(d, cls) for d in docs]


class _Udf:
    """The reference WSGATLayer's UDF trio (GATLayer.py:89-102), one head."""

    def __init__(self, seed, in_dim=16, out_dim=8, feat=50):
        g = torch.Generator().manual_seed(seed)
        self.fc = torch.randn(out_dim, in_dim, generator=g, dtype=torch.float64) / 4
        self.ffc = torch.randn(out_dim, feat, generator=g, dtype=torch.float64) / 7
        self.attn = torch.randn(1, 3 * out_dim, generator=g, dtype=torch.float64) / 5

    def edge_attention(self, edges):
        dfeat = edges.data["tfidfembed"] @ self.ffc.t()
        z2 = torch.cat([edges.src["z"], edges.dst["z"], dfeat], dim=1)
        return {"e": F.leaky_relu(z2 @ self.attn.t())}

    def message_func(self, edges):
        return {"e": edges.data["e"], "z": edges.src["z"]}

    def reduce_func(self, nodes):
        alpha = F.softmax(nodes.mailbox["e"], dim=1)
        return {"sh": torch.sum(alpha * nodes.mailbox["z"], dim=1)}


def _run_udf(G, udf, h, T):
    wnode = G.filter_nodes(lambda n: n.data["unit"] == 0)
    snode = G.filter_nodes(lambda n: n.data["unit"] == 1)
    wsedge = G.filter_edges(lambda e: (e.src["unit"] == 0) & (e.dst["unit"] == 1))
    dt0 = G.filter_edges(lambda e: e.data["dtype"] == 0)
    G.edges[dt0].data["tfidfembed"] = T[G.edata["tffrac"][dt0]]
    G.nodes[wnode].data["z"] = h @ udf.fc.t()
    G.apply_edges(udf.edge_attention, edges=wsedge)
    G.pull(snode, udf.message_func, udf.reduce_func)
    return G.ndata.pop("sh")[snode]


def test_generic_udf_apply_edges_pull_match_dgl04_semantics():
    from hetersumgraph_amd import graph as hg
    docs = _docs()
    udf = _Udf(1)
    T = torch.randn(10, 50, generator=torch.Generator().manual_seed(2), dtype=torch.float64)
    outs = []
    for mod in (hg, dgl_shim):
        G = mod.batch(_graphs(docs, mod.DGLGraph))
        n_w = int((G.ndata["unit"] == 0).sum())
        h = torch.randn(n_w, 16, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
        outs.append(_run_udf(G, udf, h, T))
    assert outs[0].shape == outs[1].shape
    assert torch.equal(outs[0], outs[1])


def test_predecessors_in_edge_id_order():
    from hetersumgraph_amd import graph as hg
    docs = _docs(4)
    G = hg.batch(_graphs(docs, hg.DGLGraph))
    S = dgl_shim.batch(_graphs(docs, dgl_shim.DGLGraph))
    for v in range(G.number_of_nodes()):
        assert G.predecessors(v).tolist() == S.predecessors(v).tolist()


def test_batch_unbatch_round_trip():
    from hetersumgraph_amd import graph as hg
    docs = _docs(5)
    gs = _graphs(docs, hg.DGLGraph)
    G = hg.batch(gs)
    assert G.batch_size == 3 and G.number_of_nodes() == sum(g.number_of_nodes() for g in gs)
    back = hg.unbatch(G)
    for a, b in zip(back, gs):
        assert a.number_of_nodes() == b.number_of_nodes() and a.number_of_edges() == b.number_of_edges()
        ua, va = a.edges()
        ub, vb = b.edges()
        assert torch.equal(ua, ub) and torch.equal(va, vb)
        for k in b.ndata.keys():
            assert torch.equal(a.ndata[k], b.ndata[k]), k
        for k in b.edata.keys():
            assert torch.equal(a.edata[k], b.edata[k]), k


def _same_graph(a, b):
    assert a.number_of_nodes() == b.number_of_nodes() and a.number_of_edges() == b.number_of_edges()
    ua, va = a.edges()
    ub, vb = b.edges()
    assert torch.equal(ua, ub) and torch.equal(va, vb)
    assert sorted(a.ndata.keys()) == sorted(b.ndata.keys()) and sorted(a.edata.keys()) == sorted(b.edata.keys())
    for k in b.ndata.keys():
        assert torch.equal(a.ndata[k], b.ndata[k]), k
    for k in b.edata.keys():
        assert torch.equal(a.edata[k], b.edata[k]), k


def test_save_load_graphs_and_load_hi_example_set(tmp_path):
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd.dgl.data.utils import load_graphs, save_graphs
    from hetersumgraph_amd.module.dataloader import LoadHiExampleSet
    gs = _graphs(_docs(6), hg.DGLGraph)
    for i, g in enumerate(gs):                        # one graph per file, as the reference's cache
        save_graphs(str(tmp_path / f"{i}.graph.bin"), [g], {"idx": torch.tensor([i])})
    (tmp_path / "README.txt").write_text("not a graph")
    ds = LoadHiExampleSet(str(tmp_path))
    assert len(ds) == len(gs)
    for i, g in enumerate(gs):
        got, idx = ds[i]
        assert idx == i
        _same_graph(got, g)
    both, labels = load_graphs(str(tmp_path / "1.graph.bin"))
    assert len(both) == 1 and labels["idx"].tolist() == [1]
    many = str(tmp_path / "all.bin")
    save_graphs(many, gs)
    sub, _ = load_graphs(many, [0, 2])
    assert len(sub) == 2
    _same_graph(sub[1], gs[2])


class _GraphSet(torch.utils.data.Dataset):
    def __init__(self, docs):
        self.docs = docs

    def __len__(self):
        return len(self.docs)

    def __getitem__(self, i):
        from hetersumgraph_amd import graph as hg
        from hetersumgraph_amd import synth
        return synth.to_graph(self.docs[i], hg.DGLGraph), i


def test_dataloader_workers_pickle_graphs():
    from hetersumgraph_amd.module.dataloader import graph_collate_fn
    from hetersumgraph_amd import synth
    docs = [synth.make_hsg_doc(np.random.default_rng(s), N=3 + s % 4, W=12 + s, k=4) for s in range(6)]
    ds = _GraphSet(docs)
    inproc = [graph_collate_fn([ds[i] for i in range(j, j + 3)]) for j in (0, 3)]
    dl = torch.utils.data.DataLoader(ds, batch_size=3, shuffle=False, num_workers=2, collate_fn=graph_collate_fn)
    got = list(dl)
    assert len(got) == 2
    for (G, idx), (R, ridx) in zip(got, inproc):
        assert list(idx) == list(ridx)
        _same_graph(G, R)
        assert G.batch_num_nodes == R.batch_num_nodes


def test_edge_score_column_semantics():
    """g.edata['e'] (graph.EdgeScoreColumn): each relation's rows come from its latest
    segment, other rows keep what the column held, and reading materialises a plain
    [E, 1] tensor (the reference: apply_edges(edge_attention) writes only the typed
    edges of the head, GATLayer.py:112 / 148, and the column persists)."""
    from hetersumgraph_amd import graph as hg

    class Seg:
        def __init__(self, key, eid, val):
            self.key, self.eid, self.val = key, torch.tensor(eid), torch.tensor(val)

        def scores(self):
            return self.val

        def to(self, device):
            return self

    g = hg.DGLGraph()
    g.add_nodes(4)
    g.add_edges([0, 1, 2, 3, 0], [1, 2, 3, 0, 2])
    g.edata["e"] = torch.full((5, 1), 7.0)                 # a column the caller wrote
    hg.record_edge_scores(g, Seg("W2S", [0, 2], [1.0, 2.0]))
    hg.record_edge_scores(g, Seg("S2W", [1], [3.0]))
    hg.record_edge_scores(g, Seg("W2S", [0, 2], [4.0, 5.0]))   # the next W2S application
    e = g.edata["e"]
    assert isinstance(e, torch.Tensor) and e.shape == (5, 1)
    assert e[:, 0].tolist() == [4.0, 3.0, 5.0, 7.0, 7.0]
    g.edges[[3]].data["e"] = torch.tensor([[9.0]])            # a row write materialises the column
    assert g.edata["e"][:, 0].tolist() == [4.0, 3.0, 5.0, 9.0, 7.0]
    g2 = hg.DGLGraph()
    g2.add_nodes(2)
    g2.add_edges([0, 1], [1, 0])
    hg.record_edge_scores(g2, Seg("W2S", [1], [2.5]))          # no column before: zeros elsewhere
    assert g2.edata["e"][:, 0].tolist() == [0.0, 2.5]
