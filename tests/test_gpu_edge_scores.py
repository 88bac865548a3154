"""``g.edata['e']`` after a forward, as the reference leaves it (VERDICT r5 boundary
divergence #1; /root/reference/module/GATLayer.py:89-93, 112, 148).

Every reference head writes its attention logits on its typed edges and the column
stays on the graph, so after a forward each typed edge holds the last head's logit of
the last application over its relation. The HIP path never forms per-edge logits.
`graph.EdgeScoreColumn` keeps the last application's projected features and head
parameters per relation, and forms the rows when the column is read. Checked against
oracle/dgl_udf.py, which keeps the column as the reference's `apply_edges` writes it
(UdfGraph.e): the per-layer module path (W2S then S2W) and the fused n_iter = 2 stack,
both in eval mode.
"""
import numpy as np
import pytest
import torch

from helpers import build_graph, gat_inputs, seeded_gat_params, synth_fixture

pytestmark = pytest.mark.gpu


def _setup(n_docs, seed):
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.HiGraph import register_tfidf_table
    from oracle import dgl_udf, fused
    z = synth_fixture(synth.make_batch_docs("cfg2", seed=0)[:n_docs])
    dev = torch.device("cuda")
    G = build_graph(z).to(dev)
    Xw, Xs, T = gat_inputs(seed, int(z["n_w"]), int(z["n_s"]))
    Td = T.to(dev)
    register_tfidf_table(G, Td)
    w2s, s2w = seeded_gat_params(seed * 100 + 1, seed * 100 + 2)
    ug = dgl_udf.UdfGraph(z["g_src"], z["g_dst"], z["g_unit"], z["g_tffrac"], z["g_edtype"])
    p1 = fused.as_params(w2s, dtype=torch.float32)
    p2 = fused.as_params(s2w, dtype=torch.float32)
    return G, ug, (Xw, Xs, T, Td), w2s.to(dev), s2w.to(dev), p1, p2


def test_edge_scores_per_layer_path():
    from oracle import dgl_udf
    G, ug, (Xw, Xs, T, _), w2s, s2w, p1, p2 = _setup(4, 7)
    dev = torch.device("cuda")
    with torch.no_grad():
        s = w2s(G, Xw.to(dev), Xs.to(dev))
        w = s2w(G, Xw.to(dev), s)
    te = dgl_udf.tfidf_embed(ug, T)
    so = dgl_udf.wswgat(ug, "W2S", Xw, Xs, p1, te)
    dgl_udf.wswgat(ug, "S2W", Xw, so, p2, te)
    e = G.edata["e"].cpu()
    assert e.shape == ug.e.shape
    assert ug.e.abs().max() > 0
    assert (e - ug.e).abs().max().item() <= 1e-4, (e - ug.e).abs().max().item()
    assert torch.isfinite(w).all()


def test_edge_scores_fused_stack():
    from hetersumgraph_amd.stack import fused_stack_ok, gat_stack
    from oracle import dgl_udf
    G, ug, (Xw, Xs, T, Td), w2s, s2w, p1, p2 = _setup(6, 8)
    dev = torch.device("cuda")
    Xwd, Xsd = Xw.to(dev), Xs.to(dev).requires_grad_()
    assert fused_stack_ok(G, w2s, s2w, Td, Xwd, Xsd)
    s = gat_stack(G, w2s, s2w, Td, Xwd, Xsd, 2)
    s.sum().backward()                                   # the column outlives the backward
    dgl_udf.stack_step(ug, Xw, Xs, p1, p2, T, n_iter=2)
    e = G.edata["e"].cpu()
    err = (e - ug.e).abs().max().item()
    print(f"fused stack edata['e'] max|diff| {err:.3e}")
    assert ug.e.abs().max() > 0 and err <= 1e-4
    # the typed rows only; every other edge keeps the zero initializer
    typed = np.zeros(len(e), bool)
    for kind in ("W2S", "S2W"):
        typed[G.relation(kind).dev["eid"].cpu().numpy()] = True
    assert not e[torch.from_numpy(~typed)].any()
