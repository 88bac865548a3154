"""Pin the DGL-UDF-structured CPU baseline (oracle/dgl_udf.py, timed by bench.py
as cpu_baseline) to the reference's golden vectors."""
import numpy as np
import pytest
import torch

from helpers import concat_arrays, gat_inputs, load_fixture, seeded_gat_params, upstream
from oracle import dgl_udf, fused


@pytest.mark.parametrize("name,seed", [("gat_small", 1), ("gat_hdsg_small", 2), ("gat_cfg1", 3)])
def test_udf_path_matches_reference(name, seed):
    z = load_fixture(name)
    a = concat_arrays(z)
    g = dgl_udf.UdfGraph(a["src"], a["dst"], a["unit"], a["tffrac"], a["edtype"])
    Xw, Xs, T = gat_inputs(seed, int(z["n_w"]), int(z["n_s"]))
    Xs.requires_grad_()
    w2s, s2w = seeded_gat_params(seed * 100 + 1, seed * 100 + 2)
    p1 = fused.as_params(w2s, dtype=torch.float32)
    p2 = fused.as_params(s2w, dtype=torch.float32)
    te = dgl_udf.tfidf_embed(g, T)
    o1 = dgl_udf.wswgat(g, "W2S", Xw, Xs, p1, te)
    o2 = dgl_udf.wswgat(g, "S2W", Xw, Xs, p2, te)
    rows = z["rows_w"] if "rows_w" in z else slice(None)
    assert np.abs(o1.detach().numpy() - z["out_w2s"]).max() <= 2e-5
    assert np.abs(o2.detach().numpy()[rows] - z["out_s2w"]).max() <= 2e-5
    R1, R2 = upstream(seed, o1.shape, o2.shape)
    ((o1 * R1).sum() + (o2 * R2).sum()).backward()
    g64 = z["grad_Xs"]
    err = np.abs(Xs.grad.numpy() - g64)
    bad = (err.max(1) > 1e-4 * np.abs(g64).max()).sum()
    assert bad <= (2 if name == "gat_cfg1" else 0)


def test_stack_step_runs_fwd_bwd():
    from hetersumgraph_amd import synth
    docs = synth.make_batch_docs("cfg1", seed=0, n_docs=2)
    src = np.concatenate([d.src + o for d, o in zip(docs, np.cumsum([0] + [d.n_nodes for d in docs])[:-1])])
    dst = np.concatenate([d.dst + o for d, o in zip(docs, np.cumsum([0] + [d.n_nodes for d in docs])[:-1])])
    g = dgl_udf.UdfGraph(src, dst, np.concatenate([d.unit for d in docs]),
                         np.concatenate([d.tffrac for d in docs]), np.concatenate([d.edtype for d in docs]))
    Xw, Xs, T = gat_inputs(0, int((g.unit == 0).sum()), int((g.unit == 1).sum()))
    w2s, s2w = seeded_gat_params(1, 2)
    p1 = fused.as_params(w2s, dtype=torch.float32)
    p2 = fused.as_params(s2w, dtype=torch.float32)
    Xs.requires_grad_()
    s = dgl_udf.stack_step(g, Xw, Xs, p1, p2, T, n_iter=2, drop=0.1, training=True)
    s.sum().backward()
    assert torch.isfinite(Xs.grad).all()
