"""Fresh dropout masks on every replay of the captured step.

bench.py times HIP-graph replays of ``rng.advance_all()`` + the fused stack.  Since
round 5 the seed advance is no launch of its own: the forward's first kernel
(hsg_attn_params_fwd_pair_seed) performs it (rng.claim / claimed).  A replay that
re-used the captured seed would train every step on the same masks.  Here the stack
forward is captured once and replayed twice; after each replay the head-projection
keep bits the graph wrote and the FFN outputs must equal oracle/masks.py (the host
restatement pinned bit-exact in test_gpu_dropout_masks.py) at THAT replay's seed, the
second replay's seed must be the first's + 1, and the masks must differ
(GATStackLayer.py:56 head-input dropout, GATLayer.py:41 FFN dropout).
"""
import numpy as np
import pytest
import torch

from helpers import build_graph, gat_inputs, seeded_gat_params, synth_fixture

pytestmark = pytest.mark.gpu

P = 0.1


def _ln_ref(y, x, keep, scale, gamma, beta, eps):
    v = np.where(keep, y.astype(np.float64) * scale, 0.0) + x.astype(np.float64)
    mu = v.mean(1, keepdims=True)
    var = ((v - mu) ** 2).mean(1, keepdims=True)
    return (v - mu) / np.sqrt(var + eps) * gamma.astype(np.float64) + beta.astype(np.float64)


@pytest.mark.parametrize("attn_pair", ["1", "0"])
def test_graph_replays_draw_fresh_masks(attn_pair, monkeypatch):
    from hetersumgraph_amd import _lib, rng, synth
    from hetersumgraph_amd.HiGraph import register_tfidf_table
    from hetersumgraph_amd.stack import gat_stack
    from oracle import masks
    # "0": the tables launch without the seed fold, the advance runs as its own launch
    # (rng.take) -- both must draw fresh masks per replay
    monkeypatch.setitem(_lib._OPTIONS, "HSG_ATTN_PAIR", attn_pair)
    dev = torch.device("cuda")
    docs = synth.make_batch_docs("cfg2", seed=0)[:4]
    z = synth_fixture(docs)
    G = build_graph(z).to(dev)
    n_w, n_s = int(z["n_w"]), int(z["n_s"])
    Xw, Xs, T = (t.to(dev) for t in gat_inputs(5, n_w, n_s))
    T.requires_grad_()
    register_tfidf_table(G, T)
    w2s, s2w = seeded_gat_params(501, 502)
    w2s, s2w = w2s.to(dev).train(), s2w.to(dev).train()
    rng.manual_seed(9090)

    def fwd():
        rng.advance_all()
        return gat_stack(G, w2s, s2w, T, Xw, Xs, 2)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fwd()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = fwd()
    ctx = s.grad_fn
    apps = ctx.apps                        # (layer, saved, neighbour, origin, slot) per application
    assert [a[0].kind for a in apps] == ["W2S", "S2W", "W2S", "S2W", "W2S"]

    seen = []
    for _ in range(2):
        g.replay()
        torch.cuda.synchronize()
        rep = {}
        for i, (lay, saved, _, _, _) in enumerate(apps):
            hsaved, neighbor, _, fsaved = saved
            x, _, _, gamma, _, y, _, _, p, seed_t, off, _ = fsaved
            rep.setdefault("seed", int(seed_t.item()))
            assert int(seed_t.item()) == rep["seed"]            # one snapshot per step
            X, _, bits, H, _, ph = hsaved
            n, d_in = X.shape
            # head projection: drawn at offset off - 1 (head, then FFN, per application)
            ref = masks.pack_hproj_bits(masks.hproj_keep(rep["seed"], off - 1, n, d_in, H, ph))
            got = bits.cpu().numpy().reshape(ref.shape)
            assert np.array_equal(got, ref), (i, int((got != ref).sum()))
            rep[f"h{i}"] = got
            # FFN dropout: the application's output is the next one's neighbour (the last: s)
            out = (apps[i + 1][1][1] if i + 1 < len(apps) else s).detach().cpu().numpy()
            yn, xn = y.float().cpu().numpy(), x.cpu().numpy()
            keep = masks.ffn_keep(rep["seed"], off, *xn.shape, p)
            exp = _ln_ref(yn, xn, keep, masks.ffn_scale(p), gamma.detach().cpu().numpy(),
                          lay.beta.detach().cpu().numpy(), lay.eps)
            err = np.abs(out - exp).max()
            assert err <= 1e-4, (i, err)
            rep[f"f{i}"] = keep
        seen.append(rep)
    a, b = seen
    assert b["seed"] == a["seed"] + 1
    for i in range(len(apps)):
        assert not np.array_equal(a[f"h{i}"], b[f"h{i}"]), i
        assert not np.array_equal(a[f"f{i}"], b[f"f{i}"]), i
