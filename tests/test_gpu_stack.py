"""The fused WSWGAT stack (hetersumgraph_amd.stack: W2S + n_iter x (S2W, W2S) as
one autograd node, gradients summed in the kernels' epilogues) against the same
stack run layer by layer through WSWGAT.forward and autograd (HSG_FUSED_STACK=0).

Both paths launch the same kernels in the same order and draw the same dropout
masks (one RNG offset per dropout call, in call order), so outputs and every
gradient agree to fp32 summation-order noise -- checked in train mode (dropout
0.1), eval mode, with gradients accumulated over two backward passes, with and
without a gradient for the word features, and on an HDSG batch (doc nodes).
"""
import numpy as np
import pytest
import torch

from hetersumgraph_amd import _lib

pytestmark = pytest.mark.gpu


def _graph(kind, seed):
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    rng = np.random.default_rng(seed)
    if kind == "hsg":
        docs = [synth.make_hsg_doc(rng, N=9, W=60, k=7, k_jitter=3, isolated_words=2, tf_range=(0.0, 1.0)),
                synth.make_hsg_doc(rng, N=5, W=40, k=6, tf_range=(0.0, 1.0)),
                synth.make_hsg_doc(rng, N=12, W=80, k=9, tf_range=(0.0, 1.0))]
    else:
        docs = [synth.make_hdsg_example(rng, [5, 4, 6], W=70, k=6, doc_words=25),
                synth.make_hdsg_example(rng, [3, 7], W=50, k=5, doc_words=20)]
    G = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    G.to(torch.device("cuda"))
    return G


def _modules(seed, drop):
    from hetersumgraph_amd.module.GAT import WSWGAT
    torch.manual_seed(seed)
    w2s = WSWGAT(300, 64, 8, drop, 512, drop, 50, "W2S").cuda()
    s2w = WSWGAT(64, 300, 6, drop, 512, drop, 50, "S2W").cuda()
    T = torch.nn.Parameter(torch.randn(10, 50, device="cuda"))
    return w2s, s2w, T


def _run(G, w2s, s2w, T, Xw, Xs, R, n_iter, fused, reps=1):
    from hetersumgraph_amd import rng
    from hetersumgraph_amd.HiGraph import register_tfidf_table
    from hetersumgraph_amd.stack import fused_stack_ok, gat_stack
    rng.manual_seed(1234)
    register_tfidf_table(G, T)
    outs = []
    for _ in range(reps):
        assert fused_stack_ok(G, w2s, s2w, T, Xw, Xs)
        if fused:
            s = gat_stack(G, w2s, s2w, T, Xw, Xs, n_iter)
        else:
            w, s = Xw, w2s(G, Xw, Xs)
            for _ in range(n_iter):
                w = s2w(G, w, s)
                s = w2s(G, w, s)
        s.backward(R)
        outs.append(s.detach().clone())
    params = list(w2s.parameters()) + list(s2w.parameters()) + [T]
    grads = [None if p.grad is None else p.grad.detach().clone() for p in params]
    return outs, grads, [None if x.grad is None else x.grad.detach().clone() for x in (Xw, Xs)]


def _zero(mods, T, Xw, Xs):
    for m in mods:
        m.zero_grad(set_to_none=True)
    for t in (T, Xw, Xs):
        t.grad = None


@pytest.mark.parametrize("kind,train,word_grad,reps,n_iter,noh", [
    ("hsg", True, False, 1, 2, 2), ("hsg", True, True, 2, 2, 2), ("hsg", False, True, 1, 1, 2),
    ("hdsg", True, True, 1, 2, 2), ("hsg", True, False, 1, 3, 2),
    # the fused stack's S2W edge pass with a stored h and G made in the dst pass
    # (HSG_GAT_GEPI=0), and without h with G from x - origin in the dst pass
    # (hsg_gat_bwd_dst_noh), against the layer-wise path, which keeps h; noh = 2 is the
    # default: no h, G from the FFN's last GEMM epilogue (hsg_gemm_f32_psw_elug +
    # hsg_gat_bwd_dst_g)
    ("hsg", True, True, 2, 2, 0), ("hsg", True, False, 1, 2, 0),
    ("hsg", True, True, 2, 2, 1), ("hdsg", True, True, 1, 2, 1), ("hsg", False, True, 1, 1, 1)])
def test_fused_stack_matches_layerwise(monkeypatch, kind, train, word_grad, reps, n_iter, noh):
    monkeypatch.setitem(_lib._OPTIONS, "HSG_GAT_NOH", str(int(noh == 1)))
    monkeypatch.setitem(_lib._OPTIONS, "HSG_GAT_GEPI", str(int(noh == 2)))
    G = _graph(kind, 3)
    w2s, s2w, T = _modules(7, 0.1)
    for m in (w2s, s2w):
        m.train(train)
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device="cuda").manual_seed(5)
    Xw = (0.4 * torch.randn(rel_s.n_dst, 300, device="cuda", generator=gen)).requires_grad_(word_grad)
    Xs = torch.randn(rel_w.n_dst, 64, device="cuda", generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device="cuda", generator=gen)
    monkeypatch.setitem(_lib._OPTIONS, "HSG_FUSED_STACK", "1")
    fo, fg, fx = _run(G, w2s, s2w, T, Xw, Xs, R, n_iter, fused=True, reps=reps)
    _zero((w2s, s2w), T, Xw, Xs)
    lo, lg, lx = _run(G, w2s, s2w, T, Xw, Xs, R, n_iter, fused=False, reps=reps)
    for a, b in zip(fo, lo):
        assert (a - b).abs().max().item() <= 1e-5
    names = [n for n, _ in w2s.named_parameters()] + [n for n, _ in s2w.named_parameters()] + ["T"]
    for name, a, b in zip(names, fg, lg):
        assert (a is None) == (b is None), name
        if a is None:
            continue
        scale = max(b.abs().max().item(), 1e-6)
        assert (a - b).abs().max().item() <= 1e-5 * max(scale, 1.0), (name, (a - b).abs().max().item(), scale)
    for name, a, b in zip(("Xw", "Xs"), fx, lx):
        assert (a is None) == (b is None), name
        if a is not None:
            scale = max(b.abs().max().item(), 1e-6)
            assert (a - b).abs().max().item() <= 1e-5 * max(scale, 1.0), name
    if not word_grad:
        assert fx[0] is None


def test_fused_stack_is_used_by_hsumgraph(monkeypatch):
    """HSumGraph.gat_stack takes the fused node when it can (and the per-layer
    loop when HSG_FUSED_STACK=0): the output's grad_fn tells which ran."""
    G = _graph("hsg", 4)
    w2s, s2w, T = _modules(8, 0.1)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.word2sent, self.sent2word, self._n_iter = w2s, s2w, 2
            self._TFembed = torch.nn.Embedding(10, 50).cuda()

    from hetersumgraph_amd.HiGraph import HSumGraph, register_tfidf_table
    m = M()
    register_tfidf_table(G, m._TFembed.weight)
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    Xw = torch.randn(rel_s.n_dst, 300, device="cuda")
    Xs = torch.randn(rel_w.n_dst, 64, device="cuda", requires_grad=True)
    s = HSumGraph.gat_stack(m, G, Xw, Xs)
    assert type(s.grad_fn).__name__.startswith("_GatStack")
    monkeypatch.setitem(_lib._OPTIONS, "HSG_FUSED_STACK", "0")
    s = HSumGraph.gat_stack(m, G, Xw, Xs)
    assert not type(s.grad_fn).__name__.startswith("_GatStack")


def _eval_setup(seed=5):
    G = _graph("hsg", seed)
    w2s, s2w, T = _modules(seed + 4, 0.1)
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device="cuda").manual_seed(seed)
    Xw = (0.4 * torch.randn(rel_s.n_dst, 300, device="cuda", generator=gen)).requires_grad_()
    Xs = torch.randn(rel_w.n_dst, 64, device="cuda", generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device="cuda", generator=gen)
    from hetersumgraph_amd.HiGraph import register_tfidf_table
    register_tfidf_table(G, T)
    return G, w2s, s2w, T, Xw, Xs, R


def test_fused_stack_is_an_ordinary_autograd_node(monkeypatch):
    """Parameter gradients come back through autograd: autograd.grad
    leaves every .grad untouched and matches the layer-wise path, backward(inputs=)
    writes only the requested leaves, and post-accumulate-grad hooks fire."""
    from hetersumgraph_amd.stack import gat_stack
    G, w2s, s2w, T, Xw, Xs, R = _eval_setup()
    for m in (w2s, s2w):
        m.eval()
    params = list(w2s.parameters()) + list(s2w.parameters()) + [T]
    want = [Xs, w2s.ffn.w_1.weight, s2w.layer.fc_weight, T]
    s = gat_stack(G, w2s, s2w, T, Xw, Xs, 2)
    got = torch.autograd.grad((s * R).sum(), want)
    assert all(p.grad is None for p in params) and Xw.grad is None and Xs.grad is None
    monkeypatch.setitem(_lib._OPTIONS, "HSG_FUSED_STACK", "0")
    w, s = Xw, w2s(G, Xw, Xs)
    for _ in range(2):
        w = s2w(G, w, s)
        s = w2s(G, w, s)
    ref = torch.autograd.grad((s * R).sum(), want)
    for a, b in zip(got, ref):
        assert (a - b).abs().max().item() <= 1e-5 * max(b.abs().max().item(), 1.0)
    monkeypatch.setitem(_lib._OPTIONS, "HSG_FUSED_STACK", "1")
    s = gat_stack(G, w2s, s2w, T, Xw, Xs, 2)
    s.backward(R, inputs=[Xs])
    assert Xs.grad is not None and all(p.grad is None for p in params) and Xw.grad is None
    fired = []
    hs = [p.register_post_accumulate_grad_hook(lambda p: fired.append(id(p))) for p in params]
    s = gat_stack(G, w2s, s2w, T, Xw, Xs, 2)
    s.backward(R)
    for h in hs:
        h.remove()
    assert sorted(fired) == sorted(id(p) for p in params)
    assert torch.equal(Xs.grad, 2 * got[0]) or (Xs.grad - 2 * got[0]).abs().max().item() <= 1e-5


def test_dropout_masks_survive_reseed_between_forward_and_backward():
    """The backward regenerates the FFN dropout masks from a seed SNAPSHOT taken at
    forward time: advancing or reseeding the stream between forward and
    backward leaves every gradient bitwise unchanged."""
    from hetersumgraph_amd import rng
    from hetersumgraph_amd.stack import gat_stack
    G, w2s, s2w, T, Xw, Xs, R = _eval_setup(6)
    params = list(w2s.parameters()) + list(s2w.parameters()) + [T]
    grads = []
    for meddle in (False, True):
        for p in params + [Xw, Xs]:
            p.grad = None
        rng.manual_seed(4321)
        s = gat_stack(G, w2s, s2w, T, Xw, Xs, 2)
        if meddle:
            rng.advance_all()
            rng.manual_seed(99)
            gat_stack(G, w2s, s2w, T, Xw.detach(), Xs.detach(), 2)    # an unrelated forward in between
        s.backward(R)
        grads.append([p.grad.clone() for p in params] + [Xw.grad.clone(), Xs.grad.clone()])
    for a, b in zip(*grads):
        assert torch.equal(a, b)
