"""Work lists of degree-skewed relations (round 6).

The HDSG batch (config 4) gives each of its doc supernodes ~250 word edges
(/root/reference/module/dataloader.py:387-400) next to ~20 per sentence, so the
edge kernels that walk a node per block (the W2S forward over destinations, the
one-pass S2W backward over sources) ran at the pace of the doc nodes.  hsg_rel_work
splits such segments into pieces; k_gat_fwd / k_gat_bwd_src_g walk the pieces and a
merge launch combines them in a fixed order.  Checked here:

* the device work list equals its host restatement (rule written in the test);
* the pieced forward and backward equal the whole-node kernels (no work list) to fp32
  rounding, on the full cfg4 relations and on a ragged relation with empty
  destinations, phantoms on long nodes and one very long segment;
* deterministic: two runs bitwise equal.
The full cfg4 stack and model goldens (test_gpu_stack_parity.py, test_gpu_model.py)
run through the same work lists against the fp64 oracle / the reference.
"""
import ctypes

import numpy as np
import pytest
import torch

from helpers import build_graph, synth_fixture

pytestmark = pytest.mark.gpu


def host_work_list(indptr, pmin=32, mult=1):
    """Restatement of hsg_rel_work (include/hsg.h): P = max(pmin, mult * ceil(E / n));
    a node with deg > P -> ceil(deg / P) near-equal pieces (the first deg % k one
    longer), coded -(v + 1); others one item; each item (code, beg, end, first item of
    the node); empty list when no node is long."""
    n = len(indptr) - 1
    E = int(indptr[-1])
    P = max(pmin, mult * (-(-E // n)))
    items, long_ = [], False
    for v in range(n):
        b, e = int(indptr[v]), int(indptr[v + 1])
        deg = e - b
        first = len(items)
        if deg > P:
            long_ = True
            k = -(-deg // P)
            q, r = divmod(deg, k)
            for p in range(k):
                pb = b + p * q + min(p, r)
                items.append((-(v + 1), pb, pb + q + (1 if p < r else 0), first))
        else:
            items.append((v, b, e, first))
    return np.array(items, np.int32).reshape(-1, 4) if long_ else np.zeros((0, 4), np.int32)


def dev_items(t):
    """(items [n, 4], counters [n]) of a relation's flat device work list."""
    a = t.cpu().numpy()
    n = len(a) // 5
    return a[:4 * n].reshape(n, 4), a[4 * n:]


def cfg4_relations():
    from hetersumgraph_amd import synth
    docs = synth.make_batch_docs("cfg4", seed=0)
    G = build_graph(synth_fixture(docs)).to("cuda")
    return G.relation("W2S"), G.relation("S2W")


def test_cfg4_work_lists_match_host_restatement():
    rw, rs = cfg4_relations()
    # W2S: long destinations (docs) -> dwork; S2W: long sources (docs) -> swork
    for rel, key, ptr_key in ((rw, "dwork", "indptr"), (rs, "swork", "cindptr")):
        ref = host_work_list(rel.dev[ptr_key].cpu().numpy())
        assert len(ref) > 0
        got, cnt = dev_items(rel.dev[key])
        assert np.array_equal(got, ref)
        assert not cnt.any()                                  # arrival counters start at 0
        n_long = len(set(-c - 1 for c in ref[:, 0] if c < 0))
        assert n_long == 96                                   # 32 examples x 3 docs
    # the other directions have no long segment (words: <= 9 edges)
    assert "swork" not in rw.dev and "dwork" not in rs.dev
    c = rw.cstruct()
    assert c.n_dwork == len(rw.dev["dwork"]) // 5 and c.n_swork == 0


def test_no_work_list_without_skew():
    from hetersumgraph_amd import synth
    for cfg in ("cfg2", "cfg5"):
        G = build_graph(synth_fixture(synth.make_batch_docs(cfg, seed=0))).to("cuda")
        for kind in ("W2S", "S2W"):
            r = G.relation(kind)
            assert "dwork" not in r.dev and "swork" not in r.dev, (cfg, kind)


def _fwd(rel, H, D, Z, sigma, tau, origin, ws):
    from hetersumgraph_amd._lib import HSG_TAU_TABLE, check, load, ptr, stream_of
    lib = load()
    relp = ctypes.byref(rel.cstruct())
    n = rel.n_dst
    h, out = Z.new_empty(n, H * D), Z.new_empty(n, H * D)
    m, l = Z.new_empty(n, H), Z.new_empty(n, H)
    w = None
    if ws:
        nf = lib.hsg_gat_fwd_ws_floats(relp, H, D)
        assert nf > 0
        w = Z.new_empty(nf)
    check(lib.hsg_gat_fwd_ws(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(origin), ptr(h),
                             ptr(out), ptr(m), ptr(l), ptr(w), stream_of(Z)), "hsg_gat_fwd_ws")
    torch.cuda.synchronize()
    return h, out, m, l


def check_counters(t, inline=True):
    """The arrival counters of the in-kernel piece merge after complete launches: at a
    long node's first-piece slot a multiple of its piece count (positive when the
    launches merged in-kernel), 0 elsewhere."""
    items, cnt = dev_items(t)
    firsts = items[:, 3]
    for i in range(len(items)):
        if items[i, 0] < 0 and firsts[i] == i:
            np_ = int((items[:, 0] == items[i, 0]).sum())
            assert cnt[i] % np_ == 0 and (cnt[i] > 0) == inline, (i, cnt[i], np_)
        else:
            assert cnt[i] == 0, (i, cnt[i])


def _check_fwd(rel, H, D, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    Z = torch.randn(rel.n_src, H * D, device="cuda", generator=g)
    sigma = torch.randn(rel.n_src, H, device="cuda", generator=g)
    tau = torch.randn(11, H, device="cuda", generator=g)
    origin = torch.randn(rel.n_dst, H * D, device="cuda", generator=g)
    a = _fwd(rel, H, D, Z, sigma, tau, origin, ws=False)
    b = _fwd(rel, H, D, Z, sigma, tau, origin, ws=True)
    b2 = _fwd(rel, H, D, Z, sigma, tau, origin, ws=True)
    for x, y, y2, name in zip(a, b, b2, ("h", "out", "m", "l")):
        assert torch.equal(y, y2), name                       # deterministic
        err = ((x - y).abs() / (x.abs() + 1)).max().item()
        assert err <= 2e-6, (name, err)
    check_counters(rel.dev["dwork"])


def test_pieced_forward_equals_whole_nodes_cfg4():
    rw, _ = cfg4_relations()
    _check_fwd(rw, 8, 8, 1)                                    # the W2S shape (narrow rows)


def skewed_relation():
    """Ragged: empty destinations, one 1,000-edge segment, long nodes with phantoms,
    short ones; its CSC the same for the source side."""
    from hetersumgraph_amd.relation import Relation
    rng = np.random.default_rng(5)
    n_src, n_dst = 300, 120
    deg = rng.integers(0, 12, size=n_dst)
    deg[[3, 40, 41, 100]] = [1000, 300, 95, 0]
    deg[7] = 0
    e_dst = np.repeat(np.arange(n_dst), deg)
    e_src = np.concatenate([rng.choice(n_src, size=min(d, n_src), replace=False) if d <= n_src else
                            rng.integers(0, n_src, size=d) for d in deg])
    # the source side skewed too: a few sources take a quarter of the edges
    hot = rng.random(len(e_src)) < 0.25
    e_src[hot] = rng.choice([5, 6, 250], size=hot.sum())
    tf = rng.integers(0, 11, size=len(e_dst)).astype(np.uint8)
    phantom = rng.integers(0, 4, size=n_dst)
    phantom[3] = 160
    indptr = np.concatenate([[0], np.cumsum(deg)])
    corder = np.argsort(e_src, kind="stable")
    cindptr = np.concatenate([[0], np.cumsum(np.bincount(e_src, minlength=n_src))])
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    rel = Relation("S2W", n_src, n_dst, np.arange(n_src), np.arange(n_dst), i32(indptr), i32(e_src), tf,
                   np.arange(len(e_src)), i32(phantom), i32(cindptr), i32(e_dst[corder]), i32(corder),
                   len(e_src) + phantom.sum())
    return rel.to("cuda"), indptr, cindptr


def test_pieced_forward_equals_whole_nodes_ragged():
    rel, indptr, cindptr = skewed_relation()
    assert np.array_equal(dev_items(rel.dev["dwork"])[0], host_work_list(indptr))
    assert np.array_equal(dev_items(rel.dev["swork"])[0], host_work_list(cindptr))
    for H, D in ((8, 8), (6, 50), (4, 16)):
        _check_fwd(rel, H, D, H * D)


def _bwd(rel, H, D, args, ws, g_bf16=False):
    from hetersumgraph_amd._lib import check, load, ptr, stream_of
    lib = load()
    relp = ctypes.byref(rel.cstruct())
    sigma, tau, m, l, G, rho, groups, a1, Z = args
    nb = lib.hsg_gat_bwd_src_g_blocks(relp, H, D)
    dZ, dsig = torch.empty_like(Z), Z.new_empty(rel.n_src, H)
    da1p, dtp = Z.new_zeros(nb, H * D), Z.new_zeros(nb, 11, H)
    w = None
    if ws:
        nf = lib.hsg_gat_bwd_src_g_ws_floats(relp, H, D)
        assert nf > 0
        w = Z.new_empty(nf)
    check(lib.hsg_gat_bwd_src_g_ws(relp, H, D, 0.01, ptr(sigma), ptr(tau), ptr(m), ptr(l), ptr(G), int(g_bf16),
                                   ptr(rho), groups, ptr(a1), ptr(Z), ptr(dZ), ptr(dsig), ptr(da1p), ptr(dtp), ptr(w),
                                   stream_of(Z)), "hsg_gat_bwd_src_g_ws")
    torch.cuda.synchronize()
    return dZ, dsig, da1p.sum(0), dtp.sum(0)


def _check_bwd(rel, H, D, seed, g_bf16=False):
    from hetersumgraph_amd._lib import load
    gen = torch.Generator(device="cuda").manual_seed(seed)
    rn = lambda *s: torch.randn(*s, device="cuda", generator=gen)
    HD = H * D
    groups = (HD + 63) // 64
    G = rn(rel.n_dst, HD)
    if g_bf16:
        G = G.bfloat16()
    args = (rn(rel.n_src, H), rn(11, H), rn(rel.n_dst, H), rn(rel.n_dst, H).abs() + 1.0, G,
            rn(rel.n_dst, groups, 3), groups, rn(H, D), rn(rel.n_src, HD))
    assert load().hsg_gat_bwd_src_g_supported(ctypes.byref(rel.cstruct()), H, D)
    a = _bwd(rel, H, D, args, ws=False, g_bf16=g_bf16)
    b = _bwd(rel, H, D, args, ws=True, g_bf16=g_bf16)
    b2 = _bwd(rel, H, D, args, ws=True, g_bf16=g_bf16)
    for x, y, y2, name in zip(a, b, b2, ("dZ", "dsigma", "da1", "dtau")):
        assert torch.equal(y, y2), name
        err = ((x - y).abs().max() / (x.abs().max() + 1e-6)).item()
        assert err <= (2e-6 if name in ("dZ", "dsigma") else 1e-5), (name, err)   # block sums: other order
    check_counters(rel.dev["swork"], inline=False)      # the backward's pieces: merged by a second launch


@pytest.mark.parametrize("g_bf16", [False, True])
def test_pieced_backward_equals_whole_sources_cfg4(g_bf16):
    _, rs = cfg4_relations()
    _check_bwd(rs, 6, 50, 3, g_bf16)                           # the S2W shape


def test_pieced_backward_equals_whole_sources_ragged():
    rel, _, _ = skewed_relation()
    for H, D in ((6, 50), (8, 32), (2, 64)):
        _check_bwd(rel, H, D, H + D)


@pytest.mark.parametrize("mode", ["0", "3"])
def test_piece_merge_modes_bitwise_equal(monkeypatch, mode):
    """The pieces merged by a second launch (HSG_PIECE_INLINE=0), in-kernel by the last
    arriving block in both directions (3), and the default (forward in-kernel, backward
    second launch) run the same merge code in the same piece order: bitwise equal
    outputs (dev library: the switch is read there only)."""
    from helpers import skip_unless_dev
    skip_unless_dev(False)
    _, rs = cfg4_relations()
    rw, _ = cfg4_relations()
    gen = torch.Generator(device="cuda").manual_seed(9)
    rn = lambda *s: torch.randn(*s, device="cuda", generator=gen)
    fa = (rn(rw.n_src, 64), rn(rw.n_src, 8), rn(11, 8), rn(rw.n_dst, 64))
    HD, groups = 300, 5
    ba = (rn(rs.n_src, 6), rn(11, 6), rn(rs.n_dst, 6), rn(rs.n_dst, 6).abs() + 1.0, rn(rs.n_dst, HD),
          rn(rs.n_dst, groups, 3), groups, rn(6, 50), rn(rs.n_src, HD))
    ref = (_fwd(rw, 8, 8, *fa, ws=True), _bwd(rs, 6, 50, ba, ws=True))
    monkeypatch.setenv("HSG_PIECE_INLINE", mode)
    got = (_fwd(rw, 8, 8, *fa, ws=True), _bwd(rs, 6, 50, ba, ws=True))
    for r, g in zip(ref, got):
        for x, y in zip(r, g):
            assert torch.equal(x, y)
    check_counters(rw.dev["dwork"])
    check_counters(rs.dev["swork"], inline=mode == "3")
