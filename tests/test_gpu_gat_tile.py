"""The destination-tile forward (k_gat_fwd_tile, round 6) against the per-destination
kernel it replaces for short segments (k_gat_fwd, one destination per wave):
bitwise-equal h / x, m and l, and bitwise-equal bf16 x rows.

It runs on full relations whose source windows behave differently:
* cfg2 S2W: 35 sentences per document, so a 48-row window covers each tile, except
  tiles that straddle two documents, which fall back to global rows;
* cfg5 S2W: 80 sentences per document, so many sources lie outside the window;
* cfg4 S2W: the sources are sentences and doc nodes.
It also runs on a ragged relation built with `oracle/fused.typed_relation` semantics
(empty destinations, long segments past the staged-edge cap).

Both kernels run in one process. The tile kernel is chosen with
`HSG_GAT_FWD_TILE=1`, which only the dev library reads; on the product library the
test checks the default kernel against itself.
"""
import ctypes

import numpy as np
import pytest
import torch

from helpers import build_graph, dev_lib, synth_fixture

pytestmark = pytest.mark.gpu


def _run(rel, H, D, Z, sigma, tau, origin, x16=False, keep_h=True):
    from hetersumgraph_amd._lib import HSG_TAU_TABLE, check, load, ptr, stream_of
    lib = load()
    relp = ctypes.byref(rel.cstruct())
    n, HD = rel.n_dst, H * D
    m, l = Z.new_empty(n, H), Z.new_empty(n, H)
    h = Z.new_empty(n, HD) if keep_h else None
    nf = lib.hsg_gat_fwd_ws_floats(relp, H, D)
    ws = Z.new_empty(nf) if nf else None
    if x16:
        ld = (HD + 7) // 8 * 8
        out = torch.full((n, ld), float("nan"), device="cuda").bfloat16()
        check(lib.hsg_gat_fwd_ws16(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(origin),
                                   ptr(h), None, ptr(m), ptr(l), ptr(ws), ptr(out), ld, stream_of(Z)), "ws16")
    else:
        out = Z.new_empty(n, HD)
        check(lib.hsg_gat_fwd_ws(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(origin),
                                 ptr(h), ptr(out), ptr(m), ptr(l), ptr(ws), stream_of(Z)), "ws")
    torch.cuda.synchronize()
    return h, out, m, l


def _compare(rel, H, D, seed, monkeypatch):
    g = torch.Generator(device="cuda").manual_seed(seed)
    HD = H * D
    Z = torch.randn(rel.n_src, HD, device="cuda", generator=g)
    sigma = torch.randn(rel.n_src, H, device="cuda", generator=g)
    tau = torch.randn(11, H, device="cuda", generator=g)
    origin = torch.randn(rel.n_dst, HD, device="cuda", generator=g)
    for x16 in (False, True):
        monkeypatch.setenv("HSG_GAT_FWD_TILE", "0")
        a = _run(rel, H, D, Z, sigma, tau, origin, x16=x16)
        monkeypatch.setenv("HSG_GAT_FWD_TILE", "1")
        b = _run(rel, H, D, Z, sigma, tau, origin, x16=x16)
        for p, q in zip(a, b):
            assert torch.equal(p, q), (x16, (p.float() - q.float()).abs().max().item())
        # no origin: h only
    monkeypatch.setenv("HSG_GAT_FWD_TILE", "0")
    a = _run(rel, H, D, Z, sigma, tau, None)
    monkeypatch.setenv("HSG_GAT_FWD_TILE", "1")
    b = _run(rel, H, D, Z, sigma, tau, None)
    assert torch.equal(a[0], b[0]) and torch.equal(a[2], b[2]) and torch.equal(a[3], b[3])


@pytest.mark.parametrize("config", ["cfg2", "cfg5", "cfg4"])
def test_tile_forward_bitwise_equal(config, monkeypatch):
    from hetersumgraph_amd import synth
    G = build_graph(synth_fixture(synth.make_batch_docs(config, seed=0))).to("cuda")
    rel = G.relation("S2W")
    if not dev_lib():
        monkeypatch.setenv("HSG_GAT_FWD_TILE", "0")
    _compare(rel, 6, 50, 17, monkeypatch)


def test_tile_forward_ragged(monkeypatch):
    """Empty destinations, one destination with 700 in-edges (past the 512 staged
    edges of its tile), sources scattered over the whole range (outside the window)."""
    from hetersumgraph_amd.relation import Relation, attach_work_lists  # noqa: F401
    from hetersumgraph_amd import graph as hg
    rng = np.random.default_rng(5)
    n_s, n_w = 300, 2000
    g = hg.DGLGraph()
    g.add_nodes(n_s + n_w)
    unit = np.concatenate([np.ones(n_s), np.zeros(n_w)]).astype(np.float32)
    g.ndata["unit"] = torch.from_numpy(unit)
    g.ndata["dtype"] = torch.from_numpy(unit.copy())
    src, dst = [], []
    for w in range(n_w):
        k = 0 if w % 7 == 0 else (700 if w == 1500 else int(rng.integers(1, 4)))
        ss = rng.choice(n_s, size=min(k, n_s), replace=False) if k <= n_s else rng.integers(0, n_s, size=k)
        src += list(ss)
        dst += [n_s + w] * len(ss)
    g.add_edges(src, dst)
    g.edata["dtype"] = torch.zeros(len(src))
    g.edata["tffrac"] = torch.from_numpy(rng.integers(0, 10, size=len(src)))
    g.to("cuda")
    rel = g.relation("S2W")
    assert rel.n_dst == n_w and rel.n_src == n_s
    _compare(rel, 6, 50, 23, monkeypatch)
