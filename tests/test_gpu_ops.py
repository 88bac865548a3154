"""Kernel-level checks of the C ABI ops (hsg_gat_fwd / bwd_dst / bwd_src /
attn_src_logits) through ``ops.gat_aggregate`` against the fp64 op restatement
``oracle.fused.gat_aggregate_ref`` (smooth inputs: no ReLU kinks involved)."""
import numpy as np
import pytest
import torch

from helpers import skip_unless_dev

pytestmark = pytest.mark.gpu


def random_relation(rng, n_src, n_dst, max_deg, phantom_max=3):
    from hetersumgraph_amd.relation import Relation
    deg = rng.integers(0, max_deg + 1, size=n_dst)
    e_dst = np.repeat(np.arange(n_dst), deg)
    e_src = np.concatenate([rng.choice(n_src, size=d, replace=False) if d <= n_src else
                            rng.integers(0, n_src, size=d) for d in deg]) if deg.sum() else np.zeros(0, int)
    tf = rng.integers(0, 11, size=len(e_dst)).astype(np.uint8)
    phantom = rng.integers(0, phantom_max + 1, size=n_dst)
    indptr = np.concatenate([[0], np.cumsum(deg)])
    corder = np.argsort(e_src, kind="stable")
    cindptr = np.concatenate([[0], np.cumsum(np.bincount(e_src, minlength=n_src))])
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    rel = Relation("W2S", n_src, n_dst, np.arange(n_src), np.arange(n_dst), i32(indptr), i32(e_src), tf,
                   np.arange(len(e_src)), i32(phantom), i32(cindptr), i32(e_dst[corder]), i32(corder),
                   len(e_src) + phantom.sum())
    return rel, e_src, e_dst, tf, phantom


@pytest.mark.parametrize("H,D,max_deg,origin,per_edge", [
    (8, 8, 40, True, False), (6, 50, 5, True, False), (6, 50, 90, True, False), (8, 8, 150, False, False),
    (1, 64, 10, True, False), (16, 4, 70, True, True), (3, 16, 20, False, True), (6, 50, 3, True, True)])
def test_gat_aggregate_matches_op_restatement(H, D, max_deg, origin, per_edge):
    from hetersumgraph_amd.ops import gat_aggregate, HSG_TAU_PER_EDGE, HSG_TAU_TABLE
    from oracle.fused import gat_aggregate_ref
    rng = np.random.default_rng(H * 1000 + D + max_deg)
    n_src, n_dst = 97, 61
    rel, e_src, e_dst, tf, phantom = random_relation(rng, n_src, n_dst, max_deg)
    reld = rel.to("cuda")
    Z = torch.randn(n_src, H * D, dtype=torch.float64)
    a1 = torch.randn(H, D, dtype=torch.float64) * 0.3
    ntau = len(e_src) if per_edge else 11
    tau = torch.randn(ntau, H, dtype=torch.float64)
    org = torch.randn(n_dst, H * D, dtype=torch.float64) if origin else None
    R = torch.randn(n_dst, H * D, dtype=torch.float64)
    leaves = [t.clone().requires_grad_() for t in (Z, a1, tau)] + ([org.clone().requires_grad_()] if origin else [])
    rows = np.arange(len(e_src)) if per_edge else tf
    ref = gat_aggregate_ref(e_src, e_dst, rows, phantom, n_dst, leaves[0], leaves[1], leaves[2],
                            leaves[3] if origin else None)
    (ref * R).sum().backward()
    dl = [t.float().cuda().requires_grad_() for t in (Z, a1, tau)] + (
        [org.float().cuda().requires_grad_()] if origin else [])
    out = gat_aggregate(dl[0], dl[1], dl[2], dl[3] if origin else None, reld, H, D,
                        tau_mode=HSG_TAU_PER_EDGE if per_edge else HSG_TAU_TABLE)
    (out * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    err = lambda a, b: (a.detach().cpu().double() - b.detach()).abs().max().item()
    assert err(out, ref) < 2e-5
    for name, got, want in zip(("Z", "a1", "tau", "origin"), dl, leaves):
        scale = want.grad.abs().max().item() + 1e-6
        assert err(got.grad, want.grad) <= 2e-5 * max(1.0, scale), (name, err(got.grad, want.grad), scale)


@pytest.mark.parametrize("lpn", ["16", "32", "64", "64-nopf"])
@pytest.mark.parametrize("H,D,skew,per_edge", [(6, 50, False, False), (6, 50, True, False), (8, 16, True, True),
                                               (1, 300, True, False), (16, 8, False, False)])
def test_forward_lanes_per_node_variants(monkeypatch, lpn, H, D, skew, per_edge):
    """Every forward work split (one destination per wave -- with the next
    destination's indptr prefetched (default) or not (HSG_GAT_FWD_PF=0) -- or 2 / 4
    per wave in LPN-lane groups, HSG_GAT_LPN) against the fp64 restatement, on short
    segments with a few long ones (skew: > 32 edges -> multi-chunk groups)."""
    from hetersumgraph_amd.ops import gat_aggregate, HSG_TAU_PER_EDGE, HSG_TAU_TABLE
    from hetersumgraph_amd.relation import Relation
    from oracle.fused import gat_aggregate_ref
    skip_unless_dev(lpn == "64")
    monkeypatch.setenv("HSG_GAT_LPN", lpn.split("-")[0])
    monkeypatch.setenv("HSG_GAT_FWD_PF", "0" if lpn.endswith("nopf") else "1")
    rng = np.random.default_rng(H * 31 + D + skew)
    n_src, n_dst = 150, 203
    deg = rng.integers(0, 4, size=n_dst)
    if skew:
        deg[rng.choice(n_dst, 5, replace=False)] = [33, 40, 64, 65, 100]
    e_dst = np.repeat(np.arange(n_dst), deg)
    e_src = rng.integers(0, n_src, size=len(e_dst))
    tf = rng.integers(0, 11, size=len(e_dst)).astype(np.uint8)
    phantom = rng.integers(0, 3, size=n_dst)
    indptr = np.concatenate([[0], np.cumsum(deg)])
    corder = np.argsort(e_src, kind="stable")
    cindptr = np.concatenate([[0], np.cumsum(np.bincount(e_src, minlength=n_src))])
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    rel = Relation("S2W", n_src, n_dst, np.arange(n_src), np.arange(n_dst), i32(indptr), i32(e_src), tf,
                   np.arange(len(e_src)), i32(phantom), i32(cindptr), i32(e_dst[corder]), i32(corder),
                   len(e_src) + phantom.sum()).to("cuda")
    f64 = dict(dtype=torch.float64)
    Z = torch.randn(n_src, H * D, **f64)
    a1 = torch.randn(H, D, **f64) * 0.3
    tau = torch.randn(len(e_src) if per_edge else 11, H, **f64)
    org = torch.randn(n_dst, H * D, **f64)
    R = torch.randn(n_dst, H * D, **f64)
    leaves = [t.clone().requires_grad_() for t in (Z, a1, tau, org)]
    rows = np.arange(len(e_src)) if per_edge else tf
    ref = gat_aggregate_ref(e_src, e_dst, rows, phantom, n_dst, *leaves)
    (ref * R).sum().backward()
    dl = [t.float().cuda().requires_grad_() for t in (Z, a1, tau, org)]
    out = gat_aggregate(*dl[:3], dl[3], rel, H, D, tau_mode=HSG_TAU_PER_EDGE if per_edge else HSG_TAU_TABLE)
    (out * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    err = lambda a, b: (a.detach().cpu().double() - b.detach()).abs().max().item()
    assert err(out, ref) < 2e-5
    for name, got, want in zip(("Z", "a1", "tau", "origin"), dl, leaves):
        scale = want.grad.abs().max().item() + 1e-6
        assert err(got.grad, want.grad) <= 2e-5 * max(1.0, scale), (name, err(got.grad, want.grad), scale)


def tau_table_ref(attn, T, wf, bf, D):
    """fp64 restatement of the edge-type term (GATLayer.py:84-93 / 123-131):
    tau[t, k] = attn_fc_k[2D:] . feat_fc_k(T[t]) for t < 10, row 10 = feat_fc_k(0)."""
    a3 = attn[:, 2 * D:]
    feat = torch.einsum("kdf,tf->tkd", wf, T)                       # [10, H, D]
    if bf is not None:
        feat = feat + bf
    rows = (feat * a3).sum(-1)                                      # [10, H]
    zero = (a3 * bf).sum(-1, keepdim=True).t() if bf is not None else torch.zeros(1, attn.shape[0],
                                                                                   dtype=attn.dtype)
    return torch.cat([rows, zero], 0)


@pytest.mark.parametrize("H,D,F,max_deg,bias", [(8, 8, 50, 40, False), (6, 50, 50, 5, True),
                                                 (3, 16, 20, 12, True), (16, 4, 7, 30, False)])
def test_gat_heads_table_matches_restatement(H, D, F, max_deg, bias):
    """The fused table path (hsg_attn_params_fwd/bwd + edge kernels) against the fp64
    composition tau_table_ref -> gat_aggregate_ref, outputs and every gradient."""
    from hetersumgraph_amd.ops import gat_heads_table
    from oracle.fused import gat_aggregate_ref
    rng = np.random.default_rng(7 * H + D + F)
    n_src, n_dst = 211, 77
    rel, e_src, e_dst, tf, phantom = random_relation(rng, n_src, n_dst, max_deg)
    reld = rel.to("cuda")
    f64 = dict(dtype=torch.float64)
    Z = torch.randn(n_src, H * D, **f64)
    attn = torch.randn(H, 3 * D, **f64) * 0.3
    T = torch.randn(10, F, **f64)
    wf = torch.randn(H, D, F, **f64) / F ** 0.5
    bf = torch.randn(H, D, **f64) * 0.2 if bias else None
    org = torch.randn(n_dst, H * D, **f64)
    R = torch.randn(n_dst, H * D, **f64)
    ins = [Z, attn, T, wf, bf, org]
    leaves = [t.clone().requires_grad_() if t is not None else None for t in ins]
    Zr, attnr, Tr, wfr, bfr, orgr = leaves
    tau = tau_table_ref(attnr, Tr, wfr, bfr, D)
    ref = gat_aggregate_ref(e_src, e_dst, tf, phantom, n_dst, Zr, attnr[:, :D], tau, orgr)
    (ref * R).sum().backward()
    dl = [t.float().cuda().requires_grad_() if t is not None else None for t in ins]
    out = gat_heads_table(dl[0], dl[1], dl[2], dl[3], dl[4], dl[5], reld, H, D)
    (out * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    err = lambda a, b: (a.detach().cpu().double() - b.detach()).abs().max().item()
    assert err(out, ref) < 2e-5
    for name, got, want in zip(("Z", "attn", "T", "wf", "bf", "origin"), dl, leaves):
        if want is None:
            continue
        scale = want.grad.abs().max().item() + 1e-6
        assert err(got.grad, want.grad) <= 2e-5 * max(1.0, scale), (name, err(got.grad, want.grad), scale)


@pytest.mark.parametrize("nq", ["0", "-1", "1", "2", "3", "5", "8"])
@pytest.mark.parametrize("H,D,dense_band,per_edge", [(6, 50, False, False), (6, 50, True, False), (4, 3, True, False),
                                                     (1, 300, False, True), (16, 8, True, False), (2, 2, False, False)])
def test_forward_row_tile_variants(monkeypatch, nq, H, D, dense_band, per_edge):
    """The row-tile forward (k_gat_fwd_rows, float4 slots, HSG_GAT_ROWS = slots per
    thread; 0 = one destination per wave) against the fp64 restatement.  dense_band
    puts 24 consecutive destinations of 100 in-edges each among short segments, so a
    block's edge range exceeds the 512-edge LDS chunk and later chunks recompute
    their alphas; D = 3 and D = 2 put two heads into one float4 slot."""
    from hetersumgraph_amd.ops import gat_aggregate, HSG_TAU_PER_EDGE, HSG_TAU_TABLE
    from hetersumgraph_amd.relation import Relation
    from oracle.fused import gat_aggregate_ref
    skip_unless_dev(nq == "0")
    monkeypatch.setenv("HSG_GAT_ROWS", nq)
    rng = np.random.default_rng(H * 17 + D + dense_band)
    n_src, n_dst = 120, 700
    deg = rng.integers(0, 4, size=n_dst)
    if dense_band:
        deg[300:324] = 100
    e_dst = np.repeat(np.arange(n_dst), deg)
    e_src = rng.integers(0, n_src, size=len(e_dst))
    tf = rng.integers(0, 11, size=len(e_dst)).astype(np.uint8)
    phantom = rng.integers(0, 3, size=n_dst)
    indptr = np.concatenate([[0], np.cumsum(deg)])
    corder = np.argsort(e_src, kind="stable")
    cindptr = np.concatenate([[0], np.cumsum(np.bincount(e_src, minlength=n_src))])
    i32 = lambda a: np.ascontiguousarray(a, np.int32)
    rel = Relation("S2W", n_src, n_dst, np.arange(n_src), np.arange(n_dst), i32(indptr), i32(e_src), tf,
                   np.arange(len(e_src)), i32(phantom), i32(cindptr), i32(e_dst[corder]), i32(corder),
                   len(e_src) + phantom.sum()).to("cuda")
    f64 = dict(dtype=torch.float64)
    Z = torch.randn(n_src, H * D, **f64)
    a1 = torch.randn(H, D, **f64) * 0.3
    tau = torch.randn(len(e_src) if per_edge else 11, H, **f64)
    org = torch.randn(n_dst, H * D, **f64)
    R = torch.randn(n_dst, H * D, **f64)
    leaves = [t.clone().requires_grad_() for t in (Z, a1, tau, org)]
    rows = np.arange(len(e_src)) if per_edge else tf
    ref = gat_aggregate_ref(e_src, e_dst, rows, phantom, n_dst, *leaves)
    (ref * R).sum().backward()
    dl = [t.float().cuda().requires_grad_() for t in (Z, a1, tau, org)]
    out = gat_aggregate(*dl[:3], dl[3], rel, H, D, tau_mode=HSG_TAU_PER_EDGE if per_edge else HSG_TAU_TABLE)
    (out * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    err = lambda a, b: (a.detach().cpu().double() - b.detach()).abs().max().item()
    assert err(out, ref) < 2e-5
    for name, got, want in zip(("Z", "a1", "tau", "origin"), dl, leaves):
        scale = want.grad.abs().max().item() + 1e-6
        assert err(got.grad, want.grad) <= 2e-5 * max(1.0, scale), (name, err(got.grad, want.grad), scale)


@pytest.mark.parametrize("hl", ["0", "1"])
@pytest.mark.parametrize("H,n_src,max_deg,per_edge", [(8, 300, 4, False), (8, 1000, 6, True), (5, 257, 3, False),
                                                     (8, 64, 20, False)])
def test_src_pass_head_lane_variant(monkeypatch, hl, H, n_src, max_deg, per_edge):
    """The head-lane src pass (k_gat_bwd_src_hl: D = 8, short CSC segments -- the W2S
    word sources) and the one-source-per-wave kernel (HSG_GAT_SRC_HL=0) against the
    fp64 restatement: sources without edges, H < nextpow2(H) (idle head lanes), odd
    segment lengths (the unpaired last edge), both tau modes."""
    from hetersumgraph_amd.ops import gat_aggregate, HSG_TAU_PER_EDGE, HSG_TAU_TABLE
    from oracle.fused import gat_aggregate_ref
    skip_unless_dev(hl == "1")
    monkeypatch.setenv("HSG_GAT_SRC_HL", hl)
    D = 8
    rng = np.random.default_rng(n_src + H + max_deg)
    rel, e_src, e_dst, tf, phantom = random_relation(rng, n_src, 40, max_deg * n_src // 40)
    reld = rel.to("cuda")
    f64 = dict(dtype=torch.float64)
    Z = torch.randn(n_src, H * D, **f64)
    a1 = torch.randn(H, D, **f64) * 0.3
    tau = torch.randn(len(e_src) if per_edge else 11, H, **f64)
    org = torch.randn(40, H * D, **f64)
    R = torch.randn(40, H * D, **f64)
    leaves = [t.clone().requires_grad_() for t in (Z, a1, tau, org)]
    rows = np.arange(len(e_src)) if per_edge else tf
    ref = gat_aggregate_ref(e_src, e_dst, rows, phantom, 40, *leaves)
    (ref * R).sum().backward()
    dl = [t.float().cuda().requires_grad_() for t in (Z, a1, tau, org)]
    out = gat_aggregate(*dl[:3], dl[3], reld, H, D, tau_mode=HSG_TAU_PER_EDGE if per_edge else HSG_TAU_TABLE)
    (out * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    err = lambda a, b: (a.detach().cpu().double() - b.detach()).abs().max().item()
    assert err(out, ref) < 2e-5
    for name, got, want in zip(("Z", "a1", "tau", "origin"), dl, leaves):
        scale = want.grad.abs().max().item() + 1e-6
        assert err(got.grad, want.grad) <= 2e-5 * max(1.0, scale), (name, err(got.grad, want.grad), scale)


def test_attn_tables_pair_equals_per_layer():
    """hsg_attn_params_fwd_pair (both layers' tables in one launch, the fused stack's
    forward) writes bitwise what two hsg_attn_params_fwd launches write (W2S-like
    layer without feat_fc bias, S2W-like layer with it)."""
    from types import SimpleNamespace
    from hetersumgraph_amd.ops import attn_tables, attn_tables_pair
    torch.manual_seed(5)
    dev = "cuda"
    T = torch.randn(10, 50, device=dev)
    l0 = SimpleNamespace(H=8, D=8, attn=torch.randn(8, 24, device=dev), wf=torch.randn(8, 8, 50, device=dev), bf=None)
    l1 = SimpleNamespace(H=6, D=50, attn=torch.randn(6, 150, device=dev), wf=torch.randn(6, 50, 50, device=dev),
                         bf=torch.randn(6, 50, device=dev))
    got = attn_tables_pair(l0, l1, T)
    for lay, (a1, tau) in zip((l0, l1), got):
        ra1, rtau = attn_tables(lay.attn, T, lay.wf, lay.bf, lay.H, lay.D)
        assert torch.equal(a1, ra1) and torch.equal(tau, rtau)


def test_dropmasks_with_weight_transpose():
    """hsg_dropmask_multi_wt: the masks are bitwise those of hsg_dropmask_multi and the
    folded weight transpose equals hsg_hproj_wt's."""
    from hetersumgraph_amd.hproj import dropmasks, transposed_weight
    dev = torch.device("cuda")
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    jobs = [(19200, 300, 8, 0.1, seed, 3), (1120, 64, 6, 0.1, seed, 7), (777, 300, 8, 0.1, seed, 11)]
    W = torch.randn(64, 300, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    ref = dropmasks(jobs, dev, st)
    got, Wt = dropmasks(jobs, dev, st, wt=(W, 8, 8))
    assert all(torch.equal(a, b) for a, b in zip(ref, got))
    assert torch.equal(Wt, transposed_weight(W, 8, 8))


@pytest.mark.parametrize("shared_dT,acc", [(True, (0, 2)), (False, (0, 0)), (True, (3, 3))])
def test_attn_params_finish_pair_equals_two_launches(shared_dT, acc):
    """hsg_attn_params_finish_pair (the stack backward's two layers in one launch)
    against two hsg_attn_params_finish launches in order: bitwise equal gradients,
    including the dT both layers write (layer 0's update first) and accumulation."""
    from types import SimpleNamespace
    from hetersumgraph_amd.ops import attn_params_finish, attn_params_finish_pair, attn_params_workspace
    torch.manual_seed(9)
    dev = "cuda"
    T = torch.randn(10, 50, device=dev)
    lays = [SimpleNamespace(H=8, D=8, attn=torch.randn(8, 24, device=dev), wf=torch.randn(8, 8, 50, device=dev),
                            bf=None),
            SimpleNamespace(H=6, D=50, attn=torch.randn(6, 150, device=dev), wf=torch.randn(6, 50, 50, device=dev),
                            bf=torch.randn(6, 50, device=dev))]
    wss = []
    for lay in lays:
        ws = attn_params_workspace(T, lay.H, lay.D)
        ws.copy_(torch.randn_like(ws))
        wss.append(ws)

    def dsts(dT_shared):
        out = []
        for q, lay in enumerate(lays):
            dT = dT_shared if dT_shared is not None else torch.randn_like(T)
            acc_T = bool(acc[q] & 2) or (dT_shared is not None and q == 1)
            out.append([torch.randn_like(lay.attn), torch.randn_like(lay.wf),
                        torch.randn_like(lay.bf) if lay.bf is not None else None, dT, bool(acc[q] & 1), acc_T])
        return out

    torch.manual_seed(1)
    d_ref = dsts(torch.randn_like(T) if shared_dT else None)
    torch.manual_seed(1)
    d_got = dsts(torch.randn_like(T) if shared_dT else None)
    for q, lay in enumerate(lays):
        attn_params_finish(wss[q], lay.attn, T, lay.wf, lay.bf, lay.H, lay.D, d_ref[q])
    attn_params_finish_pair((wss[0], lays[0], d_got[0]), (wss[1], lays[1], d_got[1]), T)
    torch.cuda.synchronize()
    for a, b in zip(d_ref, d_got):
        for x, y in zip(a[:4], b[:4]):
            if x is not None:
                assert torch.equal(x, y)


def test_step_prologue_weight_split_equals_hsg_wsplit():
    """hsg_step_prologue: the masks, the folded weight transpose AND the wide FFN's
    limb planes in one launch equal hsg_dropmask_multi / hsg_hproj_wt / hsg_wsplit."""
    from hetersumgraph_amd.dense import split_weights
    from hetersumgraph_amd.hproj import dropmasks, transposed_weight
    dev = torch.device("cuda")
    seed = torch.tensor([77], dtype=torch.int64, device=dev)
    jobs = [(19200, 300, 8, 0.1, seed, 3), (1120, 64, 6, 0.1, seed, 7)]
    W = torch.randn(64, 300, device=dev)
    w1, w2 = torch.randn(512, 300, device=dev), torch.randn(300, 512, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    specs = ((w1, False), (w2, False), (w2, True), (w1, True))
    ref_masks = dropmasks(jobs, dev, st)
    ref_split = split_weights(*specs)
    pre, job = split_weights(*specs, launch=False)
    got_masks, Wt = dropmasks(jobs, dev, st, wt=(W, 8, 8), wsplit_job=job)
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(ref_masks, got_masks))
    assert torch.equal(Wt, transposed_weight(W, 8, 8))
    for a, b in zip(ref_split, pre):
        assert torch.equal(a.planes, b.planes)
