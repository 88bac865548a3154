"""The edge layer's ELU gate fused into the FFN backward's last GEMM
(hsg_gemm_f32_psw_elug) and the dst pass that reads the resulting G rows
(hsg_gat_bwd_dst_g) -- GAT.py:56-57 backward (G = dOut * elu'(h)), GATLayer.py:95-102
backward -- against fp64 torch and against the dst pass that makes G itself."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(19200, 300, 512), (777, 300, 512), (130, 64, 96)])
def test_psw_elug_matches_fp64(M, N, K):
    from hetersumgraph_amd.dense import gemm_psw_elug, split_weights
    torch.manual_seed(M)
    dH = torch.randn(M, K, device="cuda")
    W1 = torch.randn(K, N, device="cuda") / K ** 0.5          # dx += dH W1: B = W1^T planes
    (S,) = split_weights((W1, True))
    ds = torch.randn(M, N, device="cuda")
    origin = torch.randn(M, N, device="cuda")
    h = 2 * torch.randn(M, N, device="cuda")
    h[::7] = 0.0                                               # elu' at the kink
    x = torch.nn.functional.elu(h) + origin
    out = ds.clone()
    G = torch.empty_like(ds)
    assert gemm_psw_elug(dH, S, out, x, origin, G)
    ref = ds.double() + dH.double() @ W1.double()
    e = (x.double() - origin.double())
    gref = torch.where(e > 0, ref, ref * (e + 1))
    assert (out.double() - ref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())
    # G against the exact gate exp(h): the rounding of x - origin moves it by ~ulp(x)
    gexact = torch.where(h.double() > 0, ref, ref * torch.exp(h.double()))
    assert (G.double() - gref).abs().max().item() <= 1e-4 * max(1.0, ref.abs().max().item())
    assert (G.double() - gexact).abs().max().item() <= 2e-4 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_psw_elug_gate_from_large_origin(mode):
    """the gate elu'(h) = exp(h) (h <= 0) comes from e = x - origin, so
    its absolute error is ~ulp(origin) whatever exp(h) is: relative accuracy of
    exp(h) is lost for strongly negative h beside a large residual.  Pinned here on
    rows with |origin| >> |elu(h)| (|origin| up to ~200, h down to -14) against
    fp64 dOut * elu'(h) from the TRUE h, in both GEMM modes.  Bound: the gate's
    error stays within 4 ulp(|x| + |origin|) (the fp32 rounding of x and of the
    subtraction) plus the roundings of e + 1 and of the product, i.e. |G - G_exact|
    <= |dOut| (4 * 2^-23 (|x| + |origin|) + 2^-23) + 2^-23 |G_exact|, with G_exact
    taken on the dx the kernel produced (its own error is pinned above)."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_psw_elug, split_weights
    M, N, K = 4096, 300, 512
    torch.manual_seed(7)
    dH = torch.randn(M, K, device="cuda")
    W1 = torch.randn(K, N, device="cuda") / K ** 0.5
    with gemm_dtype(mode):
        (S,) = split_weights((W1, True))
    assert S.mode == mode
    ds = torch.randn(M, N, device="cuda")
    origin = 50 * torch.randn(M, N, device="cuda")
    h = torch.empty(M, N, device="cuda").uniform_(-14.0, 2.0)
    x = torch.nn.functional.elu(h) + origin
    out = ds.clone()
    G = torch.empty_like(ds)
    assert gemm_psw_elug(dH, S, out, x, origin, G)
    if mode == "bf16":      # the GEMM itself on bf16-rounded operands (hsg_gemm_bf16 semantics)
        ref = ds.double() + dH.bfloat16().double() @ W1.bfloat16().double()
    else:
        ref = ds.double() + dH.double() @ W1.double()
    scale = max(1.0, ref.abs().max().item())
    tol_gemm = 1e-4 * scale if mode == "f32" else 2e-2 * scale
    assert (out.double() - ref).abs().max().item() <= tol_gemm
    gate = torch.where(h.double() > 0, torch.ones_like(ref), torch.exp(h.double()))
    gexact = out.double() * gate                 # the exact gate on the dx the kernel produced
    # e = x - origin carries <= 4 ulp(|x| + |origin|); e + 1 and the product v (e + 1)
    # each round once more (<= 2^-24 of 1 and of |G|)
    gate_err = 4 * 2.0 ** -23 * (x.double().abs() + origin.double().abs()) + 2.0 ** -23
    bound = out.double().abs() * gate_err + 2.0 ** -23 * gexact.abs() + 1e-12
    excess = ((G.double() - gexact).abs() - bound).max().item()
    neg = h < -8
    rel_neg = ((G.double() - gexact).abs() / gexact.abs().clamp_min(1e-30))[neg].max().item()
    print(f"{mode}: worst |G - G_exact| beyond bound {excess:.3e}; relative error of the gate at h < -8: "
          f"{rel_neg:.2e} (absolute, not relative, accuracy is the contract)")
    assert excess <= 0.0


def test_psw_elug_declines_unaligned():
    from hetersumgraph_amd.dense import gemm_psw_elug, split_weights
    W1 = torch.randn(64, 30, device="cuda")
    (S,) = split_weights((W1, True))                           # N = 30: not whole quads
    t = torch.randn(50, 30, device="cuda")
    assert not gemm_psw_elug(torch.randn(50, 64, device="cuda"), S, t.clone(), t, t, torch.empty_like(t))


def test_dst_pass_with_given_G_equals_noh_pass():
    """hsg_gat_bwd_dst_g with the G rows hsg_gat_bwd_dst_noh wrote: bitwise the same
    dpre and d tau partials (the same kernel body, G read instead of made)."""
    import ctypes
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd._lib import HSG_TAU_TABLE, load, ptr
    from hetersumgraph_amd.relation import N_BOX
    lib = load()
    rng = np.random.default_rng(3)
    docs = [synth.make_hsg_doc(rng, N=35, W=600, k=36) for _ in range(4)]
    G_ = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    G_.to(torch.device("cuda"))
    rel = G_.relation("S2W")
    relp = ctypes.byref(rel.cstruct())
    H, D = 6, 50
    assert lib.hsg_gat_bwd_dst_noh_supported(relp, H, D)
    torch.manual_seed(0)
    Z = torch.randn(rel.n_src, H * D, device="cuda")
    sigma = torch.randn(rel.n_src, H, device="cuda")
    tau = torch.randn(N_BOX + 1, H, device="cuda")
    m = torch.randn(rel.n_dst, H, device="cuda").abs()
    l = torch.rand(rel.n_dst, H, device="cuda") + 1
    x = torch.randn(rel.n_dst, H * D, device="cuda")
    org = torch.randn(rel.n_dst, H * D, device="cuda")
    dout = torch.randn(rel.n_dst, H * D, device="cuda")
    nb = lib.hsg_gat_bwd_blocks(relp)
    outs = []
    Gn = torch.empty_like(dout)
    for given in (False, True):
        dpre = torch.empty(rel.n_typed, H, device="cuda")
        dtp = torch.empty(nb, N_BOX + 1, H, device="cuda")
        if given:
            rc = lib.hsg_gat_bwd_dst_g(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(m), ptr(l),
                                       ptr(Gn), ptr(dpre), ptr(dtp), None)
        else:
            rc = lib.hsg_gat_bwd_dst_noh(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(x),
                                         ptr(org), ptr(m), ptr(l), ptr(dout), ptr(Gn), ptr(dpre), ptr(dtp), None)
        assert rc == 0
        torch.cuda.synchronize()
        outs.append((dpre, dtp))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


def _rho_ref(G, h, D, gw=64):
    """fp64 rho partials: [M, ceil(N/gw), 3], slot s of gw-column group g = the sum of
    G * h over the group's columns in head gw g // D + s (hsg_gemm_psw_elug_rho; gw = 64,
    or 112 on the fp32 mode's 112-wide dx tiles)."""
    M, N = G.shape
    ng = (N + gw - 1) // gw
    prod = G.double() * h.double()
    out = torch.zeros(M, ng, 3, dtype=torch.float64, device=G.device)
    for g in range(ng):
        hb = gw * g // D
        for s in range(3):
            cols = [c for c in range(gw * g, min(gw * g + gw, N)) if c // D == hb + s]
            if cols:
                out[:, g, s] = prod[:, cols].sum(1)
    return out


@pytest.mark.parametrize("mode", ["f32", "bf16"])
@pytest.mark.parametrize("M", [19200, 777])
def test_psw_elug_rho_partials(M, mode):
    """hsg_gemm_psw_elug_rho: the same C and G as hsg_gemm_f32_psw_elug (bitwise), and
    rho = per-head sums of G * h over each 64-column group, h = elu^-1(x - origin),
    against fp64 on the kernel's own G with the TRUE h.  G h = v (1 + e) log(1 + e)
    is taken from the rounded e = x - origin, whose error delta is <= 4 ulp(|x| +
    |origin|) + ulp(1); its derivative in e is v (h + 1), so the bound per entry is
    sum |v| delta (|h| + 1) + 1e-5 sum |G| (|h| + 1) over the entry's columns (the
    second term: the log and the summation roundings; the kernel takes u log u with
    u = 1 + e rounded, whose rounding moves G h by <= |v| ulp(1)).  Rows with h = -20
    take the e <= -1 branch (G h = 0) where e + 1 rounds to zero or below."""
    from hetersumgraph_amd.dense import elug_rho_groups, gemm_dtype, gemm_psw_elug, split_weights
    N, K, D = 300, 512, 50
    torch.manual_seed(M + 1)
    dH = torch.randn(M, K, device="cuda")
    W1 = torch.randn(K, N, device="cuda") / K ** 0.5
    with gemm_dtype(mode):
        (S,) = split_weights((W1, True))
    ds = torch.randn(M, N, device="cuda")
    origin = torch.randn(M, N, device="cuda")
    h = 2 * torch.randn(M, N, device="cuda")
    h[::7] = 0.0
    h[1::11] = -20.0                                           # exp(h) ~ 2e-9: e + 1 rounds to ~0
    x = torch.nn.functional.elu(h) + origin
    outs = []
    for with_rho in (False, True):
        out = ds.clone()
        G = torch.empty_like(ds)
        ng = elug_rho_groups(S, M, D)                          # f32: 112-wide groups (3), bf16: 64 (5)
        rho = torch.full((M, ng, 3), float("nan"), device="cuda") if with_rho else None
        assert gemm_psw_elug(dH, S, out, x, origin, G, rho, D if with_rho else 0)
        outs.append((out, G, rho))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    G, rho = outs[1][1], outs[1][2]
    gw = 112 if rho.shape[1] == (N + 111) // 112 and rho.shape[1] != (N + 63) // 64 else 64
    # 112-wide tiles (and rho groups) where they take fewer rounds x width than 64-wide
    # ones (hsg_gemm.hip wide112_pays): the cfg2 rows, not a 777-row GEMM
    assert gw == (112 if mode == "f32" and M == 19200 else 64)
    ref = _rho_ref(G, h, D, gw)
    out = outs[1][0]
    delta = 4 * 2.0 ** -23 * (x.abs() + origin.abs()) + 2.0 ** -23
    bound = (_rho_ref(out.abs(), delta * (h.abs() + 1), D, gw) + 1e-5 * _rho_ref(G.abs(), h.abs() + 1, D, gw)
             + 1e-12)
    err = (rho.double() - ref).abs()
    print(f"{mode} M={M}: worst rho error / bound {(err / bound).max().item():.3f}")
    assert torch.isfinite(rho).all()
    assert (err <= bound).all()


@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_psw_elug_rho_under_big_tile_switch(mode, monkeypatch):
    """the dev library's HSG_GEMM11=1 routes the psw GEMMs to k_gemm11,
    whose epilogue writes C and G but no rho.  The rho GEMM must decline it and run on
    k_gemm7: rho fully written (no NaN left from the prefill) and bitwise equal to the
    run without the switch, C and G too.  Dev library only."""
    from helpers import skip_unless_dev
    skip_unless_dev(False)
    from hetersumgraph_amd.dense import elug_rho_groups, gemm_dtype, gemm_psw_elug, split_weights
    M, N, K, D = 19200, 300, 512, 50
    torch.manual_seed(5)
    dH = torch.randn(M, K, device="cuda")
    W1 = torch.randn(K, N, device="cuda") / K ** 0.5
    with gemm_dtype(mode):
        (S,) = split_weights((W1, True))
    ds = torch.randn(M, N, device="cuda")
    origin = torch.randn(M, N, device="cuda")
    x = torch.nn.functional.elu(2 * torch.randn(M, N, device="cuda")) + origin
    outs = []
    for switch in ("0", "1"):
        monkeypatch.setenv("HSG_GEMM11", switch)
        out, G = ds.clone(), torch.empty_like(ds)
        rho = torch.full((M, elug_rho_groups(S, M, D), 3), float("nan"), device="cuda")
        assert gemm_psw_elug(dH, S, out, x, origin, G, rho, D)
        outs.append((out, G, rho))
    torch.cuda.synchronize()
    assert torch.isfinite(outs[1][2]).all()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_psw_elug_rho_declines_bad_head_dim():
    from hetersumgraph_amd.dense import elug_rho_groups, gemm_psw_elug, split_weights
    W1 = torch.randn(64, 300, device="cuda")
    (S,) = split_weights((W1, True))
    t = torch.randn(50, 300, device="cuda")
    for hd in (16, 70):                                         # < 32 / does not divide N
        rho = torch.empty(50, elug_rho_groups(S, 50, hd), 3, device="cuda")
        assert not gemm_psw_elug(torch.randn(50, 64, device="cuda"), S, t.clone(), t, t, torch.empty_like(t),
                                 rho, hd)


@pytest.mark.parametrize("gw", [64, 112])
@pytest.mark.parametrize("n_docs,N,W,k", [(4, 35, 600, 36), (3, 20, 200, 24)])
def test_one_pass_edge_bwd_equals_two_pass(n_docs, N, W, k, gw):
    """hsg_gat_bwd_src_g (one source-centric pass on G and the rho partials) against
    hsg_gat_bwd_dst_g + hsg_gat_bwd_src on the same S2W application, forward stats
    from a real forward: dZ and every attention-parameter gradient within 1e-5 of the
    output's scale (the passes differ only in where rho = G_v . h_v is summed)."""
    import ctypes
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd._lib import load
    from hetersumgraph_amd.ops import LEAKY_SLOPE, gat_table_bwd, gat_table_fwd
    lib = load()
    rng = np.random.default_rng(n_docs)
    docs = [synth.make_hsg_doc(rng, N=N, W=W, k=k) for _ in range(n_docs)]
    Gr = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    Gr.to(torch.device("cuda"))
    rel = Gr.relation("S2W")
    H, D = 6, 50
    assert lib.hsg_gat_bwd_src_g_supported(ctypes.byref(rel.cstruct()), H, D)
    torch.manual_seed(k)
    Z = torch.randn(rel.n_src, H * D, device="cuda")
    attn = torch.randn(H, 3 * D, device="cuda") * 0.3
    T = torch.randn(10, 50, device="cuda")
    wf = torch.randn(H, D, 50, device="cuda") * 0.1
    bf = torch.randn(H, D, device="cuda") * 0.1
    org = torch.randn(rel.n_dst, H * D, device="cuda")
    out, saved = gat_table_fwd(Z, attn, T, wf, bf, org, rel, H, D, LEAKY_SLOPE, no_h=True)
    assert saved[16] is not None
    dout = torch.randn_like(out)
    e = (out - org).double()
    G = torch.where(e > 0, dout.double(), dout.double() * (e + 1)).float()
    h = torch.where(e > 0, e, torch.log1p(e.clamp_min(-1 + 1e-12)))
    rho = _rho_ref(G, h, D, gw).float().contiguous()          # the 64- or 112-column group layout
    res = []
    for merged in (False, True):
        dst = (torch.zeros_like(attn), torch.zeros_like(wf), torch.zeros_like(bf), torch.zeros_like(T), False, False)
        dZ = gat_table_bwd(saved, dout, dst=dst, G=G, rho=rho if merged else None)
        res.append((dZ,) + dst[:4])
    torch.cuda.synchronize()
    for name, a, b in zip(("dZ", "dattn", "dwf", "dbf", "dT"), res[1], res[0]):
        tol = 1e-5 * max(1.0, b.abs().max().item())
        err = (a - b).abs().max().item()
        print(f"{name}: max |one-pass - two-pass| {err:.3e} (tol {tol:.3e})")
        assert err <= tol, name


def test_one_pass_edge_bwd_bf16_G_rows_bitwise():
    """hsg_gat_bwd_src_g_io with G as bf16 rows (the bf16 GEMM mode) against the fp32
    call on the same values: the kernel widens each bf16 feature exactly, so dZ and
    every attention-parameter gradient are bitwise equal."""
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.ops import LEAKY_SLOPE, gat_table_bwd, gat_table_fwd
    rng = np.random.default_rng(11)
    docs = [synth.make_hsg_doc(rng, N=35, W=600, k=36) for _ in range(4)]
    Gr = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    Gr.to(torch.device("cuda"))
    rel = Gr.relation("S2W")
    H, D = 6, 50
    torch.manual_seed(2)
    Z = torch.randn(rel.n_src, H * D, device="cuda")
    attn = torch.randn(H, 3 * D, device="cuda") * 0.3
    T = torch.randn(10, 50, device="cuda")
    wf = torch.randn(H, D, 50, device="cuda") * 0.1
    bf = torch.randn(H, D, device="cuda") * 0.1
    org = torch.randn(rel.n_dst, H * D, device="cuda")
    out, saved = gat_table_fwd(Z, attn, T, wf, bf, org, rel, H, D, LEAKY_SLOPE, no_h=True)
    dout = torch.randn_like(out)
    Gb = torch.randn_like(out).bfloat16()
    rho = torch.randn(rel.n_dst, (H * D + 63) // 64, 3, device="cuda")
    res = []
    for G in (Gb.float().contiguous(), Gb):
        dst = (torch.zeros_like(attn), torch.zeros_like(wf), torch.zeros_like(bf), torch.zeros_like(T), False, False)
        dZ = gat_table_bwd(saved, dout, dst=dst, G=G, rho=rho)
        res.append((dZ,) + dst[:4])
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [1120, 37])
def test_narrow_ffn_gate_epilogue(n):
    """hsg_ffn_small_bwd_gate: the same dx (bitwise) as hsg_ffn_small_bwd, and G =
    dx * elu'(h) (exp(h) for h <= 0, as the W2S dst pass) and the per-head rho =
    sum over each head's 8 columns of G * h (fp64 of the kernel's own G, 1e-6 of
    sum |G h|)."""
    from hetersumgraph_amd import rng
    from hetersumgraph_amd.ffn import ffn_bwd, ffn_fwd
    torch.manual_seed(n)
    dev = "cuda"
    x = torch.randn(n, 64, device=dev)
    w1 = torch.randn(512, 64, device=dev) / 8
    b1 = torch.randn(512, device=dev) * 0.1
    w2 = torch.randn(64, 512, device=dev) / 22
    b2 = torch.randn(64, device=dev) * 0.1
    g = 1 + 0.1 * torch.randn(64, device=dev)
    bt = 0.1 * torch.randn(64, device=dev)
    dout = torch.randn(n, 64, device=dev)
    h = 2 * torch.randn(n, 64, device=dev)
    h[::5] = 0.0
    rng.manual_seed(5)
    out, saved = ffn_fwd(x, w1, b1, w2, b2, g, bt, 0.1)
    res = []
    for with_gate in (False, True):
        grads = [torch.empty_like(t) for t in (w1, w2, b1, b2, g, bt)]
        gate = (h, torch.empty_like(h), h.new_empty(n, 8)) if with_gate else None
        r = ffn_bwd(saved, dout, (grads[0], False, grads[1], False, grads[2], grads[3], grads[4], grads[5], False),
                    gate=gate)
        res.append((r, gate))
    torch.cuda.synchronize()
    dx0 = res[0][0]
    (dx1, done), (_, G, rho) = res[1]
    assert done and torch.equal(dx0, dx1)
    gref = torch.where(h > 0, dx1, dx1 * torch.exp(h))
    assert (G - gref).abs().max().item() <= 1e-6 * max(1.0, gref.abs().max().item())
    prod = (G.double() * h.double()).view(n, 8, 8)
    err = (rho.double() - prod.sum(2)).abs()
    assert (err <= 1e-6 * prod.abs().sum(2) + 1e-12).all()


@pytest.mark.parametrize("n_docs,N,W,k", [(4, 35, 600, 36), (2, 9, 40, 5)])
def test_one_pass_w2s_edge_bwd_equals_two_pass(n_docs, N, W, k):
    """W2S (D = 8 narrow heads, h stored): hsg_gat_bwd_src_g with per-head rho
    (the head-lane kernel forming dpre itself) against the dst + src pair on the
    same G rows -- dZ and every attention-parameter gradient within 1e-5 of scale."""
    import ctypes
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd._lib import load
    from hetersumgraph_amd.ops import LEAKY_SLOPE, gat_table_bwd, gat_table_fwd
    lib = load()
    rng_ = np.random.default_rng(n_docs + 10)
    docs = [synth.make_hsg_doc(rng_, N=N, W=W, k=k) for _ in range(n_docs)]
    Gr = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    Gr.to(torch.device("cuda"))
    rel = Gr.relation("W2S")
    H, D = 8, 8
    assert lib.hsg_gat_bwd_src_g_supported(ctypes.byref(rel.cstruct()), H, D)
    torch.manual_seed(k)
    Z = torch.randn(rel.n_src, H * D, device="cuda")
    attn = torch.randn(H, 3 * D, device="cuda") * 0.3
    T = torch.randn(10, 50, device="cuda")
    wf = torch.randn(H, D, 50, device="cuda") * 0.1
    bf = None
    org = torch.randn(rel.n_dst, H * D, device="cuda")
    out, saved = gat_table_fwd(Z, attn, T, wf, bf, org, rel, H, D, LEAKY_SLOPE)
    h = saved[8]
    assert h is not None
    dout = torch.randn_like(out)
    G = torch.where(h > 0, dout, dout * torch.exp(h)).contiguous()
    rho = (G.double() * h.double()).view(-1, H, D).sum(2).float().contiguous()
    res = []
    for merged in (False, True):
        dst = (torch.zeros_like(attn), torch.zeros_like(wf), None, torch.zeros_like(T), False, False)
        if merged:
            dZ = gat_table_bwd(saved, dout, dst=dst, G=G, rho=rho)
        else:
            dZ = gat_table_bwd(saved, dout, dst=dst)
        res.append((dZ, dst[0], dst[1], dst[3]))
    torch.cuda.synchronize()
    for name, a, b in zip(("dZ", "dattn", "dwf", "dT"), res[1], res[0]):
        tol = 1e-5 * max(1.0, b.abs().max().item())
        err = (a - b).abs().max().item()
        print(f"{name}: max |one-pass - two-pass| {err:.3e} (tol {tol:.3e})")
        assert err <= tol, name


@pytest.mark.parametrize("shape", ["wide", "narrow"])
def test_one_pass_edge_bwd_ragged_relations(shape):
    """The one-pass backwards on random ragged relations (sources without out-edges,
    destinations without in-edges, phantom in-edges, repeated boxes) against the
    two-pass ones: wide heads (H = 6, D = 50, long CSC segments, rho as 64-column
    partials) and narrow heads (H = 8, D = 8, short segments, per-head rho)."""
    import ctypes
    from test_gpu_ops import random_relation
    from hetersumgraph_amd._lib import load
    from hetersumgraph_amd.ops import LEAKY_SLOPE, gat_table_bwd, gat_table_fwd
    lib = load()
    rng_ = np.random.default_rng(77 if shape == "wide" else 78)
    if shape == "wide":
        H, D = 6, 50
        rel, *_ = random_relation(rng_, 20, 300, 3)
    else:
        H, D = 8, 8
        rel, *_ = random_relation(rng_, 400, 30, 40)
    rel = rel.to("cuda")
    relp = ctypes.byref(rel.cstruct())
    assert lib.hsg_gat_bwd_src_g_supported(relp, H, D)
    torch.manual_seed(H + D)
    Z = torch.randn(rel.n_src, H * D, device="cuda")
    attn = torch.randn(H, 3 * D, device="cuda") * 0.3
    T = torch.randn(10, 50, device="cuda")
    wf = torch.randn(H, D, 50, device="cuda") * 0.1
    bf = torch.randn(H, D, device="cuda") * 0.1 if shape == "wide" else None
    org = torch.randn(rel.n_dst, H * D, device="cuda")
    out, saved = gat_table_fwd(Z, attn, T, wf, bf, org, rel, H, D, LEAKY_SLOPE, no_h=shape == "wide")
    dout = torch.randn_like(out)
    if shape == "wide":
        assert saved[16] is not None
        e = (out - org).double()
        G = torch.where(e > 0, dout.double(), dout.double() * (e + 1)).float().contiguous()
        h = torch.where(e > 0, e, torch.log1p(e.clamp_min(-1 + 1e-12)))
        rho = _rho_ref(G, h, D).float().contiguous()
    else:
        h = saved[8]
        G = torch.where(h > 0, dout, dout * torch.exp(h)).contiguous()
        rho = (G.double() * h.double()).view(-1, H, D).sum(2).float().contiguous()
    res = []
    for merged in (False, True):
        dst = (torch.zeros_like(attn), torch.zeros_like(wf), torch.zeros_like(bf) if bf is not None else None,
               torch.zeros_like(T), False, False)
        if merged:
            dZ = gat_table_bwd(saved, dout, dst=dst, G=G, rho=rho)
        elif shape == "wide":
            dZ = gat_table_bwd(saved, dout, dst=dst, G=G)
        else:
            dZ = gat_table_bwd(saved, dout, dst=dst)
        res.append((dZ, dst[0], dst[1], dst[3]) + ((dst[2],) if bf is not None else ()))
    torch.cuda.synchronize()
    for name, a, b in zip(("dZ", "dattn", "dwf", "dT", "dbf"), res[1], res[0]):
        tol = 1e-5 * max(1.0, b.abs().max().item())
        err = (a - b).abs().max().item()
        print(f"{shape} {name}: max |one-pass - two-pass| {err:.3e} (tol {tol:.3e})")
        assert err <= tol, name
    # sources without out-edges get dZ = 0 from both paths (and no NaN anywhere)
    assert torch.isfinite(res[1][0]).all()
