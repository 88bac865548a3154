"""bf16 rows for the S2W node states in the config-5 mode (round 6).

In the bf16 GEMM mode the S2W edge layer's output x = elu(h) + origin
(/root/reference/module/GAT.py:56-57; the stack at /root/reference/HiGraph.py:100-106)
is stored once as bf16 rows (hsg_gat_fwd_ws16, pitch ceil8(d), zero pad) and read as
bf16 by every consumer: the first FFN GEMM (A operand), the LayerNorm forward and
backward (the residual, hsg_ln_fwd_x16 / hsg_ln_bwd_x16), the dx GEMM's ELU gate
(elu(h) = x - origin, hsg_gemm_bf16_psw_elug_rho_x16) and dW1 = dH^T x
(hsg_gemm_dw_slabs_io).  Checked here:

* each consumer on the bf16 rows equals its fp32-row call on the same (bf16) values,
  bitwise -- the only new rounding is the store of x itself;
* hsg_gat_fwd_ws16's rows are RNE(x) of hsg_gat_fwd_ws, with the zero pad, on the full
  cfg5 S2W relation and on the cfg4 W2S relation with its work list (pieces merged
  in-kernel);
* the error budget of that rounding: |x16 - x| <= 2^-9 |x| per element (RNE), which
  moves a LayerNorm output row by at most 2^-9 |gamma| |x|_inf rstd per element;
* the cfg5-bf16 stack with bf16 x rows against the fp32-x-row run (HSG_FFN_BF16_X=0)
  within the bf16 budget; the fp64-oracle parity of that stack is
  test_gpu_stack_parity.py's cfg5-bf16 cases (bf16 x on by default).
"""
import ctypes

import numpy as np
import pytest
import torch

from helpers import build_graph, synth_fixture

pytestmark = pytest.mark.gpu


def _bf16_rows(t, pad_to=8):
    n, d = t.shape
    ld = (d + pad_to - 1) // pad_to * pad_to
    buf = torch.zeros(n, ld, dtype=torch.bfloat16, device=t.device)
    buf[:, :d] = t.bfloat16()
    return buf[:, :d]


@pytest.mark.parametrize("n,p_drop", [(28800, 0.1), (1001, 0.0)])
def test_ln_x16_equals_fp32_rows_on_the_same_values(n, p_drop):
    from hetersumgraph_amd import rng as hsg_rng
    from hetersumgraph_amd._lib import load, ptr
    lib = load()
    d = 300
    torch.manual_seed(n + 7)
    yb = torch.randn(n, d, device="cuda").bfloat16()
    x16 = _bf16_rows(torch.randn(n, d, device="cuda"))
    xf = x16.float().contiguous()
    gamma, beta = 1 + 0.1 * torch.randn(d, device="cuda"), 0.1 * torch.randn(d, device="cuda")
    hsg_rng.manual_seed(19)
    seed_t, off = hsg_rng.get(xf.device).take() if p_drop > 0 else (None, 0)
    outs = []
    for x, f16 in ((xf, False), (x16, True)):
        out, mean, rstd = torch.empty_like(xf), xf.new_empty(n), xf.new_empty(n)
        if f16:
            rc = lib.hsg_ln_fwd_x16(n, d, ptr(yb), ptr(x), x.stride(0), ptr(gamma), ptr(beta), 1e-5, p_drop,
                                    ptr(seed_t), off, ptr(out), ptr(mean), ptr(rstd), None)
        else:
            rc = lib.hsg_ln_fwd_y16(n, d, ptr(yb), ptr(x), ptr(gamma), ptr(beta), 1e-5, p_drop, ptr(seed_t), off,
                                    ptr(out), ptr(mean), ptr(rstd), None)
        assert rc == 0
        outs.append((out, mean, rstd))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    mean, rstd = outs[0][1], outs[0][2]
    dout = torch.randn(n, d, device="cuda")
    nb = lib.hsg_ln_bwd_blocks(n)
    res = []
    for x, f16 in ((xf, False), (x16, True)):
        dy = torch.full((n, 304), float("nan"), device="cuda").bfloat16()
        dx, part = torch.empty_like(xf), xf.new_empty(nb, 3, d)
        if f16:
            rc = lib.hsg_ln_bwd_x16(n, d, ptr(dout), ptr(yb), ptr(x), x.stride(0), ptr(gamma), ptr(mean), ptr(rstd),
                                    p_drop, ptr(seed_t), off, ptr(dy), 304, ptr(dx), ptr(part), None)
        else:
            rc = lib.hsg_ln_bwd_dy16(n, d, ptr(dout), ptr(yb), 1, ptr(x), ptr(gamma), ptr(mean), ptr(rstd), p_drop,
                                     ptr(seed_t), off, ptr(dy), 304, ptr(dx), ptr(part), None)
        assert rc == 0
        res.append((dy, dx, part))
    torch.cuda.synchronize()
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_ln_x16_refuses_bad_pitch():
    from hetersumgraph_amd._lib import HSG_EINVAL, load, ptr
    lib = load()
    n, d = 64, 300
    y = torch.zeros(n, d, dtype=torch.bfloat16, device="cuda")
    x = torch.zeros(n, 304, dtype=torch.bfloat16, device="cuda")
    g = torch.ones(d, device="cuda")
    out, mean, rstd = torch.empty(n, d, device="cuda"), torch.empty(n, device="cuda"), torch.empty(n, device="cuda")
    for ldx in (300, 302, 296):                  # not a multiple of 8, or below ceil8(d)
        assert lib.hsg_ln_fwd_x16(n, d, ptr(y), ptr(x), ldx, ptr(g), ptr(g), 1e-5, 0.0, None, 0, ptr(out),
                                  ptr(mean), ptr(rstd), None) == HSG_EINVAL


@pytest.mark.parametrize("M", [28800, 777])
def test_elug_x16_bitwise(M):
    """hsg_gemm_bf16_psw_elug_rho_x16 (x as bf16 rows) against the fp32-x call on the
    same values: dx, bf16 G and rho bitwise equal."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_psw_elug, split_weights
    N, K, D = 300, 512, 50
    torch.manual_seed(M + 3)
    dHb = _bf16_rows(torch.randn(M, K, device="cuda"))
    W1 = torch.randn(K, N, device="cuda") / K ** 0.5
    with gemm_dtype("bf16"):
        (S,) = split_weights((W1, True))
    ds = torch.randn(M, N, device="cuda")
    origin = torch.randn(M, N, device="cuda")
    x16 = _bf16_rows(torch.nn.functional.elu(2 * torch.randn(M, N, device="cuda")) + origin)
    outs = []
    for x in (x16.float().contiguous(), x16):
        out, G = ds.clone(), torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        rho = torch.empty(M, (N + 63) // 64, 3, device="cuda")
        assert gemm_psw_elug(dHb, S, out, x, origin, G, rho, D)
        outs.append((out, G, rho))
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_dw_pair_bf16_x_operand_bitwise():
    """dW1 = dH^T x with x as strided bf16 rows (pitch 304) against its fp32 copy."""
    from hetersumgraph_amd.dense import gemm_dtype, gemm_dw_slabs
    K, d, dh = 57600, 300, 512                    # cfg5: two S2W applications x 28,800 words
    torch.manual_seed(5)
    DY = _bf16_rows(torch.randn(K, d, device="cuda"))
    Hh = torch.randn(K, dh, device="cuda").bfloat16()
    DH = torch.randn(K, dh, device="cuda").bfloat16()
    X16 = _bf16_rows(torch.randn(K, d, device="cuda"))
    with gemm_dtype("bf16"):
        a = gemm_dw_slabs([(DY, Hh), (DH, X16)])
        b = gemm_dw_slabs([(DY, Hh), (DH, X16.float().contiguous())])
    torch.cuda.synchronize()
    assert a is not None and b is not None
    for (wa, sa), (wb, sb) in zip(a, b):
        assert sa == sb and torch.equal(wa, wb)


def _fwd_pair(rel, H, D, seed):
    from hetersumgraph_amd._lib import HSG_TAU_TABLE, check, load, ptr, stream_of
    lib = load()
    relp = ctypes.byref(rel.cstruct())
    g = torch.Generator(device="cuda").manual_seed(seed)
    HD = H * D
    Z = torch.randn(rel.n_src, HD, device="cuda", generator=g)
    sigma = torch.randn(rel.n_src, H, device="cuda", generator=g)
    tau = torch.randn(11, H, device="cuda", generator=g)
    origin = torch.randn(rel.n_dst, HD, device="cuda", generator=g)
    n = rel.n_dst
    nf = lib.hsg_gat_fwd_ws_floats(relp, H, D)
    ws = Z.new_empty(nf) if nf else None
    res = []
    for f16 in (False, True):
        m, l = Z.new_empty(n, H), Z.new_empty(n, H)
        if f16:
            ld = (HD + 7) // 8 * 8
            out = torch.full((n, ld), float("nan"), device="cuda").bfloat16()
            check(lib.hsg_gat_fwd_ws16(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(origin),
                                       None, None, ptr(m), ptr(l), ptr(ws), ptr(out), ld, stream_of(Z)),
                  "hsg_gat_fwd_ws16")
        else:
            out = Z.new_empty(n, HD)
            check(lib.hsg_gat_fwd_ws(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(sigma), ptr(tau), ptr(origin),
                                     None, ptr(out), ptr(m), ptr(l), ptr(ws), stream_of(Z)), "hsg_gat_fwd_ws")
        res.append((out, m, l))
    torch.cuda.synchronize()
    return res, HD


@pytest.mark.parametrize("config,kind,H,D", [("cfg5", "S2W", 6, 50), ("cfg2", "S2W", 6, 50), ("cfg4", "W2S", 8, 8),
                                             ("cfg4", "W2S", 6, 50)])
def test_gat_fwd_ws16_rows_are_rne_of_fp32(config, kind, H, D):
    """hsg_gat_fwd_ws16 stores RNE(elu(h) + origin) with the zero pad; (m, l) as the
    fp32 launch.  cfg4 W2S carries the doc supernodes' work list (pieces merged
    in-kernel by the last arriving block, which then writes the bf16 row)."""
    from hetersumgraph_amd import synth
    G = build_graph(synth_fixture(synth.make_batch_docs(config, seed=0))).to("cuda")
    rel = G.relation(kind)
    if config == "cfg4":
        assert "dwork" in rel.dev
    (of, mf, lf), (o16, m16, l16) = _fwd_pair(rel, H, D, 21)[0]
    HD = H * D
    assert torch.equal(o16[:, :HD], of.bfloat16())
    assert not o16[:, HD:].float().any()
    assert torch.equal(mf, m16) and torch.equal(lf, l16)
    # per element: the one rounding of the store
    err = (o16[:, :HD].float() - of).abs()
    assert bool((err <= of.abs() * 2.0 ** -8).all())


def test_gat_fwd_ws16_refuses_bad_rows():
    from hetersumgraph_amd import synth
    from hetersumgraph_amd._lib import HSG_EINVAL, HSG_TAU_TABLE, load, ptr
    lib = load()
    G = build_graph(synth_fixture(synth.make_batch_docs("cfg2", seed=0)[:4])).to("cuda")
    rel = G.relation("S2W")
    relp = ctypes.byref(rel.cstruct())
    H, D = 6, 50
    Z = torch.zeros(rel.n_src, H * D, device="cuda")
    s = torch.zeros(rel.n_src, H, device="cuda")
    t = torch.zeros(11, H, device="cuda")
    org = torch.zeros(rel.n_dst, H * D, device="cuda")
    m, l = torch.empty(rel.n_dst, H, device="cuda"), torch.empty(rel.n_dst, H, device="cuda")
    buf = torch.zeros(rel.n_dst, 312, dtype=torch.bfloat16, device="cuda")
    for ld, o in ((300, org), (302, org), (304, None)):      # pitch below ceil8 / not % 8; no origin
        assert lib.hsg_gat_fwd_ws16(relp, H, D, HSG_TAU_TABLE, 0.01, ptr(Z), ptr(s), ptr(t), ptr(o), None, None,
                                    ptr(m), ptr(l), None, ptr(buf), ld, None) == HSG_EINVAL


def _stack_run(z, seed, R, x16, train, monkeypatch):
    from hetersumgraph_amd import _lib
    from hetersumgraph_amd.dense import gemm_dtype
    from test_gpu_stack_parity import gpu_stack
    monkeypatch.setitem(_lib._OPTIONS, "HSG_FFN_BF16_X", "1" if x16 else "0")
    with gemm_dtype("bf16"):
        return gpu_stack(z, seed, R, train_seed=77 if train else None)


@pytest.mark.parametrize("train", [False, True])
def test_cfg5_stack_bf16_x_rows_within_budget(train, monkeypatch):
    """The cfg5-bf16 stack with the bf16 x rows against the same stack on fp32 x rows:
    one extra rounding of x per S2W application -- output <= 5e-3, state and parameter
    gradients <= 2e-2 relative (Frobenius; attention parameters 5e-2, cancelling sums)."""
    from hetersumgraph_amd import synth
    docs = synth.make_batch_docs("cfg5", seed=0)
    z = synth_fixture(docs)
    R = torch.from_numpy(np.random.default_rng(13).standard_normal((int(z["n_s"]), 64)))
    a = _stack_run(z, 13, R, False, train, monkeypatch)
    b = _stack_run(z, 13, R, True, train, monkeypatch)
    err = (a["s"] - b["s"]).abs().max().item()
    print(f"cfg5 bf16 x rows vs fp32 x rows: output {err:.3e}")
    assert 0 < err <= 5e-3                          # the x rounding is real, and small
    for k in ("Xw", "Xs", "T"):
        rel = ((a[k] - b[k]).norm() / a[k].norm()).item()
        assert rel <= 2e-2, (k, rel)
    for m in ("w2s", "s2w"):
        for (n, p), (_, q) in zip(a[m].named_parameters(), b[m].named_parameters()):
            if p.grad is None:
                continue
            tol = 5e-2 if ("feat_" in n or "attn_" in n) else 2e-2
            rel = ((p.grad - q.grad).norm() / p.grad.norm().clamp_min(1e-30)).item()
            assert rel <= tol, (m, n, rel)


def test_stack_keeps_bf16_x_buffers(monkeypatch):
    """The fused stack's S2W FFN-input buffer is bf16 (pitch 304) in the bf16 mode and
    fp32 with HSG_FFN_BF16_X=0 or in the f32 mode; W2S (d = 64) stays fp32."""
    from hetersumgraph_amd import _lib, synth
    from hetersumgraph_amd.HiGraph import register_tfidf_table
    from hetersumgraph_amd.dense import gemm_dtype
    from hetersumgraph_amd.stack import gat_stack
    from helpers import gat_inputs, seeded_gat_params
    dev = torch.device("cuda")
    z = synth_fixture(synth.make_batch_docs("cfg2", seed=0)[:6])
    G = build_graph(z).to(dev)
    n_w, n_s = int(z["n_w"]), int(z["n_s"])
    Xw, Xs, T = (t.to(dev) for t in gat_inputs(5, n_w, n_s))
    register_tfidf_table(G, T)
    w2s, s2w = seeded_gat_params(501, 502)
    w2s, s2w = w2s.to(dev).eval(), s2w.to(dev).eval()
    for dt, flag, want in (("bf16", "1", torch.bfloat16), ("bf16", "0", torch.float32), ("f32", "1", torch.float32)):
        monkeypatch.setitem(_lib._OPTIONS, "HSG_FFN_BF16_X", flag)
        with gemm_dtype(dt):
            s = gat_stack(G, w2s, s2w, T, Xw, Xs, 2)
        ctx = s.grad_fn
        X = ctx.bufs[id(ctx.cfg[2])][0]                   # the S2W layer's FFN-input buffer
        assert X.dtype == want, (dt, flag)
        if want == torch.bfloat16:
            assert X.stride(1) == 304
        assert ctx.bufs[id(ctx.cfg[1])][0].dtype == torch.float32
