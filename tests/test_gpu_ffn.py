"""Fused FFN (MFMA GEMMs + LN/dropout row kernels) vs PyTorch fp64, and the
dropout semantics of the row kernel."""
import pytest
import torch
import torch.nn.functional as F

from hetersumgraph_amd import _lib

pytestmark = pytest.mark.gpu


def ref_ffn(x, w1, b1, w2, b2, g, b):
    y = F.relu(x @ w1.t() + b1) @ w2.t() + b2
    return F.layer_norm(y + x, (x.shape[1],), g, b, 1e-5)


@pytest.mark.parametrize("n,d,dh", [(1120, 64, 512), (3000, 300, 512), (77, 300, 100)])
def test_ffn_eval_matches_fp64(n, d, dh):
    from hetersumgraph_amd.ffn import ffn_forward
    torch.manual_seed(n)
    x = torch.randn(n, d, dtype=torch.float64)
    ps = [torch.randn(dh, d, dtype=torch.float64) / d ** 0.5, 0.1 * torch.randn(dh, dtype=torch.float64),
          torch.randn(d, dh, dtype=torch.float64) / dh ** 0.5, 0.1 * torch.randn(d, dtype=torch.float64),
          1 + 0.1 * torch.randn(d, dtype=torch.float64), 0.1 * torch.randn(d, dtype=torch.float64)]
    R = torch.randn(n, d, dtype=torch.float64)
    leaves = [t.clone().requires_grad_() for t in [x] + ps]
    (ref_ffn(*leaves) * R).sum().backward()
    dl = [t.float().cuda().requires_grad_() for t in [x] + ps]
    out = ffn_forward(*dl, p_drop=0.0)
    (out * R.float().cuda()).sum().backward()
    ref = ref_ffn(*[t.detach() for t in leaves])
    assert (out.detach().cpu().double() - ref).abs().max().item() < 2e-5
    for a, b in zip(dl, leaves):
        scale = b.grad.abs().max().item()
        err = (a.grad.cpu().double() - b.grad).abs().max().item()
        assert err <= 1e-4 * max(scale, 1.0), (err, scale)


def test_ffn_dropout_semantics():
    """Train mode: drop rate ~p, kept values scaled by 1/(1-p), and a new call gives a
    new mask (the numeric forward/backward with the same mask:
    test_ffn_train_matches_fp64_with_same_mask)."""
    from hetersumgraph_amd import rng
    from hetersumgraph_amd.ffn import ffn_forward
    torch.manual_seed(0)
    n, d, dh, p = 4000, 300, 512, 0.1
    x = torch.randn(n, d, device="cuda")
    w1 = torch.randn(dh, d, device="cuda") / d ** 0.5
    w2 = torch.randn(d, dh, device="cuda") / dh ** 0.5
    b1 = torch.zeros(dh, device="cuda")
    b2 = torch.zeros(d, device="cuda")
    g = torch.ones(d, device="cuda")
    b = torch.zeros(d, device="cuda")
    # isolate the mask: with W2 = 0, b2 = 1 the dropped branch is exactly 0 or 1/(1-p)
    w2z = torch.zeros_like(w2)
    b2o = torch.ones(d, device="cuda")
    x0 = torch.zeros(n, d, device="cuda", requires_grad=True)
    out = ffn_forward(x0, w1, b1, w2z, b2o, g, b, p_drop=p)
    # LN of a 0/scale row: recover the mask from the sign pattern of the output
    kept = (out > 0)
    rate = 1 - kept.float().mean().item()
    assert abs(rate - p) < 0.005, rate
    out2 = ffn_forward(x0, w1, b1, w2z, b2o, g, b, p_drop=p)
    assert not torch.equal(out2 > 0, kept)             # new offset -> new mask


@pytest.mark.parametrize("n,d,dh,seed", [(3000, 300, 512, 21), (1120, 64, 512, 22), (37, 64, 512, 23),
                                         (77, 300, 100, 24)])
def test_ffn_train_matches_fp64_with_same_mask(n, d, dh, seed):
    """Train mode (dropout 0.1, GATLayer.py:41) -- forward and every gradient against
    an fp64 torch reference fed the same keep-mask, computed on the host from
    (seed, offset) by oracle/masks.py (bit-exact vs the kernels:
    test_gpu_dropout_masks.py).  d = 300: split GEMMs + hsg_ln_fwd / hsg_ln_bwd; d = 64:
    the one-launch hsg_ffn_small_fwd / _bwd.  Tolerances as the eval test."""
    from hetersumgraph_amd import rng
    from hetersumgraph_amd.ffn import ffn_forward
    from oracle import masks
    p = 0.1
    torch.manual_seed(seed)
    x = torch.randn(n, d, dtype=torch.float64)
    ps = [torch.randn(dh, d, dtype=torch.float64) / d ** 0.5, 0.1 * torch.randn(dh, dtype=torch.float64),
          torch.randn(d, dh, dtype=torch.float64) / dh ** 0.5, 0.1 * torch.randn(d, dtype=torch.float64),
          1 + 0.1 * torch.randn(d, dtype=torch.float64), 0.1 * torch.randn(d, dtype=torch.float64)]
    R = torch.randn(n, d, dtype=torch.float64)
    dl = [t.float().cuda().requires_grad_() for t in [x] + ps]
    rng.manual_seed(seed)
    out = ffn_forward(*dl, p_drop=p)
    off = rng.get("cuda").offset
    (out * R.float().cuda()).sum().backward()
    keep = torch.from_numpy(masks.ffn_keep(seed, off, n, d, p)).double()
    scale = masks.ffn_scale(p)
    leaves = [t.clone().requires_grad_() for t in [x] + ps]
    xr, w1, b1, w2, b2, g, b = leaves
    y = (F.relu(xr @ w1.t() + b1) @ w2.t() + b2) * keep * scale
    ref = F.layer_norm(y + xr, (d,), g, b, 1e-5)
    (ref * R).sum().backward()
    assert 0.05 < 1 - keep.mean().item() < 0.15
    assert (out.detach().cpu().double() - ref.detach()).abs().max().item() < 2e-5
    for name, a, r in zip(("x", "w1", "b1", "w2", "b2", "gamma", "beta"), dl, leaves):
        scale_g = r.grad.abs().max().item()
        err = (a.grad.cpu().double() - r.grad).abs().max().item()
        assert err <= 1e-4 * max(scale_g, 1.0), (name, err, scale_g)


@pytest.mark.parametrize("n,p", [(1120, 0.1), (1120, 0.0), (37, 0.1), (1, 0.3), (16 * 97 + 5, 0.1)])
def test_one_launch_narrow_ffn_matches_split_path(monkeypatch, n, p):
    """hsg_ffn_small_fwd (the W2S FFN, d = 64, d_hid = 512, one launch) against the
    split path (two hsg_gemm_f32 + hsg_ln_fwd, HSG_FFN_FUSED=0): the saved H and y,
    mean / rstd and the LN output agree to fp32 summation-order noise, the dropout
    mask is the same (same hash, same index), and the backward -- which consumes the
    saved tensors -- gives the same gradients; ragged row counts."""
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
    res = {}
    for flag in ("0", "1"):
        monkeypatch.setitem(_lib._OPTIONS, "HSG_FFN_FUSED", flag)
        rng.manual_seed(5)
        out, saved = ffn_fwd(x, w1, b1, w2, b2, g, bt, p)
        grads = [torch.empty_like(t) for t in (w1, w2, b1, b2, g, bt)]
        dx = ffn_bwd(saved, dout, (grads[0], False, grads[1], False, grads[2], grads[3], grads[4], grads[5], False))
        res[flag] = (out, saved[4], saved[5], saved[6], saved[7], dx, grads)
    torch.cuda.synchronize()
    a, b = res["0"], res["1"]
    for name, u, v in zip(("out", "H", "y", "mean", "rstd", "dx"), a[:6], b[:6]):
        tol = 2e-5 * max(1.0, u.abs().max().item())
        assert (u - v).abs().max().item() <= tol, (name, (u - v).abs().max().item())
    for name, u, v in zip(("dw1", "dw2", "db1", "db2", "dgamma", "dbeta"), a[6], b[6]):
        tol = 1e-4 * max(1.0, u.abs().max().item())
        assert (u - v).abs().max().item() <= tol, (name, (u - v).abs().max().item())
    # dropout actually applied (same mask on both paths: out agrees above)
    if p > 0:
        y, out = b[2], b[0]
        assert torch.isfinite(out).all() and y.shape == (n, 64)


@pytest.mark.parametrize("variant", ["1024,1", "512,2", "7,1", "3,2"])
@pytest.mark.parametrize("n,p", [(3000, 0.1), (77, 0.0), (1, 0.1)])
def test_ln_fwd_persistent_variant_bitwise(monkeypatch, variant, n, p):
    """The persistent LayerNorm forward (k_ln_fwd4p, the product default for 257..512
    columns: next row group's loads ahead; dev grids / two-row groups) against the
    one-round k_ln_fwd4 (HSG_LN_FWDP=0): the same per-row arithmetic, so out, mean and
    rstd are bitwise equal; tiny grids force many groups per wave, odd n a ragged pair."""
    from helpers import skip_unless_dev
    from hetersumgraph_amd._lib import check, load
    skip_unless_dev(False)
    torch.manual_seed(n)
    d = 300
    y, x = torch.randn(n, d, device="cuda"), torch.randn(n, d, device="cuda")
    g, b = 1 + 0.1 * torch.randn(d, device="cuda"), 0.1 * torch.randn(d, device="cuda")
    seed = torch.tensor([77], dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for v in ("0,1", variant):
        blocks, r = v.split(",")
        monkeypatch.setenv("HSG_LN_FWDP", blocks)
        monkeypatch.setenv("HSG_LN_FWDP_R", r)
        out, mean, rstd = torch.empty_like(y), torch.empty(n, device="cuda"), torch.empty(n, device="cuda")
        check(load().hsg_ln_fwd(n, d, y.data_ptr(), x.data_ptr(), g.data_ptr(), b.data_ptr(), 1e-5, p,
                                seed.data_ptr(), 9, out.data_ptr(), mean.data_ptr(), rstd.data_ptr(), st),
              "hsg_ln_fwd")
        res[v] = (out, mean, rstd)
    torch.cuda.synchronize()
    for a, c in zip(res["0,1"], res[variant]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("cap", ["512", "1024", "3"])
@pytest.mark.parametrize("n,p", [(3000, 0.1), (77, 0.0), (1, 0.1), (4097, 0.1)])
def test_ln_bwd_vector_variant(monkeypatch, cap, n, p):
    """k_ln_bwd4p (the product default for 257..512 columns: float4 columns, next row's
    loads ahead) against k_ln_bwd (HSG_LN_BWDP=0) on the same grid (HSG_LN_BWD_CAP): dgamma / dbeta partials bitwise
    (same rows per block, same per-column order), dx / dy / db2 partials to fp32 noise
    (the row sums add a lane's columns in another order); tiny caps walk many rows per
    wave."""
    from helpers import skip_unless_dev
    from hetersumgraph_amd._lib import check, load
    skip_unless_dev(False)
    torch.manual_seed(n)
    d = 300
    dev = "cuda"
    y, x, dout = (torch.randn(n, d, device=dev) for _ in range(3))
    g = 1 + 0.1 * torch.randn(d, device=dev)
    s = y + x
    mean = s.mean(1)
    rstd = torch.rsqrt(s.var(1, unbiased=False) + 1e-5)
    seed = torch.tensor([91], dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    monkeypatch.setenv("HSG_LN_BWD_CAP", cap)
    lib = load()
    res = {}
    for v in ("0", "1"):
        monkeypatch.setenv("HSG_LN_BWDP", v)
        nb = lib.hsg_ln_bwd_blocks(n)
        dy, dx = torch.empty_like(y), torch.empty_like(y)
        part = torch.empty(nb, 3, d, device=dev)
        check(lib.hsg_ln_bwd(n, d, dout.data_ptr(), y.data_ptr(), x.data_ptr(), g.data_ptr(), mean.data_ptr(),
                             rstd.data_ptr(), p, seed.data_ptr(), 5, dy.data_ptr(), dx.data_ptr(), part.data_ptr(), st),
              "hsg_ln_bwd")
        res[v] = (dx, dy, part)
    torch.cuda.synchronize()
    a, b = res["0"], res["1"]
    assert torch.equal(a[2][:, :2], b[2][:, :2])
    for u, w in ((a[0], b[0]), (a[1], b[1]), (a[2][:, 2], b[2][:, 2])):
        assert (u - w).abs().max().item() <= 2e-6 * max(1.0, u.abs().max().item())
