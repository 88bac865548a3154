"""Sentence CNN encoder on the GPU (hetersumgraph_amd.cnn -> hsg_cnn_* + hsg_gemm_f32
through the C ABI) against the reference's own sentEncoder outputs (golden) and the
fp64 direct-convolution oracle (oracle/cnn.py) at CNN/DM sizes.

Tolerances: outputs 5e-5 absolute (fp32 sums of h*D = 600..2100 products of O(1)
terms); gradients 1e-4 relative to the largest entry.  A max-pool gradient is
discontinuous where two windows tie within rounding, so the large-size gradient test
zeroes the upstream gradient of the (sentence, channel) pairs whose top-two distinct
windows are closer than 1e-4 (in fp64) and of those whose max sits within 1e-4 of the
ReLU kink; every other pair must route to the same window as the reference.
"""
import numpy as np
import pytest
import torch

import weights
from helpers import load_fixture
from oracle import cnn as ocnn
from test_encoder_oracle import SEED, encoder_params

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.detach().cpu().double(), torch.as_tensor(b).double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


def gpu_params(dt=torch.float32):
    emb, pos, cw, cb = encoder_params(dt)
    out = [t.cuda().requires_grad_() for t in [emb] + cw + cb]
    return out[0], pos.cuda(), out[1:7], out[7:]


def test_encoder_matches_reference_golden():
    from hetersumgraph_amd.cnn import sent_cnn
    z = load_fixture("encoder")
    ids = torch.from_numpy(z["ids"]).cuda()
    emb, pos, cw, cb = gpu_params()
    feat = sent_cnn(ids, emb, pos, cw, cb, padding_idx=0)
    torch.cuda.synchronize()
    assert feat.shape == (ids.shape[0], 300)
    assert (feat.detach().cpu().double() - torch.from_numpy(z["feat64"]).double()).abs().max() < 5e-5
    assert (feat.detach().cpu().double() - torch.from_numpy(z["feat32"]).double()).abs().max() < 5e-5
    R = torch.from_numpy(weights.feature(SEED, "dfeat", tuple(feat.shape))).cuda()
    (feat * R).sum().backward()
    assert rel_err(emb.grad, z["embed_grad64"]) < 1e-4
    assert emb.grad[0].abs().max().item() == 0.0        # padding_idx row
    for i in range(6):
        assert rel_err(cw[i].grad, z[f"conv{i}_wgrad64"]) < 1e-4, i
        assert rel_err(cb[i].grad, z[f"conv{i}_bgrad64"]) < 1e-4, i


def cnndm_ids(n, L, V, seed):
    """CNN/DM-shaped token ids: trailing padding, lengths 0, 1, 6, L and U(5, 60)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(5, 61, n)
    lens[:4] = [0, 1, 6, L]
    ids = np.zeros((n, L), np.int64)
    for i, m in enumerate(lens):
        ids[i, :m] = rng.integers(1, V, m)
    return torch.from_numpy(ids)


def unambiguous(ids, emb, pos, cw, cb, tol=1e-4):
    """[n, 300] mask of (sentence, channel) pairs whose max-pool winner is stable."""
    L = ids.shape[1]
    x = (torch.nn.functional.embedding(ids, emb) + pos[ocnn.positions(ids, L)]).unsqueeze(1)
    length = (ids != 0).sum(1)
    keep = []
    for w, b in zip(cw, cb):
        y = torch.nn.functional.conv2d(x, w, b).squeeze(3)        # [n, 50, T]
        T = y.shape[2]
        # windows past len_s are copies of window len_s: keep one of them
        t = torch.arange(T).view(1, 1, T)
        y = torch.where(t <= length.view(-1, 1, 1), y, torch.full_like(y, -1e30))
        top = y.topk(min(2, T), dim=2).values
        gap = top[..., 0] - top[..., 1] if T > 1 else torch.full_like(top[..., 0], 1e30)
        keep.append((gap > tol) & (top[..., 0].abs() > tol))
    return torch.cat(keep, 1)


def test_encoder_cnndm_size_vs_oracle():
    from hetersumgraph_amd.cnn import sent_cnn
    n, L, V, D = 192, 100, 5000, 300
    torch.manual_seed(3)
    ids = cnndm_ids(n, L, V, 3)
    emb = 0.5 * torch.randn(V, D, dtype=torch.float64)
    from hetersumgraph_amd.module.PositionEmbedding import get_sinusoid_encoding_table
    pos = get_sinusoid_encoding_table(L + 1, D, padding_idx=0).double()
    cw = [torch.randn(50, 1, h, D, dtype=torch.float64) / np.sqrt(h * D) for h in range(2, 8)]
    cb = [0.1 * torch.randn(50, dtype=torch.float64) for _ in range(6)]
    mask = unambiguous(ids, emb, pos, cw, cb)
    assert mask.float().mean() > 0.95
    R = torch.randn(n, 300, dtype=torch.float64) * mask
    # oracle (fp64, CPU, direct convolution over the padded input)
    leaves = [t.clone().requires_grad_() for t in [emb] + cw + cb]
    ref = ocnn.sent_encoder(ids, leaves[0], pos, leaves[1:7], leaves[7:])
    (ref * R).sum().backward()
    # GPU
    g = [t.float().cuda().requires_grad_() for t in [emb] + cw + cb]
    feat = sent_cnn(ids.cuda(), g[0], pos.float().cuda(), g[1:7], g[7:], padding_idx=0)
    (feat * R.float().cuda()).sum().backward()
    torch.cuda.synchronize()
    assert (feat.detach().cpu().double() - ref.detach()).abs().max() < 5e-5
    for i, (a, b) in enumerate(zip(g, leaves)):
        assert rel_err(a.grad, b.grad) < 1e-4, i


def test_encoder_edge_cases():
    from hetersumgraph_amd.cnn import sent_cnn
    emb, pos, cw, cb = gpu_params()
    # no sentences
    out = sent_cnn(torch.zeros(0, 20, dtype=torch.long, device="cuda"), emb, pos, cw, cb)
    assert out.shape == (0, 300)
    # all-padding batch: every window is the pad window
    ids = torch.zeros(3, 20, dtype=torch.long, device="cuda")
    out = sent_cnn(ids, emb, pos, cw, cb)
    ref = ocnn.sent_encoder(ids.cpu(), emb.detach().cpu().double(), pos.cpu().double(),
                            [w.detach().cpu().double() for w in cw], [b.detach().cpu().double() for b in cb])
    assert (out.detach().cpu().double() - ref).abs().max() < 5e-5
    with pytest.raises(ValueError, match="trailing"):
        sent_cnn(torch.tensor([[1, 0, 2] + [0] * 17], device="cuda"), emb, pos, cw, cb)
    with pytest.raises(ValueError, match="widest kernel"):
        sent_cnn(torch.ones(2, 6, dtype=torch.long, device="cuda"), emb, pos, cw, cb)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        sent_cnn(ids.cpu(), emb.detach().cpu(), pos.cpu(), [w.detach().cpu() for w in cw],
                 [b.detach().cpu() for b in cb])
