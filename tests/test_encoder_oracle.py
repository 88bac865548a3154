"""Pin the sentence-CNN oracle (oracle/cnn.py) against the reference's own sentEncoder
(tests/golden/encoder.npz, made by tests/golden/make_encoder_golden.py), and check the
host-side pieces of hetersumgraph_amd.cnn that need no GPU (tap stacking, layout)."""
import numpy as np
import torch

import weights
from helpers import load_fixture
from oracle import cnn as ocnn

SEED, V, D = 21, 64, 300


def encoder_params(dt=torch.float64):
    """The golden script's seeded sentEncoder parameters (weights.seed_module keys)."""
    from hetersumgraph_amd.module.PositionEmbedding import get_sinusoid_encoding_table
    emb = torch.from_numpy(weights.param_value(SEED, "embed.weight", (V, D))).to(dt)
    L = 20
    pos = get_sinusoid_encoding_table(L + 1, D, padding_idx=0).to(dt)
    cw = [torch.from_numpy(weights.param_value(SEED, f"convs.{i}.weight", (50, 1, h, D))).to(dt)
          for i, h in enumerate(range(2, 8))]
    cb = [torch.from_numpy(weights.param_value(SEED, f"convs.{i}.bias", (50,))).to(dt) for i in range(6)]
    return emb, pos, cw, cb


def test_cnn_oracle_matches_reference():
    z = load_fixture("encoder")
    ids = torch.from_numpy(z["ids"])
    emb, pos, cw, cb = encoder_params()
    for t in [emb] + cw + cb:
        t.requires_grad_()
    feat = ocnn.sent_encoder(ids, emb, pos, cw, cb)
    np.testing.assert_allclose(feat.detach().numpy(), z["feat64"], atol=2e-6, rtol=0)
    np.testing.assert_allclose(feat.detach().numpy(), z["feat32"], atol=2e-5, rtol=0)
    R = torch.from_numpy(weights.feature(SEED, "dfeat", tuple(feat.shape))).double()
    (feat * R).sum().backward()
    np.testing.assert_allclose(emb.grad.numpy(), z["embed_grad64"], atol=1e-5, rtol=1e-6)
    for i in range(6):
        np.testing.assert_allclose(cw[i].grad.numpy(), z[f"conv{i}_wgrad64"], atol=1e-5, rtol=1e-6)
        np.testing.assert_allclose(cb[i].grad.numpy(), z[f"conv{i}_bgrad64"], atol=1e-5, rtol=1e-6)


def test_stacked_taps_restatement():
    """Y = X Wall^T + shifted sum == the direct convolution (the algebra the kernels use)."""
    from hetersumgraph_amd.cnn import CHANNELS, HEIGHTS, stack_taps
    g = torch.Generator().manual_seed(0)
    Dm, L = 12, 9
    cw = [torch.randn(50, 1, h, Dm, generator=g, dtype=torch.float64) for h in HEIGHTS]
    cb = [torch.randn(50, generator=g, dtype=torch.float64) for _ in HEIGHTS]
    x = torch.randn(3, L, Dm, generator=g, dtype=torch.float64)
    wall = stack_taps(cw)
    assert wall.shape == (sum(HEIGHTS) * CHANNELS, Dm)
    Y = x @ wall.T                                           # [3, L, 1350]
    base = 0
    for h, w, b in zip(HEIGHTS, cw, cb):
        direct = torch.nn.functional.conv2d(x.unsqueeze(1), w, b).squeeze(3)      # [3, 50, L-h+1]
        shifted = sum(Y[:, i:L - h + 1 + i, (base + i) * 50:(base + i + 1) * 50] for i in range(h)) + b
        torch.testing.assert_close(shifted.transpose(1, 2), direct)
        base += h


def test_layout_rejects_inner_padding():
    from hetersumgraph_amd.cnn import _layout
    ids = torch.tensor([[3, 4, 0, 0], [5, 0, 6, 0]])
    try:
        _layout(ids)
    except ValueError as e:
        assert "trailing" in str(e)
    else:
        raise AssertionError("non-trailing padding accepted")
    length, rowoff, rows = _layout(torch.tensor([[3, 4, 0, 0], [0, 0, 0, 0], [1, 2, 3, 4]]))
    assert length.tolist() == [2, 0, 4] and rowoff.tolist() == [0, 3, 4, 9] and rows == 9
