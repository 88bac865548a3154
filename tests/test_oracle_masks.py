"""CPU checks of the host restatement of the dropout masks (oracle/masks.py):
rates, independence across heads / calls / seeds, and the packed-bit layout.
Bit-exactness against the kernels is pinned on the GPU (test_gpu_dropout_masks.py)."""
import numpy as np

from oracle import masks


def test_head_mask_rate_and_independence():
    k = masks.hproj_keep(5, 1, 4096, 300, 8, 0.1)
    assert k.shape == (8, 4096, 300)
    assert abs((1 - k.mean()) - 0.1) < 0.005
    kf = k.astype(np.float64)
    assert abs((kf[0] * kf[1]).mean() - 0.81) < 0.01            # heads of one pair
    assert abs((kf[0] * kf[2]).mean() - 0.81) < 0.01            # different pairs
    k2 = masks.hproj_keep(5, 2, 4096, 300, 8, 0.1)
    assert (k != k2).mean() > 0.1                               # another call
    k3 = masks.hproj_keep(6, 1, 4096, 300, 8, 0.1)
    assert (k != k3).mean() > 0.1                               # another seed
    assert np.array_equal(k, masks.hproj_keep(5, 1, 4096, 300, 8, 0.1))


def test_head_mask_prefix_rows_and_odd_heads():
    """A mask depends on n only through the word count: rows of a shorter call are
    the leading rows of the longer one when the 32-row word grid is the same."""
    a = masks.hproj_keep(9, 4, 64, 33, 3, 0.3)
    b = masks.hproj_keep(9, 4, 50, 33, 3, 0.3)
    assert np.array_equal(a[:, :50], b)
    assert abs((1 - a.mean()) - 0.3) < 0.05


def test_pack_layout():
    rng = np.random.default_rng(0)
    keep = rng.random((3, 70, 13)) > 0.5
    w = masks.pack_hproj_bits(keep).view(np.uint32)
    assert w.shape == (3, 3, 16)
    for k, i, c in [(0, 0, 0), (2, 69, 12), (1, 33, 5), (2, 31, 7)]:
        assert ((int(w[k, i // 32, c]) >> (i % 32)) & 1) == int(keep[k, i, c])
    assert (w[:, :, 13:] == 0).all() and (w[:, 2] >> 6 == 0).all()


def test_ffn_mask_rate_and_scale():
    k = masks.ffn_keep(3, 2, 2000, 300, 0.1)
    assert abs((1 - k.mean()) - 0.1) < 0.003
    assert not np.array_equal(k, masks.ffn_keep(3, 3, 2000, 300, 0.1))
    assert masks.ffn_threshold(0.1) == int(np.float64(np.float32(0.1)) * 2 ** 32)
    assert abs(masks.ffn_scale(0.1) - 1 / 0.9) < 1e-6
    assert abs(masks.hproj_scale(0.1) - 1 / (1 - 6553 / 65536)) < 1e-6
    assert masks.ffn_threshold(0.0) == 0 and masks.ffn_keep(1, 1, 4, 4, 0.0).all()
