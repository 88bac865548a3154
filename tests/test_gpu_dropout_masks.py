"""The kernels' dropout masks against the host restatement in oracle/masks.py,
bit for bit -- the pin that lets the train-mode parity tests
(test_gpu_stack_parity.py::test_train_stack_vs_oracle_full_size, test_gpu_ffn.py)
feed the fp64 oracle the masks computed on the host from (seed, offset) alone.

* head projection (GATStackLayer.py:56, per-head input dropout): the keep-bits of
  hsg_dropmask and of the batched hsg_dropmask_multi the fused stack uses;
* FFN output dropout (GATLayer.py:41): the keep pattern of both FFN forward paths
  (split GEMMs + hsg_ln_fwd for d = 300, the one-launch hsg_ffn_small_fwd for d = 64),
  read back through an FFN whose dropped branch is exactly 0 or 1/(1-p).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d_in,H,p,seed,off", [(19200, 300, 8, 0.1, 7, 1), (1120, 64, 6, 0.1, 7, 3),
                                                 (333, 70, 3, 0.25, -5, 9), (31, 33, 1, 0.1, 2 ** 40 + 3, 77),
                                                 (65, 4, 5, 0.5, 0, 0xFFFFFFFF)])
def test_head_masks_match_host_restatement(n, d_in, H, p, seed, off):
    from hetersumgraph_amd._lib import load, ptr
    from oracle import masks
    lib = load()
    s = torch.tensor([seed], dtype=torch.int64, device="cuda")
    bits = torch.empty(lib.hsg_dropmask_words(n, d_in, H), dtype=torch.int32, device="cuda")
    assert lib.hsg_dropmask(n, d_in, H, float(p), ptr(s), off, ptr(bits), None) == 0
    torch.cuda.synchronize()
    ref = masks.pack_hproj_bits(masks.hproj_keep(seed, off, n, d_in, H, p))
    got = bits.cpu().numpy().reshape(ref.shape)
    assert np.array_equal(got, ref), int((got != ref).sum())
    assert abs(float(lib.hsg_dropmask_scale(float(p))) - masks.hproj_scale(p)) == 0.0


def test_batched_head_masks_match_host_restatement():
    from hetersumgraph_amd.hproj import dropmasks
    from oracle import masks
    seed = torch.tensor([424242], dtype=torch.int64, device="cuda")
    jobs = [(19200, 300, 8, 0.1, seed, 1), (1120, 64, 6, 0.1, seed, 3), (19200, 300, 8, 0.1, seed, 5)]
    got = dropmasks(jobs, torch.device("cuda"), None)
    torch.cuda.synchronize()
    for (n, d_in, H, p, _, off), g in zip(jobs, got):
        ref = masks.pack_hproj_bits(masks.hproj_keep(424242, off, n, d_in, H, p))
        assert np.array_equal(g.cpu().numpy().reshape(ref.shape), ref), off


@pytest.mark.parametrize("n,d,seed", [(4000, 300, 11), (1120, 64, 12), (37, 64, 13), (77, 300, -3)])
def test_ffn_masks_match_host_restatement(n, d, seed):
    from hetersumgraph_amd import rng
    from hetersumgraph_amd.ffn import ffn_forward
    from oracle import masks
    p, dh = 0.1, 512
    dev = "cuda"
    w1 = torch.randn(dh, d, device=dev) / d ** 0.5
    b1 = torch.zeros(dh, device=dev)
    w2z = torch.zeros(d, dh, device=dev)         # dropped branch = dropout(b2 = 1): 0 or 1/(1-p)
    b2o = torch.ones(d, device=dev)
    g = torch.ones(d, device=dev)
    b = torch.zeros(d, device=dev)
    x0 = torch.zeros(n, d, device=dev)
    rng.manual_seed(seed)
    r = rng.get(dev)
    out = ffn_forward(x0, w1, b1, w2z, b2o, g, b, p_drop=p)
    off = r.offset
    torch.cuda.synchronize()
    got = (out > 0).cpu().numpy()
    ref = masks.ffn_keep(seed, off, n, d, p)
    # rows with every element kept (or dropped) normalise to 0: exclude them
    mixed = ref.any(1) & ~ref.all(1)
    assert mixed.sum() >= n * 0.9
    assert np.array_equal(got[mixed], ref[mixed]), int((got[mixed] != ref[mixed]).sum())
