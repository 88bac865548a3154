"""Regression tests for the two GPU faults of round 5
and the host-side guards that came with them.  CPU only: each checks the host code
that sized or chose a device buffer, so the pre-fix code fails here without touching
a GPU.

* profiles/r05_faults/r05f_pytest.log (gpurun_out/r05f): hipErrorIllegalAddress in test_dw_pair_bf16_operands_bitwise --
  the k_dw partial slabs (fp32 stores) were allocated with a bf16 operand's
  ``new_empty``: half the bytes;
* profiles/r05_faults/r05j_pytest.log (gpurun_out/r05j): abort in the cfg5-bf16 stack backward -- the rho partials of the dx
  GEMM's ELU-gate epilogue (fp32 stores) were allocated with the bf16 G rows'
  ``new_empty``: half the bytes.
"""
import pytest
import torch


@pytest.mark.parametrize("adt,bdt", [(torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
                                     (torch.float32, torch.bfloat16), (torch.float32, torch.float32)])
def test_dw_slab_workspaces_are_fp32_of_the_full_size(adt, bdt):
    from hetersumgraph_amd.dense import dw_slab_workspaces
    K, splits = 64, 3
    pairs = [(torch.zeros(K, 300, dtype=adt), torch.zeros(K, 512, dtype=bdt)),
             (torch.zeros(K, 512, dtype=bdt), torch.zeros(K, 300, dtype=adt))]
    ws = dw_slab_workspaces(pairs, splits)
    assert len(ws) == 2
    for w in ws:
        assert w.dtype == torch.float32
        assert w.numel() * w.element_size() == splits * 300 * 512 * 4   # the bytes k_dw stores


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_rho_partials_are_fp32(gdt):
    from hetersumgraph_amd.stack import rho_partials
    G = torch.zeros(28800, 300, dtype=gdt)                 # cfg5's S2W destinations
    rho = rho_partials(G, 5)
    assert rho.shape == (28800, 5, 3) and rho.dtype == torch.float32 and rho.is_contiguous()


def test_bf16_rows_predicate_matches_the_kernels():
    """bf16 activation rows only where hsg_ln_fwd_y16 /
    hsg_ln_bwd_dy16 (257..512 columns, d % 4 == 0) and the bf16-A GEMMs (d_hid % 8 == 0)
    take the shape."""
    from hetersumgraph_amd.ffn import bf16_rows_ok
    assert bf16_rows_ok(300, 512)                     # cfg2 / cfg4 / cfg5 S2W FFN
    assert bf16_rows_ok(512, 2048) and bf16_rows_ok(260, 8)
    assert not bf16_rows_ok(256, 512)                 # a 256-wide word embedding
    assert not bf16_rows_ok(768, 512)
    assert not bf16_rows_ok(64, 512)                  # the W2S width, off the fused narrow FFN
    assert not bf16_rows_ok(300, 500)                 # ffn_inner_hidden_size % 8 != 0
    assert not bf16_rows_ok(302, 512)


def test_seed_advance_claim_stays_pending_until_launched():
    """a claimed seed advance whose launch never happened must still be
    performed by the next take(), or the step reuses the previous step's masks."""
    from hetersumgraph_amd.rng import DropoutRNG
    r = DropoutRNG("cpu", seed=5)
    flushed = []
    r._flush = lambda: flushed.append(r._pending) or setattr(r, "_pending", False)
    r._snap = torch.empty_like(r.seed)
    r._pending = True                              # what advance() leaves on a GPU
    adv = r.claim()
    assert adv is not None and adv[0] is r.seed and adv[1] is r._snap
    assert r._pending                              # not yet launched
    r.take()                                       # the launch failed: take() does the advance
    assert flushed == [True]
    r._pending = True
    assert r.claim() is not None
    r.claimed()                                    # launched
    assert not r._pending and r.claim() is None
