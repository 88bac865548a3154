"""bench.py's roofline arithmetic against SURVEY §8(d)'s published figures for
config 2 (CPU only, no HIP library: relation sizes from the oracle's host-side
restatement; the dW tile count from bench.dw_tiles, the host mirror pinned to the
library in tests/test_abi.py)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def cfg2_rels():
    from types import SimpleNamespace
    from hetersumgraph_amd import synth
    from oracle import fused
    docs = synth.make_batch_docs("cfg2", seed=0)
    offs = np.cumsum([0] + [d.n_nodes for d in docs])
    cat = lambda f: np.concatenate([f(d, o) for d, o in zip(docs, offs[:-1])])
    src, dst, unit = cat(lambda d, o: d.src + o), cat(lambda d, o: d.dst + o), cat(lambda d, o: d.unit)
    tf, et = cat(lambda d, o: d.tffrac), cat(lambda d, o: d.edtype)
    rels = [fused.typed_relation(k, src, dst, unit, tf, et) for k in ("W2S", "S2W")]
    return [SimpleNamespace(n_src=r["n_src"], n_dst=r["n_dst"], n_typed=len(r["e_src"])) for r in rels]


def test_edge_bytes_match_survey(cfg2_rels):
    import bench
    rw, rs = cfg2_rels
    assert (rw.n_src, rw.n_dst, rw.n_typed) == (19200, 1120, 40320)
    mb = lambda b: round(b / 1e6, 2)
    assert mb(bench.edge_bytes_fwd(rw, 8, 8)) == 6.10
    assert mb(bench.edge_bytes_bwd(rw, 8, 8)) == 12.27
    assert mb(bench.edge_bytes_fwd(rs, 6, 50)) == 25.69
    assert mb(bench.edge_bytes_bwd(rs, 6, 50)) == 50.31
    step = 3 * (bench.edge_bytes_fwd(rw, 8, 8) + bench.edge_bytes_bwd(rw, 8, 8)) + \
        2 * (bench.edge_bytes_fwd(rs, 6, 50) + bench.edge_bytes_bwd(rs, 6, 50))
    assert round(step / 1e6, 1) == 207.1


def test_full_stack_floor(cfg2_rels):
    """Dense work ≈79 GFLOP per step at cfg2 (>= 0.50 ms at the f32 peak)."""
    import bench
    rw, rs = cfg2_rels
    items = bench.step_work(rw, rs, 2, "f32")
    floor, edge, dense, gflop = bench.full_stack_floor(items)
    assert 74 <= gflop <= 80
    assert 0.45e-3 <= dense <= 0.54e-3          # incl. the ~20 us of split-K slab bytes
    assert abs(edge - 207.1e6 / 8e12) < 1e-7
    # the weight gradients' split-K slabs, each written and read once, at the
    # slice counts of the one-launch pair (dense.gemm_dw_slabs): S2W 32 x
    # [300 x 512] per weight (16 tiles, two blocks per CU), W2S 21 x [64 x 512] (8 tiles:
    # 64 slices capped at 4 K tiles each over its 105, then made non-empty)
    slabs = {n: b for n, b, _, _ in items if n.startswith("ffn_dw_slabs")}
    assert bench.dw_slab_splits(38400, 300, 512) == 32 and bench.dw_slab_splits(3360, 64, 512) == 21
    assert round(slabs["ffn_dw_slabs_S2W"] / 1e6, 1) == round(2 * 2 * 4 * 32 * 300 * 512 / 1e6, 1)
    assert round(slabs["ffn_dw_slabs_W2S"] / 1e6, 1) == round(2 * 2 * 4 * 21 * 64 * 512 / 1e6, 1)


def test_dense_roofline_peak_follows_the_path():
    """the f32 (split) GEMM issues six bf16 products per fp32-accurate
    product, so its roofline is the bf16 MFMA peak on 6x the useful flops; the
    fp32-equivalent figure is kept separately."""
    import bench
    r = bench.dense_roofline("hsg_gemm_f32_psw", 19200, 100.0, 5.9e9, 0.059, "f32")
    assert r["peak"] == bench.BF16_MFMA_PEAK_TFLOPS and abs(r["achieved"] - 600.0) < 1e-9
    assert abs(r["frac"] - 600.0 / 2500.0) < 1e-12
    assert abs(r["fp32_equivalent"]["frac"] - 100.0 / bench.FP32_MFMA_PEAK_TFLOPS) < 1e-12
    b = bench.dense_roofline("hsg_gemm_*", 19200, 900.0, 5.9e9, 0.0066, "bf16")
    assert b["achieved"] == 900.0 and "fp32_equivalent" not in b
