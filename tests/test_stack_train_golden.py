"""Train-mode golden of the timed stack, made by the REFERENCE's own WSWGAT modules
(tests/golden/make_golden.py --only stack_train_cfg2; VERDICT r5 weak #7: the
full-size reference goldens were eval mode only).

The fixture chains /root/reference/module/GAT.py's WSWGAT as HiGraph.py:99-106 does
(W2S, then 2 x (S2W, W2S)) on the bench's full cfg2 batch (159,040 edges), in train
mode. Every `nn.Dropout` call is replaced by the keep-mask and scale the fused stack
draws for that call: oracle/masks.py, pinned bit-exact to the device generators. There
are 8 or 6 head-input calls per application (GATStackLayer.py:56) and one FFN-output
call (GATLayer.py:41). Here the fp64 oracle (oracle/fused.py), fed the same masks,
must reproduce the fixture:
* output, state gradients and parameter gradients (the full ones and the random
  projections of the large ones) within 1e-6 of their largest entry: both runs are
  fp64 with the same masks, so the same ReLU gates.
tests/test_gpu_stack_train_golden.py checks the GPU's fused stack against the same
fixture.
"""
import numpy as np
import torch

from helpers import load_fixture, projections


def test_oracle_reproduces_reference_train_stack():
    from test_gpu_stack_parity import oracle_stack, train_masks
    from hetersumgraph_amd.module.GATStackLayer import reference_named_grads  # noqa: F401 (names)
    z = load_fixture("stack_train_cfg2")
    seed, drop_seed, off0 = int(z["seed"]), int(z["drop_seed"]), int(z["off0"])
    n_w, n_s = int(z["n_w"]), int(z["n_s"])
    ms = train_masks(drop_seed, off0, n_w, n_s, p=float(z["p"]), n_iter=int(z["n_iter"]))
    o = oracle_stack(z, seed, masks=ms, n_iter=int(z["n_iter"]))
    ref = z["out64"].astype(np.float64)
    assert np.abs(o["s"].numpy() - ref).max() <= 1e-6 * np.abs(ref).max()
    for key, got in (("grad_Xs", o["Xs"]), ("grad_T", o["T"])):
        r = z[key].astype(np.float64)
        assert np.abs(got.numpy() - r).max() <= 1e-6 * np.abs(r).max(), key
    rows = z["rows_w"]
    r = z["grad_Xw_rows"].astype(np.float64)
    assert np.abs(o["Xw"].numpy()[rows] - r).max() <= 1e-6 * np.abs(r).max()
    got = projections(o["Xw"], seed, "grad_Xw")
    assert np.abs(got - z["proj_grad_Xw"]).max() <= 1e-6 * np.abs(z["proj_grad_Xw"]).max()
    # parameters: the oracle's fp64 copies carry the reference's key names
    n = 0
    for tag, pd in (("w2s", o["p1"]), ("s2w", o["p2"])):
        for k, t in pd.items():
            if t.grad is None:
                continue
            key = f"grad.{tag}.{k}"
            g = t.grad.detach().double()
            if key in z:
                r = z[key].astype(np.float64)
                assert np.abs(g.numpy().reshape(r.shape) - r).max() <= 1e-6 * max(np.abs(r).max(), 1e-12), key
            elif "proj." + key in z:
                r = z["proj." + key]
                assert np.abs(projections(g, seed, key) - r).max() <= 1e-6 * np.abs(r).max(), key
            else:
                continue
            n += 1
    assert n >= 30, n
