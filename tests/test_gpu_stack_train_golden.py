"""The fused stack (the timed path) in TRAIN mode against the reference's own
WSWGAT modules at the bench's full cfg2 size (tests/golden/stack_train_cfg2.npz,
made by tests/golden/make_golden.py with the stack's dropout masks injected; the
fp64 oracle reproduces it to 1e-6, tests/test_stack_train_golden.py).

The golden's output is the reference CPU path in fp32; its gradients come from the
fp64 run, so fp32 ReLU-gate flips at near-zero pre-activations show up in the
comparison. The tolerances are those of the eval-mode reference goldens
(tests/test_gpu_model.py):
* output ≤ 1e-4 absolute against both the fp32 and the fp64 reference;
* every gradient entry ≤ 2e-3 of the largest (random projections: ≤ 2e-3 of the
  largest projection + 1e-5);
* state gradients also in the bulk: relative Frobenius error ≤ 2e-4 over the rows
  within 2e-4 · max (test_gpu_stack_parity.grad_stats).
"""
import numpy as np
import pytest
import torch

from helpers import load_fixture, projections

pytestmark = pytest.mark.gpu


def test_fused_stack_matches_reference_train_golden():
    from test_gpu_stack_parity import grad_stats, gpu_stack
    from hetersumgraph_amd.module.GATStackLayer import reference_named_grads
    z = load_fixture("stack_train_cfg2")
    seed, drop_seed = int(z["seed"]), int(z["drop_seed"])
    R = torch.from_numpy(np.random.default_rng(seed).standard_normal((int(z["n_s"]), 64)))
    r = gpu_stack(z, seed, R, train_seed=drop_seed, n_iter=int(z["n_iter"]))
    assert r["off0"] == int(z["off0"])                  # the masks the golden injected
    s = r["s"].cpu().double().numpy()
    err32, err64 = np.abs(s - z["out"]).max(), np.abs(s - z["out64"]).max()
    print(f"train cfg2 vs reference: output {err32:.3e} (fp32) / {err64:.3e} (fp64)")
    assert err32 <= 1e-4 and err64 <= 1e-4
    for key, got in (("grad_Xs", r["Xs"]), ("grad_T", r["T"]), ("grad_Xw_rows", r["Xw"][z["rows_w"]])):
        ref = z[key].astype(np.float64)
        g = got.detach().cpu().double().numpy()
        assert np.abs(g - ref).max() <= 2e-3 * np.abs(ref).max(), key
        st = grad_stats(g, ref)
        print(f"  {key:14s} fro {st['fro']:.2e} worst {st['worst']:.2e} bad {st['bad_rows']}/{st['rows']}")
        assert st["fro"] <= 2e-4, (key, st)
    pr = z["proj_grad_Xw"]
    assert np.abs(projections(r["Xw"], seed, "grad_Xw") - pr).max() <= 2e-3 * np.abs(pr).max() + 1e-5
    n = 0
    for tag, mod in (("w2s", r["w2s"]), ("s2w", r["s2w"])):
        for k, grad in reference_named_grads(mod):
            key = f"grad.{tag}.{k}"
            if grad is None:
                continue
            g = grad.detach().cpu().double()
            if key in z:
                ref = z[key].astype(np.float64)
                assert np.abs(g.numpy().reshape(ref.shape) - ref).max() <= 2e-3 * max(np.abs(ref).max(), 1e-3), key
            elif "proj." + key in z:
                ref = z["proj." + key]
                assert np.abs(projections(g, seed, key) - ref).max() <= 2e-3 * np.abs(ref).max() + 1e-5, key
            else:
                continue
            n += 1
    assert n == 8 * 3 + 6 * 4 + 12
