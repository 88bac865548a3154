"""Pin the CPU oracle (oracle/fused.py) against the reference's golden vectors.

The vectors were produced by the reference's own WSWGAT module code
(tests/golden/make_golden.py), once in fp32 (the reference CPU path) and once in
fp64.  Checks:
  * oracle (fp64) vs reference fp64 outputs and gradients: 1e-6 (the fixtures
    store fp64 results rounded to fp32);
  * oracle (fp64) vs reference fp32 outputs: 2e-5 (the reference's own rounding).
Gradients are compared against the fp64 run only: an fp32 ReLU network's
gradient is discontinuous where a pre-activation is within rounding of 0 (the
cfg1 fixture has one such unit: |W1 x + b1| = 2.7e-8 for word 479), so fp32
gradients of two correct implementations can differ by O(0.1) there.
"""
import numpy as np
import pytest
import torch

from helpers import concat_arrays, gat_inputs, load_fixture, projections, seeded_gat_params, upstream
from oracle import fused

CASES = [("gat_small", 1), ("gat_hdsg_small", 2), ("gat_cfg1", 3)]


def run_oracle(z, seed):
    a = concat_arrays(z)
    rel_ws = fused.typed_relation("W2S", a["src"], a["dst"], a["unit"], a["tffrac"], a["edtype"])
    rel_sw = fused.typed_relation("S2W", a["src"], a["dst"], a["unit"], a["tffrac"], a["edtype"])
    n_w, n_s = int(z["n_w"]), int(z["n_s"])
    Xw, Xs, T = gat_inputs(seed, n_w, n_s)
    Xw = Xw.double().requires_grad_()
    Xs = Xs.double().requires_grad_()
    T = T.double().requires_grad_()
    w2s, s2w = seeded_gat_params(seed * 100 + 1, seed * 100 + 2)
    p1 = fused.as_params(w2s)
    p2 = fused.as_params(s2w)
    o1 = fused.wswgat_layer("W2S", rel_ws, Xw, Xs, p1, T)
    o2 = fused.wswgat_layer("S2W", rel_sw, Xw, Xs, p2, T)
    R1, R2 = upstream(seed, o1.shape, o2.shape)
    ((o1 * R1.double()).sum() + (o2 * R2.double()).sum()).backward()
    return dict(o1=o1, o2=o2, Xw=Xw, Xs=Xs, T=T, p1=p1, p2=p2)


def close(a, b, atol, rtol=0.0):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b).max() if a.size else 0.0
    bound = atol + rtol * np.abs(b).max() if b.size else atol
    assert err <= bound, f"max |diff| {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("name,seed", CASES)
def test_oracle_matches_reference(name, seed):
    z = load_fixture(name)
    r = run_oracle(z, seed)
    o1 = r["o1"].detach()
    o2 = r["o2"].detach()
    rows = z["rows_w"] if "rows_w" in z else slice(None)
    close(o1, z["out64_w2s"], 1e-6)
    close(o1, z["out_w2s"], 2e-5)
    close(o2[rows], z["out64_s2w"], 1e-6)
    close(o2[rows], z["out_s2w"], 2e-5)
    close(r["Xs"].grad, z["grad_Xs"], 1e-6, 1e-6)
    close(r["T"].grad, z["grad_T"], 1e-6, 1e-6)
    if "grad_Xw" in z:
        close(r["Xw"].grad, z["grad_Xw"], 1e-6, 1e-6)
    else:
        close(r["Xw"].grad[rows], z["grad_Xw_rows"], 1e-6, 1e-6)
        close(projections(o2, seed, "out_s2w"), z["proj_out_s2w"], 1e-6, 1e-9)
        close(projections(r["Xw"].grad, seed, "grad_Xw"), z["proj_grad_Xw"], 1e-6, 1e-9)
    n_checked = 0
    for tag, params in (("w2s", r["p1"]), ("s2w", r["p2"])):
        for k, p in params.items():
            key = f"grad.{tag}.{k}"
            if key in z:
                close(p.grad, z[key], 1e-6, 1e-6)
                n_checked += 1
            elif "proj." + key in z:
                close(projections(p.grad, seed, key), z["proj." + key], 1e-6, 1e-9)
                n_checked += 1
    assert n_checked >= 2 * 4 + 8 * 3 + 6 * 4


def test_phantom_edges_are_load_bearing():
    """Dropping the untyped in-edges (c_v = 0) must change the W2S output: the
    reference softmax runs over all in-edges."""
    z = load_fixture("gat_small")
    a = concat_arrays(z)
    rel = fused.typed_relation("W2S", a["src"], a["dst"], a["unit"], a["tffrac"], a["edtype"])
    assert rel["phantom"].max() > 0
    Xw, Xs, T = gat_inputs(1, int(z["n_w"]), int(z["n_s"]))
    w2s, _ = seeded_gat_params(101, 102)
    p = fused.as_params(w2s, requires_grad=False)
    with torch.no_grad():
        base = fused.wswgat_layer("W2S", rel, Xw.double(), Xs.double(), p, T.double())
        rel0 = dict(rel, phantom=np.zeros_like(rel["phantom"]))
        nop = fused.wswgat_layer("W2S", rel0, Xw.double(), Xs.double(), p, T.double())
    close(base, z["out64_w2s"], 1e-6)
    assert (base - nop).abs().max() > 1e-2


def test_oracle_ffn_gate_band():
    """oracle.fused.ffn with an implementation's ReLU gates: the fp64 gates reproduce
    the plain ReLU path exactly; a gate flipped inside the fp32 band around zero is
    followed (the backward takes that branch); one flipped outside it is rejected."""
    import pytest
    import torch
    from oracle import fused
    torch.manual_seed(0)
    n, d, dh = 40, 16, 32
    x = torch.randn(n, d, dtype=torch.float64)
    params = {"ffn.w_1.weight": torch.randn(dh, d, dtype=torch.float64) * 0.3,
              "ffn.w_1.bias": torch.randn(dh, dtype=torch.float64) * 0.1,
              "ffn.w_2.weight": torch.randn(d, dh, dtype=torch.float64) * 0.3,
              "ffn.w_2.bias": torch.randn(d, dtype=torch.float64) * 0.1,
              "ffn.layer_norm.weight": torch.ones(d, dtype=torch.float64),
              "ffn.layer_norm.bias": torch.zeros(d, dtype=torch.float64)}
    # put one pre-activation inside the band: v[3, 5] = 1e-9 * (its magnitude sum)
    v = x @ params["ffn.w_1.weight"].t() + params["ffn.w_1.bias"]
    mag = (x.abs() @ params["ffn.w_1.weight"].abs().t() + params["ffn.w_1.bias"].abs())[3, 5]
    params["ffn.w_1.bias"][5] -= v[3, 5] - 1e-9 * mag
    v = x @ params["ffn.w_1.weight"].t() + params["ffn.w_1.bias"]
    gate = v > 0
    assert torch.equal(fused.ffn(x, params), fused.ffn(x, params, gate=gate))
    flipped = gate.clone()
    flipped[3, 5] = ~flipped[3, 5]
    R = torch.randn(n, d, dtype=torch.float64)         # (a plain sum of LN rows has no gradient)
    xg = x.clone().requires_grad_()
    (fused.ffn(xg, params, gate=flipped) * R).sum().backward()
    xr = x.clone().requires_grad_()
    (fused.ffn(xr, params) * R).sum().backward()
    assert not torch.allclose(xg.grad[3], xr.grad[3]) and torch.allclose(xg.grad[4:], xr.grad[4:])
    far = gate.clone()
    i, j = [int(t) for t in torch.nonzero(v.abs() > 0.1)[0]]
    far[i, j] = ~far[i, j]
    with pytest.raises(AssertionError):
        fused.ffn(x, params, gate=far)
