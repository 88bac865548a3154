"""S2S (``WSWGAT(layerType="S2S")``, /root/reference/module/GAT.py:38-39, 49-51;
``MultiHeadSGATLayer`` GATStackLayer.py:27-44 of ``SGATLayer`` GATLayer.py:49-78) on
the CPU: the UDF oracle against the reference's own golden vectors
(tests/golden/s2s_small.npz, made by tests/golden/make_golden.py --only s2s_small),
and the score shift the HIP path uses (module/GATLayer.sgat_heads) restated with the
op-level oracle, against the UDF oracle.

The reference's S2S pull onto a unit-1 node v reads ALL its in-edges: from unit-1
nodes with e = 0 (never written) and message z_u, from words with e = leaky(a2.z_v)
and message 0 (words hold the zero z column).  The HIP path runs it as the S2S
relation (typed = unit-1 -> unit-1, phantoms = word in-edges) with every score of v
shifted by -leaky(a2.z_v)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import weights
from helpers import concat_arrays, load_fixture
from oracle import dgl_udf, fused

CASES = [("hsg", 31), ("hdsg", 32)]


def _case(tag):
    z = load_fixture("s2s_small")
    return {k[len(tag) + 1:]: v for k, v in z.items() if k.startswith(tag + ".")}


def _module(seed, d=64, H=8):
    from hetersumgraph_amd.module.GAT import WSWGAT
    return weights.seed_module(WSWGAT(d, d, H, 0.1, 512, 0.1, 50, "S2S"), seed * 100 + 3).eval()


def _graph(z):
    a = concat_arrays(z)
    return dgl_udf.UdfGraph(a["src"], a["dst"], a["unit"], a["tffrac"], a["edtype"]), a


def test_state_dict_speaks_reference_keys():
    z = _case("hsg")
    ref = sorted(k[len("grad.s2s."):] for k in z if k.startswith("grad.s2s."))
    m = _module(31)
    assert sorted(m.state_dict().keys()) == ref
    for k, v in m.state_dict().items():
        assert tuple(v.shape) == z["grad.s2s." + k].shape
    m2 = _module(99)
    m2.load_state_dict(m.state_dict())
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), m2.state_dict().values()))


@pytest.mark.parametrize("tag,seed", CASES)
def test_udf_oracle_matches_reference(tag, seed):
    z = _case(tag)
    g, _ = _graph(z)
    p = fused.as_params(_module(seed), dtype=torch.float64)
    Xs = torch.from_numpy(weights.feature(seed, "Xs", (int(z["n_s"]), 64), 1.0)).double().requires_grad_()
    out = dgl_udf.wswgat(g, "S2S", Xs, Xs, p, None)
    assert np.abs(out.detach().numpy() - z["out64_s2s"]).max() <= 1e-5
    assert np.abs(g.e.numpy() - z["e64"]).max() <= 1e-5
    R = torch.from_numpy(weights.feature(seed, "R_s2s", tuple(out.shape))).double()
    (out * R).sum().backward()
    assert np.abs(Xs.grad.numpy() - z["grad_Xs"]).max() <= 1e-5 * max(1.0, np.abs(z["grad_Xs"]).max())
    for k, v in p.items():
        ref = z["grad.s2s." + k]
        assert np.abs(v.grad.numpy() - ref).max() <= 1e-5 * max(1.0, np.abs(ref).max()), k
    # fp32 oracle against the reference's fp32 CPU run
    p32 = fused.as_params(_module(seed), dtype=torch.float32)
    g32, _ = _graph(z)
    o32 = dgl_udf.wswgat(g32, "S2S", Xs.detach().float(), Xs.detach().float(), p32, None)
    assert np.abs(o32.detach().numpy() - z["out_s2s"]).max() <= 2e-5


def test_fixture_covers_the_edge_cases():
    """Sentences with no word in-edge (no phantom), HDSG doc nodes (s->doc typed,
    w->doc phantoms), and dtype-0 edges in both directions."""
    for tag, _ in CASES:
        z = _case(tag)
        r = fused.typed_relation("S2S", **{k: concat_arrays(z)[k] for k in ("src", "dst", "unit", "tffrac", "edtype")})
        assert (r["phantom"] > 0).any() and len(r["e_src"]) > 0
        if tag == "hsg":
            assert (r["phantom"] == 0).any()
        else:
            assert (z["g_ndtype"] == 2).any()


@pytest.mark.parametrize("tag,seed", CASES)
def test_score_shift_equals_udf_pull(tag, seed):
    """sigma = 0 and per-destination tau = t(p_v), leaky(t(p)) = -p, p_v = leaky(a2.z_v):
    the kernel's softmax over typed edges + phantoms equals the reference's pull."""
    z = _case(tag)
    g, a = _graph(z)
    r = fused.typed_relation("S2S", a["src"], a["dst"], a["unit"], a["tffrac"], a["edtype"])
    m = _module(seed)
    p = fused.as_params(m, dtype=torch.float64, requires_grad=False)
    Xs = torch.from_numpy(weights.feature(seed, "Xs", (int(z["n_s"]), 64), 1.0)).double()
    H, D = 8, 8
    W = torch.cat([p[f"layer.heads.{k}.fc.weight"] for k in range(H)])
    attn = torch.cat([p[f"layer.heads.{k}.attn_fc.weight"] for k in range(H)])
    Z = Xs @ W.t()
    pv = F.leaky_relu((Z.view(-1, H, D) * attn[:, D:]).sum(-1), dgl_udf.SLOPE)
    t = torch.where(pv > 0, pv * (-1.0 / dgl_udf.SLOPE), -pv)
    assert torch.allclose(F.leaky_relu(t, dgl_udf.SLOPE), -pv, rtol=1e-12, atol=0)
    h = fused.gat_aggregate_ref(r["e_src"], r["e_dst"], r["e_dst"], r["phantom"], r["n_dst"], Z,
                                torch.zeros(H, D, dtype=Z.dtype), t, origin=Xs)
    heads = [dgl_udf._sgat_head(g, Xs, p[f"layer.heads.{k}.fc.weight"], p[f"layer.heads.{k}.attn_fc.weight"])
             for k in range(H)]
    ref = F.elu(torch.cat(heads, 1)) + Xs
    assert (h - ref).abs().max().item() <= 1e-12
