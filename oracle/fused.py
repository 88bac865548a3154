"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline
leg, as the *checker*; never by the product path (hetersumgraph_amd/).

A float64 PyTorch-CPU restatement of one WSWGAT application, written edge-wise
like the reference (no tau-table shortcut, no fused kernels), so it checks both
the HIP kernels and the algebra they rely on.  Pinned against the golden vectors
that the reference's own module code produced (tests/golden/, see
tests/test_oracle_golden.py).

Reference lines restated:
  typed_relation  -- GATLayer.py:105-107 / 143-145 (filters) + DGL 0.4 pull's
                     in-edge set (113 / 149) incl. untyped "phantom" in-edges
  wswgat_layer    -- GAT.py:45-59, GATStackLayer.py:55-59, GATLayer.py:89-102,
                     110-116, 128-152, and PositionwiseFeedForward 35-44;
                     train mode takes explicit keep-masks for the per-head input
                     dropout (GATStackLayer.py:56) and the FFN output dropout
                     (GATLayer.py:41) -- oracle/masks.py computes the kernels' ones
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

SLOPE = 0.01


def typed_relation(kind, src, dst, unit, tffrac, edtype):
    """Typed edges and phantom counts of one layer type (numpy, edge-id order)."""
    su, du = {"W2S": (0.0, 1.0), "S2W": (1.0, 0.0), "S2S": (1.0, 1.0)}[kind]
    unit = np.asarray(unit)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    is_s, is_d = unit == su, unit == du
    s_nodes, d_nodes = np.nonzero(is_s)[0], np.nonzero(is_d)[0]
    s_rank = np.full(len(unit), -1)
    s_rank[s_nodes] = np.arange(len(s_nodes))
    d_rank = np.full(len(unit), -1)
    d_rank[d_nodes] = np.arange(len(d_nodes))
    typed = np.nonzero(is_s[src] & is_d[dst])[0]
    indeg = np.bincount(dst, minlength=len(unit))[d_nodes]
    n_typed_in = np.bincount(d_rank[dst[typed]], minlength=len(d_nodes))
    has_tf = np.asarray(edtype)[typed] == 0        # tfidfembed written on dtype-0 edges only
    return dict(e_src=s_rank[src[typed]], e_dst=d_rank[dst[typed]],
                tf=np.where(has_tf, np.asarray(tffrac)[typed], -1),
                phantom=indeg - n_typed_in, any_in=indeg > 0,
                n_src=len(s_nodes), n_dst=len(d_nodes))


def _heads(params, prefix, H):
    return [dict(fc=params[f"{prefix}layer.heads.{i}.fc.weight"],
                 feat_w=params[f"{prefix}layer.heads.{i}.feat_fc.weight"],
                 feat_b=params.get(f"{prefix}layer.heads.{i}.feat_fc.bias"),
                 attn=params[f"{prefix}layer.heads.{i}.attn_fc.weight"]) for i in range(H)]


def n_heads(params, prefix=""):
    i = 0
    while f"{prefix}layer.heads.{i}.fc.weight" in params:
        i += 1
    return i


def gat_heads(rel, X, params, T, prefix="", keep=None, scale=1.0):
    """Concatenated head outputs (before ELU) -- GATStackLayer.py:55-59.
    ``keep``: train mode, bool [H, n_src, in] per-head input keep-masks
    (GATStackLayer.py:56, ``head(g, self.dropout(h))``), kept values x ``scale``."""
    H = n_heads(params, prefix)
    e_src = torch.from_numpy(rel["e_src"])
    e_dst = torch.from_numpy(rel["e_dst"])
    tf = torch.from_numpy(rel["tf"])
    n_dst = rel["n_dst"]
    phantom = torch.from_numpy(rel["phantom"]).to(X.dtype)
    tfe = torch.where((tf >= 0).unsqueeze(1), T[tf.clamp_min(0)], torch.zeros((), dtype=X.dtype))
    outs = []
    for k, hd in enumerate(_heads(params, prefix, H)):
        Xk = X if keep is None else X * (torch.as_tensor(keep[k]).to(X.dtype) * scale)
        z = Xk @ hd["fc"].t()                                  # GATLayer.py:110 / 146
        D = z.shape[1]
        dfeat = tfe @ hd["feat_w"].t()
        if hd["feat_b"] is not None:
            dfeat = dfeat + hd["feat_b"]
        zsrc = z[e_src]
        zdst = torch.zeros_like(zsrc)                          # dst 'z' never written -> 0
        wa = torch.cat([zsrc, zdst, dfeat], 1) @ hd["attn"].t()   # attn_fc, GATLayer.py:91-92
        e = F.leaky_relu(wa.squeeze(1), SLOPE)
        # softmax over ALL in-edges of each dst: typed edges + phantoms with e = 0
        mx = torch.full((n_dst,), -torch.inf, dtype=X.dtype).scatter_reduce(0, e_dst, e, "amax")
        mx = torch.where(phantom > 0, torch.clamp_min(mx, 0.0), mx)
        mx = torch.where(torch.isinf(mx), torch.zeros_like(mx), mx).detach()
        p = torch.exp(e - mx[e_dst])
        den = torch.zeros(n_dst, dtype=X.dtype).index_add(0, e_dst, p) + phantom * torch.exp(-mx)
        alpha = p / den[e_dst]
        h = torch.zeros(n_dst, D, dtype=X.dtype).index_add(0, e_dst, alpha.unsqueeze(1) * zsrc)
        outs.append(h)
    return torch.cat(outs, 1)


# ReLU gates within fp32 resolution of zero (see ``ffn``): |v| below this fraction of
# the pre-activation's magnitude sum sum_c |x_c w_c| + |b|
GATE_BAND = 2.0 ** -16


def ffn(x, params, prefix="", keep=None, scale=1.0, gate=None):
    """PositionwiseFeedForward (GATLayer.py:35-44).  ``keep``: train mode, the bool
    [n, d] keep-mask of the output dropout (GATLayer.py:41), kept values x ``scale``.
    ``gate``: the bool [n, d_hid] ReLU gates an fp32 implementation took (H > 0).
    Where the fp64 pre-activation v lies within GATE_BAND of its magnitude sum of
    zero, fp32 rounding of the inputs decides the gate either way, so the oracle takes
    the implementation's gate there (its backward then follows the same branch; the
    forward value moves by at most |v|); everywhere else the gates must agree, which
    is asserted."""
    w1 = params[f"{prefix}ffn.w_1.weight"].squeeze(-1)
    w2 = params[f"{prefix}ffn.w_2.weight"].squeeze(-1)
    b1 = params[f"{prefix}ffn.w_1.bias"]
    v = x @ w1.t() + b1
    if gate is None:
        h = F.relu(v)
    else:
        g = torch.as_tensor(gate).to(torch.bool)
        with torch.no_grad():
            band = GATE_BAND * (x.abs() @ w1.abs().t() + b1.abs())
            prone = v.abs() < band
            on = v > 0
            bad = (on != g) & ~prone
            assert not bad.any(), f"{int(bad.sum())} ReLU gates differ outside the fp32 band"
            mask = torch.where(prone, g, on).to(v.dtype)
        h = v * mask
    y = h @ w2.t() + params[f"{prefix}ffn.w_2.bias"]
    if keep is not None:
        y = y * (torch.as_tensor(keep).to(y.dtype) * scale)
    return F.layer_norm(y + x, (x.shape[1],), params[f"{prefix}ffn.layer_norm.weight"],
                        params[f"{prefix}ffn.layer_norm.bias"], 1e-5)


def wswgat_layer(kind, rel, Xw, Xs, params, T, prefix="", masks=None, gate=None):
    """WSWGAT.forward(g, w, s) (GAT.py:45-59).  Eval mode, or train mode with
    ``masks`` = (head keep [H, n_src, in], head scale, FFN keep [n_dst, d], FFN
    scale) -- e.g. oracle/masks.py's restatement of the kernels' masks.  ``gate``:
    the FFN's ReLU gates of an fp32 run (``ffn``)."""
    origin, neighbor = (Xs, Xw) if kind == "W2S" else (Xw, Xs)
    hk, hs, fk, fs = masks if masks is not None else (None, 1.0, None, 1.0)
    h = F.elu(gat_heads(rel, neighbor, params, T, prefix, keep=hk, scale=hs)) + origin
    return ffn(h, params, prefix, keep=fk, scale=fs, gate=gate)


def as_params(module_or_dict, dtype=torch.float64, requires_grad=True):
    """name -> leaf tensor (float64) from a state_dict-like mapping."""
    src = module_or_dict.state_dict() if hasattr(module_or_dict, "state_dict") else module_or_dict
    out = {}
    for k, v in src.items():
        t = torch.as_tensor(np.asarray(v.detach().cpu() if hasattr(v, "detach") else v)).to(dtype)
        out[k] = t.clone().requires_grad_(requires_grad)
    return out


def gat_aggregate_ref(e_src, e_dst, tf_row, phantom, n_dst, Z, a1, tau, origin=None, slope=SLOPE):
    """Op-level restatement of ``hetersumgraph_amd.ops.gat_aggregate`` (the fused
    restatement of SURVEY §8a) for kernel-level checks: Z [n_src, H*D], a1 [H, D],
    tau [rows, H] indexed by ``tf_row`` per typed edge (CSR or any order)."""
    H, D = a1.shape
    Zh = Z.view(Z.shape[0], H, D)
    sigma = (Zh * a1.unsqueeze(0)).sum(-1)                          # [n_src, H]
    e_src = torch.as_tensor(e_src, dtype=torch.long)
    e_dst = torch.as_tensor(e_dst, dtype=torch.long)
    tf_row = torch.as_tensor(tf_row, dtype=torch.long)
    phantom = torch.as_tensor(phantom).to(Z.dtype)
    s = F.leaky_relu(sigma[e_src] + tau[tf_row], slope)              # [E, H]
    mx = torch.full((n_dst, H), -torch.inf, dtype=Z.dtype).scatter_reduce(
        0, e_dst.unsqueeze(1).expand(-1, H), s, "amax")
    mx = torch.where(phantom.unsqueeze(1) > 0, torch.clamp_min(mx, 0.0), mx)
    mx = torch.where(torch.isinf(mx), torch.zeros_like(mx), mx).detach()
    p = torch.exp(s - mx[e_dst])
    den = torch.zeros(n_dst, H, dtype=Z.dtype).index_add(0, e_dst, p) + phantom.unsqueeze(1) * torch.exp(-mx)
    alpha = p / den[e_dst]
    h = torch.zeros(n_dst, H, D, dtype=Z.dtype).index_add(0, e_dst, alpha.unsqueeze(-1) * Zh[e_src])
    h = h.view(n_dst, H * D)
    return h if origin is None else F.elu(h) + origin
