"""DGL-CPU baseline -- TEST/BENCH INFRASTRUCTURE ONLY (never the product path).

A float32 PyTorch-CPU restatement of the reference's WSWGAT execution with the
same *structure* as DGL 0.4 running the reference UDFs (the reference itself and
DGL cannot run on the GPU box; SURVEY §8d "CPU baseline"):

  per head (GATStackLayer.py:56):  dropout(h) -> fc -> frame write of 'z' on the
      source nodes (GATLayer.py:110-111, zero-initialised column);
  apply_edges(edge_attention) on the typed edges (GATLayer.py:89-93, 112):
      gather z at src and dst, feat_fc(tfidfembed) per edge, cat, attn_fc, leaky;
  pull(message_func, reduce_func) (GATLayer.py:95-102, 113) with DGL's degree
      bucketing: per distinct in-degree a mailbox [n_b, deg, D] of ALL in-edges,
      softmax over dim 1, weighted sum, scatter into 'sh';
  cat heads, ELU, residual, FFN (GAT.py:56-58, GATLayer.py:35-44).

bench.py times its forward+backward on the host cores as ``cpu_baseline``
(kind "port"); tests/test_dgl_udf_oracle.py pins it to the golden vectors.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

SLOPE = 0.01


class UdfGraph:
    """Structure a DGL 0.4 graph would hold + the per-relation pull schedule."""

    def __init__(self, src, dst, unit, tffrac, edtype):
        self.src = torch.from_numpy(np.asarray(src, np.int64))
        self.dst = torch.from_numpy(np.asarray(dst, np.int64))
        self.unit = np.asarray(unit)
        self.n = len(self.unit)
        self.tffrac = torch.from_numpy(np.asarray(tffrac, np.int64))
        self.edtype = np.asarray(edtype)
        self.rel = {k: self._schedule(k) for k in ("W2S", "S2W", "S2S")}
        # edata['e'] as the reference's heads leave it (GATLayer.py:89-93, 112 / 148):
        # each head's apply_edges writes its logits on its typed edges, the last one stays
        self.e = torch.zeros(len(self.src), 1)

    def _schedule(self, kind):
        su, du = {"W2S": (0.0, 1.0), "S2W": (1.0, 0.0), "S2S": (1.0, 1.0)}[kind]
        src, dst = self.src.numpy(), self.dst.numpy()
        s_nodes = np.nonzero(self.unit == su)[0]
        d_nodes = np.nonzero(self.unit == du)[0]
        typed = np.nonzero((self.unit[src] == su) & (self.unit[dst] == du))[0]
        in_d = np.isin(dst, d_nodes)
        eids = np.nonzero(in_d)[0]
        order = np.argsort(dst[eids], kind="stable")
        eids = eids[order]
        nodes, start, cnt = np.unique(dst[eids], return_index=True, return_counts=True)
        buckets = []
        for deg in np.unique(cnt):
            w = np.nonzero(cnt == deg)[0]
            mat = eids[(start[w][:, None] + np.arange(deg)[None, :])]
            buckets.append((torch.from_numpy(nodes[w]), torch.from_numpy(mat)))
        return dict(s_nodes=torch.from_numpy(s_nodes), d_nodes=torch.from_numpy(d_nodes),
                    typed=torch.from_numpy(typed), buckets=buckets)


def _head(g, kind, X, fc, feat_w, feat_b, attn, tfidfembed):
    r = g.rel[kind]
    z = X @ fc.t()
    D = z.shape[1]
    zcol = torch.zeros(g.n, D, dtype=z.dtype).index_copy(0, r["s_nodes"], z)          # frame write
    te = r["typed"]
    dfeat = F.linear(tfidfembed[te], feat_w, feat_b)
    z2 = torch.cat([zcol[g.src[te]], zcol[g.dst[te]], dfeat], 1)
    e = F.leaky_relu(z2 @ attn.t(), SLOPE)                                              # [E_T, 1]
    ecol = torch.zeros(len(g.src), 1, dtype=z.dtype).index_copy(0, te, e)
    g.e = g.e.index_copy(0, te, e.detach().to(g.e.dtype))
    sh = torch.zeros(g.n, D, dtype=z.dtype)
    for nodes, mat in r["buckets"]:                                                     # degree buckets
        mb_e = ecol[mat]                                                                # [nb, deg, 1]
        mb_z = zcol[g.src[mat]]                                                         # [nb, deg, D]
        alpha = F.softmax(mb_e, dim=1)
        sh = sh.index_copy(0, nodes, torch.sum(alpha * mb_z, dim=1))
    return sh[r["d_nodes"]]


def _sgat_head(g, X, fc, attn):
    """SGATLayer.forward (GATLayer.py:71-78): z on the unit-1 nodes (zero column
    elsewhere), e = leaky(attn_fc([z_src, z_dst])) written on the dtype-0 edges
    (GATLayer.py:56-59, 68, 74), pull over ALL in-edges of the unit-1 nodes reading
    the edge column (edges never written hold the zero initializer)."""
    r = g.rel["S2S"]
    z = X @ fc.t()
    D = z.shape[1]
    zcol = torch.zeros(g.n, D, dtype=z.dtype).index_copy(0, r["s_nodes"], z)
    te = torch.from_numpy(np.nonzero(g.edtype == 0)[0])
    e = F.leaky_relu(torch.cat([zcol[g.src[te]], zcol[g.dst[te]]], 1) @ attn.t(), SLOPE)
    ecol = torch.zeros(len(g.src), 1, dtype=z.dtype).index_copy(0, te, e)
    g.e = g.e.index_copy(0, te, e.detach().to(g.e.dtype))
    sh = torch.zeros(g.n, D, dtype=z.dtype)
    for nodes, mat in r["buckets"]:
        alpha = F.softmax(ecol[mat], dim=1)
        sh = sh.index_copy(0, nodes, torch.sum(alpha * zcol[g.src[mat]], dim=1))
    return sh[r["d_nodes"]]


def wswgat(g, kind, Xw, Xs, p, tfidfembed, prefix="", drop=0.0, training=False, head_masks=None):
    """WSWGAT.forward (GAT.py:45-59) on the UDF-structured CPU path.  ``head_masks``:
    per-head input multipliers (keep / (1 - p)) replacing F.dropout of the heads."""
    origin, neighbor = (Xs, Xw) if kind == "W2S" else (Xw, Xs)
    outs = []
    i = 0
    while f"{prefix}layer.heads.{i}.fc.weight" in p:
        q = lambda n: p.get(f"{prefix}layer.heads.{i}.{n}")
        x = neighbor * head_masks[i] if head_masks is not None else F.dropout(neighbor, drop, training)
        if kind == "S2S":
            outs.append(_sgat_head(g, x, q("fc.weight"), q("attn_fc.weight")))
        else:
            outs.append(_head(g, kind, x, q("fc.weight"), q("feat_fc.weight"), q("feat_fc.bias"),
                              q("attn_fc.weight"), tfidfembed))
        i += 1
    h = F.elu(torch.cat(outs, 1)) + origin
    x = h.t().unsqueeze(0)                                                             # Conv1d layout
    y = F.conv1d(F.relu(F.conv1d(x, p[f"{prefix}ffn.w_1.weight"], p[f"{prefix}ffn.w_1.bias"])),
                 p[f"{prefix}ffn.w_2.weight"], p[f"{prefix}ffn.w_2.bias"])
    y = F.dropout(y.squeeze(0).t(), drop, training)
    return F.layer_norm(y + h, (h.shape[1],), p[f"{prefix}ffn.layer_norm.weight"],
                        p[f"{prefix}ffn.layer_norm.bias"], 1e-5)


def tfidf_embed(g, T):
    """HiGraph.set_wnfeature's edge side channel (HiGraph.py:146-151)."""
    idx = torch.from_numpy(np.nonzero(g.edtype == 0)[0])
    return torch.zeros(len(g.src), T.shape[1], dtype=T.dtype).index_copy(0, idx, T[g.tffrac[idx]])


def stack_step(g, Xw, Xs, p_w2s, p_s2w, T, n_iter=2, drop=0.0, training=False):
    """W2S + n_iter x (S2W, W2S) (HiGraph.py:99-106) -> supernode state."""
    te = tfidf_embed(g, T)
    s = wswgat(g, "W2S", Xw, Xs, p_w2s, te, drop=drop, training=training)
    w = Xw
    for _ in range(n_iter):
        w = wswgat(g, "S2W", w, s, p_s2w, te, drop=drop, training=training)
        s = wswgat(g, "W2S", w, s, p_w2s, te, drop=drop, training=training)
    return s
