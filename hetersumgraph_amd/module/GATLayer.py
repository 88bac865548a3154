"""Per-head GAT layers and the position-wise FFN (reference: module/GATLayer.py).

State-dict names and shapes match the reference exactly, but
the computation is not per head: ``MultiHeadLayer`` keeps every head's weights in
fused tensors and runs all heads in one HIP pass
(:func:`hetersumgraph_amd.ops.gat_aggregate`).  A single head's ``forward(g, h)``
is still available and is the same kernel with H = 1.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ffn import ffn_forward
from ..dense import linear as native_linear
from ..hproj import head_projection_dropout
from ..ops import LEAKY_SLOPE, gat_aggregate, gat_heads_table, HSG_TAU_PER_EDGE, HSG_TAU_TABLE
from ..graph import record_edge_scores
from ..relation import N_BOX

# The reference asserts "no NaN" around every FFN (GATLayer.py:36, 43), a host sync
# per call.  Same error behaviour behind a switch (default off: it would serialise
# the stream and break HIP-graph capture).
CHECK_NAN = os.environ.get("HSG_CHECK_NAN", "0") == "1"

TFIDF_TAG = "tffrac@dtype0"


class PositionwiseFeedForward(nn.Module):
    """LN(x + Dropout(W2 relu(W1 x + b1) + b2)), eps 1e-5 (GATLayer.py:25-44).

    Kept as two k=1 ``Conv1d`` modules for state_dict compatibility; executed as
    MFMA GEMMs with fused epilogues (:mod:`hetersumgraph_amd.ffn`)."""

    def __init__(self, d_in, d_hid, dropout=0.1):
        super().__init__()
        self.w_1 = nn.Conv1d(d_in, d_hid, 1)
        self.w_2 = nn.Conv1d(d_hid, d_in, 1)
        self.layer_norm = nn.LayerNorm(d_in)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])            # reference feeds [1, n, d] (GAT.py:58)
        if CHECK_NAN:
            assert not torch.any(torch.isnan(x2)), "FFN input"
        p = self.dropout.p if self.training else 0.0
        y = ffn_forward(x2, self.w_1.weight.squeeze(-1), self.w_1.bias, self.w_2.weight.squeeze(-1),
                        self.w_2.bias, self.layer_norm.weight, self.layer_norm.bias, p, self.layer_norm.eps)
        if CHECK_NAN:
            assert not torch.any(torch.isnan(y)), "FFN output"
        return y.reshape(shape)


class _HeadParams(nn.Module):
    """fc / feat_fc / attn_fc of one head (GATLayer.py:82-87, 121-126).

    Built exactly like the reference head (so seeded initialisation matches); a
    MultiHeadLayer then moves the values into its fused tensors and ``bind``s the
    head, which from then on owns no parameters and reads views of the fused
    storage."""

    kind = None
    feat_bias = False

    def __init__(self, in_dim, out_dim, feat_embed_size):
        super().__init__()
        self.fc = nn.Linear(in_dim, out_dim, bias=False)
        self.feat_fc = nn.Linear(feat_embed_size, out_dim, bias=self.feat_bias)
        self.attn_fc = nn.Linear(3 * out_dim, 1, bias=False)
        self._index = 0

    def bind(self, parent, index):
        del self.fc, self.feat_fc, self.attn_fc
        # plain (non-submodule) back-reference: survives deepcopy/pickle as a cycle
        object.__setattr__(self, "_parent_layer", parent)
        self._index = index

    def params(self):
        """(fc_weight [D,in], attn_weight [1,3D], feat_weight [1,D,F], feat_bias [1,D]|None)."""
        p = self.__dict__.get("_parent_layer")
        if p is None:
            fb = self.feat_fc.bias.unsqueeze(0) if self.feat_fc.bias is not None else None
            return self.fc.weight, self.attn_fc.weight, self.feat_fc.weight.unsqueeze(0), fb
        k, D = self._index, p.head_dim
        fb = p.feat_bias[k:k + 1] if p.feat_bias is not None else None
        return p.fc_weight[k * D:(k + 1) * D], p.attn_weight[k:k + 1], p.feat_weight[k:k + 1], fb

    def forward(self, g, h):
        """One head on its own (reference signature): returns [n_dst, out_dim]."""
        return fused_heads(g, h, self.params(), self.kind, origin=None, dropout=None)


class WSGATLayer(_HeadParams):
    """Word -> sentence head (GATLayer.py:81-116): feat_fc has no bias."""

    kind = "W2S"
    feat_bias = False


class SWGATLayer(_HeadParams):
    """Sentence -> word head (GATLayer.py:120-152): feat_fc has a bias."""

    kind = "S2W"
    feat_bias = True


def edge_tau(g, rel, a3, wf, bf):
    """tau = a3 . feat_fc(tfidfembed) per (tf-idf box | edge) and head.

    Fast path: ``tfidfembed`` was written by HSumGraph.set_wnfeature as a table
    column (``_TFembed.weight`` rows selected by ``tffrac`` on dtype-0 edges,
    HiGraph.py:146-151) -> an [11, H] table (row 10 = never-written edges).
    Generic path: a dense per-edge ``tfidfembed`` from a foreign caller ->
    [E_T, H] in CSR order."""
    from ..graph import TableColumn

    col = g._eframe().cols.get("tfidfembed")
    if col is None:
        raise KeyError("tfidfembed")   # edges.data['tfidfembed'] in the reference UDF
    v = torch.einsum("kd,kdf->kf", a3, wf)                               # [H, F]
    c = (a3 * bf).sum(-1) if bf is not None else None                    # [H]
    if isinstance(col, TableColumn) and col.tag == TFIDF_TAG and col.weight.shape[0] == N_BOX:
        tau = F.pad(col.weight @ v.t(), (0, 0, 0, 1))                    # [11, H], row 10 = 0
        if c is not None:
            tau = tau + c
        return tau, HSG_TAU_TABLE
    dense = col.materialize() if isinstance(col, TableColumn) else col
    eid = rel.dev["eid"]
    tau = dense[eid].to(v.dtype) @ v.t()
    if c is not None:
        tau = tau + c
    return tau, HSG_TAU_PER_EDGE


class LastHeadScores:
    """One relation's rows of ``g.edata['e']`` (graph.EdgeScoreColumn): the last head's
    logits e = leaky_relu(a1 . z_src + a3 . feat_fc(tfidfembed)) on the typed edges
    (GATLayer.py:89-93; z_dst is the zero-initialised column there, so a2 adds
    nothing).  Holds the application's projected features Z and the head parameters
    (detached) and forms the rows on demand: per-edge logits are never built on the
    HIP path.  The edge term comes from ``T`` (the [10, F] tf-idf table), ``tau_table``
    ([11, H] per tf-idf box) or ``tau_edge`` ([E_T, H], CSR order)."""

    def __init__(self, kind, rel, Z, attn, wf, bf, T=None, tau_table=None, tau_edge=None):
        self.key = kind
        d = rel.dev
        self.eid, self.src, self.tf = d["eid"], d["src"], d["tf"]
        H = attn.shape[0]
        D = Z.shape[1] // H
        k = H - 1
        self.z = Z.detach()[:, k * D:]                                   # [n_src, D]
        self.a1 = attn.detach()[k, :D]
        self.a3 = attn.detach()[k, 2 * D:]
        self.wf = wf.detach()[k]                                         # [D, F]
        self.bf = bf.detach()[k] if bf is not None else None
        self.T = T.detach() if T is not None else None
        self.tau_table = tau_table.detach()[:, k] if tau_table is not None else None
        self.tau_edge = tau_edge.detach()[:, k] if tau_edge is not None else None

    def scores(self):
        sig = self.z @ self.a1                                           # [n_src]
        if self.T is not None:
            rows = self.T @ (self.wf.t() @ self.a3)                      # [10]
            if self.bf is not None:
                rows = rows + (self.a3 * self.bf).sum()
            tau = rows[self.tf.long()]
        elif self.tau_table is not None:
            tau = self.tau_table[self.tf.long()]
        else:
            tau = self.tau_edge
        return F.leaky_relu(sig[self.src.long()] + tau, LEAKY_SLOPE)

    def to(self, device):
        c = LastHeadScores.__new__(LastHeadScores)
        c.__dict__.update({k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.__dict__.items()})
        return c


def fused_heads(g, h, params, kind, origin=None, dropout=None):
    """All heads of one layer application in one pass (+ ELU/residual if origin).

    ``params``: a MultiHeadLayer (fused tensors) or a tuple (fc_weight [H*D, in],
    attn_weight [H, 3D], feat_weight [H, D, F], feat_bias [H, D] | None).
    ``dropout``: the MultiHeadLayer's nn.Dropout, applied to ``h`` with an
    independent mask per head in training mode (GATStackLayer.py:56)."""
    rel = g.relation(kind)
    W, attn, wf, bf = params.fused_params() if hasattr(params, "fused_params") else params
    H = attn.shape[0]
    D = W.shape[0] // H
    a1 = attn[:, :D]                                                     # z_src weights
    a3 = attn[:, 2 * D:]                                                 # feat weights (z_dst part unused)
    if h.shape[0] != rel.n_src:
        raise ValueError(f"{kind}: input has {h.shape[0]} rows, graph has {rel.n_src} source nodes")
    if dropout is not None and dropout.training and dropout.p > 0:
        Z = head_projection_dropout(h, W, H, D, dropout.p)               # per-head masks, fused
    else:
        Z = native_linear(h, W)                                          # hsg_gemm_f32 (no vendor GEMM)
    T = table_weight(g)
    if T is not None and T.shape[1] == wf.shape[2]:
        out = gat_heads_table(Z, attn, T, wf, bf, origin, rel, H, D, LEAKY_SLOPE)
        record_edge_scores(g, LastHeadScores(kind, rel, Z, attn, wf, bf, T=T))
        return out
    tau, mode = edge_tau(g, rel, a3, wf, bf)
    out = gat_aggregate(Z, a1, tau, origin, rel, H, D, LEAKY_SLOPE, mode)
    if mode == HSG_TAU_TABLE:
        record_edge_scores(g, LastHeadScores(kind, rel, Z, attn, wf, bf, tau_table=tau))
    else:
        record_edge_scores(g, LastHeadScores(kind, rel, Z, attn, wf, bf, tau_edge=tau))
    return out


def table_weight(g):
    """The [10, F] TF-IDF embedding table behind edata['tfidfembed'] when that column
    was written by HSumGraph.set_wnfeature (HiGraph.py:146-151), else None."""
    from ..graph import TableColumn

    col = g._eframe().cols.get("tfidfembed")
    if col is None:
        raise KeyError("tfidfembed")   # edges.data['tfidfembed'] in the reference UDF
    if isinstance(col, TableColumn) and col.tag == TFIDF_TAG and col.weight.shape[0] == N_BOX:
        return col.weight
    return None
