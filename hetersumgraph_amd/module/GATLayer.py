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
from ..relation import N_BOX, edge_dst

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


class SGATLayer(nn.Module):
    """Sentence -> sentence head (GATLayer.py:49-78): ``fc`` and ``attn_fc`` over
    [z_src, z_dst], no edge feature.  Only ``WSWGAT(layerType="S2S")`` builds it
    (GAT.py:38-39), through :class:`..GATStackLayer.MultiHeadSGATLayer`, which moves
    the values into fused tensors and ``bind``s the head like ``_HeadParams``."""

    kind = "S2S"

    def __init__(self, in_dim, out_dim, weight=0):
        super().__init__()
        self.weight = weight
        self.fc = nn.Linear(in_dim, out_dim, bias=False)
        self.attn_fc = nn.Linear(2 * out_dim, 1, bias=False)
        self._index = 0

    def bind(self, parent, index):
        del self.fc, self.attn_fc
        object.__setattr__(self, "_parent_layer", parent)
        self._index = index

    def params(self):
        """(fc_weight [D, in], attn_weight [1, 2D])."""
        p = self.__dict__.get("_parent_layer")
        if p is None:
            return self.fc.weight, self.attn_fc.weight
        k, D = self._index, p.head_dim
        return p.fc_weight[k * D:(k + 1) * D], p.attn_weight[k:k + 1]

    def forward(self, g, h):
        """One head on its own (reference signature): [n_unit1, out_dim]."""
        return sgat_heads(g, h, self.params(), origin=None, dropout=None)


def sgat_heads(g, h, params, origin=None, dropout=None):
    """All S2S heads in one pass of the WSWGAT edge kernel (+ ELU/residual if origin).

    What the reference computes per head (GATLayer.py:71-78): z = fc(h) on the unit-1
    nodes (words keep the zero-initialised column); e = leaky(a1.z_src + a2.z_dst) on
    the dtype-0 edges; a pull onto every unit-1 node over ALL its in-edges.  On those
    in-edges:
      * from a unit-1 node (s->s, s->doc): e is never written there (0), message z_u;
      * from a word (w->s, w->doc; dtype 0): e = leaky(a2.z_v) =: p_v for every such
        edge of v (z_src = 0), message 0.
    That is the S2S relation (relation.KINDS) with c_v = #word in-edges as phantoms,
    except that the phantoms score p_v instead of 0.  Shifting every score of v by
    -p_v (softmax is shift-invariant) gives phantoms 0 and typed edges -p_v, which the
    kernel's per-edge tau mode expresses with sigma = 0 and tau_e = t(p_v), t chosen
    so leaky(t) = -p_v.  The gradient reaches p (and a2, Z) through tau by autograd.

    ``params``: a MultiHeadSGATLayer or (fc_weight [H*D, in], attn_weight [H, 2D])."""
    rel = g.relation("S2S")
    W, attn = params.fused_params()[:2] if hasattr(params, "fused_params") else params
    H = attn.shape[0]
    D = W.shape[0] // H
    if attn.shape[1] != 2 * D:
        raise ValueError(f"S2S attn_fc has {attn.shape[1]} inputs, expected 2 * {D}")
    if h.shape[0] != rel.n_src:
        raise ValueError(f"S2S: input has {h.shape[0]} rows, graph has {rel.n_src} unit-1 nodes")
    if dropout is not None and dropout.training and dropout.p > 0:
        Z = head_projection_dropout(h, W, H, D, dropout.p)
    else:
        Z = native_linear(h, W)
    p = F.leaky_relu((Z.view(-1, H, D) * attn[:, D:]).sum(-1), LEAKY_SLOPE)       # [n, H]
    t = torch.where(p > 0, p * (-1.0 / LEAKY_SLOPE), -p)                           # leaky(t) = -p
    tau = t[edge_dst(rel)]                                                         # [E_T, H]
    out = gat_aggregate(Z, Z.new_zeros(H, D), tau, origin, rel, H, D, LEAKY_SLOPE, HSG_TAU_PER_EDGE)
    record_edge_scores(g, SGATScores(g, Z, attn))
    return out


class SGATScores:
    """The S2S rows of ``g.edata['e']``: the last head's e = leaky(a1.z_src + a2.z_dst)
    on every dtype-0 edge (GATLayer.py:56-59, 74-75), z = 0 on words.  Formed on read,
    like :class:`LastHeadScores`."""

    key = "S2S"

    def __init__(self, g, Z, attn):
        self.eid, self.srank, self.drank = _dtype0_edges(g)
        H = attn.shape[0]
        D = Z.shape[1] // H
        self.z = Z.detach()[:, (H - 1) * D:]
        self.a = attn.detach()[H - 1]

    def scores(self):
        D = self.z.shape[1]
        zero = self.z.new_zeros(1)
        s1 = torch.cat([self.z @ self.a[:D], zero])                     # row n_s: a word
        s2 = torch.cat([self.z @ self.a[D:], zero])
        return F.leaky_relu(s1[self.srank] + s2[self.drank], LEAKY_SLOPE)

    def to(self, device):
        c = SGATScores.__new__(SGATScores)
        c.__dict__.update({k: (v.to(device) if isinstance(v, torch.Tensor) else v) for k, v in self.__dict__.items()})
        return c


def _dtype0_edges(g):
    """(eid, src rank, dst rank) of the dtype-0 edges (GATLayer.py:68), ranks among the
    unit-1 nodes with n_unit1 for a word; cached per graph and device."""
    key = ("s2s_e", str(g.device))
    if key not in g._rel_cache:
        g._flush()
        ef = g._eframe().cols
        if "dtype" not in ef:
            raise KeyError("dtype")   # edges.data['dtype'] in GATLayer.py:68
        is1 = g._nframe.cols["unit"] == 1
        rank = torch.cumsum(is1.long(), 0) - 1
        rank = torch.where(is1, rank, is1.sum())
        eid = (ef["dtype"] == 0).nonzero().view(-1)
        src, dst = g._src_t(), g._dst_t()
        g._rel_cache[key] = (eid, rank[src[eid]], rank[dst[eid]])
    return g._rel_cache[key]


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
