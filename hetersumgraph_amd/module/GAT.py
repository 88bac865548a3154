"""WSWGAT -- the operator surface of the hot path (reference: module/GAT.py:30-59).

Same constructor signature and ``forward(g, w, s)`` contract:

* ``layerType="W2S"``: origin = s (sentence/doc state), neighbour = w (word state);
  returns the new supernode state [n_unit1, out_dim];
* ``layerType="S2W"``: origin = w, neighbour = s; returns the new word state
  [n_unit0, out_dim];
* ``layerType="S2S"``: w and s must be equal (GAT.py:50); origin = neighbour = s,
  heads :class:`MultiHeadSGATLayer` (sentence -> sentence over all in-edges of the
  unit-1 nodes, GATLayer.py:49-78); returns [n_unit1, out_dim];
* ``out = FFN(elu(MultiHeadLayer(g, neighbour)) + origin)``.

The ELU and residual run inside the edge kernel's epilogue.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .GATLayer import PositionwiseFeedForward, SWGATLayer, WSGATLayer
from .GATStackLayer import MultiHeadLayer, MultiHeadSGATLayer


class WSWGAT(nn.Module):
    def __init__(self, in_dim, out_dim, num_heads, attn_drop_out, ffn_inner_hidden_size, ffn_drop_out,
                 feat_embed_size, layerType):
        super().__init__()
        self.layerType = layerType
        head_dim = int(out_dim / num_heads)   # GAT.py:35, 37
        if layerType == "W2S":
            self.layer = MultiHeadLayer(in_dim, head_dim, num_heads, attn_drop_out, feat_embed_size,
                                        layer=WSGATLayer)
        elif layerType == "S2W":
            self.layer = MultiHeadLayer(in_dim, head_dim, num_heads, attn_drop_out, feat_embed_size,
                                        layer=SWGATLayer)
        elif layerType == "S2S":
            # GAT.py:38-39; no model constructs it
            self.layer = MultiHeadSGATLayer(in_dim, head_dim, num_heads, attn_drop_out)
        else:
            raise NotImplementedError("GAT Layer has not been implemented!")
        self.ffn = PositionwiseFeedForward(out_dim, ffn_inner_hidden_size, ffn_drop_out)

    def forward(self, g, w, s):
        if self.layerType == "W2S":
            origin, neighbor = s, w
        elif self.layerType == "S2S":
            if w is not s and not torch.equal(w, s):     # GAT.py:50 (a host sync there too)
                raise AssertionError("S2S: w and s differ")
            origin, neighbor = w, s
        else:
            origin, neighbor = w, s
        h = self.layer(g, neighbor, origin=origin)   # elu(heads) + origin, fused
        return self.ffn(h)
