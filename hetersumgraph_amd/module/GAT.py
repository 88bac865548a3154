"""WSWGAT -- the operator surface of the hot path (reference: module/GAT.py:30-59).

Same constructor signature and ``forward(g, w, s)`` contract:

* ``layerType="W2S"``: origin = s (sentence/doc state), neighbour = w (word state);
  returns the new supernode state [n_unit1, out_dim];
* ``layerType="S2W"``: origin = w, neighbour = s; returns the new word state
  [n_unit0, out_dim];
* ``out = FFN(elu(MultiHeadLayer(g, neighbour)) + origin)``.

The ELU and residual run inside the edge kernel's epilogue.
"""
from __future__ import annotations

import torch.nn as nn

from .GATLayer import PositionwiseFeedForward, SWGATLayer, WSGATLayer
from .GATStackLayer import MultiHeadLayer


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
            # GAT.py:38-39 builds MultiHeadSGATLayer, which no model constructs
            # (SURVEY §2 rows 1-2); it is outside this build's hot path.
            raise NotImplementedError("S2S (SGATLayer) is not part of the WSWGAT hot path")
        else:
            raise NotImplementedError("GAT Layer has not been implemented!")
        self.ffn = PositionwiseFeedForward(out_dim, ffn_inner_hidden_size, ffn_drop_out)

    def forward(self, g, w, s):
        if self.layerType == "W2S":
            origin, neighbor = s, w
        else:
            origin, neighbor = w, s
        h = self.layer(g, neighbor, origin=origin)   # elu(heads) + origin, fused
        return self.ffn(h)
