"""Multi-head wrapper (reference: module/GATStackLayer.py:46-63).

The reference loops over heads in Python, each head a full DGL pass on its own
dropout of the input, then ``torch.cat``s.  Here the heads stay separate modules
(``heads.{i}.*`` state_dict keys) but execute as one fused HIP pass.
"""
from __future__ import annotations

import torch.nn as nn

from .GATLayer import fused_heads


class MultiHeadLayer(nn.Module):
    def __init__(self, in_dim, out_dim, num_heads, attn_drop_out, feat_embed_size, layer, merge="cat"):
        super().__init__()
        if merge != "cat":
            # GATStackLayer.py:60-62 'mean' branch is never constructed by WSWGAT
            raise NotImplementedError("only merge='cat' is used by WSWGAT (GAT.py:35-37)")
        self.heads = nn.ModuleList([layer(in_dim, out_dim, feat_embed_size) for _ in range(num_heads)])
        self.merge = merge
        self.dropout = nn.Dropout(attn_drop_out)
        self.kind = layer.kind

    def forward(self, g, h, origin=None):
        """[n_dst, H*out_dim] head concat; with ``origin`` the ELU + residual of
        GAT.py:56-57 is fused in (returns elu(heads) + origin)."""
        return fused_heads(g, h, list(self.heads), self.kind, origin=origin, dropout=self.dropout)
