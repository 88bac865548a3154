"""Fixed sinusoid position table (reference: module/PositionEmbedding.py:20-38).

table[p, 2i]   = sin(p / 10000^(2i/d))
table[p, 2i+1] = cos(p / 10000^(2i/d)),  row ``padding_idx`` zeroed.
Computed in float64 and rounded once to float32, like the reference's numpy path.
"""
from __future__ import annotations

import numpy as np
import torch


def get_sinusoid_encoding_table(n_position, d_hid, padding_idx=None):
    pos = np.arange(n_position, dtype=np.float64)[:, None]
    expo = 2.0 * (np.arange(d_hid) // 2) / d_hid
    angle = pos / np.power(10000.0, expo)[None, :]
    table = np.empty_like(angle)
    table[:, 0::2] = np.sin(angle[:, 0::2])
    table[:, 1::2] = np.cos(angle[:, 1::2])
    if padding_idx is not None:
        table[padding_idx] = 0.0
    return torch.FloatTensor(table)
