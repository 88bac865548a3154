"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/ (as the checker), never by the product path.

A float64 PyTorch-CPU restatement of the sentence CNN encoder, written the way the
reference computes it -- over the full padded [n, L, D] input, one Conv2d per kernel
height, ReLU, max over every window -- so that it checks both the HIP kernels and the
restatement they rely on (only real rows + one shared pad row, the stacked-tap GEMM,
the shifted sum).  Pinned against the reference's own outputs in
tests/golden/encoder.npz (tests/test_oracle_golden.py).

Reference lines restated: module/Encoder.py:56-76 (positions 58-66, conv 68-70,
ReLU 70, max_pool1d 71, cat 72).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def positions(ids, sent_max_len):
    """Encoder.py:57-66: position t+1 for t < min(sent_max_len, #non-PAD), else 0."""
    n, L = ids.shape
    length = (ids != 0).sum(1, keepdim=True).clamp(max=sent_max_len)
    ar = torch.arange(1, L + 1, device=ids.device).unsqueeze(0)
    return torch.where(ar <= length, ar, torch.zeros_like(ar))


def sent_encoder(ids, embed_w, pos_w, conv_w, conv_b, sent_max_len=None, padding_idx=0):
    """ids [n, L] int64; embed_w [V, D] (an nn.Embedding with ``padding_idx``: that row
    gets no gradient); pos_w [sent_max_len+1, D]; conv_w / conv_b the six
    Conv2d(1, 50, (h, D)) parameters.  Autograd-tracked, dtype of embed_w."""
    sent_max_len = ids.shape[1] if sent_max_len is None else sent_max_len
    x = F.embedding(ids, embed_w, padding_idx=padding_idx) + pos_w[positions(ids, sent_max_len)]   # [n, L, D]
    x = x.unsqueeze(1)
    feats = []
    for w, b in zip(conv_w, conv_b):
        y = F.relu(F.conv2d(x, w, b)).squeeze(3)                      # [n, 50, L-h+1]
        feats.append(F.max_pool1d(y, y.size(2)).squeeze(2))
    return torch.cat(feats, 1)
