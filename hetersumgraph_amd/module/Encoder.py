"""Sentence CNN encoder (reference: module/Encoder.py:18-76).

Not part of the WSWGAT hot path but in the logits
path, so it is provided with the reference's parameter layout
(``ngram_enc.{embed,position_embedding,convs.0-5}``).  Differences in *how*:
positions are built with one tensor op on the input's device instead of a Python
loop over sentences (Encoder.py:60-66), and the six convolutions run through
MIOpen/PyTorch.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
import torch.nn.init as init

from .PositionEmbedding import get_sinusoid_encoding_table

WORD_PAD = "[PAD]"


class sentEncoder(nn.Module):
    def __init__(self, hps, embed):
        super().__init__()
        self._hps = hps
        self.sent_max_len = hps.sent_max_len
        width = hps.word_emb_dim
        self.embed = embed
        self.position_embedding = nn.Embedding.from_pretrained(
            get_sinusoid_encoding_table(self.sent_max_len + 1, width, padding_idx=0), freeze=True)
        # kernel heights 2..7, 50 channels each -> 300-d (Encoder.py:36-53)
        self.convs = nn.ModuleList([nn.Conv2d(1, 50, kernel_size=(kh, width)) for kh in range(2, 8)])
        for conv in self.convs:
            init.xavier_normal_(conv.weight.data, gain=np.sqrt(6.0))

    def forward(self, input):
        # input: [n_sent, L] token ids, PAD = 0
        L = input.shape[1]
        sent_len = (input != 0).sum(dim=1, keepdim=True)
        ar = torch.arange(1, L + 1, device=input.device).unsqueeze(0)
        lim = torch.clamp(sent_len, max=self.sent_max_len)
        pos = torch.where(ar <= lim, ar, torch.zeros_like(ar))
        x = self.embed(input) + self.position_embedding(pos)
        x = x.unsqueeze(1)                                        # [n, 1, L, D]
        feats = []
        for conv in self.convs:
            y = F.relu(conv(x)).squeeze(3)                        # [n, 50, L-kh+1]
            feats.append(torch.amax(y, dim=2))                    # max-pool over time
        return torch.cat(feats, 1)                                # [n, 300]
