"""Sentence CNN encoder (reference: module/Encoder.py:18-76).

Not part of the WSWGAT hot path but in the logits path and the
next row of SURVEY §8f (rank 3).  Same parameter layout as the reference
(``ngram_enc.{embed,position_embedding,convs.0-5}``), so state_dicts load unchanged.
Differences in *how*: no Python loop over sentences for the positions
(Encoder.py:60-66), and the six convolutions + ReLU + max-pool run as one MFMA GEMM
over the sentences' real rows plus the HIP gather / pool kernels
(:mod:`hetersumgraph_amd.cnn`, hsg_cnn.hip).  There is no CPU path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.init as init

from ..cnn import sent_cnn
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
        # input: [n_sent, L] token ids, PAD = 0 (trailing) -> [n_sent, 300]
        return sent_cnn(input, self.embed.weight, self.position_embedding.weight,
                        [c.weight for c in self.convs], [c.bias for c in self.convs],
                        padding_idx=getattr(self.embed, "padding_idx", None))
