"""Sentence CNN encoder on the MFMA GEMM + HIP gather / max-pool kernels (C ABI ops).

Reference: module/Encoder.py:56-76 -- x = embed(ids) + pos_embed(pos) over the padded
sentence ([n, L, D]), six Conv2d(1, 50, (h, D)) for h = 2..7, ReLU, max-pool over time,
concat -> [n, 300].

Here (hsg_cnn.hip, include/hsg.h "sentence CNN encoder"):
  X    = gathered rows: the len_s real rows of each sentence plus ONE pad row
         (embed[0] + pos[0]: every padded position has that value)   hsg_cnn_gather
  Y    = X Wall^T, Wall = the 27 conv taps x 50 channels stacked     hsg_gemm_f32
  feat = relu(max_t (b_h + sum_i Y[t+i, tap(h,i)]))  + first argmax   hsg_cnn_pool
Backward: dY = scatter of the ReLU-masked dfeat into each max window (hsg_cnn_pool_bwd),
dWall = dY^T X (split-K GEMM), db_h = column sums of the masked dfeat, and -- only when
the word embedding trains (train.py:342 ``--embed_train``) -- dX = dY Wall scattered
into the embedding rows.

The GEMM covers sum_s (len_s + 1) rows instead of the reference's n * L padded rows,
and computes each (row, tap) product once instead of once per window.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import check, load, ptr, stream_of
from .dense import gemm, splits_for

HEIGHTS = tuple(range(2, 8))     # Encoder.py:37-38 min/max kernel size
CHANNELS = 50                    # Encoder.py:36
TAPS = sum(HEIGHTS)              # 27
NY = TAPS * CHANNELS             # 1350 columns of Y
LDY = (NY + 3) // 4 * 4          # hsg_gemm_f32 wants 16-byte row pitch


def stack_taps(weights):
    """Conv2d weights [50, 1, h, D] (h = 2..7) -> Wall [27*50, D], row (tap(h,i))*50 + c."""
    rows = []
    for h, w in zip(HEIGHTS, weights):
        rows.append(w.reshape(CHANNELS, h, w.shape[-1]).transpose(0, 1).reshape(h * CHANNELS, w.shape[-1]))
    return torch.cat(rows, 0).contiguous()


def _layout(ids):
    """Per-sentence lengths (Encoder.py:57 ``(input != 0).sum``), rowoff [n+1] int32 and
    the total row count (one host sync).  Padding must be trailing: the reference gives
    every position t >= len_s position 0, which equals the shared pad row only if the
    token there is PAD too (the dataloader always pads at the end, dataloader.py:97-109)."""
    n, L = ids.shape
    nz = ids != 0
    length = nz.sum(1)
    ar = torch.arange(L, device=ids.device)
    bad = (nz & (ar.unsqueeze(0) >= length.unsqueeze(1))).any()
    rowoff = torch.zeros(n + 1, dtype=torch.int32, device=ids.device)
    torch.cumsum(length + 1, 0, out=rowoff[1:])
    rows, bad = torch.stack([rowoff[-1].long(), bad.long()]).tolist()
    if bad:
        raise ValueError("sentEncoder: token ids after the first PAD (0) -- padding must be trailing")
    return length, rowoff, rows


class _SentCNN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, embed_w, pos_w, wall, padding_idx, *bias):
        lib = load()
        n, L = ids.shape
        D = embed_w.shape[1]
        st = stream_of(embed_w)
        length, rowoff, rows = _layout(ids)
        X = embed_w.new_empty(rows, D)
        check(lib.hsg_cnn_gather(n, L, D, ptr(ids), ptr(embed_w), ptr(pos_w), ptr(rowoff), rows, ptr(X), st),
              "hsg_cnn_gather")
        Y = embed_w.new_empty(rows, LDY)
        gemm(X, wall, b_t=True, out=Y[:, :NY])
        feat = embed_w.new_empty(n, len(HEIGHTS) * CHANNELS)
        arg = torch.empty(n, len(HEIGHTS) * CHANNELS, dtype=torch.int32, device=ids.device)
        bptr = (ctypes.c_void_p * len(bias))(*[b.data_ptr() for b in bias])
        check(lib.hsg_cnn_pool(n, L, ptr(rowoff), ptr(Y), LDY, bptr, ptr(feat), ptr(arg), st), "hsg_cnn_pool")
        ctx.save_for_backward(ids, X, wall, rowoff, length, feat, arg)
        ctx.n_embed, ctx.padding_idx = embed_w.shape[0], padding_idx
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        lib = load()
        ids, X, wall, rowoff, length, feat, arg = ctx.saved_tensors
        n, L = ids.shape
        rows, D = X.shape
        dfeat = dfeat.contiguous()
        st = stream_of(X)
        dY = X.new_zeros(rows, LDY)
        check(lib.hsg_cnn_pool_bwd(n, ptr(rowoff), ptr(feat), ptr(arg), ptr(dfeat), ptr(dY), LDY, st),
              "hsg_cnn_pool_bwd")
        d_embed = dwall = None
        if ctx.needs_input_grad[3]:
            dwall = gemm(dY[:, :NY], X, a_t=True, splits=splits_for(NY, D, rows))
        if ctx.needs_input_grad[1]:
            dX = gemm(dY[:, :NY], wall)                                      # [rows, D]
            sent = torch.repeat_interleave(torch.arange(n, device=X.device), length + 1)
            t = torch.arange(rows, device=X.device) - rowoff[:-1].long()[sent]
            tok = torch.where(t < length[sent], ids[sent, t.clamp(max=L - 1)], torch.zeros_like(t))
            d_embed = X.new_zeros(ctx.n_embed, D).index_add_(0, tok, dX)
            if ctx.padding_idx is not None:
                d_embed[ctx.padding_idx] = 0                  # nn.Embedding(padding_idx=...) semantics
        masked = (dfeat * (feat > 0)).view(n, len(HEIGHTS), CHANNELS)
        dbias = [masked[:, g].sum(0) if ctx.needs_input_grad[5 + g] else None for g in range(len(HEIGHTS))]
        return (None, d_embed, None, dwall, None, *dbias)


def sent_cnn(ids, embed_weight, pos_weight, conv_weights, conv_biases, padding_idx=None):
    """Encoder.py:56-76 forward on the HIP path: ids [n, L] int64 (PAD = 0, trailing),
    embed_weight [V, D] (``padding_idx``: the embedding row that gets no gradient, as
    nn.Embedding), pos_weight [sent_max_len+1, D] (row 0 = padding position),
    conv_weights / conv_biases of the six Conv2d(1, 50, (h, D)).  Returns [n, 300]."""
    if not ids.is_cuda or embed_weight.dtype != torch.float32:
        raise RuntimeError("hetersumgraph_amd sentence CNN runs only on a ROCm device in fp32 (no CPU fallback)")
    n, L = ids.shape
    D = embed_weight.shape[1]
    if L < max(HEIGHTS):
        raise ValueError(f"sentEncoder: sentence length {L} < the widest kernel {max(HEIGHTS)}")
    if L > pos_weight.shape[0] - 1:
        raise ValueError(f"sentEncoder: {L} tokens but only {pos_weight.shape[0] - 1} positions")
    if D % 4:
        raise ValueError("sentEncoder: word_emb_dim must be a multiple of 4 (GEMM row pitch)")
    if n == 0:
        return embed_weight.new_zeros(0, len(HEIGHTS) * CHANNELS)
    wall = stack_taps([w.float() for w in conv_weights])
    return _SentCNN.apply(ids.long().contiguous(), embed_weight.contiguous(), pos_weight.contiguous(), wall,
                          padding_idx, *[b.contiguous() for b in conv_biases])
