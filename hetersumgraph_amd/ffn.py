"""PositionwiseFeedForward on the MFMA GEMM + fused row epilogue (C ABI ops).

Reference: module/GATLayer.py:35-44 --
    out = LayerNorm(Dropout(W2 relu(W1 x + b1) + b2) + x)     (Conv1d k=1 == GEMM)

Forward  (3 launches): H = relu(x W1^T + b1) [GEMM, bias+ReLU epilogue];
                       y = H W2^T + b2       [GEMM, bias epilogue];
                       out = LN(dropout(y) + x) [row kernel, saves mean/rstd].
Backward:              (dy, dx) = row kernel (LN + dropout backward, block partials
                       of dgamma, dbeta and db2 = colsum(dy)); dH = (dy W2) * (H > 0)
                       [GEMM, relu' epilogue]; dx += dH W1 [GEMM, accumulate
                       epilogue]; dW2 = dy^T H and dW1 = dH^T x [split-K GEMMs];
                       db1 from the dH GEMM's column-sum epilogue; one launch
                       reduces both partial slabs.
"""
from __future__ import annotations

import torch

from . import rng as hsg_rng
from ._lib import check, load, ptr, stream_of
from .dense import gemm, row_tiles

LN_EPS = 1e-5


class _FFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, p_drop, eps):
        lib = load()
        x = x.contiguous()
        n, d = x.shape
        w1 = w1.contiguous()
        w2 = w2.contiguous()
        H = gemm(x, w1, b_t=True, bias=b1, relu=True)          # [n, d_hid]
        y = gemm(H, w2, b_t=True, bias=b2)                     # [n, d]
        out = torch.empty_like(x)
        mean = x.new_empty(n)
        rstd = x.new_empty(n)
        seed_t, off = (hsg_rng.get(x.device).take() if p_drop > 0 else (None, 0))
        check(lib.hsg_ln_fwd(n, d, ptr(y), ptr(x), ptr(gamma), ptr(beta), float(eps), float(p_drop),
                             ptr(seed_t), off, ptr(out), ptr(mean), ptr(rstd), stream_of(x)), "hsg_ln_fwd")
        ctx.save_for_backward(x, w1, w2, gamma, H, y, mean, rstd)
        ctx.p_drop, ctx.seed_t, ctx.off = p_drop, seed_t, off
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = load()
        x, w1, w2, gamma, H, y, mean, rstd = ctx.saved_tensors
        dout = dout.contiguous()
        n, d = x.shape
        nb = lib.hsg_ln_bwd_blocks(n)
        d_hid = H.shape[1]
        dy = torch.empty_like(x)
        dx = torch.empty_like(x)
        part = x.new_empty(nb, 3, d)
        check(lib.hsg_ln_bwd(n, d, ptr(dout), ptr(y), ptr(x), ptr(gamma), ptr(mean), ptr(rstd),
                             float(ctx.p_drop), ptr(ctx.seed_t), ctx.off, ptr(dy), ptr(dx), ptr(part),
                             stream_of(x)), "hsg_ln_bwd")
        rt = row_tiles(n, d_hid, d)
        hpart = x.new_empty(rt, d_hid)
        dH = gemm(dy, w2, relu_mask=H, splits=1, colsum_part=hpart)   # [n, d_hid] + db1 partials
        gemm(dH, w1, out=dx, add=dx)                           # dx += dH W1
        dw2 = gemm(dy, H, a_t=True)                            # [d, d_hid]
        dw1 = gemm(dH, x, a_t=True)                            # [d_hid, d]
        db1 = x.new_empty(d_hid)
        red = x.new_empty(3, d)                                # dgamma, dbeta, db2
        check(lib.hsg_colsum2(rt, d_hid, ptr(hpart), ptr(db1), nb, 3 * d, ptr(part), ptr(red), stream_of(x)),
              "hsg_colsum2")
        dg, dbt, db2 = red
        return dx, dw1, db1, dw2, db2, dg, dbt, None, None


def ffn_forward(x, w1, b1, w2, b2, gamma, beta, p_drop=0.0, eps=LN_EPS):
    """Fused FFN; x [n, d], w1 [d_hid, d], w2 [d, d_hid] (Conv1d weights squeezed)."""
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError("hetersumgraph_amd FFN runs only on a ROCm device in fp32 (no CPU fallback)")
    return _FFN.apply(x, w1, b1, w2, b2, gamma, beta, float(p_drop), float(eps))
