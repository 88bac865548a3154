"""Head projection with per-head input dropout (C ABI: hsg_dropmask / hsg_hproj_*).

Reference semantics (module/GATStackLayer.py:56 + GATLayer.py:110/146): in
training each head k projects its own dropout of the input,
    Z[:, kD:(k+1)D] = dropout_k(h) @ W[kD:(k+1)D, :].T
The H keep-masks are generated once per call as bits (seed in device memory,
per-call offset) and shared by forward and backward; the H dropped copies of
``h`` are never materialised.
"""
from __future__ import annotations

import torch

from . import rng as hsg_rng
from ._lib import check, load, ptr, stream_of


class _HeadProj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, W, H, D, p):
        lib = load()
        X = X.contiguous()
        W = W.contiguous()
        n, d_in = X.shape
        st = stream_of(X)
        seed_t, off = hsg_rng.get(X.device).take()
        bits = torch.empty(lib.hsg_dropmask_words(n, d_in, H), dtype=torch.int32, device=X.device)
        check(lib.hsg_dropmask(n, d_in, H, float(p), ptr(seed_t), off, ptr(bits), st), "hsg_dropmask")
        Z = X.new_empty(n, H * D)
        check(lib.hsg_hproj_fwd(n, d_in, H, D, ptr(X), d_in, ptr(W), ptr(bits), float(p), ptr(Z), H * D, st),
              "hsg_hproj_fwd")
        ctx.save_for_backward(X, W, bits)
        ctx.H, ctx.D, ctx.p = H, D, p
        return Z

    @staticmethod
    def backward(ctx, dZ):
        lib = load()
        X, W, bits = ctx.saved_tensors
        H, D, p = ctx.H, ctx.D, ctx.p
        dZ = dZ.contiguous()
        n, d_in = X.shape
        st = stream_of(X)
        dX = dW = None
        if ctx.needs_input_grad[0]:
            dX = torch.empty_like(X)
            check(lib.hsg_hproj_dx(n, d_in, H, D, ptr(dZ), H * D, ptr(W), ptr(bits), float(p), ptr(dX), d_in, st),
                  "hsg_hproj_dx")
        if ctx.needs_input_grad[1]:
            dW = torch.empty_like(W)
            part = X.new_empty(lib.hsg_hproj_dw_chunks(n, d_in, H, D) * H * D * d_in)
            check(lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), float(p), ptr(part),
                                   ptr(dW), st), "hsg_hproj_dw")
        return dX, dW, None, None, None


def head_projection_dropout(X, W, H, D, p):
    """Z [n, H*D] = per-head dropout(X) projected by the fused fc weight W [H*D, in]."""
    if not X.is_cuda or X.dtype != torch.float32:
        raise RuntimeError("hetersumgraph_amd head projection runs only on a ROCm device in fp32")
    return _HeadProj.apply(X, W, int(H), int(D), float(p))


def dropmask_bits(X, H, p):
    """The keep-mask bits a projection call would draw (for tests)."""
    lib = load()
    n, d_in = X.shape
    seed_t, off = hsg_rng.get(X.device).take()
    bits = torch.empty(lib.hsg_dropmask_words(n, d_in, H), dtype=torch.int32, device=X.device)
    check(lib.hsg_dropmask(n, d_in, H, float(p), ptr(seed_t), off, ptr(bits), stream_of(X)), "hsg_dropmask")
    return bits.view(H, (n + 31) // 32, -1)[:, :, :d_in]
