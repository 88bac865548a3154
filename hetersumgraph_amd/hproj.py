"""Head projection with per-head input dropout (C ABI: hsg_dropmask / hsg_hproj_*).

Reference semantics (module/GATStackLayer.py:56 + GATLayer.py:110/146): in
training each head k projects its own dropout of the input,
    Z[:, kD:(k+1)D] = dropout_k(h) @ W[kD:(k+1)D, :].T
The H keep-masks are generated once per call as bits (seed in device memory,
per-call offset) and shared by forward and backward; the H dropped copies of
``h`` are never materialised.

``hproj_fwd`` / ``hproj_bwd`` are shared by the autograd Function below and the
fused stack (:mod:`hetersumgraph_amd.stack`).
"""
from __future__ import annotations


import torch

from . import _lib
from . import rng as hsg_rng
import ctypes

from ._lib import check, load, ptr, stream_of


def dropmasks(jobs, device, stream_of_t, wt=None, wsplit_job=None):
    """Keep-mask bits of several head projections in ONE launch
    (hsg_dropmask_multi): ``jobs`` = [(n, d_in, H, p, seed_t, offset)] with one
    shared seed tensor; returns the bit tensors, each as hsg_dropmask would draw it.
    ``wt`` = (W, H, D): the same launch also writes :func:`transposed_weight` of W
    (hsg_dropmask_multi_wt), returned as ``(masks, Wt)``.  ``wsplit_job``: a
    dense.split_weights(..., launch=False) job whose limb planes the same launch
    writes (hsg_step_prologue)."""
    lib = load()
    if not jobs:
        if wsplit_job is not None:
            check(lib.hsg_wsplit(*wsplit_job, stream_of_t), "hsg_wsplit")
        return ([], transposed_weight(*wt)) if wt is not None else []
    if len({id(j[4]) for j in jobs}) != 1:
        raise ValueError("dropmasks: one seed tensor per batch")
    out = []
    k = len(jobs)
    ns, ins, hs = (ctypes.c_int * k)(), (ctypes.c_int * k)(), (ctypes.c_int * k)()
    ps, offs, bp = (ctypes.c_float * k)(), (ctypes.c_uint32 * k)(), (ctypes.c_void_p * k)()
    for q, (n, d_in, H, p, _, off) in enumerate(jobs):
        b = torch.empty(lib.hsg_dropmask_words(n, d_in, H), dtype=torch.int32, device=device)
        out.append(b)
        ns[q], ins[q], hs[q], ps[q], offs[q], bp[q] = n, d_in, H, float(p), off, b.data_ptr()
    Wt = None
    if wt is not None:
        W, H, D = wt
        W = W.contiguous()
        Wt = torch.empty(H * W.shape[1] * D, dtype=W.dtype, device=W.device)
    for q0 in range(0, k, 8):
        q1 = min(k, q0 + 8)
        sl = slice(q0, q1)
        m = q1 - q0
        w_args = (H, D, W.shape[1], ptr(W), ptr(Wt)) if (wt is not None and q0 == 0) else (0, 0, 0, None, None)
        s_args = wsplit_job if (wsplit_job is not None and q0 == 0) else (0, None, None, None, None, None, None)
        check(lib.hsg_step_prologue(m, (ctypes.c_int * m)(*ns[sl]), (ctypes.c_int * m)(*ins[sl]),
                                    (ctypes.c_int * m)(*hs[sl]), (ctypes.c_float * m)(*ps[sl]),
                                    ptr(jobs[0][4]), (ctypes.c_uint32 * m)(*offs[sl]),
                                    (ctypes.c_void_p * m)(*bp[sl]), *w_args, *s_args, stream_of_t),
              "hsg_step_prologue")
    return (out, Wt) if wt is not None else out


def narrow_heads(d_in, H, D):
    """Whether the VALU projection (hsg_hproj_fwd_t8, D = 8) takes (d_in, H, D);
    HSG_HPROJ_FWDV=0 keeps the MFMA kernel (dev A/B)."""
    return _lib.path_option("HSG_HPROJ_FWDV", "1") != "0" and bool(load().hsg_hproj_fwd_t8_supported(d_in, H, D))


def transposed_weight(W, H, D):
    """Wt[k][c][d] = W[kD+d][c] for hsg_hproj_fwd_t8 (hsg_hproj_wt)."""
    lib = load()
    d_in = W.shape[1]
    Wt = W.new_empty(H * d_in * D)
    check(lib.hsg_hproj_wt(H, D, d_in, ptr(W), ptr(Wt), stream_of(W)), "hsg_hproj_wt")
    return Wt


def hproj_fwd(X, W, H, D, p, a1=None, bits=None, wt=None):
    """Z [n, H*D] and the state its backward needs.  X, W contiguous fp32.  With
    ``a1`` [H, D] (the attention's source part), also the source logits
    sigma [n, H] from the same launch: returns (Z, saved, sigma); sigma is None when
    the fused form does not cover (H, D) (the caller computes it separately).
    ``bits``: keep-masks already drawn for this call (:func:`dropmasks`); ``wt``:
    :func:`transposed_weight` of W when the caller shares it between calls."""
    lib = load()
    n, d_in = X.shape
    st = stream_of(X)
    if bits is None:
        seed_t, off = hsg_rng.get(X.device).take()
        bits = torch.empty(lib.hsg_dropmask_words(n, d_in, H), dtype=torch.int32, device=X.device)
        check(lib.hsg_dropmask(n, d_in, H, float(p), ptr(seed_t), off, ptr(bits), st), "hsg_dropmask")
    Z = X.new_empty(n, H * D)
    saved = (X, W, bits, H, D, float(p))
    if narrow_heads(d_in, H, D) and X.data_ptr() % 16 == 0:
        if wt is None:
            wt = transposed_weight(W, H, D)
        sigma = X.new_empty(n, H) if a1 is not None else None
        check(lib.hsg_hproj_fwd_t8(n, d_in, H, ptr(X), d_in, ptr(wt), ptr(bits), float(p), ptr(Z), H * D,
                                   ptr(a1.contiguous()) if a1 is not None else None,
                                   ptr(sigma) if sigma is not None else None, st), "hsg_hproj_fwd_t8")
        return (Z, saved, sigma) if a1 is not None else (Z, saved)
    if a1 is not None:
        if not lib.hsg_hproj_fwd_logits_supported(H, D):
            check(lib.hsg_hproj_fwd(n, d_in, H, D, ptr(X), d_in, ptr(W), ptr(bits), float(p), ptr(Z), H * D, st),
                  "hsg_hproj_fwd")
            return Z, saved, None
        sigma = X.new_empty(n, H)
        check(lib.hsg_hproj_fwd_logits(n, d_in, H, D, ptr(X), d_in, ptr(W), ptr(bits), float(p), ptr(Z), H * D,
                                       ptr(a1.contiguous()), ptr(sigma), st), "hsg_hproj_fwd_logits")
        return Z, saved, sigma
    check(lib.hsg_hproj_fwd(n, d_in, H, D, ptr(X), d_in, ptr(W), ptr(bits), float(p), ptr(Z), H * D, st),
          "hsg_hproj_fwd")
    return Z, saved


def hproj_bwd(saved, dZ, dX=None, dX_acc=False, dW=None, dW_acc=False, batch=None, key=None):
    """dX (into ``dX`` -- written or, with dX_acc, added) and dW (same, into ``dW``).
    Either destination may be None (that gradient is skipped).  ``batch`` (a
    reduce.SlabBatch) with ``key``: dW's partial slabs are recorded there and summed
    with every other call of the same key in the batch's one launch."""
    lib = load()
    X, W, bits, H, D, p = saved
    dZ = dZ.contiguous()
    n, d_in = X.shape
    st = stream_of(X)
    if dX is not None and dW is not None and batch is not None and n > 0:
        # both in one call (hsg_hproj_bwd: one launch for the small wide-head shape)
        chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
        part = X.new_empty(chunks * H * D * d_in)
        check(lib.hsg_hproj_bwd(n, d_in, H, D, ptr(dZ), H * D, ptr(W), ptr(X), d_in, ptr(bits), p, ptr(dX), d_in,
                                int(dX_acc), ptr(part), st), "hsg_hproj_bwd")
        batch.add((key, "W"), dW.view(-1), H * D * d_in, H * D * d_in, 0, lib.hsg_dropmask_scale(p), dW_acc,
                  part, chunks)
        return dX
    if dX is not None:
        check(lib.hsg_hproj_dx(n, d_in, H, D, ptr(dZ), H * D, ptr(W), ptr(bits), p, ptr(dX), d_in, int(dX_acc), st),
              "hsg_hproj_dx")
    if dW is not None:
        chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
        part = X.new_empty(chunks * H * D * d_in)
        if batch is not None and n > 0:
            check(lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), p, ptr(part), None,
                                   0, st), "hsg_hproj_dw")
            batch.add((key, "W"), dW.view(-1), H * D * d_in, H * D * d_in, 0, lib.hsg_dropmask_scale(p), dW_acc,
                      part, chunks)
        else:
            check(lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), p, ptr(part), ptr(dW),
                                   int(dW_acc), st), "hsg_hproj_dw")
    return dX


class _HeadProj(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, W, H, D, p):
        Z, saved = hproj_fwd(X.contiguous(), W.contiguous(), H, D, p)
        ctx.save_for_backward(saved[0], saved[1], saved[2])
        ctx.H, ctx.D, ctx.p = H, D, p
        return Z

    @staticmethod
    def backward(ctx, dZ):
        X, W, bits = ctx.saved_tensors
        saved = (X, W, bits, ctx.H, ctx.D, float(ctx.p))
        dX = torch.empty_like(X) if ctx.needs_input_grad[0] else None
        dW = torch.empty_like(W) if ctx.needs_input_grad[1] else None
        hproj_bwd(saved, dZ, dX=dX, dW=dW)
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
