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
                       reduces both partial slabs (hsg_ffn_colsums).

``ffn_fwd`` / ``ffn_bwd`` are the building blocks shared by the per-module
autograd Function below and the fused stack (:mod:`hetersumgraph_amd.stack`),
whose backward writes the parameter gradients straight into their destination
(overwrite or accumulate) instead of returning them.
"""
from __future__ import annotations


import torch

from . import _lib
from . import rng as hsg_rng
from ._lib import HSG_EINVAL, check, load, ptr, stream_of
from .dense import (gemm, gemm_psw, gemm_psw_elug, gemm_psw_ln, get_gemm_dtype, psw_row_tiles, row_tiles,
                    split_weights)

LN_EPS = 1e-5


def _fused_ok(lib, x, w1, w2):
    """The one-launch narrow FFN kernels (hsg_ffn_small_fwd / _bwd: the W2S FFN,
    d=64, d_hid=512) cover this call: contiguous operands.  They compute in fp32 in
    either GEMM mode (in the bf16 mode this small FFN simply stays exact).
    HSG_FFN_FUSED=0 selects the split path (A/B tests)."""
    if _lib.path_option("HSG_FFN_FUSED", "1") == "0":
        return False
    d_hid, d = w1.shape
    return (bool(lib.hsg_ffn_small_supported(d, d_hid)) and x.is_contiguous() and w1.is_contiguous()
            and w2.is_contiguous())


def bf16_rows_ok(d, d_hid):
    """The bf16 GEMM mode may keep this wide FFN's activation rows (H, y, dY, dH and the
    edge gate G) in bf16: the kernels that read or write them take the shape.  Mirrors
    their host checks -- hsg_ln_fwd_y16 / hsg_ln_bwd_dy16 (csrc/hsg_rows.hip: the
    persistent vector kernels, d % 4 == 0 and 257 <= d <= 512) and hsg_gemm_bf16_psw_io
    / hsg_gemm_bf16_psw_elug_rho_a16 (csrc/hsg_gemm.hip: a bf16 A operand needs
    lda % 8 == 0, and H / dH have d_hid columns).  Any other shape keeps fp32 rows
    (a 256- or 768-wide embedding, or ffn_inner_hidden_size % 8 != 0,
    would otherwise reach a kernel that refuses it)."""
    return d % 4 == 0 and 257 <= d <= 512 and d_hid % 8 == 0


def _draw(x, p_drop, rng):
    if p_drop <= 0:
        return None, 0
    return rng if rng is not None else hsg_rng.get(x.device).take()


def ffn_wsplit(x, w1, b1, w2, b2, launch=True):
    """The pre-split weight operands (hsg_wsplit: W1, W2 for the forward GEMMs, W2^T,
    W1^T for dH = dy W2 and dx += dH W1) of an FFN that runs on the GEMM path, or
    None: the narrow fused FFN, the 'f32mfma' GEMM mode, shapes hsg_gemm_f32_psw
    does not take, or HSG_GEMM_PSW=0 (A/B).  In the 'bf16' mode the GEMMs on these
    planes run hsg_gemm_bf16_psw (plane 0 = RNE(W), one product).  Made once per forward of the fused stack and
    shared by all applications of the layer and their backward.  ``launch=False``:
    (weights, job) with the split left to the caller's launch (hsg_step_prologue)."""
    lib = load()
    if b1 is not None and b2 is not None and _fused_ok(lib, x, w1, w2):
        return None
    if get_gemm_dtype() not in ("f32", "bf16") or _lib.path_option("HSG_GEMM_PSW", "1") == "0":
        return None
    d_hid, d = w1.shape
    if d % 4 or d_hid % 4 or not (w1.is_contiguous() and w2.is_contiguous()):
        return None
    if not launch:                       # (planes, job) for hsg_step_prologue
        out, job = split_weights((w1, False), (w2, False), (w2, True), (w1, True), launch=False)
        return tuple(out), job
    return tuple(split_weights((w1, False), (w2, False), (w2, True), (w1, True)))


def ffn_fwd(x, w1, b1, w2, b2, gamma, beta, p_drop, eps=LN_EPS, H_out=None, wsplit="auto", rng=None):
    """x [n, d] contiguous, w1 [d_hid, d], w2 [d, d_hid].  ``H_out``: a contiguous
    [n, d_hid] buffer for the hidden activations (the fused stack hands in slices of
    one per-layer buffer).  ``wsplit``: :func:`ffn_wsplit`'s result for these weights
    ("auto": made here).  ``rng``: the dropout's (seed, offset), already drawn by
    the caller (default: drawn here).  Returns (out, saved)."""
    lib = load()
    n, d = x.shape
    f32 = dict(dtype=torch.float32, device=x.device)
    out = torch.empty(n, d, **f32)
    mean = torch.empty(n, **f32)
    rstd = torch.empty(n, **f32)
    if x.dtype == torch.bfloat16:
        # the bf16 GEMM mode's bf16 x rows (round 6; the edge layer's hsg_gat_fwd_ws16
        # output, pitch % 8 == 0, zero pad): the A operand of the first GEMM and the
        # LayerNorm residual, both read as bf16
        if isinstance(wsplit, str):
            wsplit = ffn_wsplit(x, w1, b1, w2, b2)
        if (wsplit is None or wsplit[0].mode != "bf16" or b2 is None or H_out is None
                or H_out.dtype != torch.bfloat16 or not bf16_rows_ok(d, w1.shape[0])):
            raise RuntimeError("ffn_fwd: bf16 x rows belong to the bf16 GEMM mode's bf16-row FFN")
        H = gemm_psw(x, wsplit[0], bias=b1, relu=True, out=H_out)
        seed_t, off = _draw(x, p_drop, rng)
        y = torch.empty(n, d, dtype=torch.bfloat16, device=x.device)
        gemm_psw(H, wsplit[1], bias=b2, out=y)
        check(lib.hsg_ln_fwd_x16(n, d, ptr(y), ptr(x), x.stride(0), ptr(gamma), ptr(beta), float(eps),
                                 float(p_drop), ptr(seed_t), off, ptr(out), ptr(mean), ptr(rstd), stream_of(x)),
              "hsg_ln_fwd_x16")
        return out, (x, w1, w2, gamma, H, y, mean, rstd, float(p_drop), seed_t, off, wsplit)
    if b1 is not None and b2 is not None and _fused_ok(lib, x, w1, w2):
        H = H_out if H_out is not None else x.new_empty(n, w1.shape[0])
        y = torch.empty_like(x)
        seed_t, off = _draw(x, p_drop, rng)
        check(lib.hsg_ffn_small_fwd(n, d, w1.shape[0], ptr(x), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(gamma),
                                    ptr(beta), float(eps), float(p_drop), ptr(seed_t), off, ptr(H), ptr(y),
                                    ptr(out), ptr(mean), ptr(rstd), stream_of(x)), "hsg_ffn_small_fwd")
        return out, (x, w1, w2, gamma, H, y, mean, rstd, float(p_drop), seed_t, off, None)
    if isinstance(wsplit, str):
        wsplit = ffn_wsplit(x, w1, b1, w2, b2)
    if wsplit is not None:
        H = gemm_psw(x, wsplit[0], bias=b1, relu=True, out=H_out)    # [n, d_hid]
        # the second GEMM with dropout + residual + LayerNorm in its epilogue when the
        # shape has a one-round full-row plan (hsg_gemm_psw_ln), else GEMM + hsg_ln_fwd
        seed_t, off = _draw(x, p_drop, rng)
        y = torch.empty_like(x)
        if b2 is not None and gemm_psw_ln(H, wsplit[1], b2, x, gamma, beta, eps, p_drop, seed_t, off, y, out,
                                          mean, rstd):
            return out, (x, w1, w2, gamma, H, y, mean, rstd, float(p_drop), seed_t, off, wsplit)
        if (H.dtype == torch.bfloat16 and bf16_rows_ok(d, H.shape[1])
                and _lib.path_option("HSG_FFN_BF16_ROWS", "1") != "0"):
            # the bf16 GEMM mode's bf16 activations: the FFN output y (the LayerNorm
            # input) as bf16 too -- rounded once, <= 2^-9 |y| per element
            y = x.new_empty(n, d, dtype=torch.bfloat16)
            gemm_psw(H, wsplit[1], bias=b2, out=y)
            check(lib.hsg_ln_fwd_y16(n, d, ptr(y), ptr(x), ptr(gamma), ptr(beta), float(eps), float(p_drop),
                                     ptr(seed_t), off, ptr(out), ptr(mean), ptr(rstd), stream_of(x)), "hsg_ln_fwd_y16")
            return out, (x, w1, w2, gamma, H, y, mean, rstd, float(p_drop), seed_t, off, wsplit)
        gemm_psw(H, wsplit[1], bias=b2, out=y)                   # [n, d]
        check(lib.hsg_ln_fwd(n, d, ptr(y), ptr(x), ptr(gamma), ptr(beta), float(eps), float(p_drop),
                             ptr(seed_t), off, ptr(out), ptr(mean), ptr(rstd), stream_of(x)), "hsg_ln_fwd")
        return out, (x, w1, w2, gamma, H, y, mean, rstd, float(p_drop), seed_t, off, wsplit)
    else:
        H = gemm(x, w1, b_t=True, bias=b1, relu=True, out=H_out)
        y = gemm(H, w2, b_t=True, bias=b2)
    seed_t, off = _draw(x, p_drop, rng)
    check(lib.hsg_ln_fwd(n, d, ptr(y), ptr(x), ptr(gamma), ptr(beta), float(eps), float(p_drop),
                         ptr(seed_t), off, ptr(out), ptr(mean), ptr(rstd), stream_of(x)), "hsg_ln_fwd")
    return out, (x, w1, w2, gamma, H, y, mean, rstd, float(p_drop), seed_t, off, wsplit)


def ffn_bwd(saved, dout, dst, act_grads=None, batch=None, key=None, elug=None, gate=None):
    """Backward of :func:`ffn_fwd`.  ``dst`` = (dw1, acc_w1, dw2, acc_w2, db1, db2,
    dgamma, dbeta, acc_b): gradient buffers shaped [d_hid, d], [d, d_hid], [d_hid],
    [d], [d], [d] (None when not needed), each written or -- with its accumulate
    flag -- added into.  ``act_grads`` = (dy [n, d], dH [n, d_hid]) contiguous buffers
    that receive the two activation gradients; the weight gradients (dw1 = dH^T x,
    dw2 = dy^T H) are then left to the caller, which runs them once over all
    applications of a layer (pass dw1 = dw2 = None).  ``batch`` (a
    reduce.SlabBatch) with ``key``: the bias / LayerNorm column sums are recorded
    there (one job per output across every call with the same key) instead of run
    here.  ``elug`` = (origin, G): the FFN input x is the edge layer's elu(h) + origin,
    and its ELU gate G = dx * elu'(h) goes into G from the last GEMM's epilogue
    (hsg_gemm_f32_psw_elug) -- only on the pre-split-weight path; (origin, G, rho,
    head_dim): also the rho partials of the one-pass edge backward
    (hsg_gemm_psw_elug_rho).  ``gate`` = (h_edge, G, rho): the same for the narrow
    one-launch FFN (W2S: the edge layer stored h; G and per-head rho from its epilogue,
    hsg_ffn_small_bwd_gate).  Returns dx (a fresh tensor), or (dx, G produced?) with
    ``elug`` or ``gate``."""
    lib = load()
    x, w1, w2, gamma, H, y, mean, rstd, p_drop, seed_t, off, wsplit = saved
    dw1, acc_w1, dw2, acc_w2, db1, db2, dg, dbt, acc = dst
    dout = dout.contiguous()
    n, d = x.shape
    st = stream_of(x)
    d_hid = H.shape[1]
    f32 = dict(dtype=torch.float32, device=x.device)
    dy = act_grads[0] if act_grads is not None else torch.empty(n, d, **f32)
    dx = torch.empty(n, d, **f32)
    g_done = False
    x16 = x.dtype == torch.bfloat16             # the bf16 mode's bf16 x rows (ffn_fwd)
    if x16 and (act_grads is None or dy.dtype != torch.bfloat16 or y.dtype != torch.bfloat16 or wsplit is None
                or elug is None or dw1 is not None):
        raise RuntimeError("ffn_bwd: bf16 x rows come with the fused stack's bf16 rows (dy, y, G) and its "
                           "batched weight gradients")
    if _fused_ok(lib, x, w1, w2) and H.is_contiguous() and y.is_contiguous():
        # one launch: LN/dropout backward, dH = (dy W2) * relu'(H), dx = ds + dH W1
        nb = rt = lib.hsg_ffn_small_bwd_blocks(n)
        part = x.new_empty(nb, 3, d)
        hpart = x.new_empty(rt, d_hid)
        dH = act_grads[1] if act_grads is not None else x.new_empty(n, d_hid)
        args = (n, d, d_hid, ptr(dout), ptr(x), ptr(H), ptr(y), ptr(w1), ptr(w2), ptr(gamma), ptr(mean), ptr(rstd),
                p_drop, ptr(seed_t), off, ptr(dy), ptr(dH), ptr(dx), ptr(part), ptr(hpart))
        rc = HSG_EINVAL
        if gate is not None:
            rc = lib.hsg_ffn_small_bwd_gate(*args, ptr(gate[0]), ptr(gate[1]), ptr(gate[2]), st)
            g_done = rc == 0
        if rc == HSG_EINVAL:                # no gate asked, or declined: the plain launch
            rc = lib.hsg_ffn_small_bwd(*args, st)
        check(rc, "hsg_ffn_small_bwd")
    else:
        nb = lib.hsg_ln_bwd_blocks(n)
        part = torch.empty(nb, 3, d, **f32)
        if x16:
            check(lib.hsg_ln_bwd_x16(n, d, ptr(dout), ptr(y), ptr(x), x.stride(0), ptr(gamma), ptr(mean), ptr(rstd),
                                     p_drop, ptr(seed_t), off, ptr(dy), dy.stride(0), ptr(dx), ptr(part), st),
                  "hsg_ln_bwd_x16")
        elif dy.dtype == torch.bfloat16:     # the bf16 mode's bf16 dy rows (zero pad to ceil8(d))
            check(lib.hsg_ln_bwd_dy16(n, d, ptr(dout), ptr(y), int(y.dtype == torch.bfloat16), ptr(x), ptr(gamma),
                                      ptr(mean), ptr(rstd), p_drop, ptr(seed_t), off, ptr(dy), dy.stride(0), ptr(dx),
                                      ptr(part), st), "hsg_ln_bwd_dy16")
        else:
            check(lib.hsg_ln_bwd(n, d, ptr(dout), ptr(y), ptr(x), ptr(gamma), ptr(mean), ptr(rstd), p_drop,
                                 ptr(seed_t), off, ptr(dy), ptr(dx), ptr(part), st), "hsg_ln_bwd")
        rt = psw_row_tiles(n, d_hid, d, wsplit[2].mode) if wsplit is not None else row_tiles(n, d_hid, d)
        hpart = torch.empty(rt, d_hid, **f32)
        dH_out = act_grads[1] if act_grads is not None else None
        if wsplit is not None:
            dH = gemm_psw(dy, wsplit[2], relu_mask=H, colsum_part=hpart, out=dH_out)
            if elug is not None and gemm_psw_elug(dH, wsplit[3], dx, x, *elug):
                g_done = True
            elif x16:
                raise RuntimeError("ffn_bwd: the ELU-gate dx GEMM declined bf16 x rows")
            else:
                gemm_psw(dH, wsplit[3], out=dx, add=dx)
        else:
            dH = gemm(dy, w2, relu_mask=H, splits=1, colsum_part=hpart,   # [n, d_hid] + db1 partials
                      out=dH_out)
            gemm(dH, w1, out=dx, add=dx)                                  # dx += dH W1
    if dw2 is not None:
        gemm(dy, H, a_t=True, out=dw2, add=dw2 if acc_w2 else None)  # [d, d_hid]
    if dw1 is not None:
        gemm(dH, x, a_t=True, out=dw1, add=dw1 if acc_w1 else None)  # [d_hid, d]
    outs = [db1, dg, dbt, db2]
    if batch is not None:
        if db1 is not None:
            batch.add((key, "b1"), db1, d_hid, d_hid, 0, 1.0, acc, hpart, rt)
        for o, name, off in ((dg, "g", 0), (dbt, "bt", d), (db2, "b2", 2 * d)):
            if o is not None:
                batch.add((key, name), o, d, 3 * d, off, 1.0, acc, part, nb)
        return (dx, g_done) if elug is not None or gate is not None else dx
    if any(o is not None for o in outs):
        db1, dg, dbt, db2 = [o if o is not None else torch.empty(n_, **f32)
                             for o, n_ in zip(outs, (d_hid, d, d, d))]   # scratch for unneeded ones
        check(lib.hsg_ffn_colsums(rt, d_hid, ptr(hpart), ptr(db1), nb, d, ptr(part), ptr(dg), ptr(dbt), ptr(db2),
                                  int(bool(acc)), st), "hsg_ffn_colsums")
    return (dx, g_done) if elug is not None or gate is not None else dx


class _FFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, gamma, beta, p_drop, eps):
        out, saved = ffn_fwd(x.contiguous(), w1.contiguous(), b1, w2.contiguous(), b2, gamma, beta, p_drop, eps)
        x, w1, w2, gamma, H, y, mean, rstd = saved[:8]
        ctx.save_for_backward(x, w1, w2, gamma, H, y, mean, rstd)
        ctx.rest = saved[8:]
        return out

    @staticmethod
    def backward(ctx, dout):
        saved = tuple(ctx.saved_tensors) + ctx.rest
        x, w1, w2 = saved[0], saved[1], saved[2]
        d, d_hid = x.shape[1], w1.shape[0]
        dw1, dw2 = torch.empty_like(w1), torch.empty_like(w2)
        db1, db2 = x.new_empty(d_hid), x.new_empty(d)
        dg, dbt = x.new_empty(d), x.new_empty(d)
        dx = ffn_bwd(saved, dout, (dw1, False, dw2, False, db1, db2, dg, dbt, False))
        return dx, dw1, db1, dw2, db2, dg, dbt, None, None


def ffn_forward(x, w1, b1, w2, b2, gamma, beta, p_drop=0.0, eps=LN_EPS):
    """Fused FFN; x [n, d], w1 [d_hid, d], w2 [d, d_hid] (Conv1d weights squeezed)."""
    if not x.is_cuda or x.dtype != torch.float32:
        raise RuntimeError("hetersumgraph_amd FFN runs only on a ROCm device in fp32 (no CPU fallback)")
    return _FFN.apply(x, w1, b1, w2, b2, gamma, beta, float(p_drop), float(eps))
