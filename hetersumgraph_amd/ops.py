"""Autograd operators over the C ABI (libhsg.so) -- the WSWGAT hot path.

``gat_aggregate`` is one multi-head WSGAT/SWGAT application with the ELU +
residual epilogue, i.e. module/GATLayer.py:104-116 (or 142-152) for every head of
module/GATStackLayer.py:55-59 followed by module/GAT.py:56-57, expressed as the
fused restatement of SURVEY §8a:

    sigma[u,k] = <Z[u,k,:], a1_k>                        (z_src part of attn_fc)
    s_e,k      = leaky_relu(sigma[u,k] + tau[t_e,k])     (z_dst part is 0, GATLayer.py:111)
    alpha      = softmax over ALL in-edges of v (phantoms: e = 0, z = 0)
    out[v]     = elu(sum_e alpha z_u) + origin[v]

Everything runs on the current HIP stream; nothing synchronises, so a whole
training step can be captured into a HIP graph.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import HSG_TAU_PER_EDGE, HSG_TAU_TABLE, check, load, ptr, stream_of


def _clock_start(tag, t):
    clk = _lib.CLOCK
    return None if clk is None else clk.start(tag, t.device)


def _clock_stop(tok, t):
    if tok is not None:
        _lib.CLOCK.stop(tok, t.device)


def _clock_abort(tok):
    if tok is not None:
        _lib.KernelClock.disarm()


from .relation import N_BOX

LEAKY_SLOPE = 0.01   # F.leaky_relu default (GATLayer.py:92, 131)


def _require_device(*ts):
    for t in ts:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                "hetersumgraph_amd WSWGAT runs only on a ROCm device (libhsg.so HIP kernels); "
                f"got a tensor on {t.device}. There is no CPU fallback.")
        if t.dtype != torch.float32:
            raise TypeError(f"hetersumgraph_amd WSWGAT computes in fp32; got {t.dtype}")


class _GatAggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Z, a1, tau, origin, rel, H, D, slope, tau_mode):
        lib = load()
        Z = Z.contiguous()
        a1 = a1.contiguous()
        tau = tau.contiguous()
        origin = None if origin is None else origin.contiguous()
        n_src, n_dst, HD = rel.n_src, rel.n_dst, H * D
        if Z.shape != (n_src, HD):
            raise ValueError(f"Z has shape {tuple(Z.shape)}, relation expects ({n_src}, {HD})")
        if origin is not None and origin.shape != (n_dst, HD):
            raise ValueError(f"origin has shape {tuple(origin.shape)}, expected ({n_dst}, {HD})")
        st = stream_of(Z)
        relp = ctypes.byref(rel.cstruct())
        sigma = Z.new_empty(n_src, H)
        check(lib.hsg_attn_src_logits(n_src, H, D, ptr(Z), ptr(a1), ptr(sigma), st),
              "hsg_attn_src_logits")
        h = Z.new_empty(n_dst, HD)
        out = Z.new_empty(n_dst, HD) if origin is not None else None
        m = Z.new_empty(n_dst, H)
        l = Z.new_empty(n_dst, H)
        ws = fwd_workspace(lib, relp, H, D, Z)
        check(lib.hsg_gat_fwd_ws(relp, H, D, tau_mode, slope, ptr(Z), ptr(sigma), ptr(tau),
                                 ptr(origin), ptr(h), ptr(out), ptr(m), ptr(l), ptr(ws), st), "hsg_gat_fwd_ws")
        ctx.save_for_backward(Z, a1, sigma, tau, h, m, l)
        ctx.rel, ctx.H, ctx.D, ctx.slope, ctx.tau_mode = rel, H, D, slope, tau_mode
        ctx.has_origin = origin is not None
        return out if origin is not None else h

    @staticmethod
    def backward(ctx, dout):
        lib = load()
        Z, a1, sigma, tau, h, m, l = ctx.saved_tensors
        rel, H, D, slope, mode = ctx.rel, ctx.H, ctx.D, ctx.slope, ctx.tau_mode
        dout = dout.contiguous()
        st = stream_of(Z)
        relp = ctypes.byref(rel.cstruct())
        G = torch.empty_like(h)
        dpre = Z.new_empty(rel.n_typed, H)
        nb = lib.hsg_gat_bwd_blocks(relp)
        dtp = Z.new_empty(nb, N_BOX + 1, H) if mode == HSG_TAU_TABLE else None
        check(lib.hsg_gat_bwd_dst(relp, H, D, mode, int(ctx.has_origin), slope, ptr(Z), ptr(sigma),
                                  ptr(tau), ptr(h), ptr(m), ptr(l), ptr(dout), ptr(G), ptr(dpre),
                                  ptr(dtp), st), "hsg_gat_bwd_dst")
        dZ = torch.empty_like(Z)
        dsig = torch.empty_like(sigma)
        check(lib.hsg_gat_bwd_src(relp, H, D, mode, slope, ptr(sigma), ptr(tau), ptr(m), ptr(l),
                                  ptr(G), ptr(dpre), ptr(a1), None, ptr(dZ), ptr(dsig), None, st),
              "hsg_gat_bwd_src")
        da1 = None
        if ctx.needs_input_grad[1]:
            da1 = torch.einsum("uk,ukd->kd", dsig, Z.view(-1, H, D))
        dtau = dtp.sum(0) if mode == HSG_TAU_TABLE else dpre
        return dZ, da1, dtau, (dout if ctx.has_origin else None), None, None, None, None, None


def fwd_workspace(lib, relp, H, D, like):
    """Scratch of hsg_gat_fwd_ws for the relation's CSR work list (the pieces of its long
    destinations), or None when it has none."""
    n = lib.hsg_gat_fwd_ws_floats(relp, H, D)
    return like.new_empty(n) if n else None


def attn_tables(attn, T, wf, bf, H, D):
    """(a1 [H, D], tau [11, H]) of one layer's attention parameters: the source part
    of attn_fc and the per-box edge term (hsg_attn_params_fwd).  They depend on the
    parameters only, so every application of a layer in one step can share them."""
    lib = load()
    a1 = attn.new_empty(H, D)
    tau = attn.new_empty(N_BOX + 1, H)
    check(lib.hsg_attn_params_fwd(H, D, T.shape[1], ptr(attn), ptr(wf), ptr(bf), ptr(T), ptr(a1), ptr(tau),
                                  stream_of(attn)), "hsg_attn_params_fwd")
    return a1, tau


def attn_tables_pair(lay0, lay1, T, seed_advance=None):
    """:func:`attn_tables` of two layers sharing T in ONE launch
    (hsg_attn_params_fwd_pair): [(a1, tau) of lay0, (a1, tau) of lay1]; a layer is any
    object with attn / wf / bf / H / D.  ``seed_advance``: a pending dropout-seed
    advance claimed from rng (its (seed, snap) tensors), performed by the same launch
    (hsg_attn_params_fwd_pair_seed)."""
    lib = load()
    outs = []
    for lay in (lay0, lay1):
        outs.append((lay.attn.new_empty(lay.H, lay.D), lay.attn.new_empty(N_BOX + 1, lay.H)))
    (a0, t0), (a1, t1) = outs
    seed, snap = seed_advance if seed_advance is not None else (None, None)
    check(lib.hsg_attn_params_fwd_pair_seed(lay0.H, lay0.D, ptr(lay0.attn), ptr(lay0.wf), ptr(lay0.bf), ptr(a0),
                                            ptr(t0), lay1.H, lay1.D, ptr(lay1.attn), ptr(lay1.wf), ptr(lay1.bf),
                                            ptr(a1), ptr(t1), T.shape[1], ptr(T), ptr(seed), ptr(snap),
                                            stream_of(T)), "hsg_attn_params_fwd_pair_seed")
    return outs


def gat_table_fwd(Z, attn, T, wf, bf, origin, rel, H, D, slope, tables=None, out=None, sigma=None, keep_h=True,
                  no_h=False):
    """Forward of one multi-head application with the TF-IDF-table edge term:
    3 launches (attention parameters -> tau table, sigma, edge pass; 2 when
    ``tables`` = :func:`attn_tables` of this layer is passed in).  ``out``: a contiguous
    [n_dst, H*D] buffer for the result (with an origin).  ``sigma``: the source logits
    when the head projection already produced them.  ``keep_h=False`` (with an origin,
    where hsg_gat_bwd_dst_noh covers the shape, and HSG_GAT_NOH=1): h is not stored; the
    backward takes elu'(h) from out - origin and G.h from the edge dots.  Opt-in: at
    cfg2 the S2W forward drops 22.6 -> 18.3 us but the dst pass, which then reads out
    and origin instead of h, rises 33 -> 39.6 us (step +8 us).  ``no_h``:
    the same without the switch -- for a caller whose backward hands
    :func:`gat_table_bwd` the G rows from the FFN's last GEMM epilogue
    (hsg_gemm_f32_psw_elug), so the dst pass reads neither h nor x / origin.  A bf16
    ``out`` ([n_dst, H*D] view of rows with pitch % 8 == 0, round 6): x is stored as
    bf16 rows there (hsg_gat_fwd_ws16, the bf16 GEMM mode's bf16 x; with ``no_h`` only,
    as the backward's G then comes from the FFN epilogue).  Returns (out, saved)."""
    lib = load()
    n_src, n_dst, HD = rel.n_src, rel.n_dst, H * D
    if Z.shape != (n_src, HD):
        raise ValueError(f"Z has shape {tuple(Z.shape)}, relation expects ({n_src}, {HD})")
    if origin is not None and origin.shape != (n_dst, HD):
        raise ValueError(f"origin has shape {tuple(origin.shape)}, expected ({n_dst}, {HD})")
    st = stream_of(Z)
    a1, tau = tables if tables is not None else attn_tables(attn, T, wf, bf, H, D)
    if sigma is None:                   # else: from the projection's epilogue (hsg_hproj_fwd_logits)
        sigma = Z.new_empty(n_src, H)
        check(lib.hsg_attn_src_logits(n_src, H, D, ptr(Z), ptr(a1), ptr(sigma), st), "hsg_attn_src_logits")
    relp = ctypes.byref(rel.cstruct())
    no_h = ((no_h or (not keep_h and _lib.path_option("HSG_GAT_NOH", "0") == "1")) and origin is not None
            and bool(lib.hsg_gat_bwd_dst_noh_supported(relp, H, D)))
    h = None if no_h else Z.new_empty(n_dst, HD)
    if origin is None:
        out = None
    elif out is None:
        out = Z.new_empty(n_dst, HD)
    x16 = out is not None and out.dtype == torch.bfloat16
    if x16 and (not no_h or out.shape != (n_dst, HD) or out.stride(1) != 1 or out.stride(0) % 8):
        raise ValueError("gat_table_fwd: bf16 x rows need the no-h forward and an [n_dst, H*D] view of rows "
                         "with a pitch of a multiple of 8")
    m = Z.new_empty(n_dst, H)
    l = Z.new_empty(n_dst, H)
    tok = _clock_start(("gat_fwd", rel.kind), Z)
    try:
        ws = fwd_workspace(lib, relp, H, D, Z)
        if x16:
            check(lib.hsg_gat_fwd_ws16(relp, H, D, HSG_TAU_TABLE, slope, ptr(Z), ptr(sigma), ptr(tau), ptr(origin),
                                       ptr(h), None, ptr(m), ptr(l), ptr(ws), ptr(out), out.stride(0), st),
                  "hsg_gat_fwd_ws16")
        else:
            check(lib.hsg_gat_fwd_ws(relp, H, D, HSG_TAU_TABLE, slope, ptr(Z), ptr(sigma), ptr(tau),
                                     ptr(origin), ptr(h), ptr(out), ptr(m), ptr(l), ptr(ws), st), "hsg_gat_fwd_ws")
    except BaseException:
        _clock_abort(tok)
        raise
    _clock_stop(tok, Z)
    saved = (Z, attn, T, wf, bf, a1, sigma, tau, h, m, l, rel, H, D, slope, origin is not None,
             (out, origin) if no_h else None)
    return (out if origin is not None else h), saved


def gat_table_bwd(saved, dout, dZ=True, dst=None, stage=None, G=None, rho=None):
    """Backward of :func:`gat_table_fwd`: 3 launches (dst pass, src pass with the
    d a1 partials, parameter backward).  Returns dZ (None with dZ=False).  ``dst`` =
    (dattn, dwf, dbf, dT, acc_head, acc_T): gradient buffers written or added into
    (dbf None on W2S).  ``stage`` = (workspace, accumulate) instead: only reduce this
    application's partials into a per-layer workspace (hsg_attn_params_stage); the
    caller runs :func:`attn_params_finish` once for all applications of the layer.
    The origin gradient is ``dout`` itself.  ``G``: the rows dOut * elu'(h), already
    made by the FFN's last GEMM (a forward without h): the dst pass reads them
    (hsg_gat_bwd_dst_g).  ``rho`` (with G): that GEMM's per-64-column partials of
    G_v . h_v (hsg_gemm_psw_elug_rho, [n_dst, groups, 3]) or, for narrow heads, the
    per-head G_v . h_v of the narrow FFN's epilogue (hsg_ffn_small_bwd_gate, [n_dst, H])
    -- the whole backward is then ONE source-centric launch (hsg_gat_bwd_src_g) instead
    of the dst + src pair."""
    lib = load()
    Z, attn, T, wf, bf, a1, sigma, tau, h, m, l, rel, H, D, slope, has_origin, xo = saved
    dout = dout.contiguous()
    st = stream_of(Z)
    relp = ctypes.byref(rel.cstruct())
    g_given = G is not None
    if not g_given:
        G = torch.empty_like(dout)
    merged = rho is not None
    if merged and not g_given:
        raise ValueError("gat_table_bwd: rho partials without their G rows")
    if merged and rho.dtype != torch.float32:
        raise ValueError("gat_table_bwd: rho partials are fp32")
    if G.dtype == torch.bfloat16 and not merged:
        raise ValueError("gat_table_bwd: bf16 G rows are read by the one-pass backward only")
    nbs = lib.hsg_gat_bwd_src_g_blocks(relp, H, D) if merged else lib.hsg_gat_bwd_src_blocks(relp)
    nbd = nbs if merged else lib.hsg_gat_bwd_blocks(relp)
    dtp = Z.new_empty(nbd, N_BOX + 1, H)
    dZt = torch.empty_like(Z)
    da1p = Z.new_empty(nbs, H * D)
    tok = _clock_start(("gat_bwd", rel.kind), Z)
    try:
        if g_given and not merged and xo is None:
            raise ValueError("gat_table_bwd: G rows given for a forward that stored h")
        if merged:                          # one source-centric pass (G and rho from the FFN epilogue)
            # rho [n_dst, groups, 3]: 64-column-group partials (wide heads); [n_dst, H]: per head
            groups = rho.shape[1] if rho.dim() == 3 else 0
            # (G bf16: the bf16 GEMM mode's bf16 G rows; ws: the pieces of the relation's
            # long sources, when it has a CSC work list)
            n_ws = lib.hsg_gat_bwd_src_g_ws_floats(relp, H, D)
            ws = Z.new_empty(n_ws) if n_ws else None
            check(lib.hsg_gat_bwd_src_g_ws(relp, H, D, slope, ptr(sigma), ptr(tau), ptr(m), ptr(l), ptr(G),
                                           int(G.dtype == torch.bfloat16), ptr(rho), groups, ptr(a1), ptr(Z),
                                           ptr(dZt), None, ptr(da1p), ptr(dtp), ptr(ws), st), "hsg_gat_bwd_src_g_ws")
        else:
            dpre = Z.new_empty(rel.n_typed, H)
            if g_given:                     # G from the FFN epilogue (forward without h)
                check(lib.hsg_gat_bwd_dst_g(relp, H, D, HSG_TAU_TABLE, slope, ptr(Z), ptr(sigma), ptr(tau), ptr(m),
                                            ptr(l), ptr(G), ptr(dpre), ptr(dtp), st), "hsg_gat_bwd_dst_g")
            elif xo is not None:            # forward without h (keep_h=False)
                if xo[0].dtype != torch.float32:
                    raise ValueError("gat_table_bwd: a forward with bf16 x rows needs its G rows from the FFN "
                                     "epilogue (hsg_gemm_bf16_psw_elug_rho_x16)")
                check(lib.hsg_gat_bwd_dst_noh(relp, H, D, HSG_TAU_TABLE, slope, ptr(Z), ptr(sigma), ptr(tau),
                                              ptr(xo[0]), ptr(xo[1]), ptr(m), ptr(l), ptr(dout), ptr(G), ptr(dpre),
                                              ptr(dtp), st), "hsg_gat_bwd_dst_noh")
            else:
                check(lib.hsg_gat_bwd_dst(relp, H, D, HSG_TAU_TABLE, int(has_origin), slope, ptr(Z), ptr(sigma),
                                          ptr(tau), ptr(h), ptr(m), ptr(l), ptr(dout), ptr(G), ptr(dpre),
                                          ptr(dtp), st), "hsg_gat_bwd_dst")
            check(lib.hsg_gat_bwd_src(relp, H, D, HSG_TAU_TABLE, slope, ptr(sigma), ptr(tau), ptr(m), ptr(l),
                                      ptr(G), ptr(dpre), ptr(a1), ptr(Z), ptr(dZt), None, ptr(da1p), st),
                  "hsg_gat_bwd_src")
    except BaseException:
        _clock_abort(tok)
        raise
    _clock_stop(tok, Z)
    if stage is not None and len(stage) == 3:       # (batch, key, workspace): staged with every application
        batch, key, ws = stage
        nt = (N_BOX + 1) * H
        rows = ws.numel() // (nt + H * D)                # the workspace's stage rows
        batch.add((key, "dtau"), ws[:rows * nt], nt, nt, 0, 1.0, False, dtp, nbd, out_rows=rows)
        batch.add((key, "da1"), ws[rows * nt:], H * D, H * D, 0, 1.0, False, da1p, nbs, out_rows=rows)
    elif stage is not None:
        ws, acc = stage
        check(lib.hsg_attn_params_stage(H, D, nbd, ptr(dtp), nbs, ptr(da1p), ptr(ws), int(bool(acc)), st),
              "hsg_attn_params_stage")
    elif dst is not None:
        dattn, dwf, dbf, dT, acc_head, acc_T = dst
        ws = Z.new_empty(lib.hsg_attn_params_bwd_workspace_floats(H, D))
        check(lib.hsg_attn_params_bwd(H, D, T.shape[1], nbd, ptr(dtp), nbs, ptr(da1p), ptr(attn), ptr(wf),
                                      ptr(bf), ptr(T), ptr(dattn), ptr(dwf), ptr(dbf), ptr(dT), ptr(ws),
                                      int(bool(acc_head)) | (2 if acc_T else 0), st), "hsg_attn_params_bwd")
    return dZt if dZ else None


def attn_params_workspace(Z, H, D):
    """A stage workspace for :func:`gat_table_bwd` / :func:`attn_params_finish`."""
    return Z.new_empty(load().hsg_attn_params_bwd_workspace_floats(H, D))


def attn_params_finish(ws, attn, T, wf, bf, H, D, dst):
    """Parameter gradients from a stage workspace (hsg_attn_params_finish); ``dst``
    as in :func:`gat_table_bwd`."""
    dattn, dwf, dbf, dT, acc_head, acc_T = dst
    check(load().hsg_attn_params_finish(H, D, T.shape[1], ptr(ws), ptr(attn), ptr(wf), ptr(bf), ptr(T), ptr(dattn),
                                        ptr(dwf), ptr(dbf), ptr(dT), int(bool(acc_head)) | (2 if acc_T else 0),
                                        stream_of(ws)), "hsg_attn_params_finish")


def attn_params_finish_pair(job0, job1, T):
    """:func:`attn_params_finish` of two layers sharing T in ONE launch
    (hsg_attn_params_finish_pair); ``job`` = (ws, layer, dst) with ``dst`` as in
    :func:`gat_table_bwd`, in the order the two separate calls would run."""
    args = []
    for ws, lay, dst in (job0, job1):
        dattn, dwf, dbf, dT, acc_head, acc_T = dst
        args += [lay.H, lay.D, ptr(ws), ptr(lay.attn), ptr(lay.wf), ptr(lay.bf), ptr(dattn), ptr(dwf), ptr(dbf),
                 ptr(dT), int(bool(acc_head)) | (2 if acc_T else 0)]
    check(load().hsg_attn_params_finish_pair(*args, T.shape[1], ptr(T), stream_of(T)), "hsg_attn_params_finish_pair")


class _GatHeadsTable(torch.autograd.Function):
    """One multi-head application whose edge-type term comes from the TF-IDF table.

    Same math as ``_GatAggregate`` with ``tau`` built in-kernel from the layer's
    attention parameters (include/hsg.h, hsg_attn_params_fwd), so forward is 3
    launches (params, sigma, edge pass) and backward 3 (dst pass, src pass with
    the d a1 partials, params backward) with every parameter gradient written
    directly -- no per-parameter slicing, einsum or reduction kernels."""

    @staticmethod
    def forward(ctx, Z, attn, T, wf, bf, origin, rel, H, D, slope):
        Z = Z.contiguous()
        origin = None if origin is None else origin.contiguous()
        out, saved = gat_table_fwd(Z, attn, T, wf, bf, origin, rel, H, D, slope)
        ctx.save_for_backward(*saved[:11])
        ctx.rest = saved[11:]
        return out

    @staticmethod
    def backward(ctx, dout):
        saved = tuple(ctx.saved_tensors) + ctx.rest
        attn, T, wf, bf = saved[1:5]
        has_origin = saved[15]
        dattn, dwf, dT = torch.empty_like(attn), torch.empty_like(wf), torch.empty_like(T)
        dbf = torch.empty_like(bf) if bf is not None else None
        need = ctx.needs_input_grad
        dZ = gat_table_bwd(saved, dout, dZ=need[0], dst=(dattn, dwf, dbf, dT, False, False))
        return (dZ, dattn if need[1] else None, dT if need[2] else None,
                dwf if need[3] else None, dbf if need[4] else None,
                (dout if has_origin else None), None, None, None, None)


def gat_heads_table(Z, attn, T, wf, bf, origin, rel, H, D, slope=LEAKY_SLOPE):
    """Multi-head aggregation with the TF-IDF-table edge term (+ ELU + residual).

    Z [n_src, H*D]; attn [H, 3D] (attn_fc weights [a1|a2|a3] of every head);
    T [10, F] TF-IDF embedding table; wf [H, D, F], bf [H, D] | None (feat_fc);
    origin [n_dst, H*D] | None.  Returns [n_dst, H*D]."""
    _require_device(Z, attn, T, wf, bf, origin)
    attn, T, wf = attn.contiguous(), T.contiguous(), wf.contiguous()
    bf = bf.contiguous() if bf is not None else None
    return _GatHeadsTable.apply(Z, attn, T, wf, bf, origin, rel, H, D, float(slope))


def gat_aggregate(Z, a1, tau, origin, rel, H, D, slope=LEAKY_SLOPE, tau_mode=HSG_TAU_TABLE):
    """Fused multi-head edge-softmax aggregation (+ ELU + residual when ``origin``).

    Z [n_src, H*D], a1 [H, D], tau [11, H] (table) or [E_T, H] (per edge, CSR
    order), origin [n_dst, H*D] or None.  Returns [n_dst, H*D]."""
    _require_device(Z, a1, tau, origin)
    return _GatAggregate.apply(Z, a1, tau, origin, rel, H, D, float(slope), int(tau_mode))
