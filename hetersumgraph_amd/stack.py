"""The WSWGAT stack as one autograd node (HiGraph.py:99-106).

``HSumGraph.forward`` runs W2S, then ``n_iter`` x (S2W, W2S), over the same two
modules: word2sent is applied n_iter+1 times, sent2word n_iter times, and every
application reads the shared ``_TFembed`` table.  Run layer by layer through
autograd, each extra application of a parameter costs a gradient-accumulation
kernel (``p.grad += g``), and each state tensor used both as a residual origin and
as the next layer's neighbour costs another (~30 small launches per cfg2 step).

Here the whole stack is one ``torch.autograd.Function``: the forward runs the
same C-ABI kernels in the same order (so dropout masks, drawn in call order, are
the per-layer path's), and the backward walks the applications in reverse and
lets the kernels do the sums in their epilogues:

* a parameter's gradient buffer is written by its first contribution and added
  into by every later application of the same layer (GEMM ADD epilogue, and the
  ``accumulate`` flag of hsg_hproj_dw / hsg_attn_params_bwd / hsg_ffn_colsums);
  the buffers are then RETURNED to autograd like any Function's input gradients,
  so ``AccumulateGrad`` installs them (``zero_grad(set_to_none=True)``: the buffer
  becomes ``p.grad`` with no copy) or adds them, and ``torch.autograd.grad``,
  ``backward(inputs=...)``, tensor / post-accumulate hooks and DDP-style reducers
  see an ordinary autograd node;
* a state's gradient starts as the FFN backward's residual-branch ``dx`` of the
  layer it was the origin of, and the head-projection backward of the layer it
  was the neighbour of adds into it (hsg_hproj_dx accumulate).

``HSumGraph`` falls back to the per-layer path (module/GAT.py) for anything this
node does not cover (CPU tensors, a foreign ``tfidfembed`` column,
HSG_CHECK_NAN=1).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import rng as hsg_rng
from ._lib import load, stream_of
from .dense import elug_rho_groups, gemm, gemm_dw_slabs, gemm_slabs
from .graph import record_edge_scores
from .ffn import bf16_rows_ok, ffn_bwd, ffn_fwd, ffn_wsplit
from .hproj import dropmasks, hproj_bwd, hproj_fwd, narrow_heads, transposed_weight
from .reduce import SlabBatch
from .ops import (LEAKY_SLOPE, attn_params_finish, attn_params_finish_pair, attn_params_workspace, attn_tables,
                  attn_tables_pair, gat_table_bwd, gat_table_fwd)


class _Grads:
    """The parameter-gradient buffers of one backward of the stack, keyed by
    parameter: created (written, not zero-filled) by a parameter's first
    contribution, added into by the later ones.  Returned to autograd at the end.

    All buffers are views of ONE flat tensor, in parameter order, so that a
    data-parallel reducer can all-reduce the stack's gradients in place as a single
    bucket once autograd has installed them as ``p.grad`` (parallel.flat_gradients)
    -- no concatenation before the collective and no copy back after it."""

    def __init__(self, params=()):
        self.buf = {}
        live = [p for p in params if p is not None and p.requires_grad]
        self.flat = None
        self.views = {}
        if live:
            self.flat = torch.empty(sum(p.numel() for p in live), dtype=live[0].dtype, device=live[0].device)
            o = 0
            for p in live:
                self.views[id(p)] = self.flat[o:o + p.numel()].view_as(p)
                o += p.numel()

    def _new(self, p, zero=False):
        g = self.views.get(id(p))
        if g is None:
            g = torch.zeros_like(p) if zero else torch.empty_like(p)
        elif zero:
            g.zero_()
        self.buf[id(p)] = g
        return g

    def dst(self, p):
        """(buffer, accumulate) for p's gradient; (None, False) if p needs none."""
        if p is None or not p.requires_grad:
            return None, False
        g = self.buf.get(id(p))
        if g is None:
            return self._new(p), False
        return g, True

    def group(self, ps):
        """Buffers for parameters whose gradients one kernel writes together under
        one accumulate flag: all fresh -> written; otherwise missing ones start at 0."""
        live = [p for p in ps if p is not None and p.requires_grad]
        if not live:
            return [None] * len(ps), False
        if all(id(p) not in self.buf for p in live):
            for p in live:
                self._new(p)
            acc = False
        else:
            for p in live:
                if id(p) not in self.buf:
                    self._new(p, zero=True)
            acc = True
        return [self.buf[id(p)] if (p is not None and p.requires_grad) else None for p in ps], acc

    def get(self, p):
        return self.buf.get(id(p))


class _Layer:
    """The tensors of one WSWGAT module (module/GAT.py:31-43) as the kernels take them."""

    def __init__(self, m):
        L, f = m.layer, m.ffn
        self.kind = m.layerType
        self.H, self.D = L.num_heads, L.head_dim
        self.W, self.attn, self.wf, self.bf = L.fused_params()
        self.w1, self.b1, self.w2, self.b2 = f.w_1.weight, f.w_1.bias, f.w_2.weight, f.w_2.bias
        self.gamma, self.beta, self.eps = f.layer_norm.weight, f.layer_norm.bias, f.layer_norm.eps
        self.p_attn = L.dropout.p if (L.dropout.training and L.dropout.p > 0) else 0.0
        self.p_ffn = f.dropout.p if (f.dropout.training and f.dropout.p > 0) else 0.0

    def params(self):
        return [p for p in (self.W, self.attn, self.wf, self.bf, self.w1, self.b1, self.w2, self.b2,
                            self.gamma, self.beta) if p is not None]


def _apply_fwd(lay, rel, T, neighbor, origin, tables=None, x_out=None, H_out=None, wsplit="auto", draws=(None, None),
               wt=None):
    """out = FFN(elu(MultiHeadLayer(neighbor)) + origin) -- module/GAT.py:45-59.
    ``tables``: the layer's (a1, tau) from :func:`ops.attn_tables`, shared by its
    applications within one forward; ``x_out`` / ``H_out``: this application's slots
    of the layer's FFN-input and hidden-activation buffers; ``wsplit``: the layer's
    pre-split FFN weights (ffn.ffn_wsplit), likewise shared; ``draws`` = (head
    projection keep-mask bits, FFN dropout (seed, offset)) drawn up front by the
    caller, or None each (drawn here); ``wt``: the layer's transposed head weights for
    the narrow-head projection (hproj.transposed_weight), shared likewise."""
    H, D = lay.H, lay.D
    sigma = None
    if lay.p_attn > 0 and tables is not None:     # source logits from the projection's epilogue
        Z, hsaved, sigma = hproj_fwd(neighbor, lay.W, H, D, lay.p_attn, a1=tables[0], bits=draws[0], wt=wt)
    elif lay.p_attn > 0:
        Z, hsaved = hproj_fwd(neighbor, lay.W, H, D, lay.p_attn, bits=draws[0], wt=wt)
    else:
        Z, hsaved = gemm(neighbor, lay.W, b_t=True, dtype="f32"), None      # fp32 in every GEMM mode, as hproj
    # with the FFN on the pre-split-weight GEMMs, its backward's last GEMM also makes the
    # edge layer's G rows (hsg_gemm_f32_psw_elug), so the forward need not store h
    # (HSG_GAT_GEPI=0: h stored and G made in the dst pass, for A/B tests)
    g_epi = wsplit is not None and not isinstance(wsplit, str) and _lib.path_option("HSG_GAT_GEPI", "1") != "0"
    x, gsaved = gat_table_fwd(Z, lay.attn, T, lay.wf, lay.bf, origin, rel, H, D, LEAKY_SLOPE, tables=tables,
                              out=x_out, sigma=sigma, keep_h=False, no_h=g_epi)
    d_hid, d = lay.w1.shape[0], lay.w1.shape[1]
    out, fsaved = ffn_fwd(x, lay.w1.view(d_hid, d), lay.b1, lay.w2.view(d, d_hid), lay.b2, lay.gamma, lay.beta,
                          lay.p_ffn, lay.eps, H_out=H_out, wsplit=wsplit, rng=draws[1])
    return out, (hsaved, neighbor, gsaved, fsaved)


def _attn_dst(grads, lay, T):
    """(dattn, dwf, dbf, dT, acc_head, acc_T) for the attention-parameter backward of
    ``lay``, or None when none of them needs a gradient (scratch for unneeded ones:
    the kernel writes all four)."""
    (dattn, dwf, dbf), a_h = grads.group([lay.attn, lay.wf, lay.bf])
    dT, a_T = grads.dst(T)
    if not any(t is not None for t in (dattn, dwf, dbf, dT)):
        return None
    dattn, dwf, dT = [t if t is not None else torch.empty_like(p)
                      for t, p in ((dattn, lay.attn), (dwf, lay.wf), (dT, T))]
    if lay.bf is not None and dbf is None:
        dbf = torch.empty_like(lay.bf)
    return dattn, dwf, dbf, dT, a_h, a_T


def rho_partials(G, groups):
    """The rho partials [n_dst, groups, 3] the dx GEMM's ELU-gate epilogue writes beside
    the G rows: fp32 whatever G's dtype (hsg_gemm_bf16_psw_elug_rho_a16 stores fp32
    sums; the one-pass edge backward reads fp32).  Round 5's first bf16-G run made them
    with ``G.new_empty(...)``, i.e. bf16 -- half the bytes -- and the epilogue's stores
    ran past the buffer into the allocator's neighbours: the abort in the cfg5-bf16
    stack backward.  Pinned on the CPU by tests/test_fault_regressions.py."""
    return G.new_empty(G.shape[0], groups, 3, dtype=torch.float32)


def _x16_ok(lay, rel, wsplit, d, d_hid):
    """The bf16 GEMM mode keeps this application's edge-layer output x (the wide FFN's
    A operand, LayerNorm residual and dW1 operand) as bf16 rows (round 6, VERDICT r5
    #8): the FFN runs on the bf16 rows (ffn.bf16_rows_ok), the forward stores no h
    (its backward's G comes from the dx GEMM's epilogue, which then reads the bf16 x:
    hsg_gemm_bf16_psw_elug_rho_x16) and that backward is the one-pass source-centric
    launch (bf16 G).  HSG_FFN_BF16_X=0: fp32 x rows (A/B)."""
    if wsplit is None or isinstance(wsplit, str) or wsplit[0].mode != "bf16" or not bf16_rows_ok(d, d_hid):
        return False
    if any(_lib.path_option(k, "1") == "0" for k in ("HSG_FFN_BF16_X", "HSG_FFN_BF16_ROWS", "HSG_FFN_BF16_ACT",
                                                     "HSG_GAT_GEPI", "HSG_GAT_MERGED")):
        return False
    if lay.H * lay.D != d:
        return False
    lib, relp = load(), ctypes.byref(rel.cstruct())
    return (bool(lib.hsg_gat_bwd_dst_noh_supported(relp, lay.H, lay.D))
            and bool(lib.hsg_gat_bwd_src_g_supported(relp, lay.H, lay.D)))


def _merged_bwd(gsaved):
    """The one-pass edge backward (hsg_gat_bwd_src_g) covers this application's
    relation and head shape (HSG_GAT_MERGED=0: the dst + src pair, for A/B tests)."""
    if _lib.path_option("HSG_GAT_MERGED", "1") == "0":
        return False
    rel, H, D = gsaved[11], gsaved[12], gsaved[13]
    return bool(load().hsg_gat_bwd_src_g_supported(ctypes.byref(rel.cstruct()), H, D))


def _apply_bwd(grads, lay, T, saved, dout, nb_grad, nb_acc, stage=None, act_grads=None, batch=None):
    """Backward of one application.  Parameter gradients go to ``grads``; the
    neighbour's gradient is written (or added, nb_acc) into ``nb_grad`` when that is
    not None.  ``stage`` = (workspace, accumulate): the attention-parameter partials
    only go into the layer's stage workspace (finished once per layer by the caller).
    ``act_grads`` = (dy, dH) slots: the FFN's activation gradients go there and its
    weight gradients are left to the caller (one GEMM per weight over all
    applications).  ``batch``: a reduce.SlabBatch collecting the column sums of the
    FFN bias / LayerNorm and head-projection dW partials (summed once per backward).
    Returns the origin's gradient (the FFN's residual-branch dx)."""
    hsaved, neighbor, gsaved, fsaved = saved
    d_hid, d = lay.w1.shape[0], lay.w1.shape[1]
    # forward without h and the FFN on the pre-split path: the G rows of the edge
    # backward come out of the FFN's last GEMM (dx epilogue)
    G = rho = None
    # (the bf16 GEMM mode's bf16 activations, fsaved[4] = H bf16: G bf16 too when the one
    # source-centric backward -- the only reader that takes bf16 G -- runs)
    merged = gsaved[16] is not None and fsaved[11] is not None and _merged_bwd(gsaved)
    gdt = torch.bfloat16 if (merged and fsaved[4].dtype == torch.bfloat16
                             and _lib.path_option("HSG_FFN_BF16_ROWS", "1") != "0") else torch.float32
    elug = (gsaved[16][1], torch.empty(fsaved[0].shape, dtype=gdt, device=fsaved[0].device)) \
        if gsaved[16] is not None and fsaved[11] is not None else None
    if elug is not None and merged:
        # ... and the rho partials, so the edge backward is one source-centric pass
        n_dst, HD = elug[1].shape
        groups = elug_rho_groups(fsaved[11][3], n_dst, gsaved[13])     # the dx GEMM's (W1^T split)
        elug += (rho_partials(elug[1], groups), gsaved[13])
    # narrow heads (W2S) with h stored: the narrow FFN's backward epilogue makes G and the
    # per-head rho, and the edge backward is one head-lane pass over the words
    gate = None
    if elug is None and gsaved[8] is not None and gsaved[13] == 8 and _merged_bwd(gsaved):
        h = gsaved[8]
        gate = (h, torch.empty_like(h), h.new_empty(h.shape[0], gsaved[12]))
    if act_grads is None:
        dw1, a_w1 = grads.dst(lay.w1)
        dw2, a_w2 = grads.dst(lay.w2)
    else:
        dw1, a_w1, dw2, a_w2 = None, False, None, False
    (db1, db2, dg, dbt), a_b = grads.group([lay.b1, lay.b2, lay.gamma, lay.beta])
    dx = ffn_bwd(fsaved, dout, (dw1.view(d_hid, d) if dw1 is not None else None, a_w1,
                                dw2.view(d, d_hid) if dw2 is not None else None, a_w2, db1, db2, dg, dbt, a_b),
                 act_grads=act_grads, batch=batch, key=id(lay), elug=elug, gate=gate)
    if elug is not None:
        dx, g_done = dx
        G = elug[1] if g_done else None
        rho = elug[2] if g_done and len(elug) > 2 else None
    elif gate is not None:
        dx, g_done = dx
        G, rho = (gate[1], gate[2]) if g_done else (None, None)
    need_dz = nb_grad is not None or lay.W.requires_grad
    if stage is not None:
        dZ = gat_table_bwd(gsaved, dx, dZ=need_dz, stage=stage, G=G, rho=rho)
    else:
        dZ = gat_table_bwd(gsaved, dx, dZ=need_dz, dst=_attn_dst(grads, lay, T), G=G, rho=rho)
    if need_dz:
        dW, a_W = grads.dst(lay.W)
        if hsaved is not None:
            hproj_bwd(hsaved, dZ, dX=nb_grad, dX_acc=nb_acc, dW=dW, dW_acc=a_W, batch=batch, key=id(lay))
        else:                                   # eval-mode projection Z = neighbor W^T
            if nb_grad is not None:
                gemm(dZ, lay.W, out=nb_grad, add=nb_grad if nb_acc else None, dtype="f32")
            if dW is not None:
                gemm(dZ, neighbor, a_t=True, out=dW, add=dW if a_W else None, dtype="f32")
    return dx


class _GatStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, w0, s0, *params):
        G, w2s, s2w, T, n_iter = cfg
        rw, rs = G.relation("W2S"), G.relation("S2W")
        states = {("w", 0): w0.contiguous(), ("s", 0): s0.contiguous()}
        apps = []                               # (layer, saved, neighbour key, origin key, slot)
        # every application of a layer writes its FFN input and hidden activations
        # into one [applications, rows, width] buffer per layer, so the backward runs
        # each FFN weight gradient as ONE GEMM over all applications' rows
        n_app = {id(w2s): n_iter + 1, id(s2w): n_iter}
        bufs, slot = {}, {id(w2s): 0, id(s2w): 0}

        # every dropout draw of the forward, in the order the layer-by-layer path takes
        # them (per application: head projection, then FFN), so both paths see the
        # same masks; the head-projection keep-masks are then made in ONE launch
        seq = [(w2s, rw)] + [(s2w, rs), (w2s, rw)] * n_iter
        gen = hsg_rng.get(w0.device)
        # the attention tables depend on the parameters only: once per layer, in the
        # forward's first launch, which also performs the step's pending dropout-seed
        # advance (before any draw below reads the seed)
        if _lib.path_option("HSG_ATTN_PAIR", "1") != "0":      # both layers' tables in one launch
            adv = gen.claim()
            tables = dict(zip((id(w2s), id(s2w)), attn_tables_pair(w2s, s2w, T, seed_advance=adv)))
            if adv is not None:                 # launched (check() raised otherwise): done
                gen.claimed()
        else:
            tables = {id(lay): attn_tables(lay.attn, T, lay.wf, lay.bf, lay.H, lay.D) for lay in (w2s, s2w)}
        draws = []
        for lay, _ in seq:
            hm = gen.take() if lay.p_attn > 0 else None
            fr = gen.take() if lay.p_ffn > 0 else None
            draws.append([hm, fr])
        jobs = [(rel.n_src, lay.W.shape[1], lay.H, lay.p_attn, d[0][0], d[0][1])
                for (lay, rel), d in zip(seq, draws) if d[0] is not None]
        # the narrow-head (VALU) projection's transposed weight comes out of the same
        # launch as the masks (hsg_dropmask_multi_wt; HSG_WT_FOLD=0: its own launch)
        narrow = [lay for lay in (w2s, s2w) if lay.p_attn > 0 and narrow_heads(lay.W.shape[1], lay.H, lay.D)]
        fold = narrow[0] if narrow and jobs and _lib.path_option("HSG_WT_FOLD", "1") != "0" else None
        # ... and so are the wide FFN's weight limb planes (hsg_step_prologue: one launch
        # for masks, transpose and split; HSG_WT_FOLD=0: separate launches)
        wsplits, split_job = {}, None
        if fold is not None:
            for lay in (w2s, s2w):
                d_hid, d = lay.w1.shape[0], lay.w1.shape[1]
                args = (w0.new_empty(1, d), lay.w1.view(d_hid, d), lay.b1, lay.w2.view(d, d_hid), lay.b2)
                if split_job is not None:           # a second wide FFN: its own launch
                    wsplits[id(lay)] = ffn_wsplit(*args)
                    continue
                r = ffn_wsplit(*args, launch=False)
                wsplits[id(lay)] = r[0] if r is not None else None
                if r is not None:
                    split_job = r[1]
            mlist, wt_fold = dropmasks(jobs, w0.device, stream_of(w0), wt=(fold.W, fold.H, fold.D),
                                       wsplit_job=split_job)
        else:
            mlist, wt_fold = dropmasks(jobs, w0.device, stream_of(w0)), None
        masks = iter(mlist)
        for d in draws:
            if d[0] is not None:
                d[0] = next(masks)
        napp = [0]

        def run(lay, rel, nb, org, outk):
            key = id(lay)
            if key not in bufs:
                d_hid, d = lay.w1.shape[0], lay.w1.shape[1]
                X = states[org].new_empty(n_app[key], rel.n_dst, d)
                # the FFN weights split into limb planes once per forward (hsg_wsplit),
                # unless the prologue launch already did
                if key not in wsplits:
                    wsplits[key] = ffn_wsplit(X[0], lay.w1.view(d_hid, d), lay.b1, lay.w2.view(d, d_hid), lay.b2)
                # the bf16 GEMM mode keeps the wide FFN's hidden activations H as bf16
                # (with dY and dH in the backward): they are only GEMM operands there,
                # rounded to bf16 by the GEMM anyway -- half their bytes, the same numbers
                # (HSG_FFN_BF16_ACT=0: fp32 buffers, for the bitwise A/B test)
                bf = (wsplits[key] is not None and wsplits[key][0].mode == "bf16" and bf16_rows_ok(d, d_hid)
                      and _lib.path_option("HSG_FFN_BF16_ACT", "1") != "0")
                if _x16_ok(lay, rel, wsplits[key], d, d_hid):
                    # ... and its input x as bf16 rows, pitch ceil8(d) (zero pad: the bf16-A
                    # contract), written by the edge forward (hsg_gat_fwd_ws16)
                    X = X.new_empty(n_app[key], rel.n_dst, (d + 7) // 8 * 8, dtype=torch.bfloat16)[:, :, :d]
                bufs[key] = (X, X.new_empty(n_app[key], rel.n_dst, d_hid,
                                            dtype=torch.bfloat16 if bf else torch.float32))
            a = slot[key]
            slot[key] += 1
            out, saved = _apply_fwd(lay, rel, T, states[nb], states[org], tables[key], x_out=bufs[key][0][a],
                                    H_out=bufs[key][1][a], wsplit=wsplits[key], draws=draws[napp[0]],
                                    wt=wts[key])
            napp[0] += 1
            states[outk] = out
            apps.append((lay, saved, nb, org, a))

        # the transposed head weights of a narrow-head (VALU) projection
        wts = {id(lay): ((wt_fold if lay is fold else transposed_weight(lay.W, lay.H, lay.D))
                         if any(lay is q for q in narrow) else None)
               for lay in (w2s, s2w)}
        run(w2s, rw, ("w", 0), ("s", 0), ("s", 1))
        for i in range(n_iter):
            run(s2w, rs, ("s", i + 1), ("w", i), ("w", i + 1))
            run(w2s, rw, ("w", i + 1), ("s", i + 1), ("s", i + 2))
        # g.edata['e'] as the reference leaves it: the last head's logits of the last
        # application of each relation, formed only if someone reads the column
        from .module.GATLayer import LastHeadScores
        last = {lay.kind: (lay, saved) for lay, saved, *_ in apps}
        for kind in ("W2S", "S2W"):
            if kind in last:
                lay, saved = last[kind]
                record_edge_scores(G, LastHeadScores(kind, G.relation(kind), saved[2][0], lay.attn, lay.wf,
                                                     lay.bf, T=T))
        ctx.cfg, ctx.apps, ctx.bufs = cfg, apps, bufs
        ctx.params = params
        ctx.need = (w0.requires_grad, s0.requires_grad)
        ctx.shapes = {k: v.shape for k, v in states.items()}
        return states[("s", n_iter + 1)]

    @staticmethod
    def backward(ctx, ds):
        if ctx.apps is None:
            raise RuntimeError("the fused WSWGAT stack's saved state was freed (backward called twice?)")
        n_iter = ctx.cfg[4]
        T = ctx.cfg[3]
        grads = {("s", n_iter + 1): ds.contiguous()}
        need_w0, need_s0 = ctx.need
        skip = {("w", 0)} if not need_w0 else set()
        if not need_s0:
            skip.add(("s", 0))
        # attention-parameter partials of all applications of a layer meet in one
        # stage workspace; the parameter transform runs once per layer at the end
        stages, gbufs = {}, {}
        pgrads = _Grads(ctx.params)
        batch = SlabBatch()
        for lay, saved, nb, org, a in reversed(ctx.apps):
            dout = grads.pop((org[0], org[1] + 1))
            nb_grad, nb_acc = None, False
            if nb not in skip:
                if nb in grads:
                    nb_grad, nb_acc = grads[nb], True
                else:
                    nb_grad = saved[1].new_empty(ctx.shapes[nb])
                    grads[nb] = nb_grad
            if id(lay) not in stages:                  # the layer's staged attention partials
                stages[id(lay)] = (lay, attn_params_workspace(saved[2][0], lay.H, lay.D))
            stage = (batch, id(lay), stages[id(lay)][1])
            if id(lay) not in gbufs:
                X, Hh = ctx.bufs[id(lay)]
                if Hh.dtype == torch.bfloat16:       # bf16 dY rows padded to a multiple of 8 (zeros)
                    d = X.shape[2]
                    DY = X.new_empty(X.shape[0], X.shape[1], (d + 7) // 8 * 8, dtype=torch.bfloat16)[:, :, :d]
                else:
                    DY = torch.empty_like(X)
                gbufs[id(lay)] = (lay, DY, torch.empty_like(Hh))
            _, DY, DH = gbufs[id(lay)]
            dx = _apply_bwd(pgrads, lay, T, saved, dout, nb_grad, nb_acc, stage, act_grads=(DY[a], DH[a]),
                            batch=batch)
            if org in skip:
                continue
            if org in grads:
                grads[org].add_(dx)
            else:
                grads[org] = dx
        # FFN weight gradients, one GEMM per weight over every application's rows:
        # dW2 = dY^T H, dW1 = dH^T X with [applications * rows] as the reduction
        # -- both of a layer in ONE launch (hsg_gemm_dw_slabs; HSG_DW_PAIR=0: one
        # hsg_gemm_*_slabs launch each, for A/B)
        for lay, DY, DH in gbufs.values():
            X, Hh = ctx.bufs[id(lay)]
            d_hid, d = lay.w1.shape[0], lay.w1.shape[1]
            todo = []
            DYf = DY.reshape(-1, DY.shape[2]) if DY.is_contiguous() else \
                DY.as_strided((DY.shape[0] * DY.shape[1], DY.shape[2]), (DY.stride(1), 1))
            Xf = X.reshape(-1, d) if X.is_contiguous() else \
                X.as_strided((X.shape[0] * X.shape[1], d), (X.stride(1), 1))      # bf16 x rows, pitch ceil8(d)
            for p, A, B, (m, n) in ((lay.w2, DYf, Hh.view(-1, d_hid), (d, d_hid)),
                                    (lay.w1, DH.view(-1, d_hid), Xf, (d_hid, d))):
                dw, a_w = pgrads.dst(p)
                if dw is not None:
                    todo.append((p, A, B, m, n, dw, a_w))
            pair = gemm_dw_slabs([(A, B) for _, A, B, *_ in todo]) \
                if todo and _lib.path_option("HSG_DW_PAIR", "1") != "0" else None
            for k, (p, A, B, m, n, dw, a_w) in enumerate(todo):
                sl = pair[k] if pair is not None else gemm_slabs(A, B, a_t=True)   # split-K slabs
                if sl is not None:
                    batch.add((id(lay), id(p)), dw.view(-1), m * n, m * n, 0, 1.0, a_w, sl[0], sl[1])
                else:
                    gemm(A, B, a_t=True, out=dw.view(m, n), add=dw.view(m, n) if a_w else None)
        batch.flush()
        fin = [(ws, lay, _attn_dst(pgrads, lay, T)) for lay, ws in stages.values()]   # in order (dT flags)
        fin = [f for f in fin if f[2] is not None]
        if len(fin) == 2 and _lib.path_option("HSG_ATTN_PAIR", "1") != "0":
            attn_params_finish_pair(fin[0], fin[1], T)                # both layers in one launch
        else:
            for ws, lay, dst in fin:
                attn_params_finish(ws, lay.attn, T, lay.wf, lay.bf, lay.H, lay.D, dst)
        ctx.apps = ctx.bufs = None
        dw0 = grads.get(("w", 0)) if need_w0 else None
        ds0 = grads.get(("s", 0)) if need_s0 else None
        out = tuple(pgrads.get(p) for p in ctx.params)
        # a parameter that got no contribution has no gradient (None), as before; its
        # stretch of the flat buffer is left untouched (never read by the reducer)
        ctx.params = None
        return (None, dw0, ds0) + out


def fused_stack_ok(G, word2sent, sent2word, T, w, s):
    """Whether :func:`gat_stack` covers this call (else use the per-layer path)."""
    from .module.GATLayer import CHECK_NAN, table_weight
    if _lib.path_option("HSG_FUSED_STACK", "1") == "0":   # per-layer path (A/B tests)
        return False
    if CHECK_NAN or not (w.is_cuda and s.is_cuda) or w.dtype != torch.float32 or s.dtype != torch.float32:
        return False
    if word2sent.layerType != "W2S" or sent2word.layerType != "S2W":
        return False
    try:
        tw = table_weight(G)
    except KeyError:
        return False
    return tw is T and T.shape[1] == word2sent.layer.feat_weight.shape[2] == sent2word.layer.feat_weight.shape[2]


def gat_stack(G, word2sent, sent2word, T, w, s, n_iter):
    """Sentence (supernode) state after W2S + n_iter x (S2W, W2S) -- the loop of
    HiGraph.py:99-106 -- as one autograd node (see the module docstring).
    ``T`` is the ``_TFembed`` weight registered as the graph's tfidfembed table."""
    w2s, s2w = _Layer(word2sent), _Layer(sent2word)
    params = w2s.params() + s2w.params() + [T]
    return _GatStack.apply((G, w2s, s2w, T, int(n_iter)), w, s, *params)
