"""Dense fp32 ops over libhsg.so's MFMA GEMM (hsg_gemm_f32, include/hsg.h).

``gemm(A, B, a_t, b_t)`` computes ``op(A) @ op(B)`` for row-major tensors with
``op(X) = X.T if x_t else X``, plus the fused epilogues the FFN and the head
projection need (bias, ReLU, ReLU-backward mask, accumulate).  Everything is
enqueued on the current stream; no host synchronisation.

Operand precision, chosen process-wide with :func:`set_gemm_dtype` /
:func:`gemm_dtype` (never from the environment):
* 'f32' (default, the parity contract): hsg_gemm_f32 -- fp32 operands and
  fp32-accurate products from three bf16 limbs per operand (six limb products on
  the bf16 matrix cores, fp32 accumulation; include/hsg.h);
* 'f32mfma': hsg_gemm_f32_mfma -- the exact-f32 MFMA instruction (one fmaf rounding
  per product), kept for A/B checks;
* 'bf16' (config 5's reduced-precision mode): fp32 storage with
  bf16-rounded operands and fp32 accumulation (hsg_gemm_bf16).
"""
from __future__ import annotations

import contextlib
import ctypes

import torch

from . import _lib
from ._lib import HSG_EINVAL, HSG_EPI_ADD, HSG_EPI_RELU_BWD, HSG_EPI_STORE, check, load, ptr, stream_of


_GEMM_DTYPE = "f32"             # explicit only (set_gemm_dtype / gemm_dtype / bench --dtype)
_FNS = {"f32": "hsg_gemm_f32", "f32mfma": "hsg_gemm_f32_mfma", "bf16": "hsg_gemm_bf16"}


def set_gemm_dtype(dtype):
    """'f32' (fp32-accurate, 3-limb bf16 split), 'f32mfma' (exact-f32 instruction) or
    'bf16' (bf16 operands, fp32 accumulate) for every GEMM issued through
    :func:`gemm` without an explicit ``dtype`` (the FFN, the sentence CNN).  The
    head projection (train: hsg_hproj_*, eval: :func:`linear`) stays fp32."""
    global _GEMM_DTYPE
    if dtype not in _FNS:
        raise ValueError(f"gemm dtype must be one of {sorted(_FNS)}, not {dtype!r}")
    _GEMM_DTYPE = dtype


def get_gemm_dtype():
    return _GEMM_DTYPE


@contextlib.contextmanager
def gemm_dtype(dtype):
    prev = _GEMM_DTYPE
    set_gemm_dtype(dtype)
    try:
        yield
    finally:
        set_gemm_dtype(prev)


def _ld(t):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("gemm operands must be 2-D row-major with unit column stride")
    return t.stride(0)


def gemm(A, B, a_t=False, b_t=False, out=None, bias=None, relu=False, relu_mask=None, add=None,
         splits=0, workspace=None, colsum_part=None, dtype=None):
    """C = op(A) @ op(B) [+ bias] [relu] | * (relu_mask > 0) | + add.

    A [M,K] (or [K,M] with a_t), B [K,N] (or [N,K] with b_t), fp32 on the GPU.
    ``add`` may be ``out`` itself (accumulate).  ``colsum_part``: a tensor of
    ``row_tiles(M, N, K) * N`` floats that receives per-tile-row column sums of C
    (unsplit GEMMs).  ``dtype``: 'f32' / 'f32mfma' / 'bf16' (default: the process-wide
    setting)."""
    lib = load()
    fn = getattr(lib, _FNS[dtype or _GEMM_DTYPE])
    if not A.is_cuda or A.dtype != torch.float32 or B.dtype != torch.float32:
        raise RuntimeError("hsg gemm: fp32 ROCm tensors only (no CPU fallback)")
    M, K = (A.shape[1], A.shape[0]) if a_t else (A.shape[0], A.shape[1])
    K2, N = (B.shape[1], B.shape[0]) if b_t else (B.shape[0], B.shape[1])
    if K != K2:
        raise ValueError(f"gemm: inner dims {K} != {K2}")
    if out is None:
        out = A.new_empty(M, N)
    epi, aux = HSG_EPI_STORE, None
    if relu_mask is not None:
        epi, aux = HSG_EPI_RELU_BWD, relu_mask
    elif add is not None:
        epi, aux = HSG_EPI_ADD, add
    ws = None
    if splits == 0:
        splits = 1 if colsum_part is not None else auto_splits(M, N, K)
    if splits > 1:
        n = lib.hsg_gemm_workspace_floats(M, N, K, splits)
        ws = workspace if workspace is not None and workspace.numel() >= n else A.new_empty(n)
    check(fn(M, N, K, ptr(A), _ld(A), int(not a_t), ptr(B), _ld(B), int(b_t), ptr(out),
                           _ld(out), ptr(bias), ptr(aux), _ld(aux) if aux is not None else 0, epi,
                           int(relu), int(splits), ptr(ws), ptr(colsum_part), stream_of(A)), fn.__name__)
    return out


class SplitWeight:
    """A weight operand B [N][K] held as its three bf16 limb planes [3][Np][Kp]
    (hsg_wsplit), for gemm_psw: made once per step, reused by every GEMM that
    multiplies by B (the FFN's W1 / W2 in the forward, W1^T / W2^T in the backward)."""
    __slots__ = ("planes", "N", "K", "W", "trans", "mode")

    def __init__(self, planes, N, K, W=None, trans=False, mode="f32"):
        self.planes, self.N, self.K = planes, N, K
        self.W, self.trans = W, trans          # the fp32 weight (fallback path)
        self.mode = mode                       # GEMM mode of the step that split it: 'f32' | 'bf16'


def split_dims(N, K):
    lib = load()
    np_, kp = ctypes.c_int(), ctypes.c_int()
    lib.hsg_wsplit_dims(N, K, ctypes.byref(np_), ctypes.byref(kp))
    return np_.value, kp.value


def split_weights(*specs, launch=True):
    """[(W, trans), ...] (1..4) -> [SplitWeight]: B = W^T if trans else W, split in
    one launch.  ``launch=False``: the planes are allocated but not written; returns
    (weights, job) with ``job`` = (n, W, N, K, ldw, trans, planes) ctypes arrays for a
    caller that runs the split inside another launch (hsg_step_prologue)."""
    lib = load()
    if not 1 <= len(specs) <= 4:
        raise ValueError("split_weights: 1..4 weights per launch")
    out, Ns, Ks, lds, trs, Ws, Ps = [], [], [], [], [], [], []
    for W, trans in specs:
        if not W.is_cuda or W.dtype != torch.float32 or W.dim() != 2 or W.stride(1) != 1:
            raise RuntimeError("split_weights: 2-D row-major fp32 ROCm tensors only")
        N, K = (W.shape[1], W.shape[0]) if trans else (W.shape[0], W.shape[1])
        Np, Kp = split_dims(N, K)
        planes = torch.empty(3 * Np * Kp, dtype=torch.bfloat16, device=W.device)
        out.append(SplitWeight(planes, N, K, W, bool(trans), "bf16" if _GEMM_DTYPE == "bf16" else "f32"))
        Ns.append(N); Ks.append(K); lds.append(W.stride(0)); trs.append(int(trans))
        Ws.append(W.data_ptr()); Ps.append(planes.data_ptr())
    n = len(specs)
    arr_i = ctypes.c_int * n
    arr_p = ctypes.c_void_p * n
    job = (n, arr_p(*Ws), arr_i(*Ns), arr_i(*Ks), arr_i(*lds), arr_i(*trs), arr_p(*Ps))
    if not launch:
        return out, job
    check(lib.hsg_wsplit(*job, stream_of(specs[0][0])), "hsg_wsplit")
    return out


def _io(A, out, aux):
    """HSG_IO_* bits of a bf16-mode GEMM's bf16 operands (hsg_gemm_bf16_psw_io)."""
    bf = torch.bfloat16
    return ((_lib.HSG_IO_A_BF16 if A.dtype == bf else 0) | (_lib.HSG_IO_C_BF16 if out.dtype == bf else 0)
            | (_lib.HSG_IO_AUX_BF16 if aux is not None and aux.dtype == bf else 0))


def gemm_psw(A, Bs, out=None, bias=None, relu=False, relu_mask=None, add=None, colsum_part=None):
    """C = A @ B^T [+ bias] [relu] | * (relu_mask > 0) | + add, with B a SplitWeight
    (hsg_gemm_f32_psw: fp32-accurate as gemm(..., dtype='f32'); a weight split in the
    'bf16' mode runs hsg_gemm_bf16_psw: its plane 0 = RNE(W), one bf16 product, as
    gemm(..., dtype='bf16')).  In the 'bf16' mode A, ``out`` and ``relu_mask`` may be
    bf16 tensors (the FFN's bf16 activations, hsg_gemm_bf16_psw_io): the same products,
    since that mode rounds A to bf16 anyway; a bf16 A carries zeros in its columns K ..
    ceil8(K) - 1 (row pitch a multiple of 8)."""
    lib = load()
    if not A.is_cuda or A.dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError("hsg gemm: fp32 ROCm tensors only (no CPU fallback)")
    M, K = A.shape
    if K != Bs.K:
        raise ValueError(f"gemm_psw: inner dims {K} != {Bs.K}")
    N = Bs.N
    if out is None:
        out = A.new_empty(M, N, dtype=torch.float32)
    epi, aux = HSG_EPI_STORE, None
    if relu_mask is not None:
        epi, aux = HSG_EPI_RELU_BWD, relu_mask
    elif add is not None:
        epi, aux = HSG_EPI_ADD, add
    io = _io(A, out, aux)
    if io:
        if Bs.mode != "bf16":
            raise RuntimeError("gemm_psw: bf16 activations belong to the 'bf16' GEMM mode")
        check(lib.hsg_gemm_bf16_psw_io(M, N, K, ptr(A), _ld(A), ptr(Bs.planes), ptr(out), _ld(out), ptr(bias),
                                       ptr(aux), _ld(aux) if aux is not None else 0, epi, int(relu),
                                       ptr(colsum_part), io, stream_of(A)), "hsg_gemm_bf16_psw_io")
        return out
    if Bs.mode == "bf16":
        rc = lib.hsg_gemm_bf16_psw(M, N, K, ptr(A), _ld(A), ptr(Bs.planes), ptr(out), _ld(out), ptr(bias), ptr(aux),
                                   _ld(aux) if aux is not None else 0, epi, int(relu), ptr(colsum_part), stream_of(A))
        if rc == HSG_EINVAL and Bs.W is not None:           # unaligned / ragged quads: the unsplit weight
            if colsum_part is not None and colsum_part.shape[0] != row_tiles(M, N, K, 1):
                raise RuntimeError("gemm_psw: column partials sized for the split-weight kernel, which "
                                   "declined this call (alignment)")
            return gemm(A, Bs.W, b_t=not Bs.trans, out=out, bias=bias, relu=relu, relu_mask=relu_mask, add=add,
                        splits=1 if colsum_part is not None else 0, colsum_part=colsum_part, dtype="bf16")
        check(rc, "hsg_gemm_bf16_psw")
        return out
    check(lib.hsg_gemm_f32_psw(M, N, K, ptr(A), _ld(A), ptr(Bs.planes), ptr(out), _ld(out), ptr(bias), ptr(aux),
                               _ld(aux) if aux is not None else 0, epi, int(relu), ptr(colsum_part),
                               stream_of(A)), "hsg_gemm_f32_psw")
    return out


def gemm_psw_ln(A, Bs, bias, x, gamma, beta, eps, p_drop, seed_t, offset, y, out, mean, rstd):
    """y = A @ B^T + bias and out = LayerNorm(dropout(y) + x) (mean / rstd per row) in
    ONE launch (hsg_gemm_psw_ln: the wide FFN's second GEMM with the LayerNorm of
    GATLayer.py:40-42 in its epilogue, the dropout stream of hsg_ln_fwd).  Returns
    False (nothing launched) when the shape has no such plan; the caller then runs
    gemm_psw + hsg_ln_fwd."""
    if _lib.path_option("HSG_FFN_LN_EPI", "0") != "1":                 # opt-in (dev library): break-even
        return False
    lib = load()
    M, K = A.shape
    N = Bs.N
    if K != Bs.K or any(t.shape != (M, N) or not t.is_contiguous() for t in (x, y, out)):
        return False
    if any(t.dtype != torch.float32 for t in (A, x, y, out)):      # the kernel reads / writes fp32 rows only
        return False
    rc = lib.hsg_gemm_psw_ln(M, N, K, ptr(A), _ld(A), ptr(Bs.planes), ptr(bias), ptr(y), ptr(x), ptr(gamma),
                             ptr(beta), float(eps), float(p_drop), ptr(seed_t), offset, ptr(out), ptr(mean),
                             ptr(rstd), int(Bs.mode == "bf16"), stream_of(A))
    if rc == HSG_EINVAL:
        return False
    check(rc, "hsg_gemm_psw_ln")
    return True


def elug_rho_groups(Bs, M, head_dim):
    """Groups per row of the rho partials gemm_psw_elug writes for this weight split:
    ceil(N / W), W = hsg_gemm_psw_elug_rho_gw (64, or 112 on the fp32 mode's 112-wide
    tiles)."""
    gw = load().hsg_gemm_psw_elug_rho_gw(M, Bs.N, Bs.K, int(head_dim), int(Bs.mode == "bf16"))
    return (Bs.N + gw - 1) // gw


def gemm_psw_elug(A, Bs, out, x, origin, G, rho=None, head_dim=0):
    """out = out + A @ B^T (the FFN backward's dx += dH W1) and, in the same epilogue,
    G = out * elu'(h) with elu(h) = x - origin (hsg_gemm_f32_psw_elug: the edge
    layer's ELU gate, GAT.py:56-57, moved out of its dst pass).  ``rho`` ([M,
    elug_rho_groups(Bs, M, head_dim), 3]): also the per-column-group partials of G . h
    per head of ``head_dim`` columns (hsg_gemm_psw_elug_rho) for the one-pass edge
    backward.  Returns False
    (nothing launched) when the shape / alignment does not allow the fused epilogue."""
    lib = load()
    M, K = A.shape
    N = Bs.N
    x16 = x.dtype == torch.bfloat16              # the bf16 mode's bf16 x rows (pitch % 8 == 0), round 6
    ts = (out, origin, G) if x16 else (out, x, origin, G)
    if K != Bs.K or any(t.shape != (M, N) or not t.is_contiguous() for t in ts):
        return False
    if x16 and (x.shape != (M, N) or x.stride(1) != 1 or x.stride(0) % 8 or A.dtype != torch.bfloat16
                or G.dtype != torch.bfloat16):
        raise RuntimeError("gemm_psw_elug: bf16 x rows come with the bf16 dH and G rows")
    if rho is not None and (rho.shape != (M, elug_rho_groups(Bs, M, head_dim), 3) or not rho.is_contiguous()):
        return False
    if rho is not None and rho.dtype != torch.float32:
        raise RuntimeError("gemm_psw_elug: rho partials are fp32")
    if G.dtype == torch.bfloat16 and A.dtype != torch.bfloat16:
        raise RuntimeError("gemm_psw_elug: bf16 G rows come with the bf16 mode's bf16 dH")
    if A.dtype == torch.bfloat16:                # the bf16 mode's bf16 dH rows
        if Bs.mode != "bf16":
            raise RuntimeError("gemm_psw_elug: bf16 activations belong to the 'bf16' GEMM mode")
        rc = lib.hsg_gemm_bf16_psw_elug_rho_x16(M, N, K, ptr(A), _ld(A), ptr(Bs.planes), ptr(out), N, ptr(out),
                                                ptr(x), x.stride(0), int(x16), ptr(origin), ptr(G), N, ptr(rho),
                                                int(head_dim), int(G.dtype == torch.bfloat16), stream_of(A))
    else:
        rc = lib.hsg_gemm_psw_elug_rho(M, N, K, ptr(A), _ld(A), ptr(Bs.planes), ptr(out), N, ptr(out), ptr(x),
                                       ptr(origin), ptr(G), N, ptr(rho), int(head_dim), int(Bs.mode == "bf16"),
                                       stream_of(A))
    if rc == HSG_EINVAL:
        return False
    check(rc, "hsg_gemm_psw_elug_rho")
    return True


def gemm_slabs(A, B, a_t=False, b_t=False):
    """The split-K partial products of op(A) @ op(B) (hsg_gemm_f32_slabs in the 'f32'
    mode, hsg_gemm_bf16_slabs in 'bf16'):
    (workspace [splits*M*N], splits), summed later by hsg_slab_reduce -- or None when
    the automatic plan does not split this shape or the GEMM mode is not 'f32'."""
    lib = load()
    if _GEMM_DTYPE not in ("f32", "bf16") or not A.is_cuda or A.dtype != torch.float32 or B.dtype != torch.float32:
        return None
    M, K = (A.shape[1], A.shape[0]) if a_t else (A.shape[0], A.shape[1])
    K2, N = (B.shape[1], B.shape[0]) if b_t else (B.shape[0], B.shape[1])
    if K != K2:
        raise ValueError(f"gemm_slabs: inner dims {K} != {K2}")
    if auto_splits(M, N, K) < 2:
        return None
    # 64 K slices: the slabs are summed in the stack's one deferred reduction anyway,
    # and the smaller slices keep each slice's operand rows L2-resident (cfg2 step
    # -17..-21 us against the 32 of hsg_gemm_f32's own plan; 24 / 48 / 96 / 128 are
    # slower, tools/ab.py)
    splits = int(_lib.path_option("HSG_DW_SPLITS", "64"))          # dev A/B
    minrows = int(_lib.path_option("HSG_DW_MINROWS", "0"))         # dev A/B: rows per K slice
    if minrows > 0:
        splits = min(splits, K // minrows)
    splits = max(2, min(splits, (K + 31) // 32))
    ws = A.new_empty(lib.hsg_gemm_workspace_floats(M, N, K, splits))
    fn = lib.hsg_gemm_bf16_slabs if _GEMM_DTYPE == "bf16" else lib.hsg_gemm_f32_slabs
    check(fn(M, N, K, ptr(A), _ld(A), int(not a_t), ptr(B), _ld(B), int(b_t), splits, ptr(ws), stream_of(A)),
          "hsg_gemm_*_slabs")
    return ws, splits


def dw_slab_workspaces(pairs, splits):
    """The partial slabs hsg_gemm_dw_slabs(_io) writes, one fp32 [splits * M * N] buffer
    per (A [K, M], B [K, N]) pair WHATEVER the operands' dtype: k_dw stores fp32 partial
    products (csrc/hsg_dw.hip, dw_tile's epilogue).  Round 5's first bf16-operand run
    allocated them with ``A.new_empty(n)``, which inherits a bf16 A's dtype -- half the
    bytes -- and the kernel's stores ran past the buffer: the hipErrorIllegalAddress of
    test_dw_pair_bf16_operands_bitwise.  Pinned on the CPU by
    tests/test_fault_regressions.py."""
    return [A.new_empty(splits * A.shape[1] * B.shape[1], dtype=torch.float32) for A, B in pairs]


def gemm_dw_slabs(pairs, splits=None):
    """Split-K partial products of A_q^T B_q for up to two (A [K, M], B [K, N]) pairs
    sharing K -- a layer's two FFN weight gradients dW2 = dY^T H and dW1 = dH^T X --
    in ONE launch (hsg_gemm_dw_slabs: 160 x 128 / 128 x 160 tiles, fp32-accurate in
    'f32' mode, one bf16 product in 'bf16').  Returns [(workspace [splits*M*N],
    splits)] per pair, summed later by hsg_slab_reduce, or None when the shapes or the
    GEMM mode are not covered (the caller then uses gemm_slabs per pair).
    ``splits``: K slices (default: two blocks per CU over all pairs' tiles, at least
    4 K tiles per slice)."""
    lib = load()
    if _GEMM_DTYPE not in ("f32", "bf16") or not pairs or len(pairs) > 2:
        return None
    K = pairs[0][0].shape[0]
    okt = (torch.float32, torch.bfloat16) if _GEMM_DTYPE == "bf16" else (torch.float32,)
    for A, B in pairs:
        if (not A.is_cuda or A.dtype not in okt or B.dtype not in okt or A.dim() != 2 or B.dim() != 2
                or A.shape[0] != K or B.shape[0] != K or A.stride(1) != 1 or B.stride(1) != 1
                or A.shape[1] % 4 or B.shape[1] % 4 or _ld(A) % 4 or _ld(B) % 4
                or A.data_ptr() % 16 or B.data_ptr() % 16):
            return None
    kt = (K + 31) // 32
    if splits is None:
        tiles = sum(lib.hsg_gemm_dw_tiles(A.shape[1], B.shape[1]) for A, B in pairs)
        splits = int(_lib.path_option("HSG_DW2_SPLITS", "0")) or max(1, (2 * 256) // max(tiles, 1))   # dev A/B
        splits = max(1, min(splits, kt // 4))
    # every K slice non-empty (the kernel's slice length is ceil(kt / splits) tiles)
    per = (kt + splits - 1) // splits
    splits = (kt + per - 1) // per
    if splits < 2:
        return None
    n = len(pairs)
    arr = lambda t, xs: (t * n)(*xs)
    ws = dw_slab_workspaces(pairs, splits)
    c_i, c_p = ctypes.c_int, ctypes.c_void_p
    io = [int(A.dtype == torch.bfloat16) | (2 * int(B.dtype == torch.bfloat16)) for A, B in pairs]
    dims = (arr(c_i, [A.shape[1] for A, _ in pairs]), arr(c_i, [B.shape[1] for _, B in pairs]), K,
            arr(c_p, [A.data_ptr() for A, _ in pairs]), arr(c_i, [_ld(A) for A, _ in pairs]),
            arr(c_p, [B.data_ptr() for _, B in pairs]), arr(c_i, [_ld(B) for _, B in pairs]))
    if any(io):                              # the bf16 mode's bf16 activations
        rc = lib.hsg_gemm_dw_slabs_io(n, *dims, arr(c_i, io), splits, arr(c_p, [w.data_ptr() for w in ws]),
                                      stream_of(pairs[0][0]))
    else:
        rc = lib.hsg_gemm_dw_slabs(n, *dims, splits, int(_GEMM_DTYPE == "bf16"), arr(c_p, [w.data_ptr() for w in ws]),
                                   stream_of(pairs[0][0]))
    if rc == HSG_EINVAL:
        return None
    check(rc, "hsg_gemm_dw_slabs")
    return [(w, splits) for w in ws]


def auto_splits(M, N, K):
    """hsg_gemm_f32's splits == 0 plan (so the workspace can be sized)."""
    return load().hsg_gemm_auto_splits(M, N, K)


def row_tiles(M, N, K, splits=1):
    """Rows of hsg_gemm_f32's colsum_part slab for this shape."""
    return load().hsg_gemm_row_tiles(M, N, K, splits)


def psw_row_tiles(M, N, K, mode="f32"):
    """Rows of the colsum_part slab of gemm_psw on this shape (hsg_gemm_psw_row_tiles)."""
    return load().hsg_gemm_psw_row_tiles(M, N, K, int(mode == "bf16"))


def splits_for(M, N, K, n_cu=256):
    """Split-K factor for the weight-gradient GEMMs (tiny M x N, K = rows):
    aim at ~2 tiles per CU, at least 4 K-tiles per split."""
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    kt = (K + 31) // 32
    s = max(1, min(kt // 4, (2 * n_cu) // max(tiles, 1)))
    return s


class _Linear(torch.autograd.Function):
    """Z = X W^T on hsg_gemm_f32 with its backward (dX = dZ W, dW = dZ^T X): the
    eval-mode head projection fc (GATLayer.py:110 / 146) without a vendor GEMM.
    Always fp32-accurate ('f32'), whatever the process-wide GEMM mode: the training
    head projection (hsg_hproj_*) is fp32 too, so eval and train project alike."""

    @staticmethod
    def forward(ctx, X, W):
        ctx.save_for_backward(X, W)
        return gemm(X, W, b_t=True, dtype="f32")

    @staticmethod
    def backward(ctx, dZ):
        X, W = ctx.saved_tensors
        dZ = dZ.contiguous()
        dX = gemm(dZ, W, dtype="f32") if ctx.needs_input_grad[0] else None
        dW = gemm(dZ, X, a_t=True, dtype="f32") if ctx.needs_input_grad[1] else None
        return dX, dW


def linear(X, W):
    """X [n, in] @ W[out, in]^T with autograd, fp32 on the device (native GEMM)."""
    if not X.is_cuda or X.dtype != torch.float32:
        raise RuntimeError("hetersumgraph_amd linear runs only on a ROCm device in fp32 (no CPU fallback)")
    return _Linear.apply(X.contiguous(), W.contiguous())
