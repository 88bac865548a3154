"""ctypes binding of libhsg.so (the C ABI declared in include/hsg.h).

The library is built in-tree (``python -m hetersumgraph_amd.build`` or
``__graft_entry__.build()``).  There is deliberately no fallback: if the shared
object is missing or a call fails, a ``RuntimeError`` is raised.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HSG_LIB_PATH") or os.path.join(_HERE, "libhsg.so")   # override: dev A/B builds

HSG_EINVAL = 1001
HSG_TAU_TABLE = 0
HSG_TAU_PER_EDGE = 1

# every symbol include/hsg.h declares (checked by tests/test_abi.py)
EXPORTS = ("hsg_gat_fwd", "hsg_gat_bwd_dst", "hsg_gat_bwd_blocks", "hsg_gat_bwd_src",
           "hsg_gat_bwd_src_blocks", "hsg_attn_src_logits", "hsg_attn_params_fwd", "hsg_attn_params_fwd_pair", "hsg_attn_params_fwd_pair_seed", "hsg_attn_params_finish_pair", "hsg_attn_params_bwd",
           "hsg_attn_params_bwd_workspace_floats", "hsg_version", "hsg_gemm_f32", "hsg_gemm_f32_mfma", "hsg_gemm_bf16", "hsg_gemm_workspace_floats", "hsg_gemm_auto_splits", "hsg_gemm_row_tiles", "hsg_ffn_colsums",
           "hsg_ln_bwd_blocks", "hsg_ln_fwd", "hsg_ln_bwd",
           "hsg_dropmask_words", "hsg_dropmask_scale", "hsg_dropmask", "hsg_hproj_fwd", "hsg_hproj_dx",
           "hsg_hproj_dw_chunks", "hsg_hproj_dw", "hsg_hproj_bwd", "hsg_rel_build_workspace_bytes", "hsg_rel_build",
           "hsg_cnn_taps", "hsg_cnn_gather", "hsg_cnn_pool", "hsg_cnn_pool_bwd",
           "hsg_ffn_small_supported", "hsg_ffn_small_fwd", "hsg_ffn_small_bwd_blocks", "hsg_ffn_small_bwd",
           "hsg_attn_params_stage", "hsg_attn_params_finish", "hsg_hproj_fwd_logits_supported",
           "hsg_hproj_fwd_logits", "hsg_wsplit_dims", "hsg_wsplit", "hsg_gemm_f32_psw", "hsg_dropmask_multi", "hsg_dropmask_multi_wt", "hsg_step_prologue", "hsg_gemm_f32_slabs", "hsg_slab_reduce",
           "hsg_hproj_wt", "hsg_hproj_fwd_t8_supported", "hsg_hproj_fwd_t8", "hsg_hproj_fwd_mf_supported", "hsg_hproj_fwd_mf", "hsg_kclock_arm",
           "hsg_kclock_pending", "hsg_seed_advance", "hsg_gat_bwd_dst_noh_supported", "hsg_gat_bwd_dst_noh",
           "hsg_gat_bwd_dst_g", "hsg_gemm_f32_psw_elug", "hsg_gemm_bf16_psw",
           "hsg_gemm_bf16_slabs", "hsg_gemm_dw_slabs", "hsg_gemm_dw_tiles", "hsg_gemm_psw_row_tiles", "hsg_gemm_psw_ln",
           "hsg_gat_bwd_src_g_supported", "hsg_gat_bwd_src_g", "hsg_gemm_psw_elug_rho", "hsg_ffn_small_bwd_gate",
           "hsg_gat_bwd_src_g_blocks", "hsg_gemm_bf16_psw_io", "hsg_gemm_bf16_psw_elug_rho_a16", "hsg_gemm_psw_elug_rho_gw", "hsg_ln_bwd_dy16",
           "hsg_gemm_dw_slabs_io", "hsg_ln_fwd_y16", "hsg_gat_bwd_src_g_io", "hsg_rel_work", "hsg_gat_fwd_ws_floats",
           "hsg_gat_fwd_ws", "hsg_gat_bwd_src_g_ws_floats", "hsg_gat_bwd_src_g_ws", "hsg_gat_fwd_ws16",
           "hsg_gemm_bf16_psw_elug_rho_x16", "hsg_ln_fwd_x16", "hsg_ln_bwd_x16")

HSG_EPI_STORE = 0
HSG_EPI_RELU_BWD = 1
HSG_EPI_ADD = 2
HSG_EPI_ADD_ELUG = 3
HSG_IO_A_BF16 = 1
HSG_IO_C_BF16 = 2
HSG_IO_AUX_BF16 = 4


class HsgRel(ctypes.Structure):
    """Mirror of ``struct hsg_rel`` (include/hsg.h)."""

    _fields_ = [("n_src", ctypes.c_int32), ("n_dst", ctypes.c_int32), ("n_edges", ctypes.c_int32),
                ("indptr", ctypes.c_void_p), ("src", ctypes.c_void_p), ("tf", ctypes.c_void_p),
                ("phantom", ctypes.c_void_p), ("cindptr", ctypes.c_void_p),
                ("cdst", ctypes.c_void_p), ("cperm", ctypes.c_void_p),
                ("n_dwork", ctypes.c_int32), ("n_swork", ctypes.c_int32),
                ("dwork", ctypes.c_void_p), ("swork", ctypes.c_void_p)]


_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_RELP = ctypes.POINTER(HsgRel)

_SIGS = {
    "hsg_gat_fwd": [_RELP, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gat_bwd_dst": [_RELP, _I, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gat_bwd_blocks": [_RELP],
    "hsg_gat_bwd_src": [_RELP, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gat_bwd_src_blocks": [_RELP],
    "hsg_attn_params_fwd": [_I, _I, _I, _P, _P, _P, _P, _P, _P, _P],
    "hsg_attn_params_fwd_pair": [_I, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P],
    "hsg_attn_params_fwd_pair_seed": [_I, _I, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P],
    "hsg_attn_params_finish_pair": [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I,
                                    _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P],
    "hsg_attn_params_bwd": [_I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P],
    "hsg_attn_params_bwd_workspace_floats": [_I, _I],
    "hsg_attn_params_stage": [_I, _I, _I, _P, _I, _P, _P, _I, _P],
    "hsg_attn_params_finish": [_I, _I, _I] + [_P] * 9 + [_I, _P],
    "hsg_attn_src_logits": [_I, _I, _I, _P, _P, _P, _P],
    "hsg_version": [],
    "hsg_kclock_arm": [_P, _P, _P],
    "hsg_kclock_pending": [],
    "hsg_seed_advance": [_P, _P, _P],
    "hsg_gat_bwd_dst_noh_supported": [_RELP, _I, _I],
    "hsg_gat_bwd_dst_noh": [_RELP, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gemm_f32": [_I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _I, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "hsg_gemm_bf16": [_I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _I, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "hsg_gemm_f32_mfma": [_I, _I, _I, _P, _I, _I, _P, _I, _I, _P, _I, _P, _P, _I, _I, _I, _I, _P, _P, _P],
    "hsg_gemm_row_tiles": [_I, _I, _I, _I],
    "hsg_ffn_colsums": [_I, _I, _P, _P, _I, _I, _P, _P, _P, _P, _I, _P],
    "hsg_gemm_workspace_floats": [_I, _I, _I, _I],
    "hsg_gemm_auto_splits": [_I, _I, _I],
    "hsg_ln_bwd_blocks": [_I],
    "hsg_dropmask_words": [_I, _I, _I],
    "hsg_dropmask_scale": [_F],
    "hsg_dropmask": [_I, _I, _I, _F, _P, ctypes.c_uint32, _P, _P],
    "hsg_hproj_fwd": [_I, _I, _I, _I, _P, _I, _P, _P, _F, _P, _I, _P],
    "hsg_hproj_fwd_logits_supported": [_I, _I],
    "hsg_hproj_fwd_logits": [_I, _I, _I, _I, _P, _I, _P, _P, _F, _P, _I, _P, _P, _P],
    "hsg_hproj_wt": [_I, _I, _I, _P, _P, _P],
    "hsg_hproj_fwd_t8_supported": [_I, _I, _I],
    "hsg_hproj_fwd_t8": [_I, _I, _I, _P, _I, _P, _P, _F, _P, _I, _P, _P, _P],
    "hsg_hproj_fwd_mf_supported": [_I, _I, _I],
    "hsg_hproj_fwd_mf": [_I, _I, _I, _P, _I, _P, _I, _I, _P, _F, _P, _I, _P, _P, _P],
    "hsg_hproj_dx": [_I, _I, _I, _I, _P, _I, _P, _P, _F, _P, _I, _I, _P],
    "hsg_hproj_dw_chunks": [_I, _I, _I, _I],
    "hsg_hproj_bwd": [_I, _I, _I, _I, _P, _I, _P, _P, _I, _P, _F, _P, _I, _I, _P, _P],
    "hsg_hproj_dw": [_I, _I, _I, _I, _P, _I, _P, _I, _P, _F, _P, _P, _I, _P],
    "hsg_rel_build_workspace_bytes": [_I, _I],
    "hsg_rel_build": [_F, _F, _I, _I] + [_P] * 17 + [ctypes.c_size_t, _P],
    "hsg_cnn_taps": [],
    "hsg_cnn_gather": [_I, _I, _I, _P, _P, _P, _P, ctypes.c_long, _P, _P],
    "hsg_cnn_pool": [_I, _I, _P, _P, _I, _P, _P, _P, _P],
    "hsg_cnn_pool_bwd": [_I, _P, _P, _P, _P, _P, _I, _P],
    "hsg_ln_fwd": [_I, _I, _P, _P, _P, _P, _F, _F, _P, ctypes.c_uint32, _P, _P, _P, _P],
    "hsg_ffn_small_supported": [_I, _I],
    "hsg_ffn_small_bwd_blocks": [_I],
    "hsg_ffn_small_bwd": [_I, _I, _I] + [_P] * 9 + [_F, _P, ctypes.c_uint32] + [_P] * 6,
    "hsg_ffn_small_bwd_gate": [_I, _I, _I] + [_P] * 9 + [_F, _P, ctypes.c_uint32] + [_P] * 9,
    "hsg_ffn_small_fwd": [_I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _P, ctypes.c_uint32, _P, _P, _P, _P, _P,
                          _P],
    "hsg_ln_bwd": [_I, _I, _P, _P, _P, _P, _P, _P, _F, _P, ctypes.c_uint32, _P, _P, _P, _P],
    "hsg_wsplit_dims": [_I, _I, _P, _P],
    "hsg_dropmask_multi": [_I, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_dropmask_multi_wt": [_I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _P],
    "hsg_step_prologue": [_I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gemm_f32_slabs": [_I, _I, _I, _P, _I, _I, _P, _I, _I, _I, _P, _P],
    "hsg_gemm_bf16_slabs": [_I, _I, _I, _P, _I, _I, _P, _I, _I, _I, _P, _P],
    "hsg_gemm_dw_slabs": [_I, _P, _P, _I, _P, _P, _P, _P, _I, _I, _P, _P],
    "hsg_gemm_dw_tiles": [_I, _I],
    "hsg_gemm_psw_row_tiles": [_I, _I, _I, _I],
    "hsg_gemm_psw_ln": [_I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _F, _F, _P, ctypes.c_uint32, _P, _P, _P, _I, _P],
    "hsg_slab_reduce": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_wsplit": [_I, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gemm_f32_psw": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _I, _I, _I, _P, _P],
    "hsg_gemm_f32_psw_elug": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P, _I, _I, _P],
    "hsg_gemm_bf16_psw": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _I, _I, _I, _P, _P],
    "hsg_gat_bwd_dst_g": [_RELP, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gat_bwd_src_g_supported": [_RELP, _I, _I],
    "hsg_gat_bwd_src_g_blocks": [_RELP, _I, _I],
    "hsg_gat_bwd_src_g": [_RELP, _I, _I, _F, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gemm_psw_elug_rho": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P, _I, _P, _I, _I, _P],
    "hsg_gemm_bf16_psw_io": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _I, _I, _I, _P, _I, _P],
    "hsg_gemm_bf16_psw_elug_rho_a16": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _P, _P, _I, _P, _I, _I, _P],
    "hsg_gemm_psw_elug_rho_gw": [_I, _I, _I, _I, _I],
    "hsg_ln_bwd_dy16": [_I, _I, _P, _P, _I, _P, _P, _P, _P, _F, _P, ctypes.c_uint32, _P, _I, _P, _P, _P],
    "hsg_ln_fwd_y16": [_I, _I, _P, _P, _P, _P, _F, _F, _P, ctypes.c_uint32, _P, _P, _P, _P],
    "hsg_gat_bwd_src_g_io": [_RELP, _I, _I, _F, _P, _P, _P, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gemm_dw_slabs_io": [_I, _P, _P, _I, _P, _P, _P, _P, _P, _I, _P, _P],
    "hsg_rel_work": [_I, _P, _I, _I, _P, _I, _P, _P],
    "hsg_gat_fwd_ws_floats": [_RELP, _I, _I],
    "hsg_gat_fwd_ws": [_RELP, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "hsg_gat_fwd_ws16": [_RELP, _I, _I, _I, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P],
    "hsg_gemm_bf16_psw_elug_rho_x16": [_I, _I, _I, _P, _I, _P, _P, _I, _P, _P, _I, _I, _P, _P, _I, _P, _I, _I, _P],
    "hsg_ln_fwd_x16": [_I, _I, _P, _P, _I, _P, _P, _F, _F, _P, ctypes.c_uint32, _P, _P, _P, _P],
    "hsg_ln_bwd_x16": [_I, _I, _P, _P, _P, _I, _P, _P, _P, _F, _P, ctypes.c_uint32, _P, _I, _P, _P, _P],
    "hsg_gat_bwd_src_g_ws_floats": [_RELP, _I, _I],
    "hsg_gat_bwd_src_g_ws": [_RELP, _I, _I, _F, _P, _P, _P, _P, _P, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P],
}
_RESTYPE = {"hsg_version": ctypes.c_char_p, "hsg_wsplit_dims": None, "hsg_gemm_workspace_floats": ctypes.c_size_t,
            "hsg_attn_params_bwd_workspace_floats": ctypes.c_size_t,
            "hsg_dropmask_scale": ctypes.c_float,
            "hsg_rel_build_workspace_bytes": ctypes.c_size_t, "hsg_gat_fwd_ws_floats": ctypes.c_size_t,
            "hsg_gat_bwd_src_g_ws_floats": ctypes.c_size_t}


def load():
    """Load libhsg.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"libhsg.so not found at {LIB_PATH}: build it with `python -m hetersumgraph_amd.build` "
            "(hetersumgraph_amd has no CPU fallback for the WSWGAT hot path)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    _lib = lib
    return lib


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    return None if t is None else t.data_ptr()


def stream_of(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def check(rc: int, what: str):
    if rc != 0:
        kind = "unsupported shape" if rc == HSG_EINVAL else f"hipError {rc}"
        raise RuntimeError(f"{what} failed: {kind}")


def version() -> str:
    return load().hsg_version().decode()


_is_dev = None
_OPTIONS = {}


def is_dev() -> bool:
    """True when the loaded library is the dev build (libhsg_dev.so via HSG_LIB_PATH)."""
    global _is_dev
    if _is_dev is None:
        _is_dev = version().endswith(" dev")
    return _is_dev


def path_option(name: str, default: str) -> str:
    """A Python-side path switch (e.g. ``HSG_FUSED_STACK``): an explicit selection made
    with :func:`path_options` first; the environment variable of the same name only
    when the dev library is loaded (the A/B tools); otherwise the measured default.
    The product path therefore never changes algorithm or precision because of the
    environment (the C library's switches follow the same rule, csrc/hsg_dev.h)."""
    if name in _OPTIONS:
        return _OPTIONS[name]
    if is_dev():
        return os.environ.get(name, default)
    return default


class path_options:
    """``with path_options(HSG_FUSED_STACK="0"): ...`` -- explicit, scoped path
    selections for tests and tools (values are strings, as the environment's)."""

    def __init__(self, **kw):
        self.kw = {k: str(v) for k, v in kw.items()}

    def __enter__(self):
        self.prev = dict(_OPTIONS)
        _OPTIONS.update(self.kw)
        return self

    def __exit__(self, *exc):
        _OPTIONS.clear()
        _OPTIONS.update(self.prev)


class KernelClock:
    """In-step kernel timing for bench.py: while a clock is active (``with
    KernelClock() as clk``), tagged edge launches are timed inside an ordinary
    (eager) training step -- so each kernel runs after the step's real predecessors,
    with the caches they leave.  The two HIP events of a launch are recorded by the
    kernels' own dispatch packets (``hsg_kclock_arm`` -> hipExtLaunchKernel: start at
    the entry point's first kernel, stop at its last), not by event packets around
    them.  Off (the default), the hook costs one global read per launch."""

    def __init__(self):
        self.events = {}

    def __enter__(self):
        global CLOCK
        CLOCK = self
        return self

    def __exit__(self, *exc):
        global CLOCK
        CLOCK = None

    def start(self, tag, device):
        st = torch.cuda.current_stream(device)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)                   # creates the events; the kernels re-record them
        e1.record(st)
        load().hsg_kclock_arm(st.cuda_stream, e0.cuda_event, e1.cuda_event)
        return (tag, e0, e1)

    def stop(self, token, device):
        tag, e0, e1 = token
        if load().hsg_kclock_pending():
            load().hsg_kclock_arm(None, None, None)
            raise RuntimeError(f"kernel clock {tag}: the launch path did not record the armed events")
        self.events.setdefault(tag, []).append((e0, e1))

    @staticmethod
    def disarm():
        """Drop this thread's armed events (error path: the entry point raised before
        its launches consumed them, so they must not outlive their Event objects)."""
        load().hsg_kclock_arm(None, None, None)

    def durations_ms(self):
        """tag -> list of per-launch durations (ms); synchronises."""
        torch.cuda.synchronize()
        return {t: [a.elapsed_time(b) for a, b in evs] for t, evs in self.events.items()}


CLOCK = None
