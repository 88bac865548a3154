"""CPU ORACLE -- TEST INFRASTRUCTURE ONLY.

numpy restatement of the two dropout-mask generators of the HIP path, so the
train-mode (dropout 0.1) stack -- the configuration bench.py times -- can be
checked against the fp64 oracle fed the SAME keep-masks, computed here on the host
from (seed, offset) alone, independently of the GPU.

Reference semantics the masks stand in for:
  * per-head input dropout  -- /root/reference/module/GATStackLayer.py:56
    (``head(g, self.dropout(h))``: one independent mask per head);
  * FFN output dropout      -- /root/reference/module/GATLayer.py:41
    (``self.dropout(output)`` before the residual add and LayerNorm).
torch's Philox stream cannot be matched draw for draw (that is a property of the
RNG, not of the layer), so parity is stated on the masks the kernels use: these
functions restate csrc/hsg_rng.h (FFN) and csrc/hsg_hproj.hip's k_dropmask
(head projection) bit for bit; tests/test_gpu_dropout_masks.py pins that.

Imported only by tests/ (never by hetersumgraph_amd/).
"""
from __future__ import annotations

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
K_SEED = np.uint64(0x9E3779B97F4A7C15)
K_OFF = np.uint64(0xD1B54A32D192ED03)


def _u64(x):
    return np.asarray(x, dtype=np.uint64)


def mix64(z):
    """splitmix64 finaliser (csrc/hsg_rng.h hsg_mix64), wrapping uint64."""
    z = _u64(z)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _f32(p):
    return float(np.float32(p))        # the kernels receive p as a C float


# ------------------------------------------------------------------ FFN dropout
def ffn_threshold(p):
    """hsg_drop_threshold: floor(p * 2^32) of the float p, saturated."""
    t = _f32(p) * 4294967296.0
    return 0xFFFFFFFF if t >= 4294967295.0 else int(t)


def ffn_scale(p):
    """1 / (1 - p) as the row kernels compute it (fp32)."""
    return float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))


def ffn_keep(seed, offset, n, d, p):
    """bool [n, d]: the FFN dropout keep-mask of one call (hsg_keep32 over the
    row-major element index r * d + c with the call's key hsg_drop_key(seed, offset))
    -- csrc/hsg_rng.h, used by csrc/hsg_rows.hip k_ln_fwd* / k_ln_bwd and
    csrc/hsg_ffn.hip."""
    thr = ffn_threshold(p)
    key = _drop_key(seed, offset)
    idx = np.arange(n * d, dtype=np.uint32)
    with np.errstate(over="ignore"):
        h = _lowbias32((idx * np.uint32(0x85EBCA6B)) ^ key)
    return (h >= np.uint32(thr)).reshape(n, d)


# ------------------------------------------------------- head-projection masks
def _lowbias32(x):
    x = np.asarray(x, dtype=np.uint32)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint32(16))
        x = x * np.uint32(0x7FEB352D)
        x = x ^ (x >> np.uint32(15))
        x = x * np.uint32(0x846CA68B)
        x = x ^ (x >> np.uint32(16))
    return x


def hproj_threshold(p):
    """thr16: floor(p * 65536) of the float p (16-bit uniforms), saturated."""
    t = np.float32(p) * np.float32(65536.0)
    return 65535 if t >= np.float32(65535.0) else int(t)


def hproj_scale(p):
    """drop_scale(p) of csrc/hsg_hproj.hip: 1 / (1 - thr16 / 65536) in fp32."""
    thr = np.float32(hproj_threshold(p))
    return float(np.float32(1.0) / (np.float32(1.0) - thr / np.float32(65536.0)))


def _drop_key(seed, offset):
    with np.errstate(over="ignore"):
        k64 = mix64(_u64(np.int64(seed).astype(np.uint64)) * K_SEED + np.uint64(offset & 0xFFFFFFFF) * K_OFF)
    return np.uint32(int(k64) & 0xFFFFFFFF) ^ np.uint32(int(k64) >> 32)


def hproj_keep(seed, offset, n, d_in, H, p):
    """bool [H, n, d_in]: keep(i, k, c) of one head-projection call -- the bits
    k_dropmask writes.  Per (head pair kp, 32-row word iw, column c): one lowbias32
    hash pair of (key, word index) seeds a xorshift64 stream; 16 steps give the
    16 bit planes (most significant first) of the 32 rows' uniforms of both heads
    (low half: head 2kp, high half: head 2kp+1); keep = uniform >= thr16(p)."""
    NWI = (n + 31) // 32
    thr = hproj_threshold(p)
    key = _drop_key(seed, offset)
    KP = (H + 1) // 2
    kp, iw, c = np.meshgrid(np.arange(KP, dtype=np.uint64), np.arange(NWI, dtype=np.uint64),
                            np.arange(d_in, dtype=np.uint64), indexing="ij")
    with np.errstate(over="ignore"):
        w = (((kp * np.uint64(NWI) + iw) * np.uint64(d_in) + c) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = _lowbias32(key ^ (w * np.uint32(0x9E3779B1)))
        lo = _lowbias32(key + np.uint32(0x7F4A7C15) + w * np.uint32(0x85EBCA6B))
        x = (hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)
        x |= np.uint64(1)
        u0 = np.zeros(x.shape + (32,), dtype=np.uint16)      # per-row 16-bit uniforms
        u1 = np.zeros_like(u0)
        for b in range(15, -1, -1):
            x ^= (x << np.uint64(13)) & _M64
            x ^= x >> np.uint64(7)
            x ^= (x << np.uint64(17)) & _M64
            # bit j of the low / high word is bit b of row j's uniform (head 2kp / 2kp+1)
            bits = np.unpackbits(x[..., None].view(np.uint8), axis=-1, bitorder="little")
            u0 |= bits[..., :32].astype(np.uint16) << np.uint16(b)
            u1 |= bits[..., 32:].astype(np.uint16) << np.uint16(b)
    k0 = u0 >= thr                                            # [KP, NWI, d_in, 32]
    k1 = u1 >= thr
    both = np.stack([k0, k1], 1).reshape(2 * KP, NWI, d_in, 32)[:H]
    return both.transpose(0, 1, 3, 2).reshape(H, NWI * 32, d_in)[:, :n]


def pack_hproj_bits(keep):
    """bool [H, n, d_in] -> the int32 words layout k_dropmask writes,
    [H, NWI, LDC] with bit (i % 32) of word (k, i / 32, c) = keep(i, k, c)."""
    H, n, d_in = keep.shape
    NWI = (n + 31) // 32
    LDC = (d_in + 3) & ~3
    k = np.zeros((H, NWI * 32, LDC), dtype=np.uint64)
    k[:, :n, :d_in] = keep
    k = k.reshape(H, NWI, 32, LDC)
    words = (k << np.arange(32, dtype=np.uint64)[None, None, :, None]).sum(2)
    return words.astype(np.uint32).view(np.int32)
