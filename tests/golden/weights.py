"""Deterministic parameter/input generation shared by the golden-vector script
(run against the reference modules) and the parity tests (run against this
build's modules).  Both module trees have identical state_dict keys and shapes
(SURVEY Appendix B), so the same (seed, key) yields the same tensor on both sides.
"""
import hashlib

import numpy as np
import torch

FROZEN = ("sent_pos_embed", "position_embedding")   # fixed sinusoid tables: keep as built


def _key_seed(seed, key):
    h = hashlib.sha256(f"{seed}:{key}".encode()).digest()
    return int.from_bytes(h[:8], "little")


def param_value(seed, key, shape):
    rng = np.random.default_rng(_key_seed(seed, key))
    leaf = key.rsplit(".", 1)[-1]
    if "layer_norm" in key and leaf == "weight":
        v = 1.0 + 0.1 * rng.standard_normal(shape)
    elif leaf.startswith("bias") or leaf == "bias":
        v = 0.1 * rng.standard_normal(shape)
    elif "embed" in key.lower():
        v = 0.5 * rng.standard_normal(shape)
    else:
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
        v = rng.standard_normal(shape) / np.sqrt(max(fan_in, 1))
    return v.astype(np.float32)


def seed_module(module, seed):
    """Overwrite every non-frozen parameter/buffer of ``module`` in place."""
    seen = set()
    with torch.no_grad():
        for key, t in sorted(module.state_dict(keep_vars=True).items()):
            if any(f in key for f in FROZEN) or not t.is_floating_point():
                continue
            if t.data_ptr() in seen:
                continue
            seen.add(t.data_ptr())
            t.copy_(torch.from_numpy(param_value(seed, key, tuple(t.shape))))
    return module


def feature(seed, name, shape, scale=1.0):
    rng = np.random.default_rng(_key_seed(seed, name))
    return (scale * rng.standard_normal(shape)).astype(np.float32)
