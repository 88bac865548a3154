"""Dropout randomness for the HIP kernels.

Masks are a stateless hash of (seed, offset, element) (csrc/hsg_rng.h).  ``seed``
lives in device memory so a captured HIP graph sees a new one after every
``advance()``; ``offset`` is a host-side counter, one value per dropout call, so
calls within a step draw independent masks.  Forward and backward of a call share
(seed, offset) and therefore the mask.
"""
from __future__ import annotations

import torch

_STATE = {}


class DropoutRNG:
    def __init__(self, device, seed=None):
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.seed = torch.tensor([seed], dtype=torch.int64, device=device)
        self.offset = 0

    def take(self):
        """(seed tensor, offset) for one dropout call."""
        self.offset = (self.offset + 1) & 0xFFFFFFFF
        return self.seed, self.offset

    def advance(self):
        """New masks for the next step (device-side add: graph-capturable)."""
        self.seed.add_(1)


def get(device) -> DropoutRNG:
    device = torch.device(device)
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    if key not in _STATE:
        _STATE[key] = DropoutRNG(device)
    return _STATE[key]


def manual_seed(seed, device=None):
    """Reseed the dropout stream of ``device`` (default: current device)."""
    device = device or torch.device("cuda", torch.cuda.current_device())
    r = get(device)
    r.seed.fill_(int(seed))
    r.offset = 0


def advance_all():
    for r in _STATE.values():
        r.advance()
