"""Dropout randomness for the HIP kernels.

Masks are a stateless hash of (seed, offset, element) (csrc/hsg_rng.h).  ``seed``
lives in device memory so a captured HIP graph sees a new one after every
``advance()``; ``offset`` is a host-side counter, one value per dropout call, so
calls within a step draw independent masks.  Forward and backward of a call share
(seed, offset) and therefore the mask: ``take()`` hands out a device-side SNAPSHOT
of the seed (one 8-byte copy per seed value, taken at the first call after an
``advance()`` / ``manual_seed()``), so reseeding or advancing between a forward and
its backward (recompute, interleaved forwards) cannot change the backward's mask.
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
        self._snap = None
        self._pending = False

    def take(self):
        """(seed snapshot tensor, offset) for one dropout call."""
        self._flush()
        if self._snap is None:
            self._snap = self.seed.clone()        # device copy: graph-capturable
        self.offset = (self.offset + 1) & 0xFFFFFFFF
        return self._snap, self.offset

    def advance(self):
        """New masks for the next step (device-side: graph-capturable).  On a GPU the
        seed is incremented and the new value written into a fresh snapshot, which the
        following take() calls hand out -- by the first launch that needs it: either
        take() (one hsg_seed_advance launch) or a kernel of the step that performs the
        advance itself after :meth:`claim` (the fused stack's first launch)."""
        if self.seed.is_cuda:
            self._flush()                           # an unclaimed earlier advance still counts
            self._snap = torch.empty_like(self.seed)
            self._pending = True
        else:
            self.seed.add_(1)
            self._snap = None

    def _flush(self):
        if self._pending:
            from ._lib import check, load
            st = torch.cuda.current_stream(self.seed.device).cuda_stream
            check(load().hsg_seed_advance(self.seed.data_ptr(), self._snap.data_ptr(), st), "hsg_seed_advance")
            self._pending = False

    def claim(self):
        """(seed, snap) of a pending advance, handed to a kernel that performs it in its
        own launch -- which must come before anything reads the seed (stream order) --
        or None when no advance is pending.  The advance stays pending until the caller
        reports the launch with :meth:`claimed`: a launch that was refused (HSG_EINVAL,
        an exception before it) leaves it to the next take(), so a step never reuses the
        previous step's masks."""
        if not self._pending:
            return None
        return self.seed, self._snap

    def claimed(self):
        """The kernel handed the pending advance by :meth:`claim` was launched."""
        self._pending = False


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
    r._snap = None
    r._pending = False
    r.offset = 0


def advance_all():
    for r in _STATE.values():
        r.advance()
