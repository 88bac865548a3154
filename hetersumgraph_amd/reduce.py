"""Deferred, batched column sums of partial slabs (C ABI: hsg_slab_reduce).

The backward of the fused stack produces many small deterministic reductions: the
head-projection dW slabs of every application (hsg_hproj_dw), the FFN bias and
LayerNorm partials (hsg_ffn_small_bwd / hsg_ln_bwd / the dH GEMM's column sums) and
the split-K slabs of the FFN weight gradients.  Summed one launch each they cost a
kernel boundary apiece; a :class:`SlabBatch` collects them -- all applications of
a layer into ONE job per output, their slabs as the job's segments -- and sums
everything in one launch at the end of the backward.
"""
from __future__ import annotations

import ctypes

from ._lib import check, load, stream_of

_MAX_JOBS, _MAX_SEGS = 24, 4


class SlabBatch:
    def __init__(self):
        self.jobs = {}          # key -> [out, cols, pitch, coff, scale, acc, [(part, rows)], out_rows]
        self.order = []

    def add(self, key, out, cols, pitch, coff, scale, acc, part, rows, out_rows=1):
        """Output ``out`` (flat fp32, cols floats; [out_rows][cols] with out_rows > 1,
        row b summing the b-th of out_rows equal row ranges of every segment) +=
        scale * column sums of part[rows][pitch] at column offset coff.  A repeated
        ``key`` adds ``part`` as one more segment of the same job (out / acc of the
        first call stand)."""
        if rows <= 0:
            return
        j = self.jobs.get(key)
        if j is None:
            self.jobs[key] = [out, cols, pitch, coff, float(scale), bool(acc), [(part, rows)], int(out_rows)]
            self.order.append(key)
        else:
            if j[1] != cols or j[2] != pitch or j[3] != coff or j[4] != float(scale) or j[7] != out_rows:
                raise ValueError(f"SlabBatch: inconsistent segment for {key}")
            j[6].append((part, rows))

    def flush(self):
        """One hsg_slab_reduce launch per 24 jobs (4 segments per job; longer
        segment lists are split into chained accumulate jobs)."""
        lib = load()
        flat = []
        for key in self.order:
            out, cols, pitch, coff, scale, acc, segs, orows = self.jobs[key]
            for i in range(0, len(segs), _MAX_SEGS):
                flat.append((out, cols, pitch, coff, scale, acc if i == 0 else True, segs[i:i + _MAX_SEGS], orows))
        # a job that accumulates onto an output written by an earlier job of the same
        # launch would race: such chains go to separate launches
        while flat:
            batch, seen, rest = [], set(), []
            for f in flat:
                oid = f[0].data_ptr()
                if len(batch) < _MAX_JOBS and oid not in seen:
                    batch.append(f)
                    seen.add(oid)
                else:
                    rest.append(f)
            self._launch(lib, batch)
            flat = rest
        self.jobs, self.order = {}, []

    @staticmethod
    def _launch(lib, batch):
        k = len(batch)
        segs = [s for f in batch for s in f[6]]
        P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        check(lib.hsg_slab_reduce(
            k, (P * k)(*[f[0].data_ptr() for f in batch]), (I * k)(*[f[1] for f in batch]),
            (I * k)(*[f[7] for f in batch]), (I * k)(*[f[2] for f in batch]), (I * k)(*[f[3] for f in batch]), (F * k)(*[f[4] for f in batch]),
            (I * k)(*[int(f[5]) for f in batch]), (I * k)(*[len(f[6]) for f in batch]),
            (P * len(segs))(*[s[0].data_ptr() for s in segs]), (I * len(segs))(*[s[1] for s in segs]),
            stream_of(batch[0][0])), "hsg_slab_reduce")
