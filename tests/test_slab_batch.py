"""Host logic of the deferred slab reductions (hetersumgraph_amd/reduce.py), on CPU:
how SlabBatch groups the segments of one output into one job, splits segment lists
longer than the kernel's 4 into chained accumulate jobs, keeps jobs that write the
same output out of one launch (they would race), and caps a launch at 24 jobs.
The launch itself (hsg_slab_reduce) is replaced by a recorder that applies the
same arithmetic in numpy, so the planned launches are also checked numerically."""
import numpy as np
import torch

from hetersumgraph_amd import reduce as red


class _Rec:
    def __init__(self):
        self.launches = []

    def __call__(self, lib, batch):
        self.launches.append(batch)
        for out, cols, pitch, coff, scale, acc, segs, orows in batch:
            o = out.view(orows, cols)
            s = torch.zeros(orows, cols, dtype=torch.float64)
            for part, rows in segs:
                p = part.reshape(-1)[:rows * pitch].view(rows, pitch)[:, coff:coff + cols].double()
                per = (rows + orows - 1) // orows
                for b in range(orows):
                    s[b] += p[b * per:(b + 1) * per].sum(0)
            o.copy_((o.double() if acc else 0) + scale * s)


def _run(batch, monkeypatch):
    rec = _Rec()
    monkeypatch.setattr(red.SlabBatch, "_launch", staticmethod(rec))
    monkeypatch.setattr(red, "load", lambda: None)
    batch.flush()
    return rec.launches


def test_segments_of_one_key_form_one_job(monkeypatch):
    b = red.SlabBatch()
    out = torch.zeros(10)
    g = torch.Generator().manual_seed(3)
    parts = [torch.randn(r, 10, generator=g) for r in (3, 5, 2)]
    for p in parts:
        b.add("k", out, 10, 10, 0, 1.0, False, p, p.shape[0])
    launches = _run(b, monkeypatch)
    assert len(launches) == 1 and len(launches[0]) == 1 and len(launches[0][0][6]) == 3
    np.testing.assert_allclose(out.numpy(), sum(p.sum(0) for p in parts).numpy(), rtol=1e-5, atol=1e-5)


def test_long_segment_lists_chain_into_separate_launches(monkeypatch):
    b = red.SlabBatch()
    out = torch.full((4,), 2.0)
    g = torch.Generator().manual_seed(9)
    parts = [torch.randn(2, 4, generator=g) for _ in range(9)]
    for p in parts:
        b.add("w", out, 4, 4, 0, 0.5, True, p, 2)
    launches = _run(b, monkeypatch)
    # 9 segments -> jobs of 4, 4, 1 on the same output: three launches, the later ones accumulate
    assert [len(l) for l in launches] == [1, 1, 1]
    assert [l[0][5] for l in launches] == [True, True, True]
    # fp32 sums in another order: relative AND absolute slack (an entry may cancel to ~0)
    np.testing.assert_allclose(out.numpy(), (2.0 + 0.5 * sum(p.sum(0) for p in parts)).numpy(), rtol=1e-5, atol=1e-5)


def test_first_call_decides_overwrite(monkeypatch):
    b = red.SlabBatch()
    out = torch.full((3,), 100.0)
    p1, p2 = torch.ones(1, 3), 2 * torch.ones(1, 3)
    b.add("k", out, 3, 3, 0, 1.0, False, p1, 1)
    b.add("k", out, 3, 3, 0, 1.0, True, p2, 1)      # later acc flags are ignored
    _run(b, monkeypatch)
    np.testing.assert_allclose(out.numpy(), [3.0, 3.0, 3.0])


def test_launch_caps_and_offsets(monkeypatch):
    b = red.SlabBatch()
    outs = []
    slab = torch.randn(6, 3 * 5)
    for j in range(30):
        o = torch.zeros(5)
        outs.append(o)
        b.add(("j", j), o, 5, 15, 5 * (j % 3), 1.0, False, slab, 6)
    launches = _run(b, monkeypatch)
    assert [len(l) for l in launches] == [24, 6]
    for j, o in enumerate(outs):
        np.testing.assert_allclose(o.numpy(), slab[:, 5 * (j % 3):5 * (j % 3) + 5].sum(0).numpy(), rtol=1e-5)


def test_staged_rows_and_inconsistent_segments(monkeypatch):
    b = red.SlabBatch()
    out = torch.zeros(4 * 2)
    p = torch.arange(16.0).view(8, 2)
    b.add("s", out, 2, 2, 0, 1.0, False, p, 8, out_rows=4)
    _run(b, monkeypatch)
    np.testing.assert_allclose(out.view(4, 2).numpy(), p.view(4, 2, 2).sum(1).numpy())
    b2 = red.SlabBatch()
    b2.add("s", out, 2, 2, 0, 1.0, False, p, 8)
    try:
        b2.add("s", out, 2, 2, 0, 2.0, False, p, 8)
    except ValueError:
        pass
    else:
        raise AssertionError("a segment with another scale must be refused")
