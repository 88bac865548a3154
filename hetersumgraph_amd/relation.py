"""Typed-edge relations: the device-resident index structure of the hot path.

For a WSGATLayer (``W2S``) or SWGATLayer (``S2W``) application the reference
(module/GATLayer.py:105-115, 143-151) does, per head and per call:

* ``filter_nodes(unit == 0)`` / ``filter_nodes(unit == 1)`` -> source / destination
  sets (rows of the layer's input and output, ascending node id);
* ``filter_edges(src.unit == a & dst.unit == b)`` -> typed edges E_T;
* ``pull(dst, ...)`` -> softmax over **all** in-edges of each destination.  In-edges
  that are not typed (s->s in HSG, s->doc in HDSG) carry ``e = 0`` and ``z = 0``
  (zero initializer), so they only add ``exp(0 - max)`` to the denominator.

A :class:`Relation` precomputes all of that once per batch: CSR of typed edges by
destination rank (source rank + tf-idf box per edge), the per-destination phantom
count ``c_v = indeg(v) - |typed in-edges of v|``, and the CSC transpose used by the
backward scatter to sources.  Index arrays are int32 (n <= 2^31) and the box is
uint8; the layout is documented in DESIGN.md §3.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

# tf-idf box rows: 0..9 = _TFembed rows (HiGraph.py:52); row 10 = "no tfidfembed
# written" (zero-initialised edge column, e.g. a typed edge with dtype != 0).
N_BOX = 10
ZERO_ROW = 10

KINDS = {"W2S": (0.0, 1.0), "S2W": (1.0, 0.0), "S2S": (1.0, 1.0)}
# the relations of the two models' layers (built on every batch by DGLGraph.to);
# S2S (GAT.py:38-39, no model constructs it) is built on first use
HOT_KINDS = ("W2S", "S2W")


class Relation:
    """Host + device arrays of one typed relation (see module docstring)."""

    def __init__(self, kind, n_src, n_dst, src_nodes, dst_nodes, indptr, src, tf, eid,
                 phantom, cindptr, cdst, cperm, n_edges_total):
        self.kind = kind
        self.n_src, self.n_dst = int(n_src), int(n_dst)
        self.n_typed = int(len(src))
        self.n_edges_total = int(n_edges_total)
        self.host = dict(src_nodes=src_nodes, dst_nodes=dst_nodes, indptr=indptr, src=src,
                         tf=tf, eid=eid, phantom=phantom, cindptr=cindptr, cdst=cdst,
                         cperm=cperm)
        self.device = torch.device("cpu")
        self.dev = None
        self._cstruct = None

    @classmethod
    def on_device(cls, kind, n_src, n_dst, dev_arrays, n_edges_total):
        """A relation whose arrays were built on the device (no host copy)."""
        r = cls.__new__(cls)
        r.kind = kind
        r.n_src, r.n_dst = int(n_src), int(n_dst)
        r.n_typed = int(dev_arrays["src"].shape[0])
        r.n_edges_total = int(n_edges_total)
        r.host = None
        r.dev = dev_arrays
        r.device = dev_arrays["indptr"].device
        r._cstruct = None
        return r

    def to(self, device):
        device = torch.device(device)
        if self.host is None:
            if device != self.device:
                raise RuntimeError("device-built relation: rebuild it on the new device")
            return self
        r = Relation.__new__(Relation)
        r.__dict__.update(self.__dict__)
        r.device = device
        r.dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in self.host.items()}
        if device.type == "cuda":
            attach_work_lists(r.dev, self.n_src, self.n_dst, self.n_typed)
        r._cstruct = None
        return r

    def degree_stats(self):
        arr = (lambda k: self.host[k]) if self.host is not None else (lambda k: self.dev[k].cpu().numpy())
        deg = np.diff(arr("indptr"))
        cdeg = np.diff(arr("cindptr"))
        return dict(max_in=int(deg.max(initial=0)), mean_in=float(deg.mean()) if len(deg) else 0.0,
                    max_out=int(cdeg.max(initial=0)), phantom_max=int(arr("phantom").max(initial=0)))

    def cstruct(self):
        """ctypes ``hsg_rel`` (include/hsg.h) pointing at the device arrays."""
        if self._cstruct is None:
            from ._lib import HsgRel
            d = self.dev
            dw, sw = d.get("dwork"), d.get("swork")        # flat: [n][4] items + [n] counters
            self._cstruct = HsgRel(
                self.n_src, self.n_dst, self.n_typed,
                d["indptr"].data_ptr(), d["src"].data_ptr(), d["tf"].data_ptr(),
                d["phantom"].data_ptr(), d["cindptr"].data_ptr(), d["cdst"].data_ptr(),
                d["cperm"].data_ptr(),
                dw.numel() // 5 if dw is not None else 0, sw.numel() // 5 if sw is not None else 0,
                dw.data_ptr() if dw is not None else None, sw.data_ptr() if sw is not None else None)
        return self._cstruct


# Work lists of degree-skewed relations (round 6, hsg_rel_work): a node whose segment is
# longer than P = max(PIECE_MIN, PIECE_MULT * ceil(mean segment)) is walked as near-equal
# pieces, so the HDSG doc supernodes (~250 word edges each, dataloader.py:387-400, next
# to ~20 per sentence) no longer set the edge kernels' critical path.  cfg2 / cfg5 have
# no such node (no list: the kernels walk the nodes as before).  cfg4 step traces
# (profiles/r06/ab_pieces_cfg4/): no lists 1,357-1,365 us, PIECE_MULT 2 (4 pieces of ~63
# edges per doc) 1,311-1,317, PIECE_MULT 1 (8 of ~31) 1,303-1,308.
PIECE_MIN = 32
PIECE_MULT = 1


def _work_list(lib, n, indptr, n_edges, stream):
    """(work: flat int32 [5 * cap] -- items of 4 int32, then the arrival counters -- or
    None) of one CSR / CSC: launched here, its item count read back by the caller
    (``count``)."""
    from . import _lib
    pmin = int(_lib.path_option("HSG_PIECE_MIN", str(PIECE_MIN)))      # dev A/B (0: no lists)
    mult = int(_lib.path_option("HSG_PIECE_MULT", str(PIECE_MULT)))
    if n <= 0 or pmin <= 0:
        return None, None
    cap = n + 2 * n_edges // pmin + 1
    work = torch.empty(5 * cap, dtype=torch.int32, device=indptr.device)     # items (4 int32) + counters
    count = torch.zeros(1, dtype=torch.int32, device=indptr.device)
    _lib.check(lib.hsg_rel_work(n, _lib.ptr(indptr), pmin, mult, _lib.ptr(work), cap, _lib.ptr(count), stream),
               "hsg_rel_work")
    return work, count


def build_relation(kind, src, dst, unit, tffrac=None, edtype=None):
    """Device construction of a :class:`Relation` through ``hsg_rel_build``
    (include/hsg.h; csrc/hsg_relbuild.hip).

    Restates GATLayer.py:105-107 / 143-145 (node and edge filters) and DGL 0.4's
    ``pull`` in-edge set (113 / 149) as index arrays; ``tffrac``/``edtype`` give the
    tf-idf box per edge following HiGraph.py:146-151: rows of ``_TFembed`` for dtype-0
    edges, :data:`ZERO_ROW` for any other typed edge (never written -> zeros).
    All inputs are tensors on one ROCm device; one 5-int readback gives the sizes."""
    from . import _lib

    s_unit, d_unit = KINDS[kind]
    dev = src.device
    if dev.type != "cuda":
        raise RuntimeError("build_relation runs only on a ROCm device (hsg_rel_build); no CPU fallback")
    lib = _lib.load()
    src = src.to(torch.int64).contiguous()
    dst = dst.to(device=dev, dtype=torch.int64).contiguous()
    unit = unit.to(device=dev, dtype=torch.float32).contiguous()
    if tffrac is not None:
        tffrac = tffrac.to(device=dev, dtype=torch.int64).contiguous()
    if edtype is not None:
        edtype = edtype.to(device=dev, dtype=torch.float32).contiguous()
    n, E = int(unit.shape[0]), int(src.shape[0])
    i32 = lambda k: torch.empty(max(k, 1), dtype=torch.int32, device=dev)
    i64 = lambda k: torch.empty(max(k, 1), dtype=torch.int64, device=dev)
    counts = torch.zeros(5, dtype=torch.int32, device=dev)
    indptr, cindptr, phantom = i32(n + 1), i32(n + 1), i32(n)
    esrc, cdst, cperm = i32(E), i32(E), i32(E)
    tf = torch.empty(max(E, 1), dtype=torch.uint8, device=dev)
    eid, src_nodes, dst_nodes = i64(E), i64(n), i64(n)
    wsb = lib.hsg_rel_build_workspace_bytes(n, E)
    if wsb == 0:
        raise RuntimeError("hsg_rel_build_workspace_bytes failed")
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.hsg_rel_build(s_unit, d_unit, n, E, _lib.ptr(src), _lib.ptr(dst), _lib.ptr(unit),
                                     _lib.ptr(tffrac), _lib.ptr(edtype), _lib.ptr(counts), _lib.ptr(indptr),
                                     _lib.ptr(esrc), _lib.ptr(tf), _lib.ptr(eid), _lib.ptr(phantom),
                                     _lib.ptr(cindptr), _lib.ptr(cdst), _lib.ptr(cperm), _lib.ptr(src_nodes),
                                     _lib.ptr(dst_nodes), _lib.ptr(ws), wsb, _lib.stream_of(src)),
                   "hsg_rel_build")
        n_src, n_dst, n_typed, bad_tf, bad_id = counts.tolist()
    if bad_id:
        raise IndexError(f"{bad_id} edges reference a node id outside [0, {n})")
    if bad_tf:
        # nn.Embedding(10, ...) would raise on the same input (HiGraph.py:52, 151)
        raise IndexError("tffrac outside the 10 tf-idf boxes")
    d = dict(src_nodes=src_nodes[:n_src], dst_nodes=dst_nodes[:n_dst], indptr=indptr[:n_dst + 1],
             src=esrc[:n_typed], tf=tf[:n_typed], eid=eid[:n_typed], phantom=phantom[:n_dst],
             cindptr=cindptr[:n_src + 1], cdst=cdst[:n_typed], cperm=cperm[:n_typed])
    attach_work_lists(d, n_src, n_dst, n_typed)
    return Relation.on_device(kind, n_src, n_dst, d, E)


def edge_dst(rel):
    """Destination rank of every typed edge in CSR order ([E_T] int64), built on first
    use and kept with the relation's device arrays (the S2S score shift reads it)."""
    d = rel.dev
    if "edst" not in d:
        ip = d["indptr"].long()
        d["edst"] = torch.repeat_interleave(torch.arange(rel.n_dst, device=ip.device), ip[1:] - ip[:-1],
                                            output_size=rel.n_typed)
    return d["edst"]


def attach_work_lists(d, n_src, n_dst, n_typed):
    """Add the CSR / CSC work lists (``dwork`` / ``swork``) of a relation's device arrays
    ``d`` when some segment is long enough to be split (hsg_rel_work)."""
    from . import _lib
    lib = _lib.load()
    dev = d["indptr"].device
    with torch.cuda.device(dev):
        st = _lib.stream_of(d["indptr"])
        dw, dc = _work_list(lib, n_dst, d["indptr"], n_typed, st)
        sw, sc = _work_list(lib, n_src, d["cindptr"], n_typed, st)
        cs = [c for c in (dc, sc) if c is not None]
        got = iter(torch.cat(cs).tolist() if cs else [])                 # one readback per batch
        cnt = [next(got) if c is not None else 0 for c in (dc, sc)]
    if cnt[0] > 0:
        d["dwork"] = dw[:5 * cnt[0]]
    if cnt[1] > 0:
        d["swork"] = sw[:5 * cnt[1]]


def _structure(g):
    """Device tensors of the structural columns (src, dst, unit, tffrac, edtype)."""
    from .graph import TableColumn

    g._flush()
    nf, ef = g._nframe.cols, g._eframe().cols
    if "unit" not in nf:
        raise KeyError("graph has no 'unit' node column (dataloader.py:216)")
    col = lambda c: None if c is None or isinstance(c, TableColumn) else c
    return g._src_t(), g._dst_t(), nf["unit"], col(ef.get("tffrac")), col(ef.get("dtype"))


def get_relation(g, kind):
    """Relation of ``kind`` on the graph's current device (cached per batch)."""
    key = ("rel", kind, str(g.device))
    if key not in g._rel_cache:
        g._rel_cache[key] = build_relation(kind, *_structure(g))
    return g._rel_cache[key]


def prefetch_relations(g, device):
    """Called by ``DGLGraph.to``: build both relations once per batch, on the device."""
    if "unit" not in g._nframe.cols:
        return
    for kind in HOT_KINDS:
        get_relation(g, kind)
