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

KINDS = {"W2S": (0.0, 1.0), "S2W": (1.0, 0.0)}


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

    def to(self, device):
        device = torch.device(device)
        r = Relation.__new__(Relation)
        r.__dict__.update(self.__dict__)
        r.device = device
        r.dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in self.host.items()}
        r._cstruct = None
        return r

    def degree_stats(self):
        deg = np.diff(self.host["indptr"])
        cdeg = np.diff(self.host["cindptr"])
        return dict(max_in=int(deg.max(initial=0)), mean_in=float(deg.mean()) if len(deg) else 0.0,
                    max_out=int(cdeg.max(initial=0)), phantom_max=int(self.host["phantom"].max(initial=0)))

    def cstruct(self):
        """ctypes ``hsg_rel`` (include/hsg.h) pointing at the device arrays."""
        if self._cstruct is None:
            from ._lib import HsgRel
            d = self.dev
            self._cstruct = HsgRel(
                self.n_src, self.n_dst, self.n_typed,
                d["indptr"].data_ptr(), d["src"].data_ptr(), d["tf"].data_ptr(),
                d["phantom"].data_ptr(), d["cindptr"].data_ptr(), d["cdst"].data_ptr(),
                d["cperm"].data_ptr())
        return self._cstruct


def build_relation(kind, src, dst, unit, tffrac=None, edtype=None):
    """Host construction of a :class:`Relation` from COO edges (numpy).

    Restates GATLayer.py:105-107 / 143-145 (node and edge filters) and DGL 0.4's
    ``pull`` in-edge set (113 / 149) as index arrays.  ``tffrac``/``edtype`` give the
    tf-idf box per edge following HiGraph.py:146-151: rows of ``_TFembed`` for dtype-0
    edges, :data:`ZERO_ROW` for any other typed edge (never written -> zeros)."""
    s_unit, d_unit = KINDS[kind]
    unit = np.asarray(unit)
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    n = len(unit)
    is_src = unit == s_unit
    is_dst = unit == d_unit
    src_nodes = np.nonzero(is_src)[0]
    dst_nodes = np.nonzero(is_dst)[0]
    src_rank = np.full(n, -1, np.int64)
    src_rank[src_nodes] = np.arange(len(src_nodes))
    dst_rank = np.full(n, -1, np.int64)
    dst_rank[dst_nodes] = np.arange(len(dst_nodes))

    typed = is_src[src] & is_dst[dst]
    te = np.nonzero(typed)[0]
    # stable sort by destination keeps DGL's edge-id order inside each mailbox
    order = np.argsort(dst_rank[dst[te]], kind="stable")
    eid = te[order]
    e_dst = dst_rank[dst[eid]]
    e_src = src_rank[src[eid]]
    n_dst = len(dst_nodes)
    n_src = len(src_nodes)
    typed_cnt = np.bincount(e_dst, minlength=n_dst)
    indptr = np.zeros(n_dst + 1, np.int64)
    np.cumsum(typed_cnt, out=indptr[1:])
    indeg_all = np.bincount(dst, minlength=n)
    phantom = indeg_all[dst_nodes] - typed_cnt

    if tffrac is None:
        tf = np.full(len(eid), ZERO_ROW, np.uint8)
    else:
        tffrac = np.asarray(tffrac, np.int64)
        et = np.zeros(len(src)) if edtype is None else np.asarray(edtype)
        box = tffrac[eid]
        has = et[eid] == 0
        if has.any() and (box[has].min() < 0 or box[has].max() >= N_BOX):
            # nn.Embedding(10, ...) would raise on the same input (HiGraph.py:52, 151)
            raise IndexError("tffrac outside the 10 tf-idf boxes")
        tf = np.where(has, box, ZERO_ROW).astype(np.uint8)

    corder = np.argsort(e_src, kind="stable")
    cperm = corder
    cdst = e_dst[corder]
    ccnt = np.bincount(e_src, minlength=n_src)
    cindptr = np.zeros(n_src + 1, np.int64)
    np.cumsum(ccnt, out=cindptr[1:])
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    return Relation(kind, n_src, n_dst, src_nodes, dst_nodes, i32(indptr), i32(e_src), tf,
                    eid.astype(np.int64), i32(phantom), i32(cindptr), i32(cdst), i32(cperm),
                    len(src))


def _host_relation(g, kind):
    key = ("rel_host", kind)
    if key not in g._rel_cache:
        g._flush()
        unit = g.host_column("unit")
        if unit is None:
            raise KeyError("graph has no 'unit' node column (dataloader.py:216)")
        g._rel_cache[key] = build_relation(kind, g._src, g._dst, unit,
                                           g.host_column("tffrac"), g.host_column("edtype"))
    return g._rel_cache[key]


def get_relation(g, kind):
    """Relation of ``kind`` on the graph's current device (cached per batch)."""
    key = ("rel", kind, str(g.device))
    if key not in g._rel_cache:
        g._rel_cache[key] = _host_relation(g, kind).to(g.device)
    return g._rel_cache[key]


def prefetch_relations(g, device):
    """Called by ``DGLGraph.to``: build both relations while the structural columns
    are still on the host, and upload them with the frames."""
    if "unit" not in g._nframe.cols:
        return
    for kind in KINDS:
        get_relation(g, kind)
