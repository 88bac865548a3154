"""DGL-0.4-compatible batched document graph (the hot path's input surface).

The reference drives WSWGAT through a DGL 0.4 ``DGLGraph`` (third-party, not
vendored).  This module provides the subset of that API the
reference's call sites use with DGL 0.4 semantics:

* construction: ``add_nodes``, ``add_edges`` (scalar / list / broadcast forms),
  ``add_edge`` -- dataloader.py:214-263, 354-400;
* frames with a zero initializer, ``ndata``/``edata`` (incl. in-place slice
  writes), ``nodes[ids].data`` / ``edges[ids].data`` get/set, ``ndata.pop``;
* ``filter_nodes`` / ``filter_edges`` / ``predecessors`` -- GATLayer.py:105-107,
  HiGraph.py:146-147, 237;
* generic UDF message passing ``apply_edges`` / ``pull`` with degree bucketing
  (for foreign UDF callers; the WSWGAT hot path never uses it);
* ``batch`` / ``unbatch`` / ``sum_nodes`` -- dataloader.py:480, HiGraph.py:248,
  train.py:118; in-place ``to(device)`` -- train.py:112.

What DGL does not have and the hot path needs: a cached, device-resident
*relation* (typed-edge CSR by destination + CSC by source + per-destination
phantom in-edge counts) per layer type, built once per batch
(:mod:`hetersumgraph_amd.relation`).  Graphs stay pickleable so they can be
built in DataLoader workers (train.py:354).
"""
from __future__ import annotations

import numpy as np
import torch

ALL = slice(None)


def zero_initializer(shape, dtype, ctx, id_range=None):
    """``dgl.init.zero_initializer`` (dataloader.py:215, 245)."""
    return torch.zeros(shape, dtype=dtype, device=ctx)


class TableColumn:
    """An edge column defined as ``weight[index]`` with rows ``index < 0`` equal to
    the frame initializer (zeros).  ``HSumGraph.set_wnfeature`` writes
    ``tfidfembed = _TFembed(tffrac)`` on dtype-0 edges (HiGraph.py:150-151); storing
    the table instead of the gathered [E, 50] tensor lets WSWGAT collapse the
    per-edge ``feat_fc`` projection into a 10-row table.  Reading the column
    materialises it (autograd flows to ``weight`` either way)."""

    def __init__(self, weight: torch.Tensor, index: torch.Tensor, tag: str = ""):
        self.weight = weight
        self.index = index          # int64 [E], -1 => initializer row
        self.tag = tag

    @property
    def shape(self):
        return (self.index.shape[0],) + tuple(self.weight.shape[1:])

    def materialize(self) -> torch.Tensor:
        idx = self.index.to(self.weight.device)
        rows = self.weight[idx.clamp_min(0)]
        mask = (idx >= 0).to(rows.dtype).view(-1, *([1] * (rows.dim() - 1)))
        return rows * mask

    def to(self, device):
        return TableColumn(self.weight, self.index.to(device), self.tag)


class EdgeScoreColumn(TableColumn):
    """``g.edata['e']`` as the reference's WSWGAT leaves it, materialised on read.

    Every head of the reference writes its attention logits
    ``e = leaky_relu(attn_fc([z_src, z_dst, feat_fc(tfidfembed)]))`` into ``g.edata['e']``
    on its typed edges (GATLayer.py:89-93 via ``apply_edges`` at :112 / :148), and the
    column stays on the graph (GATLayer.py:111-115 pops only ``z`` and ``sh``).  Heads
    run in order (GATStackLayer.py:56-58) and ``apply_edges`` writes only its rows, so
    after a forward each typed edge holds the LAST head's logit of the LAST application
    over its relation; the other rows keep what they held (zeros from the initializer).
    The HIP path never forms per-edge logits, so the column keeps one ``segment`` per
    relation (an object with ``eid`` [E_T] and ``scores()`` [E_T], see
    ``module.GATLayer.LastHeadScores``) over an optional ``base`` tensor and computes the
    rows only when someone reads the column.  Values are detached (the reference's
    column carries autograd history, which no reference caller differentiates)."""

    def __init__(self, n: int, segments, base=None):
        self.n = n
        self.segments = list(segments)
        self.base = base
        self.tag = "e"

    @property
    def shape(self):
        return (self.n, 1)

    def materialize(self) -> torch.Tensor:
        dev = self.segments[0].eid.device if self.segments else (self.base.device if self.base is not None else None)
        out = self.base.detach().clone() if self.base is not None else torch.zeros(self.n, 1, device=dev)
        for seg in self.segments:
            v = seg.scores().to(out.dtype).reshape(-1, *out.shape[1:])
            out = out.index_copy(0, seg.eid.to(out.device), v.to(out.device))
        return out

    def to(self, device):
        return EdgeScoreColumn(self.n, [s.to(device) for s in self.segments],
                               self.base.to(device) if self.base is not None else None)


def record_edge_scores(g, segment):
    """Set ``g.edata['e']`` to ``segment``'s rows over whatever the column held (a later
    segment of the same relation replaces the earlier one: its rows are the same)."""
    f = g._eframe()
    cur = f.cols.get("e")
    if isinstance(cur, EdgeScoreColumn):
        segs = [s for s in cur.segments if s.key != segment.key] + [segment]
        f.cols["e"] = EdgeScoreColumn(f.n, segs, cur.base)
    else:
        f.cols["e"] = EdgeScoreColumn(f.n, [segment], cur.materialize() if isinstance(cur, TableColumn) else cur)


def _as_index(ids, n, device):
    """Normalise a DGL id argument to an int64 tensor on ``device`` (or ALL)."""
    if isinstance(ids, slice):
        if ids == ALL:
            return ALL
        return torch.arange(n, device=device)[ids]
    if isinstance(ids, torch.Tensor):
        t = ids.reshape(-1)
        if t.dtype == torch.bool:
            t = t.nonzero().view(-1)
        return t.to(device=device, dtype=torch.int64)
    if isinstance(ids, (int, np.integer)):
        return torch.tensor([int(ids)], dtype=torch.int64, device=device)
    if isinstance(ids, np.ndarray):
        return torch.from_numpy(ids.astype(np.int64).reshape(-1)).to(device)
    # list / tuple, possibly of 0-d tensors (HiGraph.py:238)
    return torch.tensor([int(x) for x in ids], dtype=torch.int64, device=device)


class Frame:
    """Column store with DGL-0.4 zero-initialiser semantics."""

    def __init__(self, n: int, device=torch.device("cpu")):
        self.n = n
        self.cols: dict = {}
        self.initializer = zero_initializer
        self.device = torch.device(device)

    # full-column access ------------------------------------------------------
    def get(self, key):
        c = self.cols[key]
        if isinstance(c, TableColumn):
            return c.materialize()
        return c

    def set(self, key, val):
        if isinstance(val, TableColumn):
            assert val.shape[0] == self.n
            self.cols[key] = val
            return
        if not isinstance(val, torch.Tensor):
            val = torch.as_tensor(val)
        if val.shape[0] != self.n:
            raise ValueError(f"column '{key}' has {val.shape[0]} rows, frame has {self.n}")
        self.cols[key] = val

    def pop(self, key):
        v = self.get(key)
        del self.cols[key]
        return v

    # row-subset access -------------------------------------------------------
    def get_rows(self, key, idx):
        c = self.get(key)
        return c if idx is ALL else c[idx]

    def set_rows(self, key, idx, val):
        if idx is ALL:
            self.set(key, val)
            return
        if not isinstance(val, torch.Tensor):
            val = torch.as_tensor(val)
        if val.dim() == 0 or val.shape[0] != idx.shape[0]:
            val = val.expand((idx.shape[0],) + tuple(val.shape[1:] if val.dim() else ()))
        if key not in self.cols:
            base = self.initializer((self.n,) + tuple(val.shape[1:]), val.dtype, val.device)
        else:
            base = self.get(key)
            if val.dtype != base.dtype:
                val = val.to(base.dtype)
        idx = idx.to(base.device)
        # out-of-place scatter keeps autograd history (DGL 0.4 scatter_row)
        self.cols[key] = base.index_copy(0, idx, val.to(base.device))

    def extend(self, m: int):
        """Append ``m`` initializer rows to every column (add_nodes/add_edges)."""
        for k, c in list(self.cols.items()):
            if isinstance(c, TableColumn):
                c = c.materialize()
            pad = self.initializer((m,) + tuple(c.shape[1:]), c.dtype, c.device)
            self.cols[k] = torch.cat([c, pad], 0)
        self.n += m

    def to(self, device):
        device = torch.device(device)
        for k, c in self.cols.items():
            self.cols[k] = c.to(device)
        self.device = device

    def keys(self):
        return self.cols.keys()


class _DataView:
    """``g.ndata`` / ``g.edata`` / ``g.nodes[ids].data`` mapping."""

    def __init__(self, graph, is_node, idx=ALL):
        self._g, self._node, self._idx = graph, is_node, idx

    def _frame(self):
        return self._g._nframe if self._node else self._g._eframe()

    def __getitem__(self, key):
        return self._frame().get_rows(key, self._idx)

    def __setitem__(self, key, val):
        f = self._frame()
        f.set_rows(key, self._idx, val)
        self._g._touch_column(key, self._node)

    def __contains__(self, key):
        return key in self._frame().cols

    def __delitem__(self, key):
        del self._frame().cols[key]

    def pop(self, key):
        assert self._idx is ALL, "pop only on full frames"
        return self._frame().pop(key)

    def keys(self):
        return self._frame().keys()

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def __len__(self):
        return len(self._frame().cols)

    def __repr__(self):
        return f"<{'n' if self._node else 'e'}data {list(self.keys())}>"


class _Space:
    def __init__(self, graph, is_node, idx):
        self.data = _DataView(graph, is_node, idx)


class _View:
    def __init__(self, graph, is_node):
        self._g, self._node = graph, is_node

    def __getitem__(self, ids):
        n = self._g.number_of_nodes() if self._node else self._g.number_of_edges()
        return _Space(self._g, self._node, _as_index(ids, n, self._g.device))

    def __call__(self, *args, **kwargs):
        if self._node:
            return torch.arange(self._g.number_of_nodes(), device=self._g.device)
        return self._g.all_edges(*args, **kwargs)

    def __len__(self):
        return self._g.number_of_nodes() if self._node else self._g.number_of_edges()


class NodeBatch:
    """Argument of node UDFs / filter predicates (``nodes.data``, ``nodes.mailbox``)."""

    def __init__(self, graph, idx, data=None, mailbox=None):
        self._g, self._idx = graph, idx
        self._data = data
        self.mailbox = mailbox or {}

    @property
    def data(self):
        if self._data is None:
            f = self._g._nframe
            self._data = {k: f.get_rows(k, self._idx) for k in f.keys()}
        return self._data

    def nodes(self):
        return self._idx


class EdgeBatch:
    """Argument of edge UDFs / filter predicates (``edges.src/dst/data``)."""

    def __init__(self, graph, eids):
        self._g, self._eids = graph, eids
        self._src_ids = graph._src_t()[eids] if eids is not ALL else graph._src_t()
        self._dst_ids = graph._dst_t()[eids] if eids is not ALL else graph._dst_t()

    @property
    def src(self):
        f = self._g._nframe
        return {k: f.get(k)[self._src_ids] for k in f.keys()}

    @property
    def dst(self):
        f = self._g._nframe
        return {k: f.get(k)[self._dst_ids] for k in f.keys()}

    @property
    def data(self):
        f = self._g._eframe()
        return {k: f.get_rows(k, self._eids) for k in f.keys()}


class DGLGraph:
    """Directed multigraph with node/edge frames (DGL 0.4 ``DGLGraph`` surface)."""

    def __init__(self):
        self._n = 0
        self._src = np.zeros(0, np.int64)
        self._dst = np.zeros(0, np.int64)
        self._pending = []                # [(u, v, data)] appended by add_edges
        self._nframe = Frame(0)
        self._ef = Frame(0)
        self._n_init = zero_initializer
        self._e_init = zero_initializer
        self.device = torch.device("cpu")
        self._dev_src = None              # device copies of src/dst
        self._dev_dst = None
        self._rel_cache = {}
        self._host_cols = {}              # CPU snapshots of structural columns
        self._version = 0

    # ------------------------------------------------------------------ build
    def add_nodes(self, num, data=None):
        self._nframe.extend(int(num))
        self._n += int(num)
        if data:
            idx = torch.arange(self._n - num, self._n)
            for k, v in data.items():
                self._nframe.set_rows(k, idx, v)
        self._mutated()

    def add_edges(self, u, v, data=None):
        u = np.asarray(u.cpu() if isinstance(u, torch.Tensor) else u, dtype=np.int64).reshape(-1)
        v = np.asarray(v.cpu() if isinstance(v, torch.Tensor) else v, dtype=np.int64).reshape(-1)
        if len(u) == 1 and len(v) > 1:
            u = np.repeat(u, len(v))
        elif len(v) == 1 and len(u) > 1:
            v = np.repeat(v, len(u))
        if len(u) != len(v):
            raise ValueError("add_edges: u and v have incompatible lengths")
        if len(u) and (u.max() >= self._n or v.max() >= self._n or u.min() < 0 or v.min() < 0):
            raise ValueError("add_edges: node id out of range")
        self._pending.append((u, v, dict(data) if data else {}))
        self._mutated()

    def add_edge(self, u, v, data=None):
        self.add_edges([int(u)], [int(v)], data)

    def _flush(self):
        if not self._pending:
            return
        pend, self._pending = self._pending, []
        us = [p[0] for p in pend]
        vs = [p[1] for p in pend]
        counts = [len(x) for x in us]
        m = int(sum(counts))
        old_n = self._ef.n
        keys = set(self._ef.keys())
        proto = {}
        for _, _, d in pend:
            for k, t in d.items():
                t = torch.as_tensor(t)
                keys.add(k)
                proto.setdefault(k, t)
        new_cols = {}
        for k in keys:
            if k in self._ef.cols:
                ref = self._ef.get(k)
            else:
                p = proto[k]
                ref = self._e_init((old_n,) + tuple(p.shape[1:]), p.dtype, self.device)
            pieces = [ref]
            for (u, _, d), cnt in zip(pend, counts):
                if k in d:
                    t = torch.as_tensor(d[k]).to(device=ref.device)
                    if t.dim() == 0 or t.shape[0] != cnt:
                        t = t.reshape(1, *t.shape[1:] if t.dim() else ()).expand(cnt, *ref.shape[1:])
                    pieces.append(t.to(ref.dtype))
                else:
                    pieces.append(self._e_init((cnt,) + tuple(ref.shape[1:]), ref.dtype, ref.device))
            new_cols[k] = torch.cat(pieces, 0)
        self._src = np.concatenate([self._src] + us)
        self._dst = np.concatenate([self._dst] + vs)
        self._ef.n = old_n + m
        self._ef.cols = new_cols
        self._dev_src = self._dev_dst = None

    def _eframe(self):
        self._flush()
        return self._ef

    def _mutated(self):
        self._version += 1
        self._rel_cache.clear()
        self._host_cols.clear()
        self._dev_src = self._dev_dst = None

    def _touch_column(self, key, is_node):
        if key in ("unit", "dtype", "tffrac"):
            self._rel_cache.clear()
            self._host_cols.clear()

    def set_n_initializer(self, initializer, field=None):
        self._n_init = initializer
        self._nframe.initializer = initializer

    def set_e_initializer(self, initializer, field=None):
        self._e_init = initializer
        self._ef.initializer = initializer

    # ------------------------------------------------------------------ query
    def number_of_nodes(self):
        return self._n

    def number_of_edges(self):
        return len(self._src) + sum(len(p[0]) for p in self._pending)

    num_nodes = number_of_nodes
    num_edges = number_of_edges

    def __len__(self):
        return self._n

    def _src_t(self):
        self._flush()
        if self._dev_src is None:
            self._dev_src = torch.from_numpy(self._src).to(self.device)
            self._dev_dst = torch.from_numpy(self._dst).to(self.device)
        return self._dev_src

    def _dst_t(self):
        self._src_t()
        return self._dev_dst

    def all_edges(self, form="uv", order=None):
        self._flush()
        if form == "eid":
            return torch.arange(self.number_of_edges(), device=self.device)
        if form == "all":
            return self._src_t(), self._dst_t(), torch.arange(self.number_of_edges(), device=self.device)
        return self._src_t(), self._dst_t()

    def find_edges(self, eid):
        idx = _as_index(eid, self.number_of_edges(), self.device)
        return self._src_t()[idx], self._dst_t()[idx]

    def in_degrees(self, v=ALL):
        self._flush()
        deg = torch.from_numpy(np.bincount(self._dst, minlength=self._n)).to(self.device)
        return deg if v is ALL else deg[_as_index(v, self._n, self.device)]

    def out_degrees(self, v=ALL):
        self._flush()
        deg = torch.from_numpy(np.bincount(self._src, minlength=self._n)).to(self.device)
        return deg if v is ALL else deg[_as_index(v, self._n, self.device)]

    def predecessors(self, v):
        """Sources of ``v``'s in-edges in edge-id order (HiGraph.py:237)."""
        self._flush()
        v = int(v)
        return torch.from_numpy(self._src[self._dst == v].copy()).to(self.device)

    def successors(self, v):
        self._flush()
        v = int(v)
        return torch.from_numpy(self._dst[self._src == v].copy()).to(self.device)

    def in_edges(self, v, form="uv"):
        self._flush()
        idx = _as_index(v, self._n, torch.device("cpu")).numpy()
        eids = np.nonzero(np.isin(self._dst, idx))[0]
        e = torch.from_numpy(eids).to(self.device)
        if form == "eid":
            return e
        return self._src_t()[e], self._dst_t()[e]

    @property
    def ndata(self):
        return _DataView(self, True)

    @property
    def edata(self):
        return _DataView(self, False)

    @property
    def nodes(self):
        return _View(self, True)

    @property
    def edges(self):
        """Callable (``g.edges()`` -> (u, v)) and indexable (``g.edges[ids].data``)."""
        return _View(self, False)

    def filter_nodes(self, predicate, nodes=ALL):
        idx = _as_index(nodes, self._n, self.device)
        mask = predicate(NodeBatch(self, idx)).reshape(-1)
        base = torch.arange(self._n, device=self.device) if idx is ALL else idx
        return base[mask.to(base.device).bool()]

    def filter_edges(self, predicate, edges=ALL):
        self._flush()
        idx = _as_index(edges, self.number_of_edges(), self.device)
        mask = predicate(EdgeBatch(self, idx)).reshape(-1)
        base = torch.arange(self.number_of_edges(), device=self.device) if idx is ALL else idx
        return base[mask.to(base.device).bool()]

    # --------------------------------------------------- generic UDF execution
    def apply_edges(self, func, edges=ALL):
        """Edge UDF over a subset (GATLayer.py:74/112/148 call shape)."""
        self._flush()
        idx = _as_index(edges, self.number_of_edges(), self.device)
        out = func(EdgeBatch(self, idx))
        for k, val in out.items():
            self._ef.set_rows(k, idx, val)

    def pull(self, v, message_func, reduce_func):
        """DGL 0.4 ``pull``: messages on ALL in-edges of ``v``, degree-bucketed
        mailbox, reduce; nodes without in-edges keep the initializer value.  This is
        the generic (slow) path for foreign UDFs -- WSWGAT does not use it."""
        self._flush()
        vidx = _as_index(v, self._n, torch.device("cpu"))
        if vidx is ALL:
            vidx = torch.arange(self._n)
        vnp = vidx.numpy()
        sel = np.nonzero(np.isin(self._dst, vnp))[0]
        if len(sel) == 0:
            return
        order = np.argsort(self._dst[sel], kind="stable")
        eids = sel[order]
        dsts = self._dst[eids]
        uniq, starts, counts = np.unique(dsts, return_index=True, return_counts=True)
        e_t = torch.from_numpy(eids).to(self.device)
        msgs = message_func(EdgeBatch(self, e_t))
        results = {}
        for deg in np.unique(counts):
            which = np.nonzero(counts == deg)[0]
            rows = (starts[which][:, None] + np.arange(deg)[None, :]).reshape(-1)
            rows_t = torch.from_numpy(rows).to(self.device)
            mb = {k: m[rows_t].reshape(len(which), int(deg), *m.shape[1:]) for k, m in msgs.items()}
            nodes_t = torch.from_numpy(uniq[which]).to(self.device)
            out = reduce_func(NodeBatch(self, nodes_t, mailbox=mb))
            for k, val in out.items():
                results.setdefault(k, []).append((nodes_t, val))
        for k, parts in results.items():
            ids = torch.cat([p[0] for p in parts])
            vals = torch.cat([p[1] for p in parts])
            self._nframe.set_rows(k, ids, vals)

    # ------------------------------------------------------------- placement
    def to(self, device, **kwargs):
        """In-place move (DGL 0.4 semantics relied on by train.py:111-112).  The
        structural host snapshot and the hot-path relations are prepared first, so
        the relation arrays ride along with the frames."""
        device = torch.device(device)
        self._flush()
        self._snapshot_host()
        self._nframe.to(device)
        self._ef.to(device)
        self.device = device
        self._dev_src = self._dev_dst = None
        if device.type != "cpu":
            from .relation import prefetch_relations
            prefetch_relations(self, device)
        return self

    def _snapshot_host(self):
        for key, frame in (("unit", self._nframe), ("ndtype", self._nframe),
                           ("tffrac", self._ef), ("edtype", self._ef)):
            col = {"ndtype": "dtype", "edtype": "dtype"}.get(key, key)
            if key not in self._host_cols and col in frame.cols:
                c = frame.cols[col]
                if isinstance(c, TableColumn):
                    continue
                self._host_cols[key] = c.detach().cpu().numpy()

    def host_column(self, key):
        """CPU numpy copy of a structural column: 'unit', 'ndtype', 'tffrac',
        'edtype'.  Cached; a device->host copy happens only if the graph was never
        seen on the host."""
        self._flush()
        if key not in self._host_cols:
            self._snapshot_host()
        return self._host_cols.get(key)

    def relation(self, kind):
        from .relation import get_relation
        return get_relation(self, kind)

    # -------------------------------------------------------------- pickling
    def __getstate__(self):
        self._flush()
        st = dict(self.__dict__)
        st["_dev_src"] = st["_dev_dst"] = None
        st["_rel_cache"] = {}
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)

    def __repr__(self):
        return (f"DGLGraph(num_nodes={self.number_of_nodes()}, num_edges={self.number_of_edges()},"
                f" ndata={list(self._nframe.keys())}, edata={list(self._eframe().keys())})")


class BatchedDGLGraph(DGLGraph):
    """Disjoint union of graphs (dgl.batch, dataloader.py:480)."""

    def __init__(self):
        super().__init__()
        self.batch_size = 0
        self.batch_num_nodes = []
        self.batch_num_edges = []


def batch(graphs):
    g = BatchedDGLGraph()
    graphs = list(graphs)
    for x in graphs:
        x._flush()
    ncols = set().union(*[set(x._nframe.keys()) for x in graphs]) if graphs else set()
    ecols = set().union(*[set(x._ef.keys()) for x in graphs]) if graphs else set()
    g._n = sum(x._n for x in graphs)
    offs = np.cumsum([0] + [x._n for x in graphs])
    g._src = np.concatenate([x._src + o for x, o in zip(graphs, offs[:-1])]) if graphs else g._src
    g._dst = np.concatenate([x._dst + o for x, o in zip(graphs, offs[:-1])]) if graphs else g._dst
    dev = graphs[0].device if graphs else torch.device("cpu")
    g.device = dev
    g._nframe = Frame(g._n, dev)
    g._ef = Frame(len(g._src), dev)

    def _cat(frames, cols, counts):
        out = {}
        for k in cols:
            proto = next(f.get(k) for f in frames if k in f.cols)
            parts = []
            for f, c in zip(frames, counts):
                parts.append(f.get(k) if k in f.cols else
                             zero_initializer((c,) + tuple(proto.shape[1:]), proto.dtype, proto.device))
            out[k] = torch.cat(parts, 0)
        return out

    g._nframe.cols = _cat([x._nframe for x in graphs], ncols, [x._n for x in graphs])
    g._ef.cols = _cat([x._ef for x in graphs], ecols, [len(x._src) for x in graphs])
    g.batch_size = len(graphs)
    g.batch_num_nodes = [x._n for x in graphs]
    g.batch_num_edges = [len(x._src) for x in graphs]
    return g


def unbatch(g):
    """Split a batched graph back into its members (HiGraph.py:248, Tester.py:106)."""
    if not isinstance(g, BatchedDGLGraph):
        return [g]
    g._flush()
    out = []
    no = np.cumsum([0] + list(g.batch_num_nodes))
    eo = np.cumsum([0] + list(g.batch_num_edges))
    for i in range(g.batch_size):
        x = DGLGraph()
        x.device = g.device
        x._n = int(g.batch_num_nodes[i])
        x._src = g._src[eo[i]:eo[i + 1]] - no[i]
        x._dst = g._dst[eo[i]:eo[i + 1]] - no[i]
        x._nframe = Frame(x._n, g.device)
        x._ef = Frame(len(x._src), g.device)
        for k in g._nframe.keys():
            x._nframe.cols[k] = g._nframe.get(k)[no[i]:no[i + 1]]
        for k in g._ef.keys():
            x._ef.cols[k] = g._ef.get(k)[eo[i]:eo[i + 1]]
        out.append(x)
    return out


def graph_ids_of_nodes(g):
    """int64 [n] graph index of every node (cached on the device)."""
    key = ("gid", g.device)
    if key not in g._rel_cache:
        counts = g.batch_num_nodes if isinstance(g, BatchedDGLGraph) else [g.number_of_nodes()]
        gid = np.repeat(np.arange(len(counts)), counts)
        g._rel_cache[key] = torch.from_numpy(gid).to(g.device)
    return g._rel_cache[key]


def sum_nodes(g, feat, weight=None):
    """Per-graph sum of a node column -> [batch_size, *] (train.py:118)."""
    x = g.ndata[feat]
    if weight is not None:
        x = x * g.ndata[weight]
    B = g.batch_size if isinstance(g, BatchedDGLGraph) else 1
    out = torch.zeros((B,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    return out.index_add(0, graph_ids_of_nodes(g), x)


def mean_nodes(g, feat):
    s = sum_nodes(g, feat)
    counts = g.batch_num_nodes if isinstance(g, BatchedDGLGraph) else [g.number_of_nodes()]
    c = torch.tensor(counts, dtype=s.dtype, device=s.device).view(-1, *([1] * (s.dim() - 1)))
    return s / c
