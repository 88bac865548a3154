"""Test-only DGL-0.4-semantics graph used to run the *reference's own module code*
in this container (DGL itself is not installed and cannot be fetched).

Independent of the product graph (hetersumgraph_amd/graph.py) on purpose: golden
vectors must not inherit a product bug.  Reproduces exactly what the reference's
hot path and HiGraph rely on:
  1. frame columns auto-created with zeros when a row subset is written;
  2. apply_edges on a subset writes only those rows;
  3. pull(v) reduces over ALL in-edges of v with per-degree mailbox buckets
     [n_bucket, deg, ...], in-edges in edge-id order;
  4. zero in-degree nodes are not reduced (keep the zero initializer);
  5. ndata.pop; 6. batch / unbatch / predecessors.
Used only by tests/golden/make_golden.py, never shipped to the GPU box.
"""
import numpy as np
import torch


def zero_initializer(shape, dtype, ctx, id_range=None):
    return torch.zeros(shape, dtype=dtype, device=ctx)


def _idx(ids, n):
    if isinstance(ids, slice):
        return torch.arange(n)[ids]
    if isinstance(ids, torch.Tensor):
        return ids.reshape(-1).long()
    if isinstance(ids, (int, np.integer)):
        return torch.tensor([int(ids)])
    return torch.tensor([int(x) for x in ids], dtype=torch.long)


class _Store(dict):
    def __init__(self, n_fn):
        super().__init__()
        self._n_fn = n_fn

    def write(self, key, idx, val):
        if key not in self:
            self[key] = torch.zeros((self._n_fn(),) + tuple(val.shape[1:]), dtype=val.dtype)
        self[key] = self[key].index_copy(0, idx, val.to(self[key].dtype))


class _Data:
    def __init__(self, store, idx):
        self.s, self.i = store, idx

    def __getitem__(self, k):
        return self.s[k][self.i]

    def __setitem__(self, k, v):
        v = torch.as_tensor(v)
        if v.dim() == 0 or v.shape[0] != len(self.i):
            v = v.reshape(1, *v.shape[1:] if v.dim() else ()).expand(len(self.i), *v.shape[1:])
        self.s.write(k, self.i, v)


class _Sub:
    def __init__(self, store, idx):
        self.data = _Data(store, idx)


class _View:
    def __init__(self, store, n_fn):
        self.s, self.n = store, n_fn

    def __getitem__(self, ids):
        return _Sub(self.s, _idx(ids, self.n()))


class _NB:
    def __init__(self, data, mailbox=None):
        self.data = data
        self.mailbox = mailbox


class _EB:
    def __init__(self, g, eids):
        self.g, self.e = g, eids

    @property
    def src(self):
        return {k: v[self.g.src[self.e]] for k, v in self.g.ndata.items()}

    @property
    def dst(self):
        return {k: v[self.g.dst[self.e]] for k, v in self.g.ndata.items()}

    @property
    def data(self):
        return {k: v[self.e] for k, v in self.g.edata.items()}


class DGLGraph:
    def __init__(self):
        self.n = 0
        self.src = torch.zeros(0, dtype=torch.long)
        self.dst = torch.zeros(0, dtype=torch.long)
        self.ndata = _Store(lambda: self.n)
        self.edata = _Store(lambda: len(self.src))
        self.batch_num_nodes = None
        self.batch_num_edges = None

    def set_n_initializer(self, f):
        pass

    def set_e_initializer(self, f):
        pass

    def add_nodes(self, m):
        for k in list(self.ndata):
            self.ndata[k] = torch.cat([self.ndata[k], torch.zeros((m,) + self.ndata[k].shape[1:],
                                                                  dtype=self.ndata[k].dtype)])
        self.n += m

    def add_edges(self, u, v, data=None):
        u, v = torch.as_tensor(u).reshape(-1).long(), torch.as_tensor(v).reshape(-1).long()
        if len(u) == 1 and len(v) > 1:
            u = u.expand(len(v))
        if len(v) == 1 and len(u) > 1:
            v = v.expand(len(u))
        m = len(u)
        for k in list(self.edata):
            self.edata[k] = torch.cat([self.edata[k], torch.zeros((m,) + self.edata[k].shape[1:],
                                                                  dtype=self.edata[k].dtype)])
        old = len(self.src)
        self.src = torch.cat([self.src, u])
        self.dst = torch.cat([self.dst, v])
        for k, val in (data or {}).items():
            self.edata.write(k, torch.arange(old, old + m), torch.as_tensor(val))

    def add_edge(self, u, v, data=None):
        self.add_edges(u, v, data)

    @property
    def nodes(self):
        return _View(self.ndata, lambda: self.n)

    @property
    def edges(self):
        return _View(self.edata, lambda: len(self.src))

    def number_of_nodes(self):
        return self.n

    def filter_nodes(self, pred):
        return torch.nonzero(pred(_NB(dict(self.ndata))).reshape(-1)).reshape(-1)

    def filter_edges(self, pred):
        return torch.nonzero(pred(_EB(self, torch.arange(len(self.src)))).reshape(-1)).reshape(-1)

    def predecessors(self, v):
        return self.src[self.dst == int(v)]

    def apply_edges(self, func, edges):
        e = torch.as_tensor(edges).long()
        for k, val in func(_EB(self, e)).items():
            self.edata.write(k, e, val)

    def pull(self, v, mfunc, rfunc):
        v = torch.as_tensor(v).long()
        vset = set(v.tolist())
        # in-edges grouped per node in edge-id order
        per = {}
        for e, d in enumerate(self.dst.tolist()):
            if d in vset:
                per.setdefault(d, []).append(e)
        buckets = {}
        for d, es in per.items():
            buckets.setdefault(len(es), []).append(d)
        for deg, nodes in sorted(buckets.items()):
            eids = torch.tensor([e for d in nodes for e in per[d]])
            msg = mfunc(_EB(self, eids))
            mb = {k: m.reshape(len(nodes), deg, *m.shape[1:]) for k, m in msg.items()}
            nidx = torch.tensor(nodes)
            out = rfunc(_NB({k: x[nidx] for k, x in self.ndata.items()}, mb))
            for k, val in out.items():
                self.ndata.write(k, nidx, val)


def batch(graphs):
    g = DGLGraph()
    off = 0
    srcs, dsts = [], []
    keys_n = set().union(*[set(x.ndata) for x in graphs])
    keys_e = set().union(*[set(x.edata) for x in graphs])
    for x in graphs:
        srcs.append(x.src + off)
        dsts.append(x.dst + off)
        off += x.n
    g.n = off
    g.src, g.dst = torch.cat(srcs), torch.cat(dsts)
    for k in keys_n:
        proto = next(x.ndata[k] for x in graphs if k in x.ndata)
        g.ndata[k] = torch.cat([x.ndata[k] if k in x.ndata else
                                torch.zeros((x.n,) + proto.shape[1:], dtype=proto.dtype) for x in graphs])
    for k in keys_e:
        proto = next(x.edata[k] for x in graphs if k in x.edata)
        g.edata[k] = torch.cat([x.edata[k] if k in x.edata else
                                torch.zeros((len(x.src),) + proto.shape[1:], dtype=proto.dtype)
                                for x in graphs])
    g.batch_num_nodes = [x.n for x in graphs]
    g.batch_num_edges = [len(x.src) for x in graphs]
    return g


def unbatch(g):
    out = []
    no, eo = 0, 0
    for nn_, ne in zip(g.batch_num_nodes, g.batch_num_edges):
        x = DGLGraph()
        x.n = nn_
        x.src = g.src[eo:eo + ne] - no
        x.dst = g.dst[eo:eo + ne] - no
        for k, v in g.ndata.items():
            x.ndata[k] = v[no:no + nn_]
        for k, v in g.edata.items():
            x.edata[k] = v[eo:eo + ne]
        out.append(x)
        no += nn_
        eo += ne
    return out


def sum_nodes(g, key):
    out = []
    no = 0
    for nn_ in g.batch_num_nodes:
        out.append(g.ndata[key][no:no + nn_].sum(0))
        no += nn_
    return torch.stack(out)


class init:  # noqa: N801  (dgl.init namespace)
    zero_initializer = staticmethod(zero_initializer)
