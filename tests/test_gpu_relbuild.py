"""hsg_rel_build (device relation construction) vs the numpy restatement
``oracle.fused.typed_relation`` -- bit-exact on every output array.

The expected CSR is the oracle's typed edge list (edge-id order) stably sorted by
destination rank (DGL 0.4 mailbox order inside a segment, GATLayer.py:113/149); the
expected CSC is that CSR stably sorted by source rank."""
import numpy as np
import pytest
import torch

from hetersumgraph_amd import synth
from hetersumgraph_amd.relation import build_relation

pytestmark = pytest.mark.gpu


def expected(kind, src, dst, unit, tffrac, edtype):
    from oracle.fused import typed_relation
    r = typed_relation(kind, src, dst, unit, tffrac, edtype)
    su, du = (0.0, 1.0) if kind == "W2S" else (1.0, 0.0)
    unit = np.asarray(unit)
    typed = np.nonzero((unit[src] == su) & (unit[dst] == du))[0]
    order = np.argsort(r["e_dst"], kind="stable")
    e_src, e_dst = r["e_src"][order], r["e_dst"][order]
    tf = np.where(r["tf"] >= 0, r["tf"], 10)[order]
    corder = np.argsort(e_src, kind="stable")
    cnt = lambda a, m: np.concatenate([[0], np.cumsum(np.bincount(a, minlength=m))])
    return dict(src_nodes=np.nonzero(unit == su)[0], dst_nodes=np.nonzero(unit == du)[0],
                indptr=cnt(e_dst, r["n_dst"]), src=e_src, tf=tf, eid=typed[order],
                phantom=r["phantom"], cindptr=cnt(e_src, r["n_src"]), cdst=e_dst[corder],
                cperm=corder)


def check(src, dst, unit, tffrac, edtype):
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.as_tensor(np.asarray(a), dtype=dt, device=dev)
    for kind in ("W2S", "S2W"):
        rel = build_relation(kind, t(src, torch.int64), t(dst, torch.int64), t(unit, torch.float32),
                             t(tffrac, torch.int64), t(edtype, torch.float32))
        exp = expected(kind, np.asarray(src), np.asarray(dst), unit, tffrac, edtype)
        assert rel.n_src == len(exp["src_nodes"]) and rel.n_dst == len(exp["dst_nodes"])
        assert rel.n_typed == len(exp["src"]) and rel.n_edges_total == len(src)
        for k, v in exp.items():
            got = rel.dev[k].cpu().numpy()
            assert got.shape == v.shape, (kind, k)
            np.testing.assert_array_equal(got.astype(np.int64), v.astype(np.int64), err_msg=f"{kind} {k}")


def batch(docs):
    off, parts = 0, {k: [] for k in ("src", "dst", "unit", "tffrac", "edtype")}
    for d in docs:
        parts["src"].append(d.src + off)
        parts["dst"].append(d.dst + off)
        parts["unit"].append(d.unit)
        parts["tffrac"].append(d.tffrac)
        parts["edtype"].append(d.edtype)
        off += d.n_nodes
    return {k: np.concatenate(v) for k, v in parts.items()}


@pytest.mark.parametrize("config,n_docs", [("cfg1", 4), ("cfg2", 32), ("cfg4", 6), ("cfg5", 3)])
def test_relbuild_synthetic_batches(config, n_docs):
    b = batch(synth.make_batch_docs(config, seed=3, n_docs=n_docs))
    check(b["src"], b["dst"], b["unit"], b["tffrac"], b["edtype"])


def test_relbuild_isolated_words_and_jitter():
    rng = np.random.default_rng(7)
    docs = [synth.make_hsg_doc(rng, 12, 80, 9, k_jitter=8, isolated_words=5) for _ in range(5)]
    b = batch(docs)
    check(b["src"], b["dst"], b["unit"], b["tffrac"], b["edtype"])


@pytest.mark.parametrize("n,E,seed", [(1, 0, 0), (5, 0, 1), (3, 7, 2), (1000, 20000, 3), (70000, 1 << 20, 4)])
def test_relbuild_random_coo(n, E, seed):
    """Random multigraph: duplicate edges, self loops, a third unit value (neither
    side), typed edges with dtype != 0 (tau row 10), unsorted edge ids."""
    rng = np.random.default_rng(seed)
    unit = rng.choice(np.array([0.0, 1.0, 2.0], np.float32), size=n, p=[0.6, 0.3, 0.1])
    src = rng.integers(0, n, size=E)
    dst = rng.integers(0, n, size=E)
    tffrac = rng.integers(0, 10, size=E)
    edtype = rng.choice(np.array([0.0, 1.0, 2.0], np.float32), size=E, p=[0.8, 0.1, 0.1])
    check(src, dst, unit, tffrac, edtype)


def test_relbuild_rejects_bad_inputs():
    dev = torch.device("cuda", 0)
    t = lambda a, dt=torch.int64: torch.tensor(a, dtype=dt, device=dev)
    unit = t([0.0, 1.0, 1.0], torch.float32)
    with pytest.raises(IndexError, match="tf-idf"):
        build_relation("W2S", t([0, 0]), t([1, 2]), unit, t([3, 10]), t([0.0, 0.0], torch.float32))
    # out-of-range box on a dtype-1 edge is never looked up (HiGraph.py:146-151)
    rel = build_relation("W2S", t([0, 0]), t([1, 2]), unit, t([3, 10]), t([0.0, 1.0], torch.float32))
    assert rel.dev["tf"].cpu().tolist() == [3, 10]
    with pytest.raises(IndexError, match="node id"):
        build_relation("W2S", t([0, 5]), t([1, 2]), unit, t([3, 4]), t([0.0, 0.0], torch.float32))


def test_graph_relation_uses_device_builder():
    """DGLGraph.to(cuda) builds both relations through hsg_rel_build; the product
    path never materialises a host copy."""
    from hetersumgraph_amd.graph import DGLGraph, batch as dgl_batch
    docs = synth.make_batch_docs("cfg1", seed=1)
    g = dgl_batch([synth.to_graph(d, DGLGraph) for d in docs])
    g.to(torch.device("cuda", 0))
    b = batch(docs)
    for kind in ("W2S", "S2W"):
        rel = g.relation(kind)
        assert rel.host is None and rel.dev["indptr"].is_cuda
        exp = expected(kind, b["src"], b["dst"], b["unit"], b["tffrac"], b["edtype"])
        np.testing.assert_array_equal(rel.dev["indptr"].cpu().numpy(), exp["indptr"])
        np.testing.assert_array_equal(rel.dev["src"].cpu().numpy(), exp["src"])
