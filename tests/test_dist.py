"""Multi-process (world size 2, gloo, CPU) checks of the data-parallel path
(DESIGN.md §5): document sharding + bucketed mean all-reduce of the
parameter gradients.  The model on CPU is the fp64 oracle of one WSWGAT layer
(the product kernels need a GPU), so the check is exactly the data-parallel
algebra: the doc-weighted sum over ranks of per-shard gradients == full-batch
gradient -- with equal shards (plain mean) and with skewed document sizes and an
odd document count (shards of 3 and 2 docs: weights n_r / N), through the
after-backward reducer and through the hook-driven GradientReducer that overlaps
the buckets with the backward.  tests/test_gpu_dist.py runs the HIP stack itself."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _docs(skewed=False):
    from hetersumgraph_amd import synth
    rng = np.random.default_rng(11)
    if skewed:       # edge weights far apart and 5 docs: the shards hold 3 and 2 docs
        return [synth.make_hsg_doc(rng, N=n, W=w, k=k) for n, w, k in
                ((12, 60, 10), (2, 10, 3), (3, 12, 4), (2, 9, 2), (6, 30, 7))]
    return [synth.make_hsg_doc(rng, N=5, W=24, k=6) for _ in range(4)]


def _params():
    from hetersumgraph_amd.module.GAT import WSWGAT
    from oracle import fused
    torch.manual_seed(3)
    return fused.as_params(WSWGAT(300, 64, 8, 0.1, 512, 0.1, 50, "W2S"))


def _loss(docs, params, T, seed_base=0):
    """Mean over documents of <W2S(doc), R_doc> (train.py:119-style per-doc mean)."""
    from oracle import fused
    total = 0.0
    for d in docs:
        rel = fused.typed_relation("W2S", d.src, d.dst, d.unit, d.tffrac, d.edtype)
        g = torch.Generator().manual_seed(int(d.wid.sum()) % (2 ** 31))
        Xw = 0.4 * torch.randn(rel["n_src"], 300, generator=g, dtype=torch.float64)
        Xs = torch.randn(rel["n_dst"], 64, generator=g, dtype=torch.float64)
        R = torch.randn(rel["n_dst"], 64, generator=g, dtype=torch.float64)
        out = fused.wswgat_layer("W2S", rel, Xw, Xs, params, T)
        total = total + (out * R).sum()
    return total / len(docs)


def _worker(rank, world, port, bucket_bytes, skewed, hooks, accum=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hetersumgraph_amd.parallel import (GradientReducer, allreduce_gradients, shard_documents,
                                                shard_fraction)
        torch.set_num_threads(2)
        docs = _docs(skewed)
        T = torch.randn(10, 50, generator=torch.Generator().manual_seed(5), dtype=torch.float64)
        # full batch on every rank (the expected result)
        full = _params()
        _loss(docs, full, T).backward()
        # this rank's shard
        mine = shard_documents(docs, rank, world)
        frac = shard_fraction(docs, rank, world)
        assert len(mine) in ((2, 3) if skewed else (len(docs) // world,))
        assert frac == len(mine) / len(docs)
        local = _params()
        scale = frac if skewed else None
        if hooks and accum:
            # gradient accumulation: the shard's documents in two micro-batches, the
            # first under no_sync(), each loss weighted by its share of the shard
            red = GradientReducer(list(local.values()), bucket_bytes=bucket_bytes, scale=scale)
            h = len(mine) // 2
            with red.no_sync():
                (_loss(mine[:h], local, T) * (h / len(mine))).backward()
            assert red.next == 0 and not red.pending
            (_loss(mine[h:], local, T) * ((len(mine) - h) / len(mine))).backward()
            red.finish()
            # a second hooked backward before finish() must raise, not drop gradients
            extra = _params()
            red2 = GradientReducer(list(extra.values()), bucket_bytes=bucket_bytes, scale=scale)
            _loss(mine, extra, T).backward()
            with pytest.raises(RuntimeError, match="second backward"):
                _loss(mine, extra, T).backward()
            red2.finish()
            red2.remove()
            # the same when the first backward left a bucket incomplete (a
            # parameter that got no gradient): the repeated hook still raises
            extra3 = _params()
            unused = torch.zeros(3, dtype=torch.float64, requires_grad=True)
            red3 = GradientReducer([unused] + list(extra3.values()), bucket_bytes=1 << 30, scale=scale)
            assert len(red3.buckets) == 1
            _loss(mine, extra3, T).backward()
            assert red3.next == 0                    # the bucket waits for `unused`
            with pytest.raises(RuntimeError, match="second backward"):
                _loss(mine, extra3, T).backward()
            red3.finish()
            red3.remove()
            red.remove()
        elif hooks:
            red = GradientReducer(list(local.values()), bucket_bytes=bucket_bytes, scale=scale)
            _loss(mine, local, T).backward()
            red.finish()
            red.remove()
        else:
            _loss(mine, local, T).backward()
            allreduce_gradients(list(local.values()), bucket_bytes=bucket_bytes, scale=scale)
        for k in full:
            a, b = local[k].grad, full[k].grad
            assert torch.allclose(a, b, rtol=1e-9, atol=1e-12), (k, (a - b).abs().max().item())
        # the shards partition the batch
        seen = [None] * world
        dist.all_gather_object(seen, sorted(int(d.wid.sum()) for d in mine))
        assert sorted(sum(seen, [])) == sorted(int(d.wid.sum()) for d in docs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes,skewed,hooks", [(8 << 20, False, False), (4096, False, False),
                                                       (4096, True, False), (65536, True, True)])
def test_sharded_allreduce_equals_full_batch(bucket_bytes, skewed, hooks):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), bucket_bytes, skewed, hooks), nprocs=world, join=True)


def test_reducer_gradient_accumulation_and_misuse():
    """two backwards before finish() -- accumulation under no_sync() gives
    the full-batch gradient; an unguarded second hooked backward raises."""
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), 65536, True, True, True), nprocs=world, join=True)


def test_shard_documents_balanced_and_deterministic():
    from hetersumgraph_amd.parallel import shard_documents

    class D:
        def __init__(self, e):
            self.src = np.zeros(e)

    docs = [D(e) for e in (50, 10, 40, 30, 20, 60, 5, 45)]
    shards = [shard_documents(docs, r, 3) for r in range(3)]
    assert sorted(id(d) for s in shards for d in s) == sorted(id(d) for d in docs)
    assert sorted(len(s) for s in shards) == [2, 3, 3]          # counts balanced first
    loads = [sum(len(d.src) for d in s) for s in shards]
    assert max(loads) - min(loads) <= 60
    # skewed sizes: still 2 + 2 docs, not 1 + 3
    two = [shard_documents([D(e) for e in (100, 10, 10, 10)], r, 2) for r in range(2)]
    assert [len(s) for s in two] == [2, 2]
    assert [shard_documents(docs, r, 3) for r in range(3)] == shards


def test_flat_gradients_detects_one_buffer():
    """parallel.flat_gradients: gradients installed by autograd as views of one flat
    tensor (what stack._Grads returns) are recognised and reduced in place; any
    other layout falls back (None)."""
    from hetersumgraph_amd.parallel import flat_gradients
    p, q = torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(2, 2))

    class F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, y):
            return x.sum() + y.sum()

        @staticmethod
        def backward(ctx, g):
            flat = torch.arange(7.0)
            return flat[0:3].view(3), flat[3:7].view(2, 2)

    F.apply(p, q).backward()
    f = flat_gradients([q, p])                      # any order of the parameter list
    assert f is not None and f.numel() == 7
    f.mul_(2)
    assert torch.equal(p.grad, torch.tensor([0.0, 2.0, 4.0])) and q.grad[1, 1].item() == 12.0
    q.grad = q.grad.clone()                          # another buffer: no single flat view
    assert flat_gradients([p, q]) is None


def test_cfg3_global_batch_shards_over_eight_ranks():
    """BASELINE configs[2] (cfg3: 256 CNN/DM-shaped docs data-parallel over 8 GPUs,
    train.py:130-135 batching): bench.make_shard's document split gives every rank 32
    whole documents, each document exactly once, edge loads within one document of
    each other, and doc-weight fractions that sum to 1."""
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.parallel import shard_fraction, shard_owners
    world = 8
    docs = synth.make_batch_docs("cfg3", seed=0, n_docs=synth.CONFIGS["cfg3"][1] * world)
    owner = shard_owners(docs, world)
    counts = [owner.count(r) for r in range(world)]
    assert counts == [32] * world
    loads = [sum(len(d.src) for d, o in zip(docs, owner) if o == r) for r in range(world)]
    assert max(loads) - min(loads) <= max(len(d.src) for d in docs)
    fr = [shard_fraction(docs, r, world) for r in range(world)]
    assert abs(sum(fr) - 1.0) < 1e-12 and all(abs(f - 1 / 8) < 1e-12 for f in fr)


def _flat_worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hetersumgraph_amd.parallel import allreduce_gradients
        # two parameters whose gradients are views of ONE flat buffer (the fused
        # stack's layout), rank-dependent values, uneven doc weights
        p, q = torch.nn.Parameter(torch.zeros(5, dtype=torch.float64)), torch.nn.Parameter(
            torch.zeros(2, 3, dtype=torch.float64))
        flat = torch.arange(11, dtype=torch.float64) * (rank + 1)
        p.grad, q.grad = flat[:5], flat[5:].view(2, 3)
        w = [(r + 1) / sum(range(1, world + 1)) for r in range(world)]
        allreduce_gradients([p, q], scale=w[rank], bucket_bytes=1 << 30)
        want = torch.arange(11, dtype=torch.float64) * sum(wr * (r + 1) for r, wr in enumerate(w))
        assert torch.allclose(torch.cat([p.grad, q.grad.reshape(-1)]), want, rtol=0, atol=1e-12)
        assert p.grad.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()   # reduced in place
    finally:
        dist.destroy_process_group()


def test_flat_doc_weighted_allreduce_world8():
    """The bench's DP exchange (one in-place doc-weighted all-reduce of the flat
    gradient buffer, bench.py allreduce) at world size 8 -- the rank count of the
    cfg3 / SCALE runs -- rehearsed on gloo: sum_r w_r g_r on every rank."""
    world = 8
    mp.spawn(_flat_worker, args=(world, _free_port()), nprocs=world, join=True)
