"""Data-parallel plumbing for the WSWGAT path.

The batched graph is a disjoint union of documents (reference dataloader.py:480,
``dgl.batch``), so the path shards by document with no data-path collective; the
one exchange per step is the mean all-reduce of parameter gradients after
backward, done in flat buckets over RCCL (``torch.distributed`` backend "nccl" on
ROCm = RCCL over xGMI).  Parameters must start identical on every rank (same seed
or a broadcast), as the reference's replicated Adam assumes.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_documents(docs, rank, world, weight=None):
    """Deterministic balanced split of ``docs`` into ``world`` shards; returns this
    rank's list.  Greedy longest-processing-time by ``weight(doc)`` (default: the
    document's edge count, ``doc.n_edges`` or ``len(doc.src)``), ties by index."""
    if weight is None:
        def weight(d):
            return getattr(d, "n_edges", None) or len(d.src)
    order = sorted(range(len(docs)), key=lambda i: (-weight(docs[i]), i))
    load = [0] * world
    owner = [0] * len(docs)
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        owner[i] = r
        load[r] += weight(docs[i])
    return [docs[i] for i in range(len(docs)) if owner[i] == rank]


def _buckets(tensors, bucket_bytes):
    cur, size = [], 0
    for t in tensors:
        nb = t.numel() * t.element_size()
        if cur and size + nb > bucket_bytes:
            yield cur
            cur, size = [], 0
        cur.append(t)
        size += nb
    if cur:
        yield cur


def allreduce_gradients(params, group=None, bucket_bytes=8 << 20):
    """Average ``p.grad`` over the process group, in flat buckets of at most
    ``bucket_bytes`` (one all-reduce each).  Parameters without a gradient are
    skipped (every rank must agree on which those are).  RCCL averages natively;
    gloo sums, then the bucket is divided by the world size."""
    if not dist.is_available() or not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    use_avg = dist.get_backend(group) == "nccl"
    for bucket in _buckets(grads, bucket_bytes):
        flat = torch.cat([g.reshape(-1) for g in bucket])
        if use_avg:
            dist.all_reduce(flat, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
            flat.div_(world)
        torch._foreach_copy_(bucket, [v.view_as(g) for v, g in
                                      zip(torch.split(flat, [g.numel() for g in bucket]), bucket)])
