"""Data-parallel plumbing for the WSWGAT path.

The batched graph is a disjoint union of documents (reference dataloader.py:480,
``dgl.batch``), so the path shards by document with no data-path collective; the
one exchange per step is the all-reduce of parameter gradients after backward,
done in buckets over RCCL (``torch.distributed`` backend "nccl" on ROCm = RCCL
over xGMI), then ``clip_grad_norm_`` on the reduced gradients and a replicated
Adam step (train.py:130-135).  Parameters must start identical on every rank
(same seed or a broadcast).

The reference's loss is a mean over the batch's documents (train.py:118-119:
``dgl.sum_nodes(G, "loss").mean()``).  A rank's loss is the mean over ITS
documents, so the global-batch gradient is sum_r (n_r / N) grad_r, not the plain
average of the per-rank gradients unless every rank holds the same number of
documents.  :func:`shard_fraction` gives n_r / N from the deterministic shard
(no communication), and both reducers below take it as ``scale``.
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist


def _doc_weight(d):
    return getattr(d, "n_edges", None) or len(d.src)


def shard_owners(docs, world, weight=None):
    """Owner rank of every document: greedy longest-processing-time by
    ``weight(doc)`` (default: the document's edge count), ties by index, with the
    document COUNT balanced first -- shards differ by at most one document, and
    among the least-filled ranks the one with the fewest edges takes the next
    (largest remaining) document."""
    weight = weight or _doc_weight
    order = sorted(range(len(docs)), key=lambda i: (-weight(docs[i]), i))
    load = [0] * world
    count = [0] * world
    owner = [0] * len(docs)
    for i in order:
        r = min(range(world), key=lambda q: (count[q], load[q], q))
        owner[i] = r
        load[r] += weight(docs[i])
        count[r] += 1
    return owner


def shard_documents(docs, rank, world, weight=None):
    """This rank's documents of a deterministic balanced split (:func:`shard_owners`),
    in their original order."""
    owner = shard_owners(docs, world, weight)
    return [docs[i] for i in range(len(docs)) if owner[i] == rank]


def shard_fraction(docs, rank, world, weight=None):
    """n_rank / N: this rank's share of the global batch's documents -- the factor
    its per-rank-mean gradient carries in the global-mean gradient."""
    owner = shard_owners(docs, world, weight)
    return sum(1 for o in owner if o == rank) / max(len(docs), 1)


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


def _launch(bucket, scale, world, group):
    """Start one bucket's all-reduce; returns (work, flat, bucket)."""
    flat = torch.cat([g.reshape(-1) for g in bucket])
    if scale is not None:
        flat.mul_(scale)                       # weighted sum = global-batch mean
        op = dist.ReduceOp.SUM
    elif dist.get_backend(group) == "nccl":
        op = dist.ReduceOp.AVG                 # RCCL averages natively
    else:
        op = dist.ReduceOp.SUM                 # gloo: sum, divided after the wait
    work = dist.all_reduce(flat, op=op, group=group, async_op=True)
    return work, flat, bucket, (scale is None and op == dist.ReduceOp.SUM)


def _finish(pending, world):
    for work, flat, bucket, divide in pending:
        work.wait()
        if divide:
            flat.div_(world)
        torch._foreach_copy_(bucket, [v.view_as(g) for v, g in
                                      zip(torch.split(flat, [g.numel() for g in bucket]), bucket)])


def flat_gradients(params):
    """A 1-D tensor over the one buffer behind every ``p.grad`` of ``params`` when the
    gradients tile that buffer exactly (the fused stack's backward writes them as
    views of one flat tensor, stack._Grads; AccumulateGrad installs them without a
    copy), else None.  Reducing it in place reduces every ``p.grad``."""
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return None
    st = grads[0].untyped_storage()
    es = grads[0].element_size()
    if any(g.untyped_storage().data_ptr() != st.data_ptr() or g.dtype != grads[0].dtype or not g.is_contiguous()
           for g in grads):
        return None
    total = sum(g.numel() for g in grads)
    if total * es != st.nbytes():
        return None
    o = 0
    for g in sorted(grads, key=lambda t: t.storage_offset()):
        if g.storage_offset() != o:
            return None
        o += g.numel()
    return torch.empty(0, dtype=grads[0].dtype, device=grads[0].device).set_(st, 0, (total,))


def reduce_flat(flat, group=None, scale=None):
    """All-reduce ONE flat gradient buffer in place: sum_r scale_r * g_r when
    ``scale`` (this rank's :func:`shard_fraction`) is given, else the mean.  No
    world-size-1 short cut, no host synchronisation and no allocation, so on the
    nccl (RCCL) backend it can be captured into the step's HIP graph after the
    backward (bench.py replays step + exchange as one graph; the communicator must
    have run one collective before the capture)."""
    if scale is not None:
        if scale != 1.0:
            flat.mul_(scale)                    # weighted sum = global-batch mean
        op = dist.ReduceOp.SUM
    elif dist.get_backend(group) == "nccl":
        op = dist.ReduceOp.AVG                  # RCCL averages natively
    else:
        op = dist.ReduceOp.SUM
    dist.all_reduce(flat, op=op, group=group)
    if scale is None and op == dist.ReduceOp.SUM:
        flat.div_(dist.get_world_size(group))


def allreduce_gradients(params, group=None, bucket_bytes=2 << 20, scale=None):
    """Reduce ``p.grad`` over the process group in flat buckets of at most
    ``bucket_bytes`` (all issued asynchronously, then waited): the mean when
    ``scale`` is None (equal shards), else sum_r scale_r * grad_r with this rank's
    ``scale`` = :func:`shard_fraction`.  Parameters without a gradient are skipped
    (every rank must agree on which those are)."""
    if not dist.is_available() or not dist.is_initialized():
        return
    world = dist.get_world_size(group)
    if world == 1:
        return
    flat = flat_gradients(params) if bucket_bytes >= (1 << 30) else None
    if flat is not None:
        # the gradients already form one flat buffer: reduce it in place (no cat /
        # copy-back); the doc-weighted sum scales it first (one elementwise pass)
        reduce_flat(flat, group, scale)
        return
    grads = [p.grad for p in params if p.grad is not None]
    pending = [_launch(b, scale, world, group) for b in _buckets(grads, bucket_bytes)]
    _finish(pending, world)


class GradientReducer:
    """Bucketed gradient all-reduce overlapped with the backward (DDP-style, for
    the eager train step, train.py:114-135).

    Parameters are bucketed in REVERSE registration order (the order backward
    finalises them: the classifier head and the GAT stack before the sentence
    encoder).  A post-accumulate-grad hook marks a parameter ready; when every
    parameter of a bucket is ready its all-reduce is launched asynchronously on
    the communicator's stream while autograd carries on with the rest of the
    backward.  Buckets are launched strictly in bucket order (a ready bucket waits
    for its predecessors), so every rank issues the same collective sequence even
    if hooks fire in a different order.  :meth:`finish` waits for the outstanding
    buckets, writes the reduced values back into ``p.grad`` and returns the
    parameters, so the caller clips (``clip_grad_norm_``) and steps the optimizer
    on the reduced gradients.

    The fused WSWGAT stack returns its parameter gradients through autograd
    (hetersumgraph_amd/stack.py), so its hooks fire when the stack node's backward
    ends -- before the encoder's backward runs.

    One reduced backward per :meth:`finish`.  Gradient accumulation runs the
    earlier micro-batches under :meth:`no_sync` (hooks idle, gradients accumulate
    locally in ``p.grad``) and the last one outside it, whose hooks then reduce the
    accumulated sums.  A second backward with hooks before :meth:`finish` raises
    instead of silently reducing only the first one.
    """

    def __init__(self, params, group=None, bucket_bytes=2 << 20, scale=None):
        self.params = [p for p in params if p.requires_grad]
        self.group, self.scale = group, scale
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.buckets = list(_buckets(list(reversed(self.params)), bucket_bytes))
        self.where = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self.where[id(p)] = bi
        self.ready = [0] * len(self.buckets)
        self.seen = set()                    # parameters whose hook fired since the last finish()
        self.next = 0                        # next bucket to launch
        self.pending = []
        self._sync = True
        self.hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params] \
            if self.world > 1 else []

    def _launch_next(self):
        b = self.buckets[self.next]
        live = [q.grad for q in b if q.grad is not None]
        if live:
            self.pending.append(_launch(live, self.scale, self.world, self.group))
        self.next += 1

    @contextlib.contextmanager
    def no_sync(self):
        """Backward passes inside this context only accumulate into ``p.grad`` (the
        micro-batches before the last one of a gradient-accumulation step)."""
        prev, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = prev

    def _on_grad(self, p):
        if not self._sync:
            return
        bi = self.where[id(p)]
        # a parameter's hook firing twice before finish() is a second backward, even
        # when the first one left its bucket incomplete (a parameter without gradient)
        if id(p) in self.seen or self.next == len(self.buckets) or self.ready[bi] >= len(self.buckets[bi]):
            raise RuntimeError("GradientReducer: a second backward before finish() -- its gradients would not "
                               "be reduced; run the earlier micro-batches under no_sync()")
        self.seen.add(id(p))
        self.ready[bi] += 1
        while self.next < len(self.buckets) and self.ready[self.next] == len(self.buckets[self.next]):
            self._launch_next()

    def finish(self):
        """Launch the buckets still outstanding (e.g. one holding a parameter that
        got no gradient this step), in order; wait for all; reset for the next step."""
        if self.world > 1:
            while self.next < len(self.buckets):
                self._launch_next()
            _finish(self.pending, self.world)
        self.pending = []
        self.next = 0
        self.ready = [0] * len(self.buckets)
        self.seen = set()
        return self.params

    def remove(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []
