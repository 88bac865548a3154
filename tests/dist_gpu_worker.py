"""One rank of tests/test_gpu_dist.py (launched by torch.distributed.run; not a test
module itself).  Every rank runs the HIP WSWGAT stack (the fused node bench.py
times) on its document shard of a skewed 5-document batch, reduces the parameter
gradients with the hook-driven GradientReducer (doc-weighted: n_r / N), clips
them (train.py:132-133), and compares with the full-batch gradient computed on
the same device: the data-parallel step must equal the single-process step."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def doc_inputs(d, dev):
    """Per-document features and upstream weights, seeded by the document itself,
    so a shard and the full batch see identical values."""
    g = torch.Generator().manual_seed(int(d.wid.sum()) % (2 ** 31))
    n_w, n_s = int((d.unit == 0).sum()), int((d.unit == 1).sum())
    Xw = 0.4 * torch.randn(n_w, 300, generator=g)
    Xs = torch.randn(n_s, 64, generator=g)
    R = torch.randn(n_s, 64, generator=g)
    return Xw.to(dev), Xs.to(dev), R.to(dev)


def loss_of(docs, stack, dev):
    """train.py:115-119 shape: per-document sum over its sentences, mean over docs."""
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    G = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    G.to(dev)
    ins = [doc_inputs(d, dev) for d in docs]
    Xw = torch.cat([i[0] for i in ins])
    Xs = torch.cat([i[1] for i in ins])
    s = stack(G, Xw, Xs)
    per_doc = [(si * i[2]).sum() for si, i in zip(torch.split(s, [i[1].shape[0] for i in ins]), ins)]
    return torch.stack(per_doc).mean()


def main():
    from bench import Stack
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.parallel import GradientReducer, shard_documents, shard_fraction
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)              # both ranks share the one GPU of the box
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(21)
    docs = [synth.make_hsg_doc(rng, N=n, W=w, k=k) for n, w, k in
            ((30, 500, 30), (4, 40, 5), (6, 60, 6), (3, 30, 4), (12, 200, 14))]
    torch.manual_seed(0)
    full = Stack(0.1, 2).to(dev).eval()
    torch.manual_seed(0)
    local = Stack(0.1, 2).to(dev).eval()
    params = [p for p in local.parameters() if p.requires_grad]
    # full-batch reference step on this device
    loss_of(docs, full, dev).backward()
    ref_grads = [p.grad.detach().clone() for p in full.parameters()]
    ref_norm = torch.nn.utils.clip_grad_norm_(full.parameters(), 1.0)
    # data-parallel step: shard, backward with overlapped buckets, clip
    mine = shard_documents(docs, rank, world)
    red = GradientReducer(params, bucket_bytes=1 << 20, scale=shard_fraction(docs, rank, world))
    assert len(red.buckets) >= 2
    loss_of(mine, local, dev).backward()
    red.finish()
    norm = torch.nn.utils.clip_grad_norm_(params, 1.0)
    red.remove()
    assert abs(norm.item() - ref_norm.item()) <= 1e-5 * ref_norm.item(), (norm.item(), ref_norm.item())
    worst = 0.0
    for (n, a), b in zip(local.named_parameters(), full.parameters()):
        scale = max(b.grad.abs().max().item(), 1e-8)
        err = (a.grad - b.grad).abs().max().item() / scale
        worst = max(worst, err)
        assert err <= 2e-5, (n, err)
    # bench.py's exchange after a graph replay: the fused stack wrote every gradient
    # into one flat buffer, reduced in place as one bucket (parallel.flat_gradients)
    from hetersumgraph_amd.parallel import allreduce_gradients, flat_gradients
    for p in params:
        p.grad = None
    loss_of(mine, local, dev).backward()
    assert flat_gradients(params) is not None
    allreduce_gradients(params, scale=shard_fraction(docs, rank, world), bucket_bytes=1 << 30)
    for (n, a), b in zip(local.named_parameters(), ref_grads):
        scale = max(b.abs().max().item(), 1e-8)
        err = (a.grad - b).abs().max().item() / scale
        assert err <= 2e-5, ("flat", n, err)
    print(f"rank {rank}: {len(mine)} docs, grad norm {norm.item():.6e} (full batch {ref_norm.item():.6e}), "
          f"max rel grad err {worst:.2e}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
