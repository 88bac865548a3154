"""Worker of tests/test_gpu_rccl.py (run as a subprocess, not a test module itself):
the data-parallel exchange of bench.py on RCCL, on the one GPU of the box.

A world-size-1 ``nccl`` process group (RCCL; file:// rendezvous) is created in this
process.  The fused WSWGAT stack runs one eager fwd+bwd (train mode, dropout 0, so
every run is bit-reproducible; the backward is deterministic), its flat gradient
buffer is cloned as the reference, then step + the doc-weighted in-place all-reduce
(parallel.reduce_flat with scale s) are captured into ONE HIP graph and replayed
twice.  After each replay every ``p.grad`` must equal s x the reference: the
captured backward rewrites the buffer and the captured collective scales and
reduces it in place (a world of one sums one contribution).  The semantics are
train.py:118-135's mean loss over documents, reduced over ranks."""
import os
import sys
import tempfile

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    from bench import Stack
    from hetersumgraph_amd import _lib
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.parallel import flat_gradients, reduce_flat
    _lib.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    fd, rdv = tempfile.mkstemp(prefix="hsg_rccl_")
    os.close(fd)
    os.unlink(rdv)
    dist.init_process_group("nccl", init_method=f"file://{rdv}", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    docs = synth.make_batch_docs("cfg2", seed=5, n_docs=6)
    G = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    G.to(dev)
    torch.manual_seed(0)
    stack = Stack(0.0, 2).to(dev).train()
    params = [p for p in stack.parameters() if p.requires_grad]
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device=dev).manual_seed(3)
    Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)
    Xs = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen)
    scale = 0.375                        # a rank holding 3 of 8 documents

    def zero():
        for p in params:
            p.grad = None
        Xs.grad = None

    def step():
        stack(G, Xw, Xs).backward(R)

    def exchange():
        flat = flat_gradients(params)
        assert flat is not None, "the fused stack's gradients do not tile one flat buffer"
        reduce_flat(flat, scale=scale)

    zero()
    step()
    flat = flat_gradients(params)
    assert flat is not None and flat.numel() == sum(p.numel() for p in params)
    ref = flat.clone()
    reduce_flat(flat, scale=scale)       # eager: also the communicator's first collective
    torch.cuda.synchronize()
    assert torch.equal(flat, ref * scale), "eager in-place exchange"

    s_side = torch.cuda.Stream(dev)
    s_side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s_side):
        for _ in range(2):
            zero()
            step()
            exchange()
    torch.cuda.current_stream(dev).wait_stream(s_side)
    zero()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
        exchange()
    torch.cuda.synchronize()
    worst = 0.0
    for rep in range(2):
        graph.replay()
        torch.cuda.synchronize()
        got = flat_gradients(params)
        assert got is not None
        err = ((got - ref * scale).abs().max() / (ref.abs().max() * scale)).item()
        worst = max(worst, err)
        assert err <= 1e-6, (rep, err)
    print(f"rccl world 1: {len(params)} params, {ref.numel()} grads in one flat buffer, "
          f"step + exchange replayed as one graph, max rel err {worst:.2e}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
