"""Dev tool: what the one hsg_slab_reduce launch of a cfg2 stack backward spends its
time on.  Runs one eager train step with SlabBatch._launch intercepted, then times
every captured job alone (same buffers, HIP events, 20 launches) and the whole batch,
and prints per job: output, columns x output rows, segments x rows, slab MB read."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def timed(f, reps=20):
    """GPU time per launch: ``reps`` launches captured in one HIP graph and replayed
    (eager ctypes launches are host-bound at ~9 us each and would hide the kernel)."""
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e3
        best = t if best is None else min(best, t)
    return best


def main(config="cfg2"):
    import bench
    from hetersumgraph_amd import reduce as red
    from hetersumgraph_amd import rng as hsg_rng
    from hetersumgraph_amd._lib import load
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    docs, G, _, _ = bench.make_shard(config, 0, 1, 0)
    G.to(dev)
    torch.manual_seed(0)
    stack = bench.Stack(0.1, 2).to(dev).train()
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device=dev).manual_seed(0)
    Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)
    Xs = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen)
    captured = []
    orig = red.SlabBatch._launch

    def spy(lib, batch):
        captured.append(list(batch))
        orig(lib, batch)
    red.SlabBatch._launch = staticmethod(spy)
    hsg_rng.advance_all()
    stack(G, Xw, Xs).backward(R)
    torch.cuda.synchronize()
    red.SlabBatch._launch = staticmethod(orig)
    lib = load()
    # keep the stack's tensors alive while timing (the slabs live in its saved state)
    for bi, batch in enumerate(captured):
        us = timed(lambda: orig(lib, batch))
        print(f"launch {bi}: {len(batch)} jobs, {us:.1f} us", flush=True)
        for f in batch:
            out, cols, pitch, coff, scale, acc, segs, orows = f
            mb = sum(r * cols * 4 for _, r in segs) / 1e6
            us1 = timed(lambda: orig(lib, [f]))
            rest = [g for g in batch if g is not f]
            us_wo = timed(lambda: orig(lib, rest)) if rest else 0.0
            print(f"   cols {cols:7d} x orows {orows:3d}  pitch {pitch:7d}  segs {[r for _, r in segs]}  "
                  f"{mb:7.2f} MB  alone {us1:6.1f} us  {mb / us1 if us1 else 0:5.2f} TB/s  "
                  f"batch without it {us_wo:6.1f} us", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
