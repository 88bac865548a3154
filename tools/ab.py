"""Dev tool: A/B the bench step (cfg2 unless HSG_AB_CONFIG; GEMM mode HSG_AB_DTYPE) under environment
variants in ONE process: for every variant 'VAR=a,VAR2=b' (the empty string is the
baseline) set the variables, re-capture the step into a HIP graph and time 100
replays; rounds interleave the variants.  Also prints each variant's in-step
edge-kernel times (HIP events inside eager steps).

usage: python tools/ab.py '' 'HSG_GAT_CAP=2048' 'HSG_GAT_CAP=1024'
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(variants):
    import numpy as np
    import torch
    import bench
    from hetersumgraph_amd import rng as hsg_rng
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from hetersumgraph_amd.dense import set_gemm_dtype
    set_gemm_dtype(os.environ.get("HSG_AB_DTYPE", "f32"))             # bench.py --dtype
    docs, G, _, _ = bench.make_shard(os.environ.get("HSG_AB_CONFIG", "cfg2"), 0, 1, 0)
    G.to(dev)
    torch.manual_seed(0)
    stack = bench.Stack(0.1, 2).to(dev).train()
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device=dev).manual_seed(0)
    Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)
    Xs = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen)
    params = list(stack.parameters())

    def step():
        hsg_rng.advance_all()
        stack(G, Xw, Xs).backward(R)

    def zero():
        for p in params:
            p.grad = None
        Xs.grad = None

    def apply(v):
        for k in [k for k in os.environ if k.startswith("HSG_") and k not in ("HSG_AB_CONFIG", "HSG_AB_DTYPE")]:
            del os.environ[k]
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=", 1)
            os.environ[k] = val

    graphs = {}
    for v in variants:
        apply(v)
        for _ in range(3):
            zero()
            step()
        torch.cuda.synchronize()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            zero()
            step()
        torch.cuda.current_stream(dev).wait_stream(s)
        zero()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        torch.cuda.synchronize()
        graphs[v] = g
    res = {v: [] for v in variants}
    for _ in range(3):
        for v in variants:
            g = graphs[v]
            for _ in range(10):
                g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(100):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 100)
    for v in variants:
        apply(v)
        kt = bench.time_edge_kernels_in_step(step, zero, 5)
        ks = "  ".join(f"{a}_{b} {ms * 1e3:.1f}" for (a, b), (ms, _) in sorted(kt.items()))
        print(f"{v or 'baseline':40s} {np.median(res[v]):.4f} ms/step (min {min(res[v]):.4f})  {ks}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or [""])
