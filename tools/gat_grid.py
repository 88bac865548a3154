"""Dev tool: time the cfg2 edge kernels (fwd + bwd dst/src, both directions) for
the grid cap in HSG_GAT_CAP (compare across runs)."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from hetersumgraph_amd import _lib
from hetersumgraph_amd.HiGraph import register_tfidf_table
from hetersumgraph_amd.ops import gat_heads_table

dev = torch.device("cuda", 0)
docs, G, _, _ = bench.make_shard("cfg2", 0, 1, 0)
G.to(dev)
torch.manual_seed(0)
stack = bench.Stack(0.1, 2).to(dev)
register_tfidf_table(G, stack._TFembed.weight)
res = []
for kind, mod, n_src_dim in (("S2W", stack.sent2word, 300), ("W2S", stack.word2sent, 64)):
    rel = G.relation(kind)
    layer = mod.layer
    H, D = layer.num_heads, layer.head_dim
    W, attn, wf, bf = layer.fused_params()
    Z = torch.randn(rel.n_src, H * D, device=dev, requires_grad=True)
    org = torch.randn(rel.n_dst, H * D, device=dev, requires_grad=True)
    T = stack._TFembed.weight
    R = torch.randn(rel.n_dst, H * D, device=dev)
    def f():
        out = gat_heads_table(Z, attn, T, wf, bf, org, rel, H, D)
        (out * R).sum().backward()
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): f()
    e1.record(); torch.cuda.synchronize()
    res.append(f"{kind} {e0.elapsed_time(e1)/20*1e3:.1f}us")
print(os.environ.get("HSG_GAT_CAP", "default"), *res)
