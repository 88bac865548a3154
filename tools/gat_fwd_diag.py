"""Dev tool: what bounds the cfg2 S2W edge forward.  Times hsg_gat_fwd back to back
(events around 200 launches) on the cfg2 S2W relation in these modes:
  out   origin read + out write (the product path, no h)
  h     no origin: writes h only (same store bytes, no residual read)
  both  origin read + out + h writes
and, with the dev library, each env variant passed on the command line
(e.g. HSG_GAT_FWD_PF=3 HSG_GAT_FWD_B=4)."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
from hetersumgraph_amd import _lib
from hetersumgraph_amd._lib import load, ptr, stream_of
from hetersumgraph_amd.HiGraph import register_tfidf_table
from hetersumgraph_amd._lib import HSG_TAU_TABLE
from hetersumgraph_amd.ops import attn_tables, LEAKY_SLOPE

dev = torch.device("cuda", 0)
docs, G, _, _ = bench.make_shard("cfg2", 0, 1, 0)
G.to(dev)
torch.manual_seed(0)
stack = bench.Stack(0.1, 2).to(dev)
register_tfidf_table(G, stack._TFembed.weight)
lib = load()
rel = G.relation("S2W")
layer = stack.sent2word.layer
H, D = layer.num_heads, layer.head_dim
W, attn, wf, bf = layer.fused_params()
T = stack._TFembed.weight
HD = H * D
Z = torch.randn(rel.n_src, HD, device=dev)
org = torch.randn(rel.n_dst, HD, device=dev)
a1, tau = attn_tables(attn, T, wf, bf, H, D)
sigma = Z.new_empty(rel.n_src, H)
lib.hsg_attn_src_logits(rel.n_src, H, D, ptr(Z), ptr(a1), ptr(sigma), stream_of(Z))
h = torch.empty(rel.n_dst, HD, device=dev)
out = torch.empty(rel.n_dst, HD, device=dev)
m = Z.new_empty(rel.n_dst, H)
l = Z.new_empty(rel.n_dst, H)
relp = ctypes.byref(rel.cstruct())
modes = {"out": (org, None, out), "h": (None, h, None), "both": (org, h, out)}


def run(mode, n):
    o, hh, oo = modes[mode]
    for _ in range(n):
        rc = lib.hsg_gat_fwd(relp, H, D, HSG_TAU_TABLE, LEAKY_SLOPE, ptr(Z), ptr(sigma), ptr(tau), ptr(o), ptr(hh),
                             ptr(oo), ptr(m), ptr(l), stream_of(Z))
        assert rc == 0, rc


res = []
for mode in modes:
    run(mode, 10)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run(mode, 200)
    e1.record()
    torch.cuda.synchronize()
    res.append(f"{mode} {e0.elapsed_time(e1) / 200 * 1e3:.2f}us")
print(" ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("HSG_GAT")) or "default", *res, flush=True)
