"""Dev tool: S2W hsg_gat_fwd (the bench roofline kernel) per forward variant on cfg2.
Arguments are VAR=VALUE env settings, one variant each, e.g.
  HSG_GAT_ROWS=0 (one destination per wave)  HSG_GAT_ROWS=0,HSG_GAT_LPN=32 (grouped)
  HSG_GAT_ROWS=5 (row-tile kernel, 5 float4 slots per thread)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
docs, G, _, _ = bench.make_shard("cfg2", 0, 1, 0)
G.to(dev)
torch.manual_seed(0)
stack = bench.Stack(0.1, 2).to(dev)
from hetersumgraph_amd.HiGraph import register_tfidf_table  # noqa: E402
register_tfidf_table(G, stack._TFembed.weight)
gen = torch.Generator(device=dev).manual_seed(0)
rel_s = G.relation("S2W")
Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)
Xs = torch.randn(rel_s.n_src, 64, device=dev, generator=gen)
for variant in sys.argv[1:] or ["HSG_GAT_ROWS=0", "HSG_GAT_ROWS=-1"]:
    saved = dict(os.environ)
    for kv in variant.split(","):
        k, v = kv.split("=")
        os.environ[k] = v
    ms, med, nbytes = bench.time_fwd_kernel(G, stack, Xw, Xs, 100)
    print(f"{variant:28s} mean {ms * 1e3:6.1f} us  median {med * 1e3:6.1f} us  "
          f"{nbytes / (ms * 1e-3) / 1e9:7.1f} GB/s", flush=True)
    os.environ.clear()
    os.environ.update(saved)
