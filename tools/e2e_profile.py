"""Dev tool (GPU): where the secondary end-to-end train step (bench.time_train_step)
spends its time on cfg2 -- synchronised wall time per phase, then the same step
under torch.profiler for the host/device split."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from hetersumgraph_amd import HiGraph  # noqa: E402
from hetersumgraph_amd import graph as hg  # noqa: E402

dev = torch.device("cuda", 0)
docs, G, _, _ = bench.make_shard(sys.argv[1] if len(sys.argv) > 1 else "cfg2", 0, 1, 0)
G.to(dev)
hps = bench._HPS(2)
torch.manual_seed(1)
embed = torch.nn.Embedding(hps.vocab_size, 300, padding_idx=0)
embed.weight.requires_grad = False
model = HiGraph.HSumGraph(hps, embed).to(dev).train()
opt = torch.optim.Adam([p for p in model.parameters() if p.requires_grad], lr=hps.lr)
crit = torch.nn.CrossEntropyLoss(reduction="none")
T = {}


def tick(name, t0):
    torch.cuda.synchronize()
    t = time.perf_counter()
    T[name] = T.get(name, 0.0) + (t - t0) * 1e3
    return t


def step(n):
    t = time.perf_counter()
    w = model.set_wnfeature(G)
    t = tick("set_wnfeature", t)
    snode_id = HiGraph.node_ids(G, "dtype", 1.0)
    ngram, cnn = model._sent_cnn_feature(G, snode_id)
    t = tick("cnn", t)
    glen = HiGraph.sentence_counts(G)
    lstm = model._sent_lstm_rows(ngram, glen)
    t = tick("lstm", t)
    s = model.n_feature_proj(torch.cat([cnn, lstm], dim=1))
    st = model.gat_stack(G, w, s)
    out = model.wh(st)
    t = tick("gat_stack", t)
    sid = G.filter_nodes(lambda nodes: nodes.data["dtype"] == 1)
    label = G.ndata["label"][sid].sum(-1)
    G.nodes[sid].data["loss"] = crit(out, label).unsqueeze(-1)
    loss = hg.sum_nodes(G, "loss").mean()
    ok = bool(torch.isfinite(loss).item())
    t = tick("loss", t)
    opt.zero_grad()
    loss.backward()
    t = tick("backward", t)
    opt.step()
    t = tick("adam", t)
    G.ndata.pop("loss")


for _ in range(3):
    step(0)
T.clear()
N = 10
for _ in range(N):
    step(0)
print({k: round(v / N, 3) for k, v in T.items()}, "total", round(sum(T.values()) / N, 3), flush=True)
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for _ in range(3):
        step(0)
print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25))
print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))
for name in ("aten::copy_", "aten::fill_", "hipDeviceSynchronize", "aten::nonzero", "aten::item"):
    print("=====", name)
    rows = [e for e in prof.key_averages(group_by_stack_n=6) if e.key == name]
    for e in sorted(rows, key=lambda e: -e.count)[:6]:
        print(e.count, "calls;", " <- ".join(fr.split("/")[-1] for fr in e.stack[:6]))
