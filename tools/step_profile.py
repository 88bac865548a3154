"""Per-kernel time of ONE bench step (cfg2 by default): run under
    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o step -- python tools/step_profile.py run [cfg]
then
    python tools/step_profile.py parse DIR/step_kernel_trace.csv [REPLAYS]
The run does 3 eager steps, captures the step into a HIP graph and replays it
REPLAYS (100) times; parse keeps only the dispatches of the replays (the last
REPLAYS x kernels-per-step rows) and prints mean microseconds per step per kernel.
"""
import csv
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REPLAYS = 100


def run(config="cfg2"):
    import torch
    import bench
    from hetersumgraph_amd import rng as hsg_rng
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from hetersumgraph_amd.dense import set_gemm_dtype
    set_gemm_dtype(os.environ.get("HSG_PROFILE_DTYPE", "f32"))       # bench.py --dtype
    docs, G, _, _ = bench.make_shard(config, 0, 1, 0)
    G.to(dev)
    torch.manual_seed(0)
    stack = bench.Stack(0.1, 2).to(dev).train()
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device=dev).manual_seed(0)
    Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)
    Xs = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen)
    params = [p for p in stack.parameters()]

    def step():
        hsg_rng.advance_all()
        stack(G, Xw, Xs).backward(R)

    def zero():
        for p in params:
            p.grad = None
        Xs.grad = None

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
    for _ in range(REPLAYS):
        g.replay()
    torch.cuda.synchronize()


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    if "(" in name:
        head = name[:name.index("(")]
        return head.replace("void ", "")
    return name


def parse(path, replays=REPLAYS):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # kernels per step: the replays repeat the same sequence; find the period from the end
    names = [short(r["Kernel_Name"]) for r in rows]
    n = len(names)
    per = None
    for p in range(10, 400):
        if names[n - p:] == names[n - 2 * p:n - p] and names[n - p:] == names[n - 3 * p:n - 2 * p]:
            per = p
            break
    if per is None:
        raise SystemExit("could not find the step period")
    tail = rows[n - replays * per:]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in tail:
        k = short(r["Kernel_Name"])
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[k] += 1
    span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3 / replays
    busy = sum(tot.values()) / replays
    print(f"kernels per step {per}; wall {span:.1f} us/step; kernel busy {busy:.1f} us/step; "
          f"gaps {span - busy:.1f} us/step")
    for k in sorted(tot, key=lambda k: -tot[k]):
        print(f"{tot[k] / replays:9.1f} us  {cnt[k] / replays:5.1f}x  {tot[k] / cnt[k]:8.2f} us/launch  {k}")
    # the step in launch order: mean time of each position (tells the W2S and S2W
    # launches of one kernel apart) and its grid size
    print("\nlaunch order (mean us per position, grid):")
    for i in range(per):
        ds = [(int(tail[j]["End_Timestamp"]) - int(tail[j]["Start_Timestamp"])) / 1e3 for j in range(i, len(tail), per)]
        g = tail[i].get("Grid_Size", tail[i].get("Grid_Size_X", "?"))
        print(f"  {i:3d} {sum(ds) / len(ds):8.2f} us  grid {g:>8}  {short(tail[i]['Kernel_Name'])}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(*sys.argv[2:3])
    else:
        parse(sys.argv[2], *(int(x) for x in sys.argv[3:4]))
