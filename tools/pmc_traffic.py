"""HBM traffic of the roofline kernel (S2W hsg_gat_fwd) from rocprofv3 PMC passes,
over IN-STEP launches: the workload is the bench's own training step (eager, train
mode, cfg2), so each counted dispatch runs after its real predecessors, with the
cache state they leave (not back-to-back repeats of one launch over a working set
the 256 MiB Infinity Cache holds).

Counters are collected in two SEPARATE passes, FETCH_SIZE and WRITE_SIZE (they do
not fit one pass on gfx950), each run with --pmc only (no trace domains):

  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python tools/pmc_traffic.py run
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python tools/pmc_traffic.py run
  python tools/pmc_traffic.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/pmc_traffic.json

The workload first runs a calibration copy of a known byte count (a 256 MiB
device-to-device copy_, one read + one write per element, far beyond the 256 MiB
Infinity Cache's residency for a streamed pair), so the counter units and the
gfx950 FETCH_SIZE half-count (MI355X_MICROARCH.md §HBM) are corrected from a
measurement rather than assumed.  The S2W launches are the k_gat_fwd dispatches
with the largest grid (19,200 word destinations vs 1,120 sentences).  bench.py
reports the resulting bytes/launch as roofline.traffic.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CAL_BYTES = 256 << 20
STEPS = 6


def run():
    import torch
    import bench
    from hetersumgraph_amd import rng as hsg_rng
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    # calibration: 256 MiB read + 256 MiB write
    a = torch.empty(CAL_BYTES // 4, device=dev)
    b = torch.empty_like(a).normal_()
    for _ in range(3):
        a.copy_(b)
    torch.cuda.synchronize()
    del a, b
    docs, G, _, _ = bench.make_shard("cfg2", 0, 1, 0)
    G.to(dev)
    torch.manual_seed(0)
    stack = bench.Stack(0.1, 2).to(dev).train()
    rel_w, rel_s = G.relation("W2S"), G.relation("S2W")
    gen = torch.Generator(device=dev).manual_seed(0)
    Xw = 0.4 * torch.randn(rel_s.n_dst, 300, device=dev, generator=gen)
    Xs = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen).requires_grad_()
    R = torch.randn(rel_w.n_dst, 64, device=dev, generator=gen)
    for _ in range(STEPS):
        for p in stack.parameters():
            p.grad = None
        hsg_rng.advance_all()
        stack(G, Xw, Xs).backward(R)
    torch.cuda.synchronize()
    H, D = stack.sent2word.layer.num_heads, stack.sent2word.layer.head_dim
    print("algorithmic_bytes", bench.edge_bytes_fwd(rel_s, H, D))


def _collect(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    gat = [r for r in rows if "k_gat_fwd" in r["Kernel_Name"]]
    big = max(int(r["Grid_Size"]) for r in gat)
    gat = [float(r["Counter_Value"]) for r in gat if int(r["Grid_Size"]) == big]
    cal = [float(r["Counter_Value"]) for r in rows if "copy" in r["Kernel_Name"].lower()
           or "elementwise" in r["Kernel_Name"]]
    return gat, cal


def parse(dfetch, dwrite, out_json):
    gf, cf = _collect(dfetch, "FETCH_SIZE")
    gw, cw = _collect(dwrite, "WRITE_SIZE")
    # calibration launches: the three big copies are the largest values
    cf, cw = sorted(cf)[-3:], sorted(cw)[-3:]
    f_scale = CAL_BYTES / (sum(cf) / len(cf))
    w_scale = CAL_BYTES / (sum(cw) / len(cw))
    fetch = sum(gf) / len(gf) * f_scale
    write = sum(gw) / len(gw) * w_scale
    res = {"kernel": "hsg_gat_fwd (S2W, cfg2), in-step launches", "launches": len(gf), "fetch_bytes": fetch,
           "write_bytes": write,
           "traffic_bytes": fetch + write, "fetch_unit_scale": f_scale, "write_unit_scale": w_scale,
           "calibration": f"{CAL_BYTES} B device copy_ (read {CAL_BYTES} B + write {CAL_BYTES} B)"}
    with open(out_json, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(*sys.argv[2:5])
