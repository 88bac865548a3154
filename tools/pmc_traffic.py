"""HBM traffic of the roofline kernel (S2W hsg_gat_fwd) from rocprofv3 PMC passes.

Counters are collected in two SEPARATE passes, FETCH_SIZE and WRITE_SIZE (they do
not fit one pass on gfx950), each run with --pmc only (no trace domains):

  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python tools/pmc_traffic.py run
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python tools/pmc_traffic.py run
  python tools/pmc_traffic.py parse gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/r01_pmc_traffic.json

The workload also runs a calibration copy of a known byte count (a 256 MiB
device-to-device copy_, one read + one write per element, far beyond the 256 MiB
Infinity Cache's residency for a streamed pair), so the counter units and the
gfx950 FETCH_SIZE half-count (MI355X_MICROARCH.md §HBM) are corrected from a
measurement rather than assumed.  bench.py reports the resulting bytes/launch as
roofline.traffic.
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CAL_BYTES = 256 << 20
REPS = 20


def run():
    import ctypes
    import torch
    import bench
    from hetersumgraph_amd import _lib
    from hetersumgraph_amd.module.GATLayer import edge_tau
    lib = _lib.load()
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
    stack = bench.Stack(0.1, 2).to(dev)
    rel = G.relation("S2W")
    layer = stack.sent2word.layer
    H, D = layer.num_heads, layer.head_dim
    gen = torch.Generator(device=dev).manual_seed(0)
    Xw = 0.4 * torch.randn(rel.n_dst, 300, device=dev, generator=gen)
    Xs = torch.randn(rel.n_src, 64, device=dev, generator=gen)
    from hetersumgraph_amd.HiGraph import register_tfidf_table
    register_tfidf_table(G, stack._TFembed.weight)
    with torch.no_grad():
        W, attn, wf, bf = layer.fused_params()
        a1, a3 = attn[:, :D].contiguous(), attn[:, 2 * D:]
        Z = torch.nn.functional.linear(Xs, W).contiguous()
        tau, mode = edge_tau(G, rel, a3, wf, bf)
        tau = tau.contiguous()
        sigma = Z.new_empty(rel.n_src, H)
        h = Xw.new_empty(rel.n_dst, H * D)
        out = torch.empty_like(h)
        m = Z.new_empty(rel.n_dst, H)
        l = Z.new_empty(rel.n_dst, H)
        st = torch.cuda.current_stream().cuda_stream
        relp = ctypes.byref(rel.cstruct())
        _lib.check(lib.hsg_attn_src_logits(rel.n_src, H, D, Z.data_ptr(), a1.data_ptr(), sigma.data_ptr(), st),
                   "sigma")
        for _ in range(REPS):
            _lib.check(lib.hsg_gat_fwd(relp, H, D, mode, 0.01, Z.data_ptr(), sigma.data_ptr(), tau.data_ptr(),
                                       Xw.data_ptr(), h.data_ptr(), out.data_ptr(), m.data_ptr(), l.data_ptr(),
                                       st), "fwd")
        torch.cuda.synchronize()
    print("algorithmic_bytes", bench.algorithmic_bytes_fwd(rel, H, D))


def _collect(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter]
    gat = [float(r["Counter_Value"]) for r in rows if "k_gat_fwd" in r["Kernel_Name"]]
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
    res = {"kernel": "hsg_gat_fwd (S2W, cfg2)", "launches": len(gf), "fetch_bytes": fetch, "write_bytes": write,
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
