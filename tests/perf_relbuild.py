"""Timing script (GPU; tests/ may use the oracle as a baseline; not collected by pytest): time hsg_rel_build (device) for the cfg2 batch against the numpy
restatement oracle.fused.typed_relation + CSR/CSC sorts (host)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np
import torch
from hetersumgraph_amd import synth
from hetersumgraph_amd.relation import build_relation
from test_gpu_relbuild import batch, expected

dev = torch.device("cuda", 0)
for cfg in ("cfg2", "cfg5"):
    b = batch(synth.make_batch_docs(cfg, seed=0))
    t = {k: torch.as_tensor(v, device=dev) for k, v in b.items()}
    for _ in range(3):
        build_relation("W2S", t["src"], t["dst"], t["unit"], t["tffrac"], t["edtype"])
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        for kind in ("W2S", "S2W"):
            build_relation(kind, t["src"], t["dst"], t["unit"], t["tffrac"], t["edtype"])
    torch.cuda.synchronize()
    dt_dev = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(3):
        for kind in ("W2S", "S2W"):
            expected(kind, b["src"], b["dst"], b["unit"], b["tffrac"], b["edtype"])
    dt_host = (time.perf_counter() - t0) / 3
    print(f"{cfg}: E={len(b['src'])} n={len(b['unit'])} both relations: device {dt_dev*1e3:.3f} ms "
          f"(incl. one readback each), numpy {dt_host*1e3:.3f} ms")
