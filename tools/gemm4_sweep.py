"""Dev tool: the step's K-contiguous FFN GEMMs on k_gemm3 (register-staged split
planes) vs k_gemm4 (LDS-DMA pipeline, fragment-time split) under each HSG_GEMM4
plan: time (HIP events, 20 back-to-back launches) and max error vs fp64 scaled by
max |ref|."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm  # noqa: E402

SHAPES = [("s2w ffn1 x.W1^T", 19200, 512, 300), ("s2w ffn2 h.W2^T", 19200, 300, 512),
          ("w2s hproj-like", 19200, 64, 300), ("cnn taps", 112000, 1350, 300)]
PLANS = {"0": "gemm3", "1": "64x64 S3", "2": "128x64 S3", "3": "64x64 S4", "4": "128x64 S2", "5": "64x64 S2",
         "6": "128x128 S2"}


def timed(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for name, M, N, K in SHAPES:
    X = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda")
    ref = X.double() @ W.double().t()
    out = torch.empty(M, N, device="cuda")
    print(f"{name:18s} {M}x{N}x{K}", flush=True)
    for g4, tag in PLANS.items():
        os.environ["HSG_GEMM4"] = g4
        us = timed(lambda: gemm(X, W, b_t=True, out=out, dtype="f32"))
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        print(f"   {tag:10s} {us:7.1f} us {2 * M * N * K / us / 1e6:6.1f} TF  err {err:.1e}", flush=True)
    os.environ.pop("HSG_GEMM4", None)
