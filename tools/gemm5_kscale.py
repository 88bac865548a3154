"""Dev tool: hsg_gemm_f32_psw (plan HSG_GEMM5, default 1) time vs K at M=19200,
N=512 -- separates the per-K-tile cost from the fixed (prologue + epilogue) cost;
plus a 39 MB fill for the output-write floor."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm, gemm_psw, split_weights  # noqa: E402


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


M, N = 19200, 512
out = torch.empty(M, N, device="cuda")
print(f"fill 39 MB: {timed(lambda: out.fill_(1.0)):.1f} us", flush=True)
for plan in ("1", "2"):
    os.environ["HSG_GEMM5"] = plan
    for K in (32, 64, 128, 300, 600, 1200):
        A = torch.randn(M, K, device="cuda")
        W = torch.randn(N, K, device="cuda")
        (S,) = split_weights((W, False))
        us = timed(lambda: gemm_psw(A, S, out=out))
        us3 = timed(lambda: gemm(A, W, b_t=True, out=out))
        print(f"plan {plan} K {K:5d}: psw {us:6.1f} us  gemm3 {us3:6.1f} us", flush=True)
