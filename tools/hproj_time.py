"""Dev tool (GPU): head-projection kernels at the cfg2 W2S shape (n = 19,200 words,
in = 300, H = 8, D = 8) and S2W shape (n = 1,120, in = 64, H = 6, D = 50), timed with
HIP events: hsg_dropmask, hsg_hproj_fwd, hsg_hproj_dx, hsg_hproj_dw."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.hproj import hproj_bwd, hproj_fwd  # noqa: E402


def timed(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    out = {}
    for name, (n, din, H, D) in {"w2s": (19200, 300, 8, 8), "s2w": (1120, 64, 6, 50)}.items():
        X = torch.randn(n, din, device="cuda")
        W = torch.randn(H * D, din, device="cuda")
        Z, saved = hproj_fwd(X, W, H, D, 0.1)
        dZ = torch.randn_like(Z)
        dX, dW = torch.empty_like(X), torch.empty_like(W)
        r = {"fwd_us": timed(lambda: hproj_fwd(X, W, H, D, 0.1)),
             "dx_us": timed(lambda: hproj_bwd(saved, dZ, dX=dX)),
             "dw_us": timed(lambda: hproj_bwd(saved, dZ, dW=dW))}
        r["gflop"] = 2 * n * din * H * D / 1e9
        out[name] = r
    print(json.dumps({"sg": os.environ.get("HSG_HPROJ_SG", "4"), **out}))


if __name__ == "__main__":
    main()
