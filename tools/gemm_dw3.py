"""Dev tool: the step's weight-gradient GEMMs (dW = dY^T X, both operands
M/N-contiguous) on the exact-f32 MFMA kernel vs the 3-limb split kernel with
transpose-read staging under each tile plan (HSG_GEMM3_TILE; VAR 3 = one-limb
probe of the same pipeline), per split count; HIP-event timed (20
back-to-back launches) with the max relative error against a float64 product."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm  # noqa: E402

SHAPES = [("s2w dW2 = dy^T.H", 300, 512, 38400), ("s2w dW1 = dH^T.x", 512, 300, 38400),
          ("w2s dW2", 64, 512, 3360), ("w2s dW1", 512, 64, 3360)]


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
    A = torch.randn(K, M, device="cuda")
    B = torch.randn(K, N, device="cuda")
    ref = A.double().t() @ B.double()
    out = torch.empty(M, N, device="cuda")
    row = [f"{name:18s}"]
    variants = [("mfma", {}, "f32mfma")] + [(f"x3t{t}{'v' + v if v else ''}", {"HSG_GEMM3_TILE": t, "HSG_GEMM3_VAR": v},
                                             "f32") for t in ("0", "1", "3") for v in ("5", "6")]
    for tag, env, dt in variants:
        for k, v in env.items():
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
        for sp in (0, 8, 16, 32):
            us = timed(lambda: gemm(A, B, a_t=True, out=out, splits=sp, dtype=dt))
            err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
            row.append(f"{tag}/s{sp}:{us:.0f}us,{err:.0e}")
        for k in env:
            os.environ.pop(k, None)
    print(f"{name:18s}", flush=True)
    for i in range(1, len(row), 4):
        print("   " + " ".join(row[i:i + 4]), flush=True)
