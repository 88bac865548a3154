"""Dev tool: the step's weight-gradient GEMM shapes (K = all rows of all
applications of a layer) on the exact-f32 MFMA kernel under each tile plan
(HSG_GEMM_TILE) and split count, HIP-event timed (20 back-to-back launches)."""
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
    out = torch.empty(M, N, device="cuda")
    row = [f"{name:18s}"]
    for tile in ("", "0", "1", "3", "4", "5", "7", "9", "11"):
        for sp in (0, 8, 16, 32, 64):
            if tile:
                os.environ["HSG_GEMM_TILE"] = tile
            else:
                os.environ.pop("HSG_GEMM_TILE", None)
            try:
                us = timed(lambda: gemm(A, B, a_t=True, out=out, splits=sp, dtype="f32mfma"))
            except Exception as e:  # noqa: BLE001
                us = float("nan")
            row.append(f"t{tile or '-'}s{sp}:{us:.0f}")
    os.environ.pop("HSG_GEMM_TILE", None)
    print(" ".join(row), flush=True)
