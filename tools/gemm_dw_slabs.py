"""Dev tool: the S2W FFN weight-gradient GEMMs as the stack runs them (gemm_slabs:
split-K slabs, 64 K slices, summed elsewhere) under HSG_GEMM3_VAR variants; HIP-event
timed (20 back-to-back launches, medians of interleaved rounds) with the max relative
error of the slab sum against a float64 product.
usage: VARS=5,7,8 python tools/gemm_dw_slabs.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm_slabs  # noqa: E402

VARS = os.environ.get("VARS", "5,7,8").split(",")
SHAPES = [("s2w dW2 = dy^T.H", 300, 512, 38400), ("s2w dW1 = dH^T.x", 512, 300, 38400)]


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
    times = {v: [] for v in VARS}
    errs = {}
    for _ in range(int(os.environ.get("ROUNDS", 3))):
        for v in VARS:
            os.environ["HSG_GEMM3_VAR"] = v
            times[v].append(timed(lambda: gemm_slabs(A, B, a_t=True)))
            if v not in errs:
                sl, rows = gemm_slabs(A, B, a_t=True)
                got = sl[:rows * M * N].view(rows, M, N).double().sum(0)
                errs[v] = ((got - ref).abs().max() / ref.abs().max()).item()
    os.environ.pop("HSG_GEMM3_VAR", None)
    print(f"{name} {M}x{N}x{K}", flush=True)
    for v in VARS:
        t = sorted(times[v])
        print(f"    var {v}: median {t[len(t) // 2]:7.1f} us  min {t[0]:7.1f}  err {errs[v]:.1e}", flush=True)
