"""Dev tool: the step's FFN GEMM shapes under hsg_gemm_f32 (3-limb bf16 split, each
k_gemm3 tile plan), hsg_gemm_f32_mfma (exact-f32 instruction) and torch.mm
(hipBLASLt): time (HIP events, 20 back-to-back launches) and error vs fp64 scaled by
sum_k |a||b| (the fp32 dot-product error unit).

usage: python tools/gemm3_sweep.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm  # noqa: E402

SHAPES = [
    ("s2w ffn1 x.W1^T", 19200, 512, 300, 0, 1, "relu"),
    ("s2w ffn2 h.W2^T", 19200, 300, 512, 0, 1, "bias"),
    ("s2w dH = dy.W2", 19200, 512, 300, 0, 0, "mask"),
    ("s2w dx += dH.W1", 19200, 300, 512, 0, 0, "add"),
    ("s2w dW2 = dy^T.H", 300, 512, 38400, 1, 0, ""),
    ("s2w dW1 = dH^T.x", 512, 300, 38400, 1, 0, ""),
    ("w2s hproj-like", 19200, 64, 300, 0, 1, ""),
    ("cnn taps", 112000, 1350, 300, 0, 1, ""),
]


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


def main():
    torch.manual_seed(0)
    for name, M, N, K, a_t, b_t, epi in SHAPES:
        A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
        B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
        out = torch.empty(M, N, device="cuda")
        kw = {}
        if epi == "relu":
            kw = dict(bias=torch.randn(N, device="cuda"), relu=True)
        elif epi == "bias":
            kw = dict(bias=torch.randn(N, device="cuda"))
        elif epi == "mask":
            kw = dict(relu_mask=torch.randn(M, N, device="cuda"), splits=1)
        elif epi == "add":
            kw = dict(add=torch.randn(M, N, device="cuda"))
        a64 = (A.t() if a_t else A).double()
        b64 = (B.t() if b_t else B).double()
        ref = a64 @ b64
        unit = a64.abs() @ b64.abs()
        flops = 2.0 * M * N * K
        row = [f"{name:18s} {M:6d}x{N:4d}x{K:5d}"]
        variants = [("mfma", "f32mfma", None, "0")] + [(f"x3t{t}", "f32", str(t), "0") for t in (0, 1)] + \
            [(f"v{v}t{t}", "f32", str(t), str(v)) for v in (1, 2, 3, 4) for t in (0, 1)]
        for tag, dt, tile, var in variants:
            os.environ["HSG_GEMM3_VAR"] = var
            if tile is None:
                os.environ.pop("HSG_GEMM3_TILE", None)
            else:
                os.environ["HSG_GEMM3_TILE"] = tile
            us = timed(lambda: gemm(A, B, bool(a_t), bool(b_t), out=out, dtype=dt, **kw))
            gemm(A, B, bool(a_t), bool(b_t), out=out, dtype=dt)          # plain product for the error
            err = ((out.double() - ref).abs() / unit.clamp_min(1e-30)).max().item()
            row.append(f"{tag} {us:6.1f} {flops / us / 1e6:5.1f}TF e{err:.0e}")
        os.environ.pop("HSG_GEMM3_TILE", None)
        os.environ.pop("HSG_GEMM3_VAR", None)
        at, bt = (A.t() if a_t else A), (B.t() if b_t else B)
        us = timed(lambda: torch.mm(at, bt, out=out))
        row.append(f"torch {us:7.1f}us {flops / us / 1e6:6.1f}TF")
        print(" | ".join(row[:4]), flush=True)
        print("      " + " | ".join(row[4:]), flush=True)


if __name__ == "__main__":
    main()
