"""Dev tool: time hsg_gemm_f32 on the FFN shapes of one WSWGAT step under env
variants (HSG_GEMM_*), next to torch.mm (hipBLASLt/rocBLAS) on the same shape.

usage: python tools/gemm_bench.py [VAR=a,b ...]    e.g. HSG_GEMM_XCD=0,1
"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm  # noqa: E402

# (name, M, N, K, a_t, b_t, epilogue)
SHAPES = [
    ("s2w ffn1 x.W1^T", 19200, 512, 300, 0, 1, "relu"),
    ("s2w ffn2 h.W2^T", 19200, 300, 512, 0, 1, "bias"),
    ("s2w dH = dy.W2", 19200, 512, 300, 0, 0, "mask"),
    ("s2w dx += dH.W1", 19200, 300, 512, 0, 0, "add"),
    ("s2w dW2 = dy^T.H", 300, 512, 19200, 1, 0, ""),
    ("s2w dW1 = dH^T.x", 512, 300, 19200, 1, 0, ""),
    ("w2s ffn1", 1120, 512, 64, 0, 1, "relu"),
    ("w2s ffn2", 1120, 64, 512, 0, 1, "bias"),
    ("w2s dW2", 64, 512, 1120, 1, 0, ""),
]


def run(sh, reps=30):
    name, M, N, K, a_t, b_t, epi = sh
    A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
    bias = torch.randn(N, device="cuda")
    aux = torch.randn(M, N, device="cuda")
    out = torch.empty(M, N, device="cuda")
    kw = {}
    if epi == "relu":
        kw = dict(bias=bias, relu=True)
    elif epi == "bias":
        kw = dict(bias=bias)
    elif epi == "mask":
        kw = dict(relu_mask=aux, splits=1)
    elif epi == "add":
        kw = dict(add=aux)
    f = lambda: gemm(A, B, bool(a_t), bool(b_t), out=out, **kw)
    ref = (A.t() if a_t else A).double() @ (B.t() if b_t else B).double()
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    # correctness of the plain product part
    if epi == "":
        err = (out.double() - ref).abs().max().item() / ref.abs().max().item()
    else:
        err = float("nan")
    return us, 2 * M * N * K / us / 1e6, err


def run_torch(sh, reps=30):
    name, M, N, K, a_t, b_t, epi = sh
    A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
    At, Bt = (A.t() if a_t else A), (B.t() if b_t else B)
    for _ in range(3):
        torch.mm(At, Bt)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.mm(At, Bt)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / reps * 1e3
    return us, 2 * M * N * K / us / 1e6


def main():
    variants = []
    for a in sys.argv[1:]:
        k, v = a.split("=")
        variants.append([(k, x) for x in v.split(",")])
    combos = list(itertools.product(*variants)) or [()]
    for sh in SHAPES:
        cells = []
        for combo in combos:
            for k, v in combo:
                os.environ[k] = v
            us, tf, err = run(sh)
            tag = ",".join(f"{k[9:]}={v}" for k, v in combo)
            cells.append(f"{tag} {us:6.1f}us {tf:5.1f}TF" + (f" err {err:.1e}" if err == err else ""))
        tus, ttf = run_torch(sh)
        print(f"{sh[0]:20s} | " + " | ".join(cells) + f" | torch.mm {tus:6.1f}us {ttf:5.1f}TF", flush=True)


if __name__ == "__main__":
    main()
