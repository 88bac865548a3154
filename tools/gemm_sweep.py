"""Dev tool: TFLOP/s of hsg_gemm_f32 vs torch on the WSWGAT stack's GEMM shapes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hetersumgraph_amd.dense import gemm, splits_for

def t(fn, reps=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3

# (name, M, N, K, a_t, b_t)
cases = [("ffn1 fwd  X W1^T", 19200, 512, 300, False, True),
         ("ffn2 fwd  H W2^T", 19200, 300, 512, False, True),
         ("ffn dH = dY W2", 19200, 512, 300, False, False),
         ("ffn dX = dH W1", 19200, 300, 512, False, False),
         ("ffn dW2 = dY^T H", 300, 512, 19200, True, False),
         ("ffn dW1 = dH^T X", 512, 300, 19200, True, False),
         ("w2s fc X W^T", 19200, 64, 300, False, True),
         ("w2s ffn1", 1120, 512, 64, False, True),
         ("w2s ffn2", 1120, 64, 512, False, True)]
for name, M, N, K, a_t, b_t in cases:
    A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
    sp = splits_for(M, N, K) if a_t else 1
    us = t(lambda: gemm(A, B, a_t, b_t, splits=sp))
    At = A.t() if a_t else A
    Bt = B.t() if b_t else B
    ut = t(lambda: torch.mm(At, Bt))
    fl = 2 * M * N * K
    print(f"{name:22s} M={M:6d} N={N:4d} K={K:6d} split={sp:3d}  hsg {us:8.1f} us {fl/us/1e6:6.1f} TF   torch {ut:8.1f} us {fl/ut/1e6:6.1f} TF", flush=True)
