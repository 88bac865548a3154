"""Dev tool: hsg_gemm_f32_psw time vs M on the two cfg2 FFN shapes, to see whether
the 128x64-tile grid pays for whole rounds of resident blocks (2 per CU = 512
slots): ffn1/dH (N = 512, K = 300) and ffn2/dx (N = 300, K = 512)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm_psw, split_weights  # noqa: E402


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


for N, K in ((512, 300), (300, 512)):
    W = torch.randn(N, K, device="cuda")
    (S,) = split_weights((W, False))
    tn = (N + 63) // 64
    for M in (4096, 8192, 12288, 13056, 16384, 19200, 24576, 26112, 32768):
        A = torch.randn(M, K, device="cuda")
        out = torch.empty(M, N, device="cuda")
        us = timed(lambda: gemm_psw(A, S, out=out))
        tiles = (M + 127) // 128 * tn
        print(f"N {N} K {K} M {M:6d}: tiles {tiles:5d} ({tiles / 512:4.2f} rounds of 512)  {us:6.1f} us  "
              f"{us / tiles * 512:6.2f} us per 512 tiles", flush=True)
