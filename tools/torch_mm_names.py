"""Dev tool (GPU, under rocprofv3 --kernel-trace): torch.mm on the S2W FFN shapes, to
read the hipBLASLt kernel names (macro tile, MFMA shape, depth) from the trace."""
import torch
shapes = [(19200, 512, 300, 0, 1), (19200, 300, 512, 0, 1), (19200, 512, 300, 0, 0), (19200, 300, 512, 0, 0)]
for M, N, K, a_t, b_t in shapes:
    A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
    At, Bt = (A.t() if a_t else A), (B.t() if b_t else B)
    for _ in range(5):
        torch.mm(At, Bt)
    torch.cuda.synchronize()
print("done")
