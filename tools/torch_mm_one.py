"""Dev tool: torch.mm (hipBLASLt) on one shape, for kernel-name / timing comparison."""
import sys
import torch
M, N, K, a_t, b_t = (int(x) for x in sys.argv[1:6])
A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
At = A.t() if a_t else A
Bt = B.t() if b_t else B
for _ in range(10):
    torch.mm(At, Bt)
torch.cuda.synchronize()
