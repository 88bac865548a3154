"""Dev tool: run one GEMM shape repeatedly (for rocprofv3 counter passes).
usage: python tools/gemm_one.py M N K a_t b_t [reps] [splits]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hetersumgraph_amd.dense import gemm

M, N, K, a_t, b_t = (int(x) for x in sys.argv[1:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
splits = int(sys.argv[7]) if len(sys.argv) > 7 else 0
A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
for _ in range(reps):
    gemm(A, B, bool(a_t), bool(b_t), splits=splits)
torch.cuda.synchronize()
print("done")
