"""Dev tool: run one FFN-shaped GEMM a few times (for rocprofv3 --pmc passes).
usage: python tools/gemm_one_run.py M N K a_t b_t dtype [tile]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm  # noqa: E402

M, N, K, a_t, b_t = (int(x) for x in sys.argv[1:6])
dt = sys.argv[6]
if len(sys.argv) > 7:
    os.environ["HSG_GEMM3_TILE"] = sys.argv[7]
A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
out = torch.empty(M, N, device="cuda")
for _ in range(5):
    gemm(A, B, bool(a_t), bool(b_t), out=out, dtype=dt)
torch.cuda.synchronize()
