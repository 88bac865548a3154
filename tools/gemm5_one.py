"""Dev tool: run the S2W ffn1 GEMM (19200x512x300) on hsg_gemm_f32_psw 20 times (for
rocprofv3 --pmc passes; plan from HSG_GEMM5)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm_psw, split_weights  # noqa: E402

x = torch.randn(19200, 300, device="cuda")
W1 = torch.randn(512, 300, device="cuda")
(s1,) = split_weights((W1, False))
out = torch.empty(19200, 512, device="cuda")
for _ in range(20):
    gemm_psw(x, s1, out=out)
torch.cuda.synchronize()
print("done")
