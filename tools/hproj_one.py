"""Dev tool (GPU, for rocprofv3 --pmc passes): the W2S head-projection forward
(n = 19,200, in = 300, H = 8, D = 8) 20 times."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.hproj import hproj_fwd  # noqa: E402

X = torch.randn(19200, 300, device="cuda")
W = torch.randn(64, 300, device="cuda")
for _ in range(20):
    hproj_fwd(X, W, 8, 8, 0.1)
torch.cuda.synchronize()
print("done")
