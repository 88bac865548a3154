"""Dev tool (GPU, for rocprofv3 passes): the W2S head projection (n = 19,200, in = 300,
H = 8, D = 8) forward, dX and dW, 20 times each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.hproj import hproj_bwd, hproj_fwd  # noqa: E402

X = torch.randn(19200, 300, device="cuda")
W = torch.randn(64, 300, device="cuda")
for _ in range(20):
    Z, saved = hproj_fwd(X, W, 8, 8, 0.1)
dZ = torch.randn_like(Z)
dX, dW = torch.empty_like(X), torch.empty_like(W)
for _ in range(20):
    hproj_bwd(saved, dZ, dX=dX)
for _ in range(20):
    hproj_bwd(saved, dZ, dW=dW)
torch.cuda.synchronize()
print("done")
