"""Dev tool: the cfg2 W2S head-projection dW (n = 19,200, in = 300, H = 8, D = 8) as the
stack runs it (partial slabs only), 200 back-to-back launches; HSG_HPROJ_DWMF=0 (dev
library) selects the 16x16x4 kernel."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hetersumgraph_amd._lib import load, ptr, stream_of
from hetersumgraph_amd.hproj import dropmask_bits

lib = load()
n, d_in, H, D, p = 19200, 300, 8, 8, 0.1
X = torch.randn(n, d_in, device="cuda")
dZ = torch.randn(n, H * D, device="cuda")
bits = dropmask_bits(X, H, p)
chunks = lib.hsg_hproj_dw_chunks(n, d_in, H, D)
part = torch.empty(chunks * H * D * d_in, device="cuda")
st = stream_of(X)
f = lambda: lib.hsg_hproj_dw(n, d_in, H, D, ptr(dZ), H * D, ptr(X), d_in, ptr(bits), p, ptr(part), None, 0, st)
for _ in range(10):
    assert f() == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    f()
e1.record()
torch.cuda.synchronize()
print(os.environ.get("HSG_HPROJ_DWMF", "default"), f"dw {e0.elapsed_time(e1) / 200 * 1e3:.2f}us", flush=True)
