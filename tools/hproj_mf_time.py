"""Dev tool: the cfg2 W2S head-projection forward (n = 19,200, in = 300, H = 8, D = 8),
VALU kernel (hsg_hproj_fwd_t8) against the bf16 limb MFMA kernel (hsg_hproj_fwd_mf),
200 back-to-back launches each, with the fused source logits."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hetersumgraph_amd._lib import load, ptr, stream_of
from hetersumgraph_amd.dense import split_dims, split_weights
from hetersumgraph_amd.hproj import dropmask_bits, transposed_weight

lib = load()
n, d_in, H, D, p = 19200, 300, 8, 8, 0.1
X = torch.randn(n, d_in, device="cuda")
W = torch.randn(H * D, d_in, device="cuda") / d_in ** 0.5
a1 = torch.randn(H, D, device="cuda")
bits = dropmask_bits(X, H, p)
(sw,) = split_weights((W, False))
Np, Kp = split_dims(H * D, d_in)
wt = transposed_weight(W, H, D)
Z = torch.empty(n, H * D, device="cuda")
sg = torch.empty(n, H, device="cuda")
st = stream_of(X)
runs = {
    "t8": lambda: lib.hsg_hproj_fwd_t8(n, d_in, H, ptr(X), d_in, ptr(wt), ptr(bits), p, ptr(Z), H * D, ptr(a1),
                                       ptr(sg), st),
    "mf": lambda: lib.hsg_hproj_fwd_mf(n, d_in, H, ptr(X), d_in, ptr(sw.planes), Np, Kp, ptr(bits), p, ptr(Z),
                                       H * D, ptr(a1), ptr(sg), st),
}
res = []
for name, f in runs.items():
    for _ in range(10):
        assert f() == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        f()
    e1.record()
    torch.cuda.synchronize()
    res.append(f"{name} {e0.elapsed_time(e1) / 200 * 1e3:.2f}us")
print(*res, flush=True)
