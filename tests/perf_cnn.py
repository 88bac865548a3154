"""Timing script (GPU; tests/ may use the oracle as a baseline; not collected by pytest): sentence CNN encoder fwd+bwd at cfg2 shapes (1,120 sentences x
L = 100 tokens, D = 300, CNN/DM-like lengths U(5, 60)) -- the HIP path
(hetersumgraph_amd.cnn) vs the reference's formulation run through PyTorch/MIOpen on
the same GPU (oracle/cnn.py's direct convolution over the padded input)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from hetersumgraph_amd.cnn import sent_cnn  # noqa: E402
from hetersumgraph_amd.module.PositionEmbedding import get_sinusoid_encoding_table  # noqa: E402
from oracle import cnn as ocnn  # noqa: E402


def timed(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    n, L, V, D = 1120, 100, 50000, 300
    rng = np.random.default_rng(0)
    lens = rng.integers(5, 61, n)
    ids = np.zeros((n, L), np.int64)
    for i, m in enumerate(lens):
        ids[i, :m] = rng.integers(1, V, m)
    ids = torch.from_numpy(ids).cuda()
    torch.manual_seed(0)
    emb = (0.5 * torch.randn(V, D, device="cuda"))
    pos = get_sinusoid_encoding_table(L + 1, D, padding_idx=0).cuda()
    cw = [(torch.randn(50, 1, h, D, device="cuda") / np.sqrt(h * D)).requires_grad_() for h in range(2, 8)]
    cb = [(0.1 * torch.randn(50, device="cuda")).requires_grad_() for _ in range(6)]
    R = torch.randn(n, 300, device="cuda")

    def hip():
        (sent_cnn(ids, emb, pos, cw, cb, padding_idx=0) * R).sum().backward()

    def miopen():
        (ocnn.sent_encoder(ids, emb, pos, cw, cb) * R).sum().backward()

    def hip_fwd():
        with torch.no_grad():
            sent_cnn(ids, emb, pos, cw, cb, padding_idx=0)

    def miopen_fwd():
        with torch.no_grad():
            ocnn.sent_encoder(ids, emb, pos, cw, cb)

    rows = int(lens.sum() + n)
    res = {"sentences": n, "L": L, "gemm_rows": rows,
           "gemm_gflop_fwd": 2 * rows * 1350 * D / 1e9,
           "hip_fwd_ms": timed(hip_fwd), "hip_fwdbwd_ms": timed(hip),
           "torch_miopen_fwd_ms": timed(miopen_fwd), "torch_miopen_fwdbwd_ms": timed(miopen)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
