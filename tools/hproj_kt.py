"""Dev tool (GPU, under rocprofv3 --kernel-trace --stats): the W2S head projection
forward (n = 19,200, in = 300, H = 8, D = 8, with the fused source logits) 30 times per
environment variant given on the command line ('VAR=a,VAR2=b'; '' = defaults), and the
dX / dW kernels 30 times each under the defaults."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.hproj import hproj_bwd, hproj_fwd  # noqa: E402


def main(variants):
    X = torch.randn(19200, 300, device="cuda")
    W = torch.randn(64, 300, device="cuda")
    a1 = torch.randn(8, 8, device="cuda")
    scrub = torch.empty(512 * 2**20 // 4, device="cuda")
    for v in variants or [""]:
        for k in [k for k in os.environ if k.startswith("HSG_")]:
            del os.environ[k]
        for kv in filter(None, v.split(",")):
            a, b = kv.split("=", 1)
            os.environ[a] = b
        for _ in range(30):
            scrub.fill_(1.0)                      # evict X from the caches between launches
            Z, saved, sigma = hproj_fwd(X, W, 8, 8, 0.1, a1=a1)
    for k in [k for k in os.environ if k.startswith("HSG_")]:
        del os.environ[k]
    dZ = torch.randn_like(Z)
    dX, dW = torch.empty_like(X), torch.empty_like(W)
    for _ in range(30):
        scrub.fill_(1.0)
        hproj_bwd(saved, dZ, dX=dX)
    for _ in range(30):
        scrub.fill_(1.0)
        hproj_bwd(saved, dZ, dW=dW)
    # the S2W shape (n = 1,120, in = 64, H = 6, D = 50)
    Xs = torch.randn(1120, 64, device="cuda")
    Ws = torch.randn(300, 64, device="cuda")
    Zs, saved_s = hproj_fwd(Xs, Ws, 6, 50, 0.1)
    dZs = torch.randn_like(Zs)
    dXs = torch.empty_like(Xs)
    for _ in range(30):
        scrub.fill_(1.0)
        hproj_bwd(saved_s, dZs, dX=dXs)
    for v in variants or [""]:
        for k in [k for k in os.environ if k.startswith("HSG_")]:
            del os.environ[k]
        for kv in filter(None, v.split(",")):
            a, b = kv.split("=", 1)
            os.environ[a] = b
        for _ in range(30):
            scrub.fill_(1.0)
            hproj_bwd(saved, dZ, dX=dX)
            hproj_bwd(saved_s, dZs, dX=dXs)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main(sys.argv[1:])
