"""Dev tool: time every hsg_gemm tile config (HSG_GEMM_TILE) on the FFN shapes."""
import os, sys, subprocess
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) > 1:
    import torch
    from hetersumgraph_amd.dense import gemm
    M, N, K, a_t, b_t, sp = (int(x) for x in sys.argv[1:7])
    A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
    f = lambda: gemm(A, B, bool(a_t), bool(b_t), splits=sp)
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): f()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{us:8.1f} us {2*M*N*K/us/1e6:6.1f} TF")
    sys.exit(0)
shapes = [(19200, 512, 300, 0, 1, 1), (19200, 300, 512, 0, 1, 1), (19200, 512, 300, 0, 0, 1),
          (19200, 300, 512, 0, 0, 1), (300, 512, 19200, 1, 0, 16), (300, 512, 19200, 1, 0, 32),
          (512, 300, 19200, 1, 0, 16), (1120, 512, 64, 0, 1, 0), (1120, 64, 512, 0, 1, 0),
          (64, 512, 1120, 1, 0, 0), (512, 64, 1120, 1, 0, 0)]
for sh in shapes:
    res = []
    for tile in (2, 4, 5, 6, 7, 8, 9):
        env = dict(os.environ, HSG_GEMM_TILE=str(tile))
        out = subprocess.run([sys.executable, __file__] + [str(x) for x in sh], env=env, capture_output=True,
                             text=True, timeout=120).stdout.strip().splitlines()
        res.append(out[-1] if out else "fail")
    print(sh, " | ".join(res), flush=True)
