"""Dev tool: hsg_gemm time vs persistent grid size (HSG_GEMM_GRID) and tile (HSG_GEMM_TILE)."""
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
    print(f"{us:7.1f}us {2*M*N*K/us/1e6:5.1f}TF")
    sys.exit(0)
shapes = [(19200, 512, 300, 0, 1, 1), (19200, 300, 512, 0, 1, 1), (300, 512, 19200, 1, 0, 32)]
for tile in (5, 4, 2):
    for sh in shapes:
        res = []
        for g in (100000, 2048, 1536, 1280, 1200, 1024, 768, 512):
            env = dict(os.environ, HSG_GEMM_TILE=str(tile), HSG_GEMM_GRID=str(g))
            out = subprocess.run([sys.executable, __file__] + [str(x) for x in sh], env=env, capture_output=True,
                                 text=True, timeout=120).stdout.strip().splitlines()
            res.append(f"g{g}:" + (out[-1] if out else "fail"))
        print("tile", tile, sh, " | ".join(res), flush=True)
