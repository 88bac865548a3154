"""Dev tool: the S2W FFN GEMMs (forward x.W1^T, h.W2^T; backward dy.W2, dH.W1) on
hsg_gemm_f32 (k_gemm3) vs hsg_gemm_f32_psw (k_gemm5, pre-split weight) under each
HSG_GEMM5 plan, plus the hsg_wsplit launch of the four weight views: time (HIP
events, 20 back-to-back launches) and max error vs fp64 scaled by max |ref|."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm_dtype, gemm_psw, split_weights  # noqa: E402

# BF16=1: the bf16-mode kernel (hsg_gemm_bf16_psw) under HSG_GEMM7B plans instead
BF16 = os.environ.get("BF16") == "1"
# 34-38: k_gemm7 dev diagnostics (no C store / no MFMA / loads only / A only / B only)
PLANS = {"27": "g7 64 lds RNE prefetch", "34": "dev: no C store", "35": "dev: no MFMA", "36": "dev: loads only",
         "37": "dev: A loads only", "38": "dev: B loads only"}
if os.environ.get("PLANS"):                 # e.g. PLANS=27,40,41
    PLANS = {k: f"plan {k}" for k in os.environ["PLANS"].split(",")}
if BF16:
    PLANS = {"0": "default (128 | 64 by N)", "9": "64 S2", "3": "128 S2"}
ENV = "HSG_GEMM7B" if BF16 else "HSG_GEMM5"


def timed(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


n, d, dh = int(os.environ.get("ROWS", 19200)), 300, 512
if BF16:
    from hetersumgraph_amd.dense import set_gemm_dtype  # noqa: E402
    set_gemm_dtype("bf16")
W1 = torch.randn(dh, d, device="cuda") * 0.05
W2 = torch.randn(d, dh, device="cuda") * 0.05
x = torch.randn(n, d, device="cuda")
H = torch.randn(n, dh, device="cuda")
dy = torch.randn(n, d, device="cuda")
us = timed(lambda: split_weights((W1, False), (W2, False), (W2, True), (W1, True)))
print(f"hsg_wsplit x4: {us:.1f} us", flush=True)
s1, s2, s2t, s1t = split_weights((W1, False), (W2, False), (W2, True), (W1, True))
cases = [("ffn1 x.W1^T", x, W1, True, s1), ("ffn2 h.W2^T", H, W2, True, s2),
         ("dH = dy.W2", dy, W2, False, s2t), ("dx = dH.W1", H, W1, False, s1t)]
ROUNDS = int(os.environ.get("ROUNDS", 5))
for name, A, W, b_t, S in cases:
    Ar, Wr = (A.bfloat16(), W.bfloat16()) if BF16 else (A, W)
    ref = Ar.double() @ (Wr.double().t() if b_t else Wr.double())
    M, N = ref.shape
    K = A.shape[1]
    out = torch.empty(M, N, device="cuda")
    times = {g5: [] for g5 in PLANS}
    errs = {}
    for _ in range(ROUNDS):                 # plans interleaved: box drift hits all alike
        for g5 in PLANS:
            os.environ[ENV] = g5
            times[g5].append(timed(lambda: gemm_psw(A, S, out=out)))
            if g5 not in errs:
                errs[g5] = ((out.double() - ref).abs().max() / ref.abs().max()).item()
    os.environ.pop(ENV, None)
    print(f"{name:14s} {M}x{N}x{K}", flush=True)
    for g5, tag in PLANS.items():
        t = sorted(times[g5])
        med = t[len(t) // 2]
        print(f"      {tag:18s} median {med:6.1f} us  min {t[0]:6.1f}  {2 * M * N * K / med / 1e6:6.1f} TF "
              f"err {errs[g5]:.1e}", flush=True)
