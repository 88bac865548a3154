"""Dev A/B: the resident-B FFN GEMM (k_gemm12) against k_gemm7 on the cfg2 wide FFN
shapes with K <= 320 (ffn1 x.W1^T + b1, ReLU; dH = (dy.W2) * (H > 0) + db1 partials).
Needs the dev library (HSG_LIB_PATH=.../libhsg_dev.so): HSG_GEMM12=1 selects k_gemm12.
Prints bitwise equality of C, the column-sum difference, and interleaved timings."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from hetersumgraph_amd.dense import gemm_psw, psw_row_tiles, split_weights  # noqa: E402


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


def with_env(v, f):
    old = os.environ.get("HSG_GEMM12")
    os.environ["HSG_GEMM12"] = v
    try:
        return f()
    finally:
        if old is None:
            del os.environ["HSG_GEMM12"]
        else:
            os.environ["HSG_GEMM12"] = old


n, d, dh = int(os.environ.get("ROWS", 19200)), 300, 512
torch.manual_seed(0)
W1 = torch.randn(dh, d, device="cuda") * 0.05
W2 = torch.randn(d, dh, device="cuda") * 0.05
b1 = torch.randn(dh, device="cuda") * 0.1
x = torch.randn(n, d, device="cuda")
H = torch.relu(torch.randn(n, dh, device="cuda"))
dy = torch.randn(n, d, device="cuda")
s1, s2t = split_weights((W1, False), (W2, True))
for name, run in (("ffn1", lambda out, part: gemm_psw(x, s1, bias=b1, relu=True, out=out)),
                  ("dH", lambda out, part: gemm_psw(dy, s2t, relu_mask=H, colsum_part=part, out=out))):
    outs, parts = {}, {}
    for v in ("1", "0"):
        rt = with_env(v, lambda: psw_row_tiles(n, dh, d))
        out = torch.empty(n, dh, device="cuda")
        part = torch.empty(rt, dh, device="cuda")
        with_env(v, lambda: run(out, part))
        torch.cuda.synchronize()
        outs[v], parts[v] = out, part.sum(0)
    ref = (x.double() @ W1.double().t() + b1.double()).relu() if name == "ffn1" else \
        (dy.double() @ W2.double()) * (H > 0)
    eq = torch.equal(outs["1"], outs["0"])
    err = ((outs["1"].double() - ref).abs().max() / ref.abs().max()).item()
    cs = (parts["1"] - parts["0"]).abs().max().item() if name == "dH" else 0.0
    print(f"{name}: k_gemm12 == k_gemm7 bitwise {eq}; err vs fp64 {err:.2e}; colsum max|diff| {cs:.2e}", flush=True)
    out = torch.empty(n, dh, device="cuda")
    part = torch.empty(max(psw_row_tiles(n, dh, d), (n + 63) // 64), dh, device="cuda")
    # variants: "pd,iglp" of k_gemm12 (HSG_GEMM12_IGLP; pd named the A prefetch depth of the
    # earlier ring versions, profiles/r06/g12/; the pipelined kernel has none), "g7" = k_gemm7
    variants = os.environ.get("VARIANTS", "4,0;g7").split(";")
    t = {v: [] for v in variants}
    for _ in range(5):
        for v in variants:
            if v == "g7":
                t[v].append(with_env("0", lambda: timed(lambda: run(out, part))))
            else:
                pd, ig = v.split(",")
                os.environ["HSG_GEMM12_PD"], os.environ["HSG_GEMM12_IGLP"] = pd, ig
                t[v].append(with_env("1", lambda: timed(lambda: run(out, part))))
    print(f"{name}: " + "  ".join(f"[{v}] {sorted(t[v])[2]:.1f} us" for v in variants), flush=True)
