"""Per-shape kernel times of the six S2W FFN GEMM shapes of a cfg2 step, on the
path the step runs, from a rocprofv3 kernel trace:

  cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
  rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o shapes -- python tools/gemm_shapes.py run
  python tools/gemm_shapes.py parse DIR/.../shapes_kernel_trace.csv > profiles/<round>/gemm_shapes.md

run: each shape REPS times back to back (forward/backward FFN GEMMs on hsg_gemm_f32_psw
with pre-split weights; the weight gradients as the step's 64-slice split-K slabs,
hsg_gemm_f32_slabs, whose sum the step does in its one hsg_slab_reduce launch), with
a 64 MiB buffer write between shapes as a separator."""
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REPS = 20
SHAPES = [("ffn1 x.W1^T + b1, ReLU", 19200, 512, 300), ("ffn2 H.W2^T + b2", 19200, 300, 512),
          ("dH = (dy.W2) * relu'(H)", 19200, 512, 300), ("dx += dH.W1", 19200, 300, 512),
          ("dW2 = dY^T.H (K = 2 applications)", 300, 512, 38400), ("dW1 = dH^T.X", 512, 300, 38400)]
PEAK = 157.3


def run():
    import torch
    from hetersumgraph_amd.dense import gemm_psw, gemm_slabs, split_weights
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    W1 = 0.05 * torch.randn(512, 300, device=dev, generator=g)
    W2 = 0.05 * torch.randn(300, 512, device=dev, generator=g)
    b1, b2 = torch.randn(512, device=dev, generator=g), torch.randn(300, device=dev, generator=g)
    x = torch.randn(19200, 300, device=dev, generator=g)
    H = torch.relu(torch.randn(19200, 512, device=dev, generator=g))
    dy = torch.randn(19200, 300, device=dev, generator=g)
    dH = torch.randn(19200, 512, device=dev, generator=g)
    DY, HH = torch.randn(38400, 300, device=dev, generator=g), torch.randn(38400, 512, device=dev, generator=g)
    DH, XX = torch.randn(38400, 512, device=dev, generator=g), torch.randn(38400, 300, device=dev, generator=g)
    s1, s2, s2t, s1t = split_weights((W1, False), (W2, False), (W2, True), (W1, True))
    o512, o300 = torch.empty(19200, 512, device=dev), torch.empty(19200, 300, device=dev)
    dx = torch.zeros(19200, 300, device=dev)
    sep = torch.empty(16 << 20, device=dev)
    calls = [lambda: gemm_psw(x, s1, bias=b1, relu=True, out=o512),
             lambda: gemm_psw(H, s2, bias=b2, out=o300),
             lambda: gemm_psw(dy, s2t, relu_mask=H, out=o512),
             lambda: gemm_psw(dH, s1t, out=dx, add=dx),
             lambda: gemm_slabs(DY, HH, a_t=True),
             lambda: gemm_slabs(DH, XX, a_t=True)]
    for f in calls:
        sep.fill_(1.0)
        for _ in range(REPS):
            f()
    torch.cuda.synchronize()


def parse(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    groups, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "fill" in name.lower() or "FillFunctor" in name:
            cur = []
            groups.append(cur)
        elif cur is not None and ("k_gemm" in name or "splitk" in name):
            cur.append(r)
    groups = groups[-len(SHAPES):]
    print("| shape | M x N x K | kernel | launches | avg us | TFLOP/s | frac of fp32 MFMA peak (157.3) |")
    print("|---|---|---|---|---|---|---|")
    for (label, M, N, K), grp in zip(SHAPES, groups):
        by = {}
        for r in grp:
            n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
            n = n[:n.index("(")] if "(" in n else n
            by.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        tot = 0.0
        for n, ds in by.items():
            avg = sum(ds) / len(ds)
            tot += avg
            tf = 2.0 * M * N * K / (avg * 1e-6) / 1e12 if "gemm" in n else None
            print(f"| {label} | {M}x{N}x{K} | `{n}` | {len(ds)} | {avg:.1f} | "
                  f"{tf:.1f} | {tf / PEAK:.2f} |" if tf else
                  f"| {label} | {M}x{N}x{K} | `{n}` | {len(ds)} | {avg:.1f} | - | - |")
        if len(by) > 1:
            tf = 2.0 * M * N * K / (tot * 1e-6) / 1e12
            print(f"| {label} | {M}x{N}x{K} | GEMM + reduce | - | {tot:.1f} | {tf:.1f} | {tf / PEAK:.2f} |")


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else parse(sys.argv[2])
