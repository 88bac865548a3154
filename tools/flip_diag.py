"""Dev tool: is a gradient difference between two GEMM plans on a golden fixture an
fp32 ReLU-gate flip?  Records the S2W FFN input x of the layer-wise path, then for
plans A and B compares the relu pattern of H = relu(x W1^T + b1) and prints the fp64
pre-activation of every flipped element (tests/test_gpu_gat.py::gat_cfg1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import torch  # noqa: E402

import hetersumgraph_amd.ffn as F  # noqa: E402
from test_gpu_gat import load_fixture, run_gat  # noqa: E402

rec = {}
orig = F.ffn_fwd


def spy(x, w1, b1, w2, b2, *a, **k):
    out, saved = orig(x, w1, b1, w2, b2, *a, **k)
    if x.shape[1] == 300:
        rec.setdefault(os.environ.get("HSG_GEMM5", "dflt"), []).append((x.clone(), w1.clone(), b1.clone(),
                                                                          saved[4].clone()))
    return out, saved


F.ffn_fwd = spy
z = load_fixture("gat_cfg1")
grads = {}
for plan in sys.argv[1:] or ["7", "27"]:
    os.environ["HSG_GEMM5"] = plan
    r = run_gat(z, 3)
    grads[plan] = r["Xs"].grad.double().cpu()
plans = list(grads)
a, b = plans[0], plans[1]
xa, w1, b1, Ha = rec[a][0]
_, _, _, Hb = rec[b][0]
pre = (xa.double() @ w1.double().t() + b1.double())
flip = (Ha > 0) != (Hb > 0)
idx = flip.nonzero()
print(f"H elements with different relu gate between plans {a} and {b}: {len(idx)}")
for i, j in idx[:20].tolist():
    print(f"  row {i} col {j}: fp64 pre-activation {pre[i, j].item():.3e} (|x|.|w1| scale "
          f"{(xa[i].double().abs() @ w1[j].double().abs()).item():.3e}), H {a}={Ha[i, j].item():.3e} {b}={Hb[i, j].item():.3e}")
ref = torch.as_tensor(z["grad_Xs"], dtype=torch.float64)
for p in plans:
    e = (grads[p] - ref).abs().max(1).values
    top = torch.topk(e, 3)
    print(f"plan {p}: worst Xs-grad rows {top.indices.tolist()} err {[round(v, 4) for v in top.values.tolist()]} "
          f"scale {ref.abs().max().item():.2f}")
