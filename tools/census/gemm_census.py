"""Dev tool: residency timeline of hsg_gemm blocks (build with -DHSG_GEMM_CENSUS into
hetersumgraph_amd/libhsg_census.so; run with HSG_LIB_PATH pointing at it)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from hetersumgraph_amd import _lib
from hetersumgraph_amd.dense import gemm
lib = _lib.load()
M, N, K, a_t, b_t = (int(x) for x in sys.argv[1:6])
A = torch.randn(K, M, device="cuda") if a_t else torch.randn(M, K, device="cuda")
B = torch.randn(N, K, device="cuda") if b_t else torch.randn(K, N, device="cuda")
for _ in range(3):
    gemm(A, B, bool(a_t), bool(b_t), splits=1)
torch.cuda.synchronize()
nb = int(sys.argv[6])
buf = (ctypes.c_ulonglong * (4 * nb))()
lib.hsg_gemm_census_read(buf, nb)
h = np.array(buf, dtype=np.uint64).reshape(nb, 4)
hw, xcc, t0, t1 = h[:, 0].astype(np.int64), h[:, 1].astype(np.int64), h[:, 2].astype(np.int64), h[:, 3].astype(np.int64)
key = xcc * 100000 + (hw & 0xFF00) + ((hw >> 13) & 7) * 16 + ((hw >> 12) & 1)
T0 = t0.min()
life = t1 - t0
print(f"blocks {nb} span {(t1.max() - T0)} cycles  life mean {life.mean():.0f} min {life.min()} max {life.max()}")
# residency per CU over time
res = []
for k in np.unique(key):
    sel = key == k
    ev = sorted([(a, 1) for a in t0[sel]] + [(b, -1) for b in t1[sel]])
    c = m = 0
    for _, d in ev:
        c += d
        m = max(m, c)
    res.append(m)
print("CUs", len(res), "max resident per CU: mean", np.mean(res), "min", np.min(res), "max", np.max(res))
# start-time distribution
st = np.sort(t0 - T0)
print("start times pct:", [int(st[int(q * (nb - 1))]) for q in (0, 0.25, 0.5, 0.75, 0.85, 0.9, 1.0)])
en = np.sort(t1 - T0)
print("end times pct:", [int(en[int(q * (nb - 1))]) for q in (0, 0.25, 0.5, 0.75, 0.9, 1.0)])
