"""Timing script (tests/ may use the oracle as a baseline; not collected by pytest): cfg2-shaped graph construction time -- native builder (datapipe,
libhsg_host.so) vs the per-edge Python restatement of CreateGraph
(oracle/create_graph.py, a lower bound for the reference, which also creates a
tensor per add_edges call).  32 docs x 35 sentences x 36 distinct words."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden"))
import numpy as np  # noqa: E402

from graph_data import MinVocab  # noqa: E402
from hetersumgraph_amd import build  # noqa: E402
from hetersumgraph_amd.datapipe import build_doc_arrays, tfidf_pairs  # noqa: E402
from oracle import create_graph as cg  # noqa: E402

build.build_host(verbose=False)
rng = np.random.default_rng(0)
words = [f"w{i}" for i in range(50000)]
vocab = MinVocab(words)
L, B, N, W, K = 100, 32, 35, 600, 36
docs, raw = [], []
for _ in range(B):
    dw = rng.choice(50000, W, replace=False) + 4
    pad, tfs, w2s = [], [], {}
    for i in range(N):
        ids = rng.choice(dw, K, replace=False).tolist()
        pad.append(ids + [0] * (L - K))
        tfw = {vocab.id2word(w): float(rng.uniform(0.05, 0.6)) for w in ids}
        w2s[str(i)] = tfw
    raw.append((pad, w2s))
t0 = time.perf_counter()
items = [dict(sent_pad=p, label=np.zeros((N, 50)), sent_tf=[tfidf_pairs(w[str(i)], vocab) for i in range(N)])
         for p, w in raw]
t1 = time.perf_counter()
for threads in (1, 8):
    t2 = time.perf_counter()
    arrs = build_doc_arrays(items, L, [0], threads=threads)
    t3 = time.perf_counter()
    print(f"native builder, {threads} thread(s): {(t3 - t2) * 1e3:.1f} ms for {B} docs "
          f"({sum(len(a.src) for a in arrs)} edges); tf-idf pair mapping {(t1 - t0) * 1e3:.1f} ms")
t4 = time.perf_counter()
for p, w in raw:
    cg.hsg_graph(p, w, vocab, {0})
t5 = time.perf_counter()
print(f"python per-edge restatement: {(t5 - t4) * 1e3:.1f} ms for {B} docs")
