"""Golden outputs of the reference's evaluation-time selection (Tester.py SLTester).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_tester_golden.py [--ref /root/reference]

Runs /root/reference/Tester.py (read-only) over batched synthetic graphs with seeded
logits from a stand-in model, with ``sys.modules['dgl']`` pointed at the test-only
DGL-0.4 shim (dgl_shim.py) and ``sys.modules['rouge']`` at an empty placeholder --
tools/utils.py imports ``rouge`` at module level (absent here) but SLTester.evaluation
and eval_label never call it.  Writes tester.json: for m in {0, 3} and blocking on/off,
every accumulated output (extracts, hyps, refer, running loss, counters, metrics).
"""
import argparse
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import dgl_shim  # noqa: E402
from hetersumgraph_amd import synth  # noqa: E402

WORDS = "the a of to in cat dog sat on mat ran far away big small red blue".split()


def make_case(seed):
    """Docs (sorted by sentence count, as graph_collate_fn), logits, article texts."""
    rng = np.random.default_rng(seed)
    shapes = [(7, 30, 5), (5, 20, 4), (5, 22, 4), (2, 9, 3), (1, 5, 2)]
    docs = [synth.make_hsg_doc(rng, N=n, W=w, k=k, vocab_size=500) for n, w, k in shapes]
    n_s = sum(int((d.ndtype == 1).sum()) for d in docs)
    logits = rng.standard_normal((n_s, 2)).astype(np.float32)
    texts = []
    for d in docs:
        N = int((d.ndtype == 1).sum())
        sents = []
        for i in range(N):
            L = int(rng.integers(3, 9))
            tail = " ".join(WORDS[j] for j in rng.integers(0, len(WORDS), L))
            # sentences i % 3 != 0 share the trigrams of a common prefix: n-gram blocking drops them
            sents.append("the cat sat on the mat " + tail if i % 3 else tail)
        texts.append({"sents": sents, "abstract": " ".join(sents[:1]) + " summary"})
    return docs, logits, texts


class _Model:
    def __init__(self, logits):
        self.logits = torch.from_numpy(logits)

    def forward(self, G):
        return self.logits.clone()


class _Example:
    def __init__(self, t):
        self.original_article_sents = t["sents"]
        self.original_abstract = t["abstract"]


class _Set:
    def __init__(self, texts):
        self.texts = texts

    def get_example(self, i):
        return _Example(self.texts[i])


def state(t):
    f = lambda x: float(x) if not isinstance(x, float) else x
    return {"extracts": t.extracts, "hyps": t._hyps, "refer": t._refer, "hyps_limited": t.hyps,
            "running_loss": f(t.running_loss), "batch_number": t.batch_number,
            "pred": int(t.pred), "true": int(t.true), "match": int(t.match), "match_true": int(t.match_true),
            "total_sentence_num": t.total_sentence_num, "example_num": t.example_num,
            "metric": [f(x) for x in (t._accu, t._precision, t._recall, t._F)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    shim = types.ModuleType("dgl")
    for k in ("DGLGraph", "batch", "unbatch", "sum_nodes", "init"):
        setattr(shim, k, getattr(dgl_shim, k))
    sys.modules["dgl"] = shim
    sys.modules["rouge"] = types.ModuleType("rouge")
    sys.modules["rouge"].Rouge = None
    import Tester  # noqa: E402  (reference)

    out = {"cases": []}
    for seed in (31, 32):
        docs, logits, texts = make_case(seed)
        for m, blocking in ((0, False), (3, False), (3, True), (2, True)):
            G = dgl_shim.batch([synth.to_graph(d, dgl_shim.DGLGraph) for d in docs])
            t = Tester.SLTester(_Model(logits), m, limited=True)
            t.evaluation(G, list(range(len(docs))), _Set(texts), blocking=blocking)
            t.getMetric()
            out["cases"].append({"seed": seed, "m": m, "blocking": blocking, "logits": logits.tolist(),
                                 "texts": texts, "state": state(t)})
    with open(os.path.join(HERE, "tester.json"), "w") as f:
        json.dump(out, f)
    print(len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
