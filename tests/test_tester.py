"""SLTester (hetersumgraph_amd/Tester.py) against the reference's own SLTester outputs
(tests/golden/tester.json, made by tests/golden/make_tester_golden.py): selected
sentence indices in order, hypotheses, counters and metrics must be identical, the
running loss equal to fp32 rounding.  Runs on CPU (the selection is host/tensor logic;
the model is a stand-in returning the fixture's logits)."""
import json
import os

import numpy as np
import pytest
import torch

from make_tester_golden import _Model, _Set, make_case

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tester.json")


def cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", cases(), ids=lambda c: f"seed{c['seed']}-m{c['m']}-block{int(c['blocking'])}")
def test_sltester_matches_reference(case):
    from hetersumgraph_amd import graph as hg
    from hetersumgraph_amd import synth
    from hetersumgraph_amd.Tester import SLTester
    docs, logits, texts = make_case(case["seed"])
    np.testing.assert_array_equal(logits, np.asarray(case["logits"], np.float32))
    assert texts == case["texts"]
    G = hg.batch([synth.to_graph(d, hg.DGLGraph) for d in docs])
    t = SLTester(_Model(logits), case["m"], limited=True)
    t.evaluation(G, list(range(len(docs))), _Set(texts), blocking=case["blocking"])
    t.getMetric()
    ref = case["state"]
    assert t.extracts == ref["extracts"]
    assert t._hyps == ref["hyps"] and t._refer == ref["refer"] and t.hyps == ref["hyps_limited"]
    for k in ("pred", "true", "match", "match_true"):
        assert int(getattr(t, k)) == ref[k], k
    assert t.total_sentence_num == ref["total_sentence_num"] and t.example_num == ref["example_num"]
    assert t.batch_number == ref["batch_number"]
    assert abs(t.running_loss - ref["running_loss"]) <= 1e-6 * max(1.0, abs(ref["running_loss"]))
    got = [float(x) for x in (t._accu, t._precision, t._recall, t._F)]
    np.testing.assert_allclose(got, ref["metric"], rtol=1e-6, atol=0)


def test_select_topk_matches_per_document_topk():
    """The batched padded top-k equals a per-document torch.topk (ragged counts, m > N)."""
    from hetersumgraph_amd.Tester import _select
    g = torch.Generator().manual_seed(0)
    counts = [9, 4, 1, 3, 7, 2]
    p = torch.randn(sum(counts), 2, generator=g)
    for m in (1, 3, 5, 12):
        got = _select(p, counts, m)
        o = 0
        for j, n in enumerate(counts):
            ref = torch.topk(p[o:o + n, 1], min(m, n))[1]
            assert got[j].tolist() == ref.tolist()
            o += n
    got = _select(p, counts, 0)
    o = 0
    for j, n in enumerate(counts):
        assert got[j].tolist() == torch.arange(n)[p[o:o + n].max(1)[1] != 0].tolist()
        o += n
