"""Golden document graphs from the REFERENCE's own graph builders.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_graph_golden.py [--ref /root/reference]

Imports /root/reference/module/dataloader.py (ExampleSet / MultiExampleSet:
Example tokenisation, AddWordNode, CreateGraph, MapSent2Doc) and
module/vocabulary.py (read-only, never copied), with two stand-ins for modules
this container lacks: ``dgl`` -> the test-only DGL-0.4 shim (tests/golden/dgl_shim.py)
and ``nltk`` -> a stub whose ``stopwords.words('english')`` is graph_data.STOPWORDS
(the real list is not installed; the same list is passed to the build's
ExampleSet).  The datasets are graph_data.make_files(); every example's graph
arrays go to tests/golden/graphs_ref.npz.  Only this script touches the reference.
"""
import argparse
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import dgl_shim  # noqa: E402
import graph_data  # noqa: E402

SENT_MAX_LEN, DOC_MAX = 12, 7


def _stubs():
    nltk = types.ModuleType("nltk")
    corpus = types.ModuleType("nltk.corpus")
    corpus.stopwords = types.SimpleNamespace(words=lambda lang: list(graph_data.STOPWORDS))
    nltk.corpus = corpus
    sys.modules["nltk"], sys.modules["nltk.corpus"] = nltk, corpus
    dgl = types.ModuleType("dgl")
    for k in ("DGLGraph", "batch", "unbatch", "sum_nodes", "init"):
        setattr(dgl, k, getattr(dgl_shim, k))
    data = types.ModuleType("dgl.data")
    utils = types.ModuleType("dgl.data.utils")
    utils.save_graphs = utils.load_graphs = None
    data.utils = utils
    dgl.data = data
    sys.modules.update({"dgl": dgl, "dgl.data": data, "dgl.data.utils": utils})


def arrays(G):
    return dict(n=np.int64(G.n), unit=G.ndata["unit"].numpy(), dtype=G.ndata["dtype"].numpy(),
                id=G.ndata["id"].numpy(), words=G.ndata["words"].numpy(), position=G.ndata["position"].numpy(),
                label=G.ndata["label"].numpy(), src=G.src.numpy(), dst=G.dst.numpy(),
                tffrac=G.edata["tffrac"].numpy(), edtype=G.edata["dtype"].numpy())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(HERE, "graphs_ref.npz"))
    args = ap.parse_args()
    _stubs()
    sys.path.insert(0, args.ref)
    from module import dataloader as ref_dl
    from module.vocabulary import Vocab
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for kind, multi in (("hsg", False), ("hdsg", True)):
            d = os.path.join(tmp, kind)
            graph_data.make_files(d, seed=11 if multi else 7, multi=multi)
            vocab = Vocab(os.path.join(d, "vocab"), 0)
            paths = [os.path.join(d, "data.jsonl"), vocab, DOC_MAX, SENT_MAX_LEN, os.path.join(d, "filter_word.txt"),
                     os.path.join(d, "w2s.jsonl")]
            ds = ref_dl.MultiExampleSet(*paths, os.path.join(d, "w2d.jsonl")) if multi else ref_dl.ExampleSet(*paths)
            for i in range(len(ds)):
                G, idx = ds[i]
                assert idx == i
                for k, v in arrays(G).items():
                    out[f"{kind}.{i}.{k}"] = v
            out[f"{kind}.n"] = np.int64(len(ds))
            out[f"{kind}.filterids"] = np.asarray(sorted(set(ds.filterids)), np.int64)
    np.savez_compressed(args.out, **out)
    print("wrote", args.out, len(out), "arrays")


if __name__ == "__main__":
    main()
