"""``dgl.data.utils.save_graphs/load_graphs`` (dataloader.py:46, 435).

The on-disk format is this build's own (a torch ``save`` of plain tensors and
numpy edge arrays, loaded with ``weights_only=True``); DGL's binary format is not
readable without DGL.
"""
import numpy as np
import torch

from ...graph import DGLGraph, Frame


def save_graphs(filename, g_list, labels=None):
    payload = {"graphs": [], "labels": labels or {}}
    for g in g_list:
        g._flush()
        payload["graphs"].append({
            "n": g.number_of_nodes(),
            "src": torch.from_numpy(g._src.copy()), "dst": torch.from_numpy(g._dst.copy()),
            "ndata": {k: v.detach().cpu() for k, v in g.ndata.items()},
            "edata": {k: v.detach().cpu() for k, v in g.edata.items()},
        })
    torch.save(payload, filename)


def load_graphs(filename, idx_list=None):
    payload = torch.load(filename, weights_only=True)
    out = []
    for i, rec in enumerate(payload["graphs"]):
        if idx_list is not None and i not in idx_list:
            continue
        g = DGLGraph()
        g._n = int(rec["n"])
        g._src = rec["src"].numpy().astype(np.int64)
        g._dst = rec["dst"].numpy().astype(np.int64)
        g._nframe = Frame(g._n)
        g._ef = Frame(len(g._src))
        g._nframe.cols = dict(rec["ndata"])
        g._ef.cols = dict(rec["edata"])
        out.append(g)
    return out, payload["labels"]
