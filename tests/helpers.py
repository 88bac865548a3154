"""Shared test helpers: rebuild graphs / modules from golden fixtures and seeds."""
import os

import numpy as np
import torch

import weights  # tests/golden/weights.py

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def fixture_docs(z, prefix="g_"):
    """Per-doc arrays (local node ids) from a fixture's batched graph arrays."""
    nn_ = z[prefix + "n_nodes"]
    ne = z[prefix + "n_edges"]
    no = np.cumsum(np.concatenate([[0], nn_]))
    eo = np.cumsum(np.concatenate([[0], ne]))
    docs = []
    for i in range(len(nn_)):
        a, b, c, d = no[i], no[i + 1], eo[i], eo[i + 1]
        docs.append(dict(unit=z[prefix + "unit"][a:b], ndtype=z[prefix + "ndtype"][a:b],
                         wid=z[prefix + "wid"][a:b].astype(np.int64),
                         src=z[prefix + "src"][c:d].astype(np.int64) - a,
                         dst=z[prefix + "dst"][c:d].astype(np.int64) - a,
                         tffrac=z[prefix + "tffrac"][c:d].astype(np.int64),
                         edtype=z[prefix + "edtype"][c:d].astype(np.float32)))
    return docs


def build_graph(z, sent_words=None, sent_label=None):
    """Product DGLGraph (batched) from a fixture, via the DGL construction API."""
    from hetersumgraph_amd import graph as hg
    docs = fixture_docs(z)
    gs = []
    s_off = 0
    for d in docs:
        g = hg.DGLGraph()
        n = len(d["unit"])
        g.add_nodes(n)
        g.set_n_initializer(hg.zero_initializer)
        g.set_e_initializer(hg.zero_initializer)
        g.ndata["unit"] = torch.from_numpy(d["unit"].copy())
        g.ndata["dtype"] = torch.from_numpy(d["ndtype"].copy())
        g.ndata["id"] = torch.from_numpy(d["wid"].copy())
        g.add_edges(torch.from_numpy(d["src"]), torch.from_numpy(d["dst"]),
                    data={"tffrac": torch.from_numpy(d["tffrac"]), "dtype": torch.from_numpy(d["edtype"])})
        sn = np.nonzero(d["ndtype"] == 1)[0]
        if sent_words is not None:
            N = len(sn)
            g.nodes[torch.from_numpy(sn)].data["words"] = torch.from_numpy(
                sent_words[s_off:s_off + N].astype(np.int64))
            g.nodes[torch.from_numpy(sn)].data["position"] = torch.arange(1, N + 1).view(-1, 1)
            g.nodes[torch.from_numpy(sn)].data["label"] = torch.from_numpy(
                sent_label[s_off:s_off + N].astype(np.int64))
            s_off += N
        gs.append(g)
    return hg.batch(gs)


def concat_arrays(z, prefix="g_"):
    return dict(src=z[prefix + "src"].astype(np.int64), dst=z[prefix + "dst"].astype(np.int64),
                unit=z[prefix + "unit"], ndtype=z[prefix + "ndtype"],
                tffrac=z[prefix + "tffrac"].astype(np.int64), edtype=z[prefix + "edtype"].astype(np.float32))


def gat_inputs(seed, n_w, n_s):
    Xw = torch.from_numpy(weights.feature(seed, "Xw", (n_w, 300), 0.4))
    Xs = torch.from_numpy(weights.feature(seed, "Xs", (n_s, 64), 1.0))
    T = torch.from_numpy(weights.param_value(seed, "_TFembed.weight", (10, 50)))
    return Xw, Xs, T


def upstream(seed, shape_w2s, shape_s2w):
    R1 = torch.from_numpy(weights.feature(seed, "R_w2s", tuple(shape_w2s)))
    R2 = torch.from_numpy(weights.feature(seed, "R_s2w", tuple(shape_s2w)))
    return R1, R2


def projections(x, seed, name, n_proj=4):
    x = x.detach().double().reshape(-1).cpu().numpy()
    rng = np.random.default_rng(weights._key_seed(seed, "proj:" + name))
    P = rng.standard_normal((n_proj, x.size))
    return np.concatenate([[x.sum(), np.sqrt((x * x).sum()), np.abs(x).max()], P @ x])


def seeded_gat_params(seed_w2s, seed_s2w):
    """State dicts of the two WSWGAT modules as seeded in make_golden.py."""
    from hetersumgraph_amd.module.GAT import WSWGAT
    w2s = weights.seed_module(WSWGAT(300, 64, 8, 0.1, 512, 0.1, 50, "W2S"), seed_w2s)
    s2w = weights.seed_module(WSWGAT(64, 300, 6, 0.1, 512, 0.1, 50, "S2W"), seed_s2w)
    return w2s.eval(), s2w.eval()


def synth_fixture(docs):
    """Fixture-like dict from synth DocArrays (no reference outputs)."""
    offs = np.cumsum([0] + [d.n_nodes for d in docs])
    cat = lambda f: np.concatenate([f(d, o) for d, o in zip(docs, offs[:-1])])
    z = {"g_n_nodes": np.array([d.n_nodes for d in docs]), "g_n_edges": np.array([len(d.src) for d in docs]),
         "g_unit": cat(lambda d, o: d.unit), "g_ndtype": cat(lambda d, o: d.ndtype),
         "g_wid": cat(lambda d, o: d.wid), "g_src": cat(lambda d, o: d.src + o),
         "g_dst": cat(lambda d, o: d.dst + o), "g_tffrac": cat(lambda d, o: d.tffrac),
         "g_edtype": cat(lambda d, o: d.edtype)}
    z["n_w"] = int((z["g_unit"] == 0).sum())
    z["n_s"] = int((z["g_unit"] == 1).sum())
    return z


def dev_lib():
    """True when the loaded library is the dev build (libhsg_dev.so via HSG_LIB_PATH):
    only it reads the A/B switches of the rejected kernel variants (csrc/hsg_dev.h);
    the product libhsg.so runs the defaults whatever the environment says."""
    from hetersumgraph_amd._lib import version
    return version().endswith(" dev")


def skip_unless_dev(variant_is_default):
    import pytest
    if not variant_is_default and not dev_lib():
        pytest.skip("dev kernel variant: runs against libhsg_dev.so (HSG_LIB_PATH); the product library "
                    "carries the default kernels only")
