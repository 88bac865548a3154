"""Generate the golden vectors by running the REFERENCE's own module code.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--ref /root/reference]

Imports /root/reference/module/{GAT,GATLayer,GATStackLayer,Encoder,PositionEmbedding}.py
and HiGraph.py (read-only, never copied) with ``sys.modules['dgl']`` pointed at the
test-only DGL-0.4-semantics shim (tests/golden/dgl_shim.py; DGL is not installed and
cannot be fetched), on CPU in fp32 -- the reference CPU path.  Writes
small ``.npz`` fixtures next to this file: graph arrays, outputs, and gradients
(full where small, otherwise checksums + random projections).  Parameters and
inputs are regenerated from seeds (tests/golden/weights.py) on both sides.

Only this script touches the reference; the GPU box never sees it.
"""
import argparse
import hashlib
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import dgl_shim  # noqa: E402
import weights  # noqa: E402
from hetersumgraph_amd import synth  # noqa: E402

N_PROJ = 4


def projections(x, seed, name):
    x = x.detach().double().reshape(-1).numpy()
    rng = np.random.default_rng(weights._key_seed(seed, "proj:" + name))
    P = rng.standard_normal((N_PROJ, x.size))
    return np.concatenate([[x.sum(), np.sqrt((x * x).sum()), np.abs(x).max()], P @ x])


def graph_arrays(docs, prefix="g_"):
    """Concatenated (batched) graph arrays of a list of DocArrays (sorted order)."""
    offs = np.cumsum([0] + [d.n_nodes for d in docs])
    cat = lambda f: np.concatenate([f(d, o) for d, o in zip(docs, offs[:-1])])
    return {
        prefix + "n_nodes": np.array([d.n_nodes for d in docs], np.int64),
        prefix + "n_edges": np.array([len(d.src) for d in docs], np.int64),
        prefix + "unit": cat(lambda d, o: d.unit), prefix + "ndtype": cat(lambda d, o: d.ndtype),
        prefix + "wid": cat(lambda d, o: d.wid).astype(np.int32),
        prefix + "src": cat(lambda d, o: d.src + o).astype(np.int32),
        prefix + "dst": cat(lambda d, o: d.dst + o).astype(np.int32),
        prefix + "tffrac": cat(lambda d, o: d.tffrac).astype(np.int8),
        prefix + "edtype": cat(lambda d, o: d.edtype).astype(np.int8),
    }


def compact(d):
    """fp64 results are stored rounded to fp32 (7 significant digits is far below
    every test tolerance); projections and scalars stay fp64."""
    out = {}
    for k, v in d.items():
        v = np.asarray(v)
        if v.dtype == np.float64 and v.size > 16 and not k.startswith("proj"):
            v = v.astype(np.float32)
        out[k] = v
    return out


def sort_by_sentences(docs):
    # graph_collate_fn (dataloader.py:472-481): descending #sentence nodes
    lens = [int((d.ndtype == 1).sum()) for d in docs]
    order = sorted(range(len(docs)), key=lambda i: -lens[i])
    return [docs[i] for i in order]


def shim_batch(docs):
    return dgl_shim.batch([synth.to_graph(d, dgl_shim.DGLGraph) for d in docs])


def import_reference(ref):
    sys.path.insert(0, ref)
    shim_mod = types.ModuleType("dgl")
    shim_mod.DGLGraph = dgl_shim.DGLGraph
    shim_mod.batch = dgl_shim.batch
    shim_mod.unbatch = dgl_shim.unbatch
    shim_mod.sum_nodes = dgl_shim.sum_nodes
    shim_mod.init = dgl_shim.init
    sys.modules["dgl"] = shim_mod
    import HiGraph  # noqa: F401  (reference)
    from module import GAT  # noqa: F401  (reference)
    return HiGraph, GAT


def ref_hashes(ref):
    out = {}
    for rel in ("module/GAT.py", "module/GATLayer.py", "module/GATStackLayer.py", "module/Encoder.py",
                "module/PositionEmbedding.py", "HiGraph.py"):
        with open(os.path.join(ref, rel), "rb") as f:
            out[rel] = hashlib.sha256(f.read()).hexdigest()[:16]
    return out


# ----------------------------------------------------------------- GAT level --
def gat_case(GAT, docs, seed, full_grads, keep_rows=None):
    """W2S and S2W WSWGAT (reference) on one batched graph, eval mode.

    Forward outputs in fp32 (the reference CPU path, ``out_*``) and fp64
    (``out64_*``); gradients from the fp64 run (fp32 gradients of a ReLU network
    flip at near-zero pre-activations, see tests/test_oracle_golden.py)."""
    res = {}
    rows = None
    for dt in (torch.float32, torch.float64):
        G = shim_batch(docs)
        n_w = int((G.ndata["unit"] == 0).sum())
        if keep_rows is not None:
            rows = np.sort(np.random.default_rng(seed).choice(n_w, size=keep_rows, replace=False))
        n_s = int((G.ndata["unit"] == 1).sum())
        Xw = torch.from_numpy(weights.feature(seed, "Xw", (n_w, 300), 0.4)).to(dt).requires_grad_()
        Xs = torch.from_numpy(weights.feature(seed, "Xs", (n_s, 64), 1.0)).to(dt).requires_grad_()
        T = torch.from_numpy(weights.param_value(seed, "_TFembed.weight", (10, 50))).to(dt).requires_grad_()
        wsedge = G.filter_edges(lambda e: e.data["dtype"] == 0)
        G.edges[wsedge].data["tfidfembed"] = F.embedding(G.edata["tffrac"][wsedge], T)
        w2s = GAT.WSWGAT(300, 64, 8, 0.1, 512, 0.1, 50, "W2S")
        s2w = GAT.WSWGAT(64, 300, 6, 0.1, 512, 0.1, 50, "S2W")
        weights.seed_module(w2s, seed * 100 + 1).eval().to(dt)
        weights.seed_module(s2w, seed * 100 + 2).eval().to(dt)
        out_ws = w2s(G, Xw, Xs)
        out_sw = s2w(G, Xw, Xs)
        if dt == torch.float32:
            res["out_w2s"] = out_ws.detach().numpy()
            res["out_s2w"] = out_sw.detach().numpy() if rows is None else out_sw.detach().numpy()[rows]
    R1 = torch.from_numpy(weights.feature(seed, "R_w2s", tuple(out_ws.shape))).double()
    R2 = torch.from_numpy(weights.feature(seed, "R_s2w", tuple(out_sw.shape))).double()
    ((out_ws * R1).sum() + (out_sw * R2).sum()).backward()
    res.update({"n_w": n_w, "n_s": n_s, "out64_w2s": out_ws.detach().numpy(),
                "grad_Xs": Xs.grad.numpy(), "grad_T": T.grad.numpy()})
    if keep_rows is None:
        res["out64_s2w"] = out_sw.detach().numpy()
        res["grad_Xw"] = Xw.grad.numpy()
    else:
        res["rows_w"] = rows
        res["out64_s2w"] = out_sw.detach().numpy()[rows]
        res["grad_Xw_rows"] = Xw.grad.numpy()[rows]
        res["proj_out_s2w"] = projections(out_sw, seed, "out_s2w")
        res["proj_grad_Xw"] = projections(Xw.grad, seed, "grad_Xw")
    for tag, mod in (("w2s", w2s), ("s2w", s2w)):
        for name, p in mod.named_parameters():
            key = f"grad.{tag}.{name}"
            if full_grads or p.numel() <= 40000:
                res[key] = p.grad.numpy()
            else:
                res["proj." + key] = projections(p.grad, seed, key)
    return res


def s2s_case(GAT, docs, seed, d=64, H=8):
    """WSWGAT(layerType="S2S") (GAT.py:38-39, 49-51: MultiHeadSGATLayer of SGATLayer
    heads, GATLayer.py:49-78) on one batched graph, eval mode.  Forward in fp32 and
    fp64, gradients of ``(out * R).sum()`` from the fp64 run, and the edge column
    ``edata['e']`` the fp64 forward leaves on the graph."""
    res = {}
    for dt in (torch.float32, torch.float64):
        G = shim_batch(docs)
        n_s = int((G.ndata["unit"] == 1).sum())
        Xs = torch.from_numpy(weights.feature(seed, "Xs", (n_s, d), 1.0)).to(dt).requires_grad_()
        s2s = GAT.WSWGAT(d, d, H, 0.1, 512, 0.1, 50, "S2S")
        weights.seed_module(s2s, seed * 100 + 3).eval().to(dt)
        out = s2s(G, Xs, Xs)
        if dt == torch.float32:
            res["out_s2s"] = out.detach().numpy()
    R = torch.from_numpy(weights.feature(seed, "R_s2s", tuple(out.shape))).double()
    (out * R).sum().backward()
    res.update({"n_s": n_s, "out64_s2s": out.detach().numpy(), "grad_Xs": Xs.grad.numpy(),
                "e64": G.edata["e"].detach().numpy()})
    for name, p in s2s.named_parameters():
        res[f"grad.s2s.{name}"] = p.grad.numpy()
    return res


# ---------------------------------------------------------- train-mode stack --
def stack_train_case(GAT, docs, seed, drop_seed, off0=0, n_iter=2, p=0.1, keep_rows=160):
    """The reference's own WSWGAT modules chained as HiGraph.py:99-106 (W2S, then
    n_iter x (S2W, W2S)) in TRAIN mode, with every ``nn.Dropout`` call (H per head
    input, GATStackLayer.py:56; one per FFN output, GATLayer.py:41) replaced by the
    keep-mask and scale the fused stack draws for it at (drop_seed, offset):
    oracle/masks.py, which restates the device generators bit for bit
    (tests/test_gpu_dropout_masks.py).  The reference's code computes everything
    else.  Outputs in fp32 and fp64, gradients of ``(s * R).sum()`` from the fp64 run."""
    sys.path.insert(0, REPO)
    from oracle import masks as om
    res = {}
    for dt in (torch.float32, torch.float64):
        G = shim_batch(docs)
        n_w = int((G.ndata["unit"] == 0).sum())
        n_s = int((G.ndata["unit"] == 1).sum())
        Xw = torch.from_numpy(weights.feature(seed, "Xw", (n_w, 300), 0.4)).to(dt).requires_grad_()
        Xs = torch.from_numpy(weights.feature(seed, "Xs", (n_s, 64), 1.0)).to(dt).requires_grad_()
        T = torch.from_numpy(weights.param_value(seed, "_TFembed.weight", (10, 50))).to(dt).requires_grad_()
        wsedge = G.filter_edges(lambda e: e.data["dtype"] == 0)
        G.edges[wsedge].data["tfidfembed"] = F.embedding(G.edata["tffrac"][wsedge], T)
        w2s = GAT.WSWGAT(300, 64, 8, p, 512, p, 50, "W2S")
        s2w = GAT.WSWGAT(64, 300, 6, p, 512, p, 50, "S2W")
        weights.seed_module(w2s, seed * 100 + 1).train().to(dt)
        weights.seed_module(s2w, seed * 100 + 2).train().to(dt)
        calls, off = [], off0
        for kind in ["W2S"] + ["S2W", "W2S"] * n_iter:
            n_src, d_in, H, n_dst, d = (n_w, 300, 8, n_s, 64) if kind == "W2S" else (n_s, 64, 6, n_w, 300)
            hk = om.hproj_keep(drop_seed, off + 1, n_src, d_in, H, p)
            calls += [(hk[k], om.hproj_scale(p)) for k in range(H)]
            calls.append((om.ffn_keep(drop_seed, off + 2, n_dst, d, p), om.ffn_scale(p)))
            off += 2
        it = iter(calls)

        class MaskDropout(torch.nn.Module):
            def forward(self, x):
                keep, scale = next(it)
                return x * torch.from_numpy(keep).to(x.dtype).reshape(x.shape) * scale

        for mod in (w2s, s2w):
            mod.layer.dropout = MaskDropout()
            mod.ffn.dropout = MaskDropout()
        w, s = Xw, w2s(G, Xw, Xs)
        for _ in range(n_iter):
            w = s2w(G, w, s)
            s = w2s(G, w, s)
        assert next(it, None) is None, "dropout calls out of step with the fused stack's draws"
        if dt == torch.float32:
            res["out"] = s.detach().numpy()
    R = torch.from_numpy(np.random.default_rng(seed).standard_normal(tuple(s.shape)))
    (s * R).sum().backward()
    rows = np.sort(np.random.default_rng(seed).choice(n_w, size=keep_rows, replace=False))
    res.update({"n_w": n_w, "n_s": n_s, "seed": np.array(seed), "drop_seed": np.array(drop_seed),
                "off0": np.array(off0), "n_iter": np.array(n_iter), "p": np.array(p),
                "out64": s.detach().numpy(), "grad_Xs": Xs.grad.numpy(), "grad_T": T.grad.numpy(),
                "rows_w": rows, "grad_Xw_rows": Xw.grad.numpy()[rows],
                "proj_grad_Xw": projections(Xw.grad, seed, "grad_Xw")})
    for tag, mod in (("w2s", w2s), ("s2w", s2w)):
        for name, q in mod.named_parameters():
            key = f"grad.{tag}.{name}"
            if q.numel() <= 40000:
                res[key] = q.grad.numpy()
            else:
                res["proj." + key] = projections(q.grad, seed, key)
    return res


# --------------------------------------------------------------- model level --
class HPS:
    def __init__(self, **kw):
        d = dict(n_iter=2, word_emb_dim=300, feat_embed_size=50, n_feature_size=128, hidden_size=64,
                 n_head=8, atten_dropout_prob=0.1, ffn_inner_hidden_size=512, ffn_dropout_prob=0.1,
                 doc_max_timesteps=50, lstm_hidden_state=128, lstm_layers=2, bidirectional=True,
                 sent_max_len=100, cuda=False, vocab_size=500)
        d.update(kw)
        self.__dict__.update(d)


def model_case(HiGraph, docs, seed, cls_name, **hps_kw):
    hps = HPS(**hps_kw)
    res = {}
    for dt in (torch.float32, torch.float64):
        torch.manual_seed(seed)
        embed = torch.nn.Embedding(hps.vocab_size, 300, padding_idx=0)
        model = getattr(HiGraph, cls_name)(hps, embed)
        weights.seed_module(model, seed)
        model.eval().to(dt)
        G = shim_batch(docs)
        logits = model(G)
        if dt == torch.float32:
            res["logits"] = logits.detach().numpy()
    snode = G.filter_nodes(lambda n: n.data["dtype"] == 1)
    label = G.ndata["label"][snode].sum(-1)
    # train.py:115-119 loss
    G.nodes[snode].data["loss"] = F.cross_entropy(logits, label, reduction="none").unsqueeze(-1)
    loss = dgl_shim.sum_nodes(G, "loss").mean()
    loss.backward()
    res.update({"logits64": logits.detach().numpy(), "loss64": np.array(loss.item())})
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        key = f"grad.{name}"
        if p.numel() <= 20000:
            res[key] = p.grad.numpy()
        else:
            res["proj." + key] = projections(p.grad, seed, key)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None, help="regenerate one fixture (file stem), e.g. model_hsg_cfg1")
    args = ap.parse_args()
    torch.set_num_threads(8)
    HiGraph, GAT = import_reference(args.ref)
    meta = {"ref_hash." + k: np.array(v) for k, v in ref_hashes(args.ref).items()}
    meta["torch"] = np.array(torch.__version__)

    def want(stem):
        return args.only is None or args.only == stem

    if want("model_hsg_cfg1"):
        # 4 config-1-shaped documents (N=30, W=400, k=20; 12,000 graph edges) through
        # the whole HSumGraph: logit parity beyond the 2-doc toy fixture
        rng = np.random.default_rng(15)
        cdocs = sort_by_sentences([synth.make_hsg_doc(rng, N=30, W=400, k=20, vocab_size=2000)
                                   for _ in range(4)])
        res = model_case(HiGraph, cdocs, 6, "HSumGraph", vocab_size=2000)
        extra = {"sent_words": np.concatenate([d.words for d in cdocs]).astype(np.int32),
                 "sent_label": np.concatenate([d.label for d in cdocs]).astype(np.int8),
                 "vocab_size": np.array(2000)}
        np.savez_compressed(os.path.join(HERE, "model_hsg_cfg1.npz"), **graph_arrays(cdocs), **compact(res),
                            **extra, **meta)
    if want("model_hsg_cfg1_n1"):
        # the same 4 config-1-shaped documents through HSumGraph at train.py's own
        # default n_iter = 1 (train.py:282): W2S, then ONE (S2W, W2S) round
        rng = np.random.default_rng(15)
        cdocs = sort_by_sentences([synth.make_hsg_doc(rng, N=30, W=400, k=20, vocab_size=2000)
                                   for _ in range(4)])
        res = model_case(HiGraph, cdocs, 7, "HSumGraph", vocab_size=2000, n_iter=1)
        extra = {"sent_words": np.concatenate([d.words for d in cdocs]).astype(np.int32),
                 "sent_label": np.concatenate([d.label for d in cdocs]).astype(np.int8),
                 "vocab_size": np.array(2000), "n_iter": np.array(1)}
        np.savez_compressed(os.path.join(HERE, "model_hsg_cfg1_n1.npz"), **graph_arrays(cdocs), **compact(res),
                            **extra, **meta)
    if args.only == "model_hsg_cfg2":
        # BASELINE config 2 at full size (32 CNN/DM-shaped documents, N=35, W=600, k=36:
        # 159,040 graph edges -- the bench's batch shape) through the whole HSumGraph;
        # generated on request only (--only model_hsg_cfg2: the reference CPU path takes
        # minutes at this size)
        cdocs = sort_by_sentences(synth.make_batch_docs("cfg2", seed=21, vocab_size=5000))
        res = model_case(HiGraph, cdocs, 8, "HSumGraph", vocab_size=5000)
        extra = {"sent_words": np.concatenate([d.words for d in cdocs]).astype(np.int32),
                 "sent_label": np.concatenate([d.label for d in cdocs]).astype(np.int8),
                 "vocab_size": np.array(5000)}
        np.savez_compressed(os.path.join(HERE, "model_hsg_cfg2.npz"), **graph_arrays(cdocs), **compact(res),
                            **extra, **meta)
    if args.only == "model_hdsg_cfg4":
        # BASELINE config 4 at full size (32 multi-document HDSG examples with doc nodes,
        # 3 x 15 sentences, W=700, k=20: 107,040 graph edges) through HSumDocGraph
        cdocs = sort_by_sentences(synth.make_batch_docs("cfg4", seed=22, vocab_size=5000))
        res = model_case(HiGraph, cdocs, 9, "HSumDocGraph", vocab_size=5000)
        extra = {"sent_words": np.concatenate([d.words for d in cdocs]).astype(np.int32),
                 "sent_label": np.concatenate([d.label for d in cdocs]).astype(np.int8),
                 "vocab_size": np.array(5000)}
        np.savez_compressed(os.path.join(HERE, "model_hdsg_cfg4.npz"), **graph_arrays(cdocs), **compact(res),
                            **extra, **meta)
    if args.only == "model_hsg_cfg5":
        # BASELINE config 5 at full size (NYT50-shaped: 32 documents, 481,280 graph edges
        # with the phantom sentence in-edges of doc_max_timesteps = 80) through HSumGraph
        cdocs = sort_by_sentences(synth.make_batch_docs("cfg5", seed=23, vocab_size=5000))
        res = model_case(HiGraph, cdocs, 10, "HSumGraph", vocab_size=5000, doc_max_timesteps=80)
        extra = {"sent_words": np.concatenate([d.words for d in cdocs]).astype(np.int32),
                 "sent_label": np.concatenate([d.label for d in cdocs]).astype(np.int8),
                 "vocab_size": np.array(5000), "doc_max_timesteps": np.array(80)}
        np.savez_compressed(os.path.join(HERE, "model_hsg_cfg5.npz"), **graph_arrays(cdocs), **compact(res),
                            **extra, **meta)
    if args.only == "stack_train_cfg2":
        # the TIMED configuration: the fused stack's train mode (dropout 0.1, masks
        # injected, see stack_train_case) on the bench's full cfg2 batch (159,040 edges)
        cdocs = sort_by_sentences(synth.make_batch_docs("cfg2", seed=0))
        res = stack_train_case(GAT, cdocs, 46, 1046)
        np.savez_compressed(os.path.join(HERE, "stack_train_cfg2.npz"), **graph_arrays(cdocs), **compact(res), **meta)
    if want("s2s_small"):
        # S2S on an HSG batch (w->s phantoms, s->s typed; a sentence with no words)
        # and an HDSG batch (doc nodes: s->doc typed, w->doc phantoms)
        rng = np.random.default_rng(16)
        hs = sort_by_sentences([synth.make_hsg_doc(rng, N=5, W=16, k=4, k_jitter=4, isolated_words=2,
                                                   vocab_size=500, tf_range=(0.0, 1.0)),
                                synth.make_hsg_doc(rng, N=3, W=9, k=3, vocab_size=500),
                                synth.make_hsg_doc(rng, N=6, W=8, k=1, k_jitter=1, vocab_size=500)])
        rng = np.random.default_rng(17)
        hd = sort_by_sentences([synth.make_hdsg_example(rng, (3, 2), W=20, k=4, doc_words=6, vocab_size=500),
                                synth.make_hdsg_example(rng, (2, 1, 2), W=15, k=3, doc_words=5, vocab_size=500)])
        out = {}
        for tag, docs, sd in (("hsg", hs, 31), ("hdsg", hd, 32)):
            out.update({f"{tag}.{k}": v for k, v in compact({**graph_arrays(docs), **s2s_case(GAT, docs, sd)}).items()})
        np.savez_compressed(os.path.join(HERE, "s2s_small.npz"), **out, **meta)
    if args.only is not None:
        return

    # edge-case graph: zero-typed sentences (phantoms only), isolated words,
    # every tf-idf box 0..9, degree-1 words
    rng = np.random.default_rng(11)
    small = [synth.make_hsg_doc(rng, N=5, W=16, k=4, k_jitter=4, isolated_words=2, vocab_size=500,
                                tf_range=(0.0, 1.0)),
             synth.make_hsg_doc(rng, N=3, W=9, k=3, vocab_size=500, tf_range=(0.0, 1.0))]
    small = sort_by_sentences(small)
    res = gat_case(GAT, small, 1, full_grads=False)
    np.savez_compressed(os.path.join(HERE, "gat_small.npz"), **graph_arrays(small), **compact(res), **meta)

    rng = np.random.default_rng(12)
    hd = [synth.make_hdsg_example(rng, (3, 2), W=20, k=4, doc_words=6, vocab_size=500,
                                  tf_range=(0.0, 1.0)),
          synth.make_hdsg_example(rng, (2, 1, 2), W=15, k=3, doc_words=5, vocab_size=500,
                                  tf_range=(0.0, 1.0))]
    hd = sort_by_sentences(hd)
    res = gat_case(GAT, hd, 2, full_grads=False)
    np.savez_compressed(os.path.join(HERE, "gat_hdsg_small.npz"), **graph_arrays(hd), **compact(res), **meta)

    cfg1 = sort_by_sentences(synth.make_batch_docs("cfg1", seed=0))
    res = gat_case(GAT, cfg1, 3, full_grads=False, keep_rows=160)
    np.savez_compressed(os.path.join(HERE, "gat_cfg1.npz"), **graph_arrays(cfg1), **compact(res), **meta)

    rng = np.random.default_rng(13)
    mdocs = sort_by_sentences([synth.make_hsg_doc(rng, N=6, W=24, k=5, k_jitter=2, vocab_size=500),
                               synth.make_hsg_doc(rng, N=4, W=14, k=4, vocab_size=500)])
    res = model_case(HiGraph, mdocs, 4, "HSumGraph")
    extra = {"sent_words": np.concatenate([d.words for d in mdocs]).astype(np.int32),
             "sent_label": np.concatenate([d.label for d in mdocs]).astype(np.int8)}
    np.savez_compressed(os.path.join(HERE, "model_hsg.npz"), **graph_arrays(mdocs), **compact(res), **extra, **meta)

    rng = np.random.default_rng(14)
    hdocs = sort_by_sentences([synth.make_hdsg_example(rng, (3, 2), W=22, k=4, doc_words=6, vocab_size=500),
                               synth.make_hdsg_example(rng, (2, 2), W=16, k=3, doc_words=5, vocab_size=500)])
    res = model_case(HiGraph, hdocs, 5, "HSumDocGraph")
    extra = {"sent_words": np.concatenate([d.words for d in hdocs]).astype(np.int32),
             "sent_label": np.concatenate([d.label for d in hdocs]).astype(np.int8)}
    np.savez_compressed(os.path.join(HERE, "model_hdsg.npz"), **graph_arrays(hdocs), **compact(res), **extra, **meta)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
