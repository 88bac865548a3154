"""Native document-graph construction (libhsg_host.so, include/hsg_graph.h).

The reference builds each document graph in Python with one ``add_edges`` call per
edge (module/dataloader.py:222-268 HSG, 328-406 HDSG).  Here the Python side only
tokenises (word ids, padding, labels -- the reference's Example / Example2) and
maps each sentence's tf-idf JSON object to (word id, value) pairs; the C++
builder discovers word nodes and emits every edge in the reference's order, for a
whole list of documents at once on a thread pool.  The result is one
:class:`~hetersumgraph_amd.synth.DocArrays` per document, turned into a
DGL-0.4-compatible graph by :func:`hetersumgraph_amd.synth.to_graph`.

The library is host-only (g++ -> libhsg_host.so, no HIP runtime), so it can run
inside DataLoader worker processes that never touch the GPU.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .synth import DocArrays

_HERE = os.path.dirname(os.path.abspath(__file__))
HOST_LIB = os.path.join(_HERE, "libhsg_host.so")
HSG_GRAPH_EINVAL = 2001

_P = ctypes.c_void_p


class HsgDocs(ctypes.Structure):
    """struct hsg_docs (include/hsg_graph.h)."""
    _fields_ = [("n_docs", ctypes.c_int32), ("sent_max_len", ctypes.c_int32),
                ("doc_nsent", _P), ("sent_ids", _P), ("sent_tf_ptr", _P), ("sent_tf_wid", _P),
                ("sent_tf_val", _P), ("doc_narticle", _P), ("sent_article", _P), ("art_word_ptr", _P),
                ("art_word_ids", _P), ("art_tf_ptr", _P), ("art_tf_wid", _P), ("art_tf_val", _P)]


_lib = None


def host_lib():
    """The native builder; raises if libhsg_host.so was not built (no Python fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(HOST_LIB):
            raise RuntimeError(f"{HOST_LIB} is missing: build it with `python -m hetersumgraph_amd.build`")
        lib = ctypes.CDLL(HOST_LIB)
        lib.hsg_graph_count.argtypes = [ctypes.POINTER(HsgDocs), ctypes.c_int64, _P, _P, _P, ctypes.c_int]
        lib.hsg_graph_fill.argtypes = [ctypes.POINTER(HsgDocs), ctypes.c_int64, _P, _P, _P] + [_P] * 8 + [ctypes.c_int]
        lib.hsg_graph_count.restype = ctypes.c_int
        lib.hsg_graph_fill.restype = ctypes.c_int
        _lib = lib
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def tfidf_pairs(tfw, vocab):
    """A sentence's (or document's) tf-idf JSON object {word: value} as id / value
    arrays: exactly the entries the reference's ``vocab.id2word(wid) in tfw`` test
    can hit, i.e. the words that map back to themselves through the vocab."""
    wids, vals = [], []
    for k, v in tfw.items():
        w = vocab.word2id(k)
        if vocab.id2word(w) == k:
            wids.append(w)
            vals.append(float(v))
    return np.asarray(wids, np.int64), np.asarray(vals, np.float64)


def _csr(parts, dtype):
    ptr = np.zeros(len(parts) + 1, np.int64)
    ptr[1:] = np.cumsum([len(p) for p in parts])
    data = np.concatenate(parts).astype(dtype) if parts and ptr[-1] else np.zeros(0, dtype)
    return ptr, data


def build_doc_arrays(docs, sent_max_len, filterids, multi=False, threads=0):
    """Graphs of many documents in one native call.

    ``docs``: list of dicts with
      ``sent_pad``  [N][sent_max_len] padded word ids (already truncated to
                    doc_max_timesteps), ``sent_tf``  N (wids, vals) pairs,
      ``label``     [N, doc_max_timesteps] (sentence node column),
    and for ``multi`` (HDSG) also
      ``sent2doc``  [N] document node of each sentence, ``n_art`` document nodes,
      ``art_words`` n_art word-id lists, ``art_tf`` n_art (wids, vals) pairs.
    Returns one DocArrays per document (local node ids)."""
    lib = host_lib()
    B = len(docs)
    L = int(sent_max_len)
    nsent = np.asarray([len(d["sent_pad"]) for d in docs], np.int32)
    sent_ids = (np.concatenate([np.asarray(d["sent_pad"], np.int64).reshape(-1, L) for d in docs])
                if nsent.sum() else np.zeros((0, L), np.int64))
    sent_ids = np.ascontiguousarray(sent_ids)
    stp, stw = _csr([t[0] for d in docs for t in d["sent_tf"]], np.int64)
    _, stv = _csr([t[1] for d in docs for t in d["sent_tf"]], np.float64)
    keep = [sent_ids, stp, stw, stv]
    s = HsgDocs(B, L, _ptr(nsent), _ptr(sent_ids), _ptr(stp), _ptr(stw), _ptr(stv))
    if multi:
        nart = np.asarray([d["n_art"] for d in docs], np.int32)
        sart = np.concatenate([np.asarray(d["sent2doc"], np.int32) for d in docs]) if nsent.sum() else \
            np.zeros(0, np.int32)
        awp, awi = _csr([np.asarray(w, np.int64) for d in docs for w in d["art_words"]], np.int64)
        atp, atw = _csr([t[0] for d in docs for t in d["art_tf"]], np.int64)
        _, atv = _csr([t[1] for d in docs for t in d["art_tf"]], np.float64)
        keep += [nart, sart, awp, awi, atp, atw, atv]
        s.doc_narticle, s.sent_article = _ptr(nart), _ptr(sart)
        s.art_word_ptr, s.art_word_ids = _ptr(awp), _ptr(awi)
        s.art_tf_ptr, s.art_tf_wid, s.art_tf_val = _ptr(atp), _ptr(atw), _ptr(atv)
    filt = np.asarray(sorted(set(int(x) for x in filterids)), np.int64)
    nn = np.zeros(B, np.int64)
    ne = np.zeros(B, np.int64)
    rc = lib.hsg_graph_count(ctypes.byref(s), len(filt), _ptr(filt), _ptr(nn), _ptr(ne), int(threads))
    if rc:
        raise ValueError(f"hsg_graph_count: invalid document arrays ({rc})")
    noff = np.concatenate([[0], np.cumsum(nn)[:-1]]).astype(np.int64)
    eoff = np.concatenate([[0], np.cumsum(ne)[:-1]]).astype(np.int64)
    Nn, Ne = int(nn.sum()), int(ne.sum())
    unit, ndt = np.empty(Nn, np.float32), np.empty(Nn, np.float32)
    wid = np.empty(Nn, np.int64)
    src, dst, tf = np.empty(Ne, np.int64), np.empty(Ne, np.int64), np.empty(Ne, np.int64)
    et = np.empty(Ne, np.float32)
    sent_node = np.empty(int(nsent.sum()), np.int64)
    rc = lib.hsg_graph_fill(ctypes.byref(s), len(filt), _ptr(filt), _ptr(noff), _ptr(eoff), _ptr(unit), _ptr(ndt),
                            _ptr(wid), _ptr(src), _ptr(dst), _ptr(tf), _ptr(et), _ptr(sent_node), int(threads))
    if rc:
        raise ValueError(f"hsg_graph_fill: invalid document arrays ({rc})")
    out = []
    s0 = 0
    for b, d in enumerate(docs):
        n0, n1 = noff[b], noff[b] + nn[b]
        e0, e1 = eoff[b], eoff[b] + ne[b]
        N = int(nsent[b])
        out.append(DocArrays(
            n_nodes=int(nn[b]), unit=unit[n0:n1].copy(), ndtype=ndt[n0:n1].copy(), wid=wid[n0:n1].copy(),
            src=src[e0:e1] - n0, dst=dst[e0:e1] - n0, tffrac=tf[e0:e1].copy(), edtype=et[e0:e1].copy(),
            sent_nodes=sent_node[s0:s0 + N] - n0,
            words=np.asarray(d["sent_pad"], np.int64).reshape(N, L),
            position=np.arange(1, N + 1, dtype=np.int64).reshape(-1, 1),
            label=np.asarray(d["label"], np.int64).reshape(N, -1)))
        s0 += N
    return out
