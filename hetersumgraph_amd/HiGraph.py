"""HSumGraph / HSumDocGraph (reference: HiGraph.py:34-255).

Same constructor ``(hps, embed)``, same ``forward(graph) -> [n_sent, 2]`` logits and
the same state_dict keys/shapes, so reference checkpoints load
and ``train.py``'s loop (train.py:101-135) runs unchanged on a
:class:`hetersumgraph_amd.graph.DGLGraph`.  Module registration order follows the
reference so that a given ``torch.manual_seed`` yields the same initial weights.

What differs is *how* the graph is read: node/edge subsets (filter_nodes /
filter_edges), per-graph sentence counts (dgl.unbatch, HiGraph.py:248) and the
HDSG doc<->sentence bookkeeping (the Python loops at HiGraph.py:219-226, 236-243)
are computed once per batch on the host and cached on the graph as index
tensors; the WSWGAT layers run the fused HIP kernels.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.utils.rnn as rnn

from .graph import TableColumn
from .module.Encoder import sentEncoder
from .module.GAT import WSWGAT
from .module.GATLayer import CHECK_NAN, TFIDF_TAG
from .module.PositionEmbedding import get_sinusoid_encoding_table
from .stack import fused_stack_ok
from .stack import gat_stack as fused_gat_stack


def _cached(graph, key, fn):
    k = (key, str(graph.device))
    if k not in graph._rel_cache:
        graph._rel_cache[k] = fn()
    return graph._rel_cache[k]


def _dev(graph, arr):
    return torch.from_numpy(np.ascontiguousarray(arr)).to(graph.device)


def node_ids(graph, column, value):
    """Cached ``filter_nodes(lambda n: n.data[column] == value)`` (ascending ids)."""
    host = {"unit": "unit", "dtype": "ndtype"}[column]

    def build():
        col = graph.host_column(host)
        return _dev(graph, np.nonzero(col == value)[0].astype(np.int64))
    return _cached(graph, ("nodes", column, value), build)


def sentence_counts(graph):
    """Sentences per member graph, in batch order (get_snode_feat, HiGraph.py:247-255)."""
    def build():
        nd = graph.host_column("ndtype")
        counts = getattr(graph, "batch_num_nodes", None) or [graph.number_of_nodes()]
        offs = np.cumsum([0] + list(counts))
        return [int((nd[offs[i]:offs[i + 1]] == 1).sum()) for i in range(len(counts))]
    return _cached(graph, "sent_counts", build)


def register_tfidf_table(graph, weight):
    """``graph.edges[dtype==0].data['tfidfembed'] = _TFembed(tffrac)`` (HiGraph.py:146-151),
    stored as a table column: rows of ``weight`` selected by ``tffrac`` on dtype-0
    edges, initializer zeros elsewhere."""
    idx = _cached(graph, "tfidf_index", lambda: torch.where(
        graph.edata["dtype"] == 0, graph.edata["tffrac"].long(),
        torch.full_like(graph.edata["tffrac"].long(), -1)))
    graph._eframe().set("tfidfembed", TableColumn(weight, idx, TFIDF_TAG))


class HSumGraph(nn.Module):
    """Single-document HeterSumGraph (HiGraph.py:34-161)."""

    def __init__(self, hps, embed):
        super().__init__()
        self._hps = hps
        self._n_iter = hps.n_iter
        self._embed = embed
        self.embed_size = hps.word_emb_dim
        self._init_sn_param()
        self._TFembed = nn.Embedding(10, hps.feat_embed_size)        # 10 tf-idf boxes
        self.n_feature_proj = nn.Linear(hps.n_feature_size * 2, hps.hidden_size, bias=False)
        self.word2sent = WSWGAT(in_dim=hps.word_emb_dim, out_dim=hps.hidden_size, num_heads=hps.n_head,
                                attn_drop_out=hps.atten_dropout_prob,
                                ffn_inner_hidden_size=hps.ffn_inner_hidden_size,
                                ffn_drop_out=hps.ffn_dropout_prob,
                                feat_embed_size=hps.feat_embed_size, layerType="W2S")
        self.sent2word = WSWGAT(in_dim=hps.hidden_size, out_dim=hps.word_emb_dim,
                                num_heads=6,                               # HiGraph.py:70
                                attn_drop_out=hps.atten_dropout_prob,
                                ffn_inner_hidden_size=hps.ffn_inner_hidden_size,
                                ffn_drop_out=hps.ffn_dropout_prob,
                                feat_embed_size=hps.feat_embed_size, layerType="S2W")
        self.n_feature = hps.hidden_size
        self.wh = nn.Linear(self.n_feature, 2)

    def _init_sn_param(self):
        hps = self._hps
        self.sent_pos_embed = nn.Embedding.from_pretrained(
            get_sinusoid_encoding_table(hps.doc_max_timesteps + 1, self.embed_size, padding_idx=0),
            freeze=True)
        self.cnn_proj = nn.Linear(self.embed_size, hps.n_feature_size)
        self.lstm_hidden_state = hps.lstm_hidden_state
        self.lstm = nn.LSTM(self.embed_size, self.lstm_hidden_state, num_layers=hps.lstm_layers,
                            dropout=0.1, batch_first=True, bidirectional=hps.bidirectional)
        mult = 2 if hps.bidirectional else 1
        self.lstm_proj = nn.Linear(self.lstm_hidden_state * mult, hps.n_feature_size)
        self.ngram_enc = sentEncoder(hps, self._embed)

    # ---------------------------------------------------------------- forward
    def gat_stack(self, graph, word_feature, sent_feature):
        """W2S, then n_iter x (S2W, W2S) (HiGraph.py:99-106) -> supernode state.

        On a ROCm device with the TF-IDF table column registered by set_wnfeature
        the stack runs as one autograd node (:mod:`hetersumgraph_amd.stack`); the
        per-layer loop below is the same computation through WSWGAT.forward."""
        T = self._TFembed.weight
        if fused_stack_ok(graph, self.word2sent, self.sent2word, T, word_feature, sent_feature):
            return fused_gat_stack(graph, self.word2sent, self.sent2word, T, word_feature, sent_feature,
                                   self._n_iter)
        word_state = word_feature
        sent_state = self.word2sent(graph, word_feature, sent_feature)
        for _ in range(self._n_iter):
            word_state = self.sent2word(graph, word_state, sent_state)
            sent_state = self.word2sent(graph, word_state, sent_state)
        return sent_state

    def forward(self, graph):
        word_feature = self.set_wnfeature(graph)
        sent_feature = self.n_feature_proj(self.set_snfeature(graph))
        sent_state = self.gat_stack(graph, word_feature, sent_feature)
        return self.wh(sent_state)

    # --------------------------------------------------------- node features
    def set_wnfeature(self, graph):
        """Word embeddings; registers ``tfidfembed = _TFembed(tffrac)`` on dtype-0
        edges (HiGraph.py:144-152) as a table column."""
        wnode_id = node_ids(graph, "unit", 0.0)
        wid = graph.ndata["id"][wnode_id]
        w_embed = self._embed(wid)
        register_tfidf_table(graph, self._TFembed.weight)
        return w_embed

    def _sent_cnn_feature(self, graph, snode_id):
        ngram_feature = self.ngram_enc(graph.ndata["words"][snode_id])           # [n_s, 300]
        snode_pos = graph.ndata["position"][snode_id].view(-1)
        cnn_feature = self.cnn_proj(ngram_feature + self.sent_pos_embed(snode_pos))
        return ngram_feature, cnn_feature

    def _sent_lstm_feature(self, features, glen):
        """HiGraph.py:135-142 on the per-document feature list (see _sent_lstm_rows)."""
        return self._sent_lstm_rows(torch.cat(features, dim=0) if len(features) != 1 else features[0], glen)

    def _sent_lstm_rows(self, ngram, glen):
        """HiGraph.py:135-142 on the documents' sentence rows laid end to end.  The
        padding to [docs, max_len] and the gather of the valid rows back are one index
        scatter and one index gather (positions cached) instead of a copy per document
        each way; the same values move, so the result is the reference's bit for bit."""
        n_doc, max_len = len(glen), max(glen)
        key = ("lstm_index", tuple(glen))
        idx = getattr(self, "_lstm_idx", None)
        if idx is None or idx[0] != key or idx[1].device != ngram.device:
            doc = torch.repeat_interleave(torch.arange(n_doc), torch.tensor(glen))
            pos = torch.cat([torch.arange(g) for g in glen])
            idx = (key, (doc * max_len + pos).to(ngram.device))
            self._lstm_idx = idx
        flat = idx[1]
        pad_seq = ngram.new_zeros(n_doc * max_len, ngram.shape[1]).index_copy(0, flat, ngram)
        lstm_input = rnn.pack_padded_sequence(pad_seq.view(n_doc, max_len, -1), glen, batch_first=True)
        lstm_output, _ = self.lstm(lstm_input)
        unpacked, _ = rnn.pad_packed_sequence(lstm_output, batch_first=True, total_length=max_len)
        return self.lstm_proj(unpacked.reshape(n_doc * max_len, -1).index_select(0, flat))

    def set_snfeature(self, graph):
        snode_id = node_ids(graph, "dtype", 1.0)
        ngram_feature, cnn_feature = self._sent_cnn_feature(graph, snode_id)
        glen = sentence_counts(graph)
        lstm_feature = self._sent_lstm_rows(ngram_feature, glen)
        return torch.cat([cnn_feature, lstm_feature], dim=1)


def _hdsg_layout(graph):
    """Host bookkeeping of HSumDocGraph.forward (HiGraph.py:191-226, 231-244)."""
    def build():
        g = graph
        g._flush()
        unit = g.host_column("unit")
        nd = g.host_column("ndtype")
        snodes = np.nonzero(nd == 1)[0]
        dnodes = np.nonzero(nd == 2)[0]
        supers = np.nonzero(unit == 1)[0]
        super_rank = np.full(len(unit), -1, np.int64)
        super_rank[supers] = np.arange(len(supers))
        s_rank = np.full(len(unit), -1, np.int64)
        s_rank[snodes] = np.arange(len(snodes))
        d_rank = np.full(len(unit), -1, np.int64)
        d_rank[dnodes] = np.arange(len(dnodes))
        # predecessors of doc nodes that are sentences (HiGraph.py:237)
        sel = np.nonzero((nd[g._src] == 1) & (nd[g._dst] == 2))[0]
        ps, pd = s_rank[g._src[sel]], d_rank[g._dst[sel]]
        cnt = np.bincount(pd, minlength=len(dnodes))
        if len(dnodes) and cnt.min() == 0:
            raise AssertionError("doc_feature_element")    # mean of no sentences is NaN (HiGraph.py:239)
        doc_of_sent = np.full(len(snodes), -1, np.int64)
        doc_of_sent[ps] = pd                                 # last write wins, like the dict
        if (doc_of_sent < 0).any():
            raise KeyError(int(snodes[np.nonzero(doc_of_sent < 0)[0][0]]))   # snid2dnid lookup
        # supernode state = init_feature[supernode_id] with sentence rows then doc rows
        pos = np.zeros(len(supers), np.int64)
        in_s = s_rank[supers] >= 0
        pos[in_s] = s_rank[supers[in_s]]
        pos[~in_s] = len(snodes) + d_rank[supers[~in_s]]
        return dict(pair_s=_dev(g, ps), pair_d=_dev(g, pd),
                    inv_cnt=_dev(g, (1.0 / np.maximum(cnt, 1)).astype(np.float32)),
                    n_docs=len(dnodes), super_pos=_dev(g, pos),
                    sent_super=_dev(g, super_rank[snodes]),
                    doc_super=_dev(g, super_rank[dnodes[doc_of_sent]]))
    return _cached(graph, "hdsg_layout", build)


class HSumDocGraph(HSumGraph):
    """Multi-document variant with doc supernodes (HiGraph.py:166-244)."""

    def __init__(self, hps, embed):
        super().__init__(hps, embed)
        self.dn_feature_proj = nn.Linear(hps.hidden_size, hps.hidden_size, bias=False)
        self.wh = nn.Linear(self.n_feature * 2, 2)

    def set_dnfeature(self, graph, sent_feature):
        """Doc init = mean of its sentences' init features (HiGraph.py:231-244) as a
        segment mean over sentence->doc edges."""
        lay = _hdsg_layout(graph)
        acc = sent_feature.new_zeros(lay["n_docs"], sent_feature.shape[1])
        acc = acc.index_add(0, lay["pair_d"], sent_feature[lay["pair_s"]])
        doc = acc * lay["inv_cnt"].unsqueeze(1)
        if CHECK_NAN:
            assert not torch.any(torch.isnan(doc)), "doc_feature_element"
        return doc

    def forward(self, graph):
        lay = _hdsg_layout(graph)
        word_feature = self.set_wnfeature(graph)
        sent_feature = self.n_feature_proj(self.set_snfeature(graph))
        doc_feature = self.dn_feature_proj(self.set_dnfeature(graph, sent_feature))
        init_state = torch.cat([sent_feature, doc_feature], 0)[lay["super_pos"]]
        super_state = self.gat_stack(graph, word_feature, init_state)
        s_state = torch.cat([super_state[lay["sent_super"]], super_state[lay["doc_super"]]], dim=-1)
        return self.wh(s_state)
