"""Dataset / graph-construction surface of the reference (module/dataloader.py),
with the graph built by the native builder (:mod:`hetersumgraph_amd.datapipe`).

Same class names, constructor arguments and item format as the reference, so
train.py's ``ExampleSet(...)`` / ``MultiExampleSet(...)`` + ``DataLoader(...,
collate_fn=graph_collate_fn)`` (train.py:345-367) run unchanged:

* ``Example`` / ``Example2`` (dataloader.py:56-137): whitespace tokens, lower-cased
  vocab ids, padding/truncation to sent_max_len, the label matrix, and the
  per-document word lists of multi-document examples;
* ``ExampleSet.__getitem__`` / ``MultiExampleSet.__getitem__`` -> ``(G, index)``;
* ``graph_collate_fn`` (dataloader.py:472-481): sort by sentence count (the
  reference's ``torch.sort(..., descending=True)``) and ``dgl.batch``;
* ``LoadHiExampleSet`` (dataloader.py:426-440): a directory of cached
  ``<index>.graph.bin`` graphs read with ``load_graphs`` -- this build's on-disk
  format (hetersumgraph_amd/dgl/data/utils.py), not DGL's binary one.

One difference: the reference's stop-word list comes from nltk
(``stopwords.words('english')``, dataloader.py:48), which is not installed here;
pass it as ``stopwords=`` (default: none; the punctuation list and the low tf-idf
filter words are applied as in the reference).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from .. import graph as hg
from ..datapipe import build_doc_arrays, tfidf_pairs
from ..synth import to_graph

PUNCTUATIONS = [',', '.', ':', ';', '?', '(', ')', '[', ']', '&', '!', '*', '@', '#', '$', '%', "''", "'", '`',
                '``', '-', '--', '|', '\\/']       # dataloader.py:49-50


def readJson(fname):  # noqa: N802 (reference name)
    with open(fname, encoding="utf-8") as f:
        return [json.loads(line) for line in f]


def readText(fname):  # noqa: N802
    with open(fname, encoding="utf-8") as f:
        return [line.strip() for line in f]


def catDoc(textlist):  # noqa: N802
    return [w for t in textlist for w in t]


class Example:
    """dataloader.py:56-109: token ids, padded ids and the label matrix of one example."""

    def __init__(self, article_sents, abstract_sents, vocab, sent_max_len, label):
        self.sent_max_len = sent_max_len
        self.original_article_sents = article_sents
        self.original_abstract = "\n".join(abstract_sents)
        if isinstance(article_sents, list) and article_sents and isinstance(article_sents[0], list):
            self.original_article_sents = [s for doc in article_sents for s in doc]
        self.enc_sent_input = [[vocab.word2id(w.lower()) for w in s.split()] for s in self.original_article_sents]
        self.enc_sent_len = [len(s.split()) for s in self.original_article_sents]
        pad_id = vocab.word2id("[PAD]")
        self.enc_sent_input_pad = [ids[:sent_max_len] + [pad_id] * max(0, sent_max_len - len(ids))
                                   for ids in self.enc_sent_input]
        self.label = label
        self.label_matrix = np.zeros((len(self.original_article_sents), len(label)), dtype=int)
        if label != []:
            self.label_matrix[np.array(label), np.arange(len(label))] = 1


class Example2(Example):
    """dataloader.py:112-137: plus per-document lengths and concatenated word ids."""

    def __init__(self, article_sents, abstract_sents, vocab, sent_max_len, label):
        super().__init__(article_sents, abstract_sents, vocab, sent_max_len, label)
        cur = 0
        self.original_articles, self.article_len, self.enc_doc_input = [], [], []
        for doc in article_sents:
            if len(doc) == 0:
                continue
            self.original_articles.append(" ".join(doc))
            self.article_len.append(len(doc))
            self.enc_doc_input.append(catDoc(self.enc_sent_input[cur:cur + len(doc)]))
            cur += len(doc)


def map_sent2doc(article_len, sent_num):
    """MultiExampleSet.MapSent2Doc (dataloader.py:316-327), including its early exit
    at ``sentNo > sentNum`` (one sentence past the truncated count is mapped)."""
    sent2doc, sent_no = {}, 0
    for i, n in enumerate(article_len):
        for _ in range(n):
            sent2doc[sent_no] = i
            sent_no += 1
            if sent_no > sent_num:
                return sent2doc
    return sent2doc


class ExampleSet(torch.utils.data.Dataset):
    """Single-document dataset (dataloader.py:142-286); graphs built natively."""

    def __init__(self, data_path, vocab, doc_max_timesteps, sent_max_len, filter_word_path, w2s_path,
                 stopwords=(), threads=1):
        self.vocab = vocab
        self.sent_max_len = sent_max_len
        self.doc_max_timesteps = doc_max_timesteps
        self.example_list = readJson(data_path)
        self.size = len(self.example_list)
        self.threads = threads
        # dataloader.py:166-179: stop words + punctuation + [PAD] + up to 5001 low tf-idf words
        self.filterwords = list(stopwords) + PUNCTUATIONS
        self.filterids = [vocab.word2id(w.lower()) for w in self.filterwords]
        self.filterids.append(vocab.word2id("[PAD]"))
        lowtfidf_num = 0
        for w in readText(filter_word_path):
            if vocab.word2id(w) != vocab.word2id("[UNK]"):
                self.filterwords.append(w)
                self.filterids.append(vocab.word2id(w))
                lowtfidf_num += 1
            if lowtfidf_num > 5000:
                break
        self.w2s_tfidf = readJson(w2s_path)

    def get_example(self, index):
        e = self.example_list[index]
        e["summary"] = e.setdefault("summary", [])
        return Example(e["text"], e["summary"], self.vocab, self.sent_max_len, e["label"])

    def pad_label_m(self, label_matrix):
        m = label_matrix[:self.doc_max_timesteps, :self.doc_max_timesteps]
        N, k = m.shape
        if k < self.doc_max_timesteps:
            return np.hstack([m, np.zeros((N, self.doc_max_timesteps - k))])
        return m

    def doc_item(self, index):
        """The native builder's input for example ``index`` (see datapipe)."""
        item = self.get_example(index)
        input_pad = item.enc_sent_input_pad[:self.doc_max_timesteps]
        w2s_w = self.w2s_tfidf[index]
        return dict(sent_pad=input_pad, label=self.pad_label_m(item.label_matrix),
                    sent_tf=[tfidf_pairs(w2s_w[str(i)], self.vocab) for i in range(len(input_pad))])

    def graph_arrays(self, indices):
        return build_doc_arrays([self.doc_item(i) for i in indices], self.sent_max_len, self.filterids,
                                threads=self.threads)

    def __getitem__(self, index):
        return to_graph(self.graph_arrays([index])[0], hg.DGLGraph), index

    def __len__(self):
        return self.size


class MultiExampleSet(ExampleSet):
    """Multi-document dataset (dataloader.py:289-423); graphs built natively."""

    def __init__(self, data_path, vocab, doc_max_timesteps, sent_max_len, filter_word_path, w2s_path, w2d_path,
                 stopwords=(), threads=1):
        super().__init__(data_path, vocab, doc_max_timesteps, sent_max_len, filter_word_path, w2s_path,
                         stopwords=stopwords, threads=threads)
        self.w2d_tfidf = readJson(w2d_path)

    def get_example(self, index):
        e = self.example_list[index]
        e["summary"] = e.setdefault("summary", [])
        return Example2(e["text"], e["summary"], self.vocab, self.sent_max_len, e["label"])

    def doc_item(self, index):
        item = self.get_example(index)
        sent_pad = item.enc_sent_input_pad[:self.doc_max_timesteps]
        N = len(sent_pad)
        sent2doc = map_sent2doc(item.article_len, N)
        n_art = len(set(sent2doc.values()))
        w2s_w, w2d_w = self.w2s_tfidf[index], self.w2d_tfidf[index]
        return dict(sent_pad=sent_pad, label=self.pad_label_m(item.label_matrix),
                    sent_tf=[tfidf_pairs(w2s_w[str(i)], self.vocab) for i in range(N)],
                    sent2doc=[sent2doc[i] for i in range(N)], n_art=n_art,
                    art_words=[item.enc_doc_input[a] for a in range(n_art)],
                    art_tf=[tfidf_pairs(w2d_w[str(a)], self.vocab) for a in range(n_art)])

    def graph_arrays(self, indices):
        return build_doc_arrays([self.doc_item(i) for i in indices], self.sent_max_len, self.filterids,
                                multi=True, threads=self.threads)


def graph_collate_fn(samples):
    """dataloader.py:472-481: batch sorted by sentence count, descending."""
    graphs, index = map(list, zip(*samples))
    graph_len = [len(g.filter_nodes(lambda nodes: nodes.data["dtype"] == 1)) for g in graphs]
    sorted_len, sorted_index = torch.sort(torch.LongTensor(graph_len), dim=0, descending=True)
    batched_graph = hg.batch([graphs[idx] for idx in sorted_index])
    return batched_graph, [index[idx] for idx in sorted_index]


class LoadHiExampleSet(torch.utils.data.Dataset):
    """dataloader.py:426-440: item ``index`` is graph 0 of ``<data_root>/<index>.graph.bin``
    (written by ``save_graphs``), returned as ``(G, index)`` like ExampleSet."""

    def __init__(self, data_root):
        super().__init__()
        self.data_root = data_root
        self.gfiles = [f for f in os.listdir(self.data_root) if f.endswith("graph.bin")]

    def __getitem__(self, index):
        from ..dgl.data.utils import load_graphs
        g, _labels = load_graphs(os.path.join(self.data_root, "%d.graph.bin" % index))
        return g[0], index

    def __len__(self):
        return len(self.gfiles)
