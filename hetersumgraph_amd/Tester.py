"""Evaluation-time sentence selection (reference: Tester.py:8-196, tools/utils.py:45-55).

Same classes, constructor arguments, ``evaluation(G, index, dataset, blocking)``
contract and accumulated state (``extracts``, ``hyps``, ``refer``, ``running_avg_loss``,
``pred/true/match/match_true``, ``getMetric`` -> accu / precision / recall / F) as the
reference, so evaluation.py's loop and ``train.py``'s validation run unchanged.

What differs is *how*: the reference unbatches the graph and, per document, filters
its sentence nodes, runs ``topk`` and compares against the labels (Tester.py:105-140)
-- a Python loop of small tensor ops per document.  Here the per-document loss sums,
the top-k selection (one ``topk`` over the [docs, max_sentences] padded score
matrix) and the match counters are batched tensor ops on the logits' device, with
one device->host copy per batch for the selected indices; only the string work
(n-gram blocking, hypothesis assembly) stays on the host.
"""
from __future__ import annotations

import datetime
import logging
import os

import torch

from .HiGraph import node_ids, sentence_counts

logger = logging.getLogger("Summarization logger")


def eval_label(match_true, pred, true, total, match):
    """tools/utils.py:45-55 (tensor arithmetic: a zero count gives nan/inf, as there)."""
    match_true, pred, true, match = (torch.as_tensor(x).float() for x in (match_true, pred, true, match))
    try:
        accu = match / total
        precision = match_true / pred
        recall = match_true / true
        F = 2 * precision * recall / (precision + recall)
    except ZeroDivisionError:
        accu, precision, recall, F = 0.0, 0.0, 0.0, 0.0
        logger.error("[Error] float division by zero")
    return accu, precision, recall, F


class TestPipLine:
    """Tester.py:8-75."""

    def __init__(self, model, m, test_dir, limited):
        self.model = model
        self.limited = limited
        self.m = m
        self.test_dir = test_dir
        self.extracts = []
        self.batch_number = 0
        self.running_loss = 0
        self.example_num = 0
        self.total_sentence_num = 0
        self._hyps = []
        self._refer = []

    def evaluation(self, G, index, valset):
        pass

    def getMetric(self):  # noqa: N802 (reference name)
        pass

    def SaveDecodeFile(self):  # noqa: N802
        now = datetime.datetime.now().strftime("%Y%m%d_%H%M%S")
        with open(os.path.join(self.test_dir, now), "wb") as f:
            for i in range(self.rougePairNum):
                f.write(b"[Reference]\t" + self._refer[i].encode("utf-8") + b"\n")
                f.write(b"[Hypothesis]\t" + self._hyps[i].encode("utf-8") + b"\n\n\n")

    @property
    def running_avg_loss(self):
        return self.running_loss / self.batch_number

    @property
    def rougePairNum(self):  # noqa: N802
        return len(self._hyps)

    @property
    def hyps(self):
        if not self.limited:
            return self._hyps
        # limited-length recall: cut each hypothesis to its reference's word count
        return [" ".join(h.split(" ")[:len(r.split(" "))]) for h, r in zip(self._hyps, self._refer)]

    @property
    def refer(self):
        return self._refer

    @property
    def extractLabel(self):  # noqa: N802
        return self.extracts


def _select(p_sent, counts, m):
    """Per-document selected sentence indices (local), in the reference's order:
    m == 0 -> argmax(p) != 0 in ascending index order (Tester.py:115-117); else
    topk(p[:, 1], min(m, N)) in descending score order (124)."""
    dev = p_sent.device
    B = len(counts)
    if m == 0:
        pred = p_sent.max(1)[1].ne(0).cpu()
        out, o = [], 0
        for n in counts:
            out.append(torch.nonzero(pred[o:o + n]).view(-1))
            o += n
        return out
    nmax = max(counts) if counts else 0
    cnt = torch.tensor(counts, device=dev)
    seg = torch.repeat_interleave(torch.arange(B, device=dev), cnt)
    start = torch.cumsum(cnt, 0) - cnt
    local = torch.arange(p_sent.shape[0], device=dev) - start[seg]
    score = p_sent.new_full((B, max(nmax, 1)), float("-inf"))
    score[seg, local] = p_sent[:, 1]
    k = min(m, nmax)
    top = torch.topk(score, k, dim=1).indices.cpu() if k > 0 else torch.zeros(B, 0, dtype=torch.long)
    return [top[j, :min(m, n)] for j, n in enumerate(counts)]


class SLTester(TestPipLine):
    """Tester.py:78-196."""

    def __init__(self, model, m, test_dir=None, limited=False, blocking_win=3):
        super().__init__(model, m, test_dir, limited)
        self.pred, self.true, self.match, self.match_true = 0, 0, 0, 0
        self._F = 0
        self.criterion = torch.nn.CrossEntropyLoss(reduction="none")
        self.blocking_win = blocking_win

    def evaluation(self, G, index, dataset, blocking=False):
        self.batch_number += 1
        outputs = self.model.forward(G)
        snode = node_ids(G, "dtype", 1.0)
        label = G.ndata["label"][snode].sum(-1)                               # [n_sent]
        counts = sentence_counts(G)
        B = len(counts)
        # dgl.sum_nodes(G, "loss").mean(): per-document sums of the sentence losses
        seg = torch.repeat_interleave(torch.arange(B, device=outputs.device),
                                      torch.tensor(counts, device=outputs.device))
        loss_s = self.criterion(outputs, label)
        per_doc = loss_s.new_zeros(B).index_add(0, seg, loss_s)
        self.running_loss += float(per_doc.mean())

        p_host = outputs.detach().cpu() if blocking else None
        sel = None if blocking else _select(outputs.detach(), counts, self.m)
        label_h = label.cpu()
        o = 0
        for j in range(B):
            N = counts[j]
            example = dataset.get_example(index[j])
            sents = example.original_article_sents
            if blocking and self.m != 0:
                pred_idx = self.ngram_blocking(sents, p_host[o:o + N, 1], self.blocking_win, min(self.m, N))
            elif blocking:
                pred_idx = _select(p_host[o:o + N], [N], 0)[0]
            else:
                pred_idx = sel[j]
            prediction = torch.zeros(N, dtype=torch.long)
            prediction[pred_idx] = 1
            lab = label_h[o:o + N]
            self.extracts.append(pred_idx.tolist())
            self.pred += prediction.sum()
            self.true += lab.sum()
            self.match_true += ((prediction == lab) & (prediction == 1)).sum()
            self.match += (prediction == lab).sum()
            self.total_sentence_num += N
            self.example_num += 1
            self._hyps.append("\n".join(sents[i] for i in pred_idx.tolist() if i < len(sents)))
            self._refer.append(example.original_abstract)
            o += N

    def getMetric(self):  # noqa: N802
        logger.info("[INFO] Validset match_true %d, pred %d, true %d, total %d, match %d",
                    self.match_true, self.pred, self.true, self.total_sentence_num, self.match)
        self._accu, self._precision, self._recall, self._F = eval_label(
            self.match_true, self.pred, self.true, self.total_sentence_num, self.match)
        logger.info("[INFO] The size of totalset is %d, sent_number is %d, accu is %f, precision is %f, "
                    "recall is %f, F is %f", self.example_num, self.total_sentence_num, self._accu,
                    self._precision, self._recall, self._F)

    def ngram_blocking(self, sents, p_sent, n_win, k):
        """Tester.py:161-191: greedy by descending score, skip a sentence sharing an
        n-gram with the ones already chosen.  Keeps the reference's window range
        ``range(len(pieces) - n_win)`` (the last n-gram of a sentence is not used)."""
        seen = set()
        chosen = []
        for idx in p_sent.sort(descending=True)[1].tolist():
            pieces = sents[idx].split()
            grams = [" ".join(pieces[i:i + n_win]) for i in range(len(pieces) - n_win)]
            if any(g in seen for g in grams):
                continue
            chosen.append(idx)
            seen.update(grams)
            if len(chosen) >= k:
                break
        return torch.LongTensor(chosen)

    @property
    def labelMetric(self):  # noqa: N802
        return self._F
