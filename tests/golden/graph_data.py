"""Seeded synthetic dataset files in the reference's on-disk formats, shared by the
graph golden generator (make_graph_golden.py) and the graph-builder tests:

* vocab file: "<word>\\t<count>" per line (module/vocabulary.py:50-62); ids 0-3 are
  [PAD] [UNK] [START] [STOP];
* data JSONL: {"text": [sentences] | [[doc sentences], ...], "summary": [...],
  "label": [sentence indices]} (dataloader.py:185-189, 306-309);
* filter-word file: one word per line, low tf-idf first (script/lowTFIDFWords.py);
* w2s / w2d JSONL: per example {"<sentence|doc index>": {word: tfidf}}
  (script/calw2sTFIDF.py, calw2dTFIDF.py).

The text mixes vocabulary words, out-of-vocabulary words, stop words,
punctuation, upper case, repeats, sentences longer than sent_max_len, more
sentences than doc_max_timesteps, words missing from the tf-idf tables and tf-idf
values on exact .5 boxes (x * 9 = k + 0.5) to exercise half-to-even rounding.
"""
import json
import os

import numpy as np

STOPWORDS = ["the", "a", "of", "and", "to", "in", "is", "it"]      # stands in for nltk's English list
PUNCT = [",", ".", ";", "(", ")", "--", "``"]


class MinVocab:
    """The reference Vocab's mapping (module/vocabulary.py:30-88) over a word list."""

    def __init__(self, words):
        self._w2i = {"[PAD]": 0, "[UNK]": 1, "[START]": 2, "[STOP]": 3}
        for w in words:
            if w not in self._w2i:
                self._w2i[w] = len(self._w2i)
        self._i2w = {i: w for w, i in self._w2i.items()}

    def word2id(self, w):
        return self._w2i.get(w, self._w2i["[UNK]"])

    def id2word(self, i):
        return self._i2w[i]

    def size(self):
        return len(self._w2i)


def _tfidf(rng, words):
    out = {}
    for w in words:
        r = rng.random()
        if r < 0.15:
            continue                                   # word without a tf-idf entry
        if r < 0.35:
            out[w] = (int(rng.integers(0, 9)) + 0.5) / 9.0   # exact half box
        else:
            out[w] = float(rng.uniform(0.0, 1.0))
    return out


def make_files(d, seed=0, n_examples=6, multi=False):
    rng = np.random.default_rng(seed)
    vocab_words = [f"w{i}" for i in range(120)] + STOPWORDS + PUNCT
    oov = [f"oov{i}" for i in range(15)]
    pool = vocab_words + oov
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "vocab"), "w", encoding="utf-8") as f:
        for w in vocab_words:
            f.write(f"{w}\t{int(rng.integers(1, 1000))}\n")
    with open(os.path.join(d, "filter_word.txt"), "w", encoding="utf-8") as f:
        for w in ["w0", "w1", "oov0", "w2", "w3"]:
            f.write(w + "\n")
    data, w2s, w2d = [], [], []
    for e in range(n_examples):
        def sentence():
            n = int(rng.integers(1, 14)) if rng.random() > 0.1 else int(rng.integers(14, 30))
            toks = [pool[int(rng.integers(0, len(pool)))] for _ in range(n)]
            if rng.random() < 0.3 and toks:
                toks.append(toks[0])                   # repeated word
            return " ".join(t.upper() if rng.random() < 0.1 else t for t in toks)
        if multi:
            docs = [[sentence() for _ in range(int(rng.integers(1, 6)))] for _ in range(int(rng.integers(1, 4)))]
            sents = [s for doc in docs for s in doc]
            text = docs
        else:
            sents = [sentence() for _ in range(int(rng.integers(2, 12)))]
            text = sents
        label = sorted(rng.choice(len(sents), size=min(3, len(sents)), replace=False).tolist())
        data.append({"text": text, "summary": ["x"], "label": label})
        w2s.append({str(i): _tfidf(rng, [t.lower() for t in s.split()]) for i, s in enumerate(sents)})
        if multi:
            w2d.append({str(i): _tfidf(rng, [t.lower() for s in doc for t in s.split()]) for i, doc in enumerate(docs)})
    for name, rows in (("data.jsonl", data), ("w2s.jsonl", w2s)) + ((("w2d.jsonl", w2d),) if multi else ()):
        with open(os.path.join(d, name), "w", encoding="utf-8") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return MinVocab(vocab_words)
