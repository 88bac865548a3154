"""Golden vectors for the sentence CNN encoder, from the REFERENCE's own module code.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_encoder_golden.py [--ref /root/reference]

Runs /root/reference/module/Encoder.py (``sentEncoder``, read-only, imported on torch
alone -- SURVEY §8c) on CPU in fp32 and fp64 over a seeded [n, L] batch of token ids
with trailing padding and edge-case lengths (0, 1, below / at / above the widest
kernel, exactly L), and writes ``encoder.npz``: ids, the fp32 and fp64 outputs, and
the gradients of every conv weight / bias and of the word embedding under a seeded
random upstream gradient.  Parameters are regenerated from seeds (weights.py) on both
sides.  Only this script touches the reference.
"""
import argparse
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import weights  # noqa: E402

SEED = 21
N, L, D, V = 14, 20, 300, 64
LENGTHS = [0, 1, 2, 6, 7, 8, 19, 20, 3, 11, 20, 5, 14, 9]


class HPS:
    sent_max_len = L
    word_emb_dim = D
    cuda = False


def make_ids():
    rng = np.random.default_rng(SEED)
    ids = np.zeros((N, L), np.int64)
    for i, n in enumerate(LENGTHS):
        ids[i, :n] = rng.integers(1, V, n)
    # a repeated-token sentence: many equal windows (first-max tie order)
    ids[12, :14] = 5
    return ids


def run(Encoder, dt, ids):
    torch.manual_seed(0)
    embed = torch.nn.Embedding(V, D, padding_idx=0)
    enc = Encoder.sentEncoder(HPS(), embed)
    weights.seed_module(enc, SEED)
    enc = enc.to(dt)
    feat = enc(torch.from_numpy(ids))
    R = torch.from_numpy(weights.feature(SEED, "dfeat", tuple(feat.shape))).to(dt)
    (feat * R).sum().backward()
    res = {"feat": feat.detach().numpy(), "embed_grad": embed.weight.grad.numpy()}
    for i, c in enumerate(enc.convs):
        res[f"conv{i}_wgrad"] = c.weight.grad.numpy()
        res[f"conv{i}_bgrad"] = c.bias.grad.numpy()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    from module import Encoder  # noqa: E402  (reference)
    torch.set_num_threads(8)
    ids = make_ids()
    out = {"ids": ids}
    for dt, tag in ((torch.float32, "32"), (torch.float64, "64")):
        for k, v in run(Encoder, dt, ids).items():
            if tag == "64" or k == "feat":      # fp32 gradients are not stored (fp64 is the target)
                out[f"{k}{tag}"] = v.astype(np.float32) if tag == "64" else v
    np.savez_compressed(os.path.join(HERE, "encoder.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
