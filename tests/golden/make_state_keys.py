"""Record the reference models' state_dict keys and shapes by
building the REFERENCE HSumGraph / HSumDocGraph (HiGraph.py, imported from
/root/reference over the test-only DGL shim, as make_golden.py does) with
train.py's argparse defaults (train.py:279-309).  Writes state_keys.json next to
this file; tests/test_state_dict.py compares this build's models against it.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_state_keys.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from make_golden import HPS, import_reference, ref_hashes  # noqa: E402


def main(ref="/root/reference"):
    HiGraph, _ = import_reference(ref)
    hps = HPS(vocab_size=50000)
    out = {"ref_hash": ref_hashes(ref)}
    for cls in ("HSumGraph", "HSumDocGraph"):
        torch.manual_seed(0)
        embed = torch.nn.Embedding(hps.vocab_size, 300, padding_idx=0)
        m = getattr(HiGraph, cls)(hps, embed)
        out[cls] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
        out[cls + ".trainable"] = sum(p.numel() for p in m.parameters() if p.requires_grad) - \
            embed.weight.numel()
    with open(os.path.join(HERE, "state_keys.json"), "w") as f:
        json.dump(out, f, indent=0)
    print({k: len(v) for k, v in out.items() if isinstance(v, list)})


if __name__ == "__main__":
    main(*sys.argv[1:2])
