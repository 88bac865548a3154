"""Checkpoint compatibility (train.py:60-64 save, evaluation.py:39-59 restore by
state_dict): this build's HSumGraph / HSumDocGraph expose exactly the reference
models' state_dict -- 100 / 101 keys, same names, same shapes, same order
(tests/golden/state_keys.json, recorded from the reference's own HiGraph.py by
tests/golden/make_state_keys.py) -- and a reference-layout state_dict loads into
the fused head tensors and reads back unchanged.  CPU only."""
import json
import os

import pytest
import torch

KEYS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "state_keys.json")))


class HPS:
    def __init__(self):
        self.__dict__.update(dict(
            vocab_size=50000, n_iter=2, word_emb_dim=300, embed_train=False, feat_embed_size=50,
            lstm_hidden_state=128, lstm_layers=2, bidirectional=True, n_feature_size=128, hidden_size=64,
            ffn_inner_hidden_size=512, n_head=8, recurrent_dropout_prob=0.1, atten_dropout_prob=0.1,
            ffn_dropout_prob=0.1, sent_max_len=100, doc_max_timesteps=50, cuda=False))


def _model(cls):
    from hetersumgraph_amd import HiGraph
    torch.manual_seed(0)
    embed = torch.nn.Embedding(50000, 300, padding_idx=0)
    embed.weight.requires_grad = False                   # train.py: hps.embed_train = False
    return getattr(HiGraph, cls)(HPS(), embed)


@pytest.mark.parametrize("cls", ["HSumGraph", "HSumDocGraph"])
def test_state_dict_keys_and_shapes_match_reference(cls):
    m = _model(cls)
    got = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    assert len(got) == len(KEYS[cls]) == (100 if cls == "HSumGraph" else 101)
    assert got == KEYS[cls]
    trainable = sum(p.numel() for p in m.parameters() if p.requires_grad)
    assert trainable == KEYS[cls + ".trainable"]          # embedding frozen (embed_train=False)


@pytest.mark.parametrize("cls", ["HSumGraph", "HSumDocGraph"])
def test_reference_layout_state_dict_round_trip(cls):
    from hetersumgraph_amd.module.GATStackLayer import MultiHeadLayer
    m = _model(cls)
    g = torch.Generator().manual_seed(1)
    ref_sd = {k: torch.randn(*shape, generator=g) for k, shape in KEYS[cls]}
    ref_sd["ngram_enc.embed.weight"] = ref_sd["_embed.weight"]     # the sentence encoder shares _embed
    missing, unexpected = m.load_state_dict(ref_sd, strict=True)
    assert not missing and not unexpected
    back = m.state_dict()
    for k, _ in KEYS[cls]:
        assert torch.equal(back[k], ref_sd[k]), k
    # the fused tensors the kernels read hold the per-head reference tensors
    for name, mod in m.named_modules():
        if not isinstance(mod, MultiHeadLayer):
            continue
        D = mod.head_dim
        for k in range(mod.num_heads):
            p = f"{name}.heads.{k}."
            assert torch.equal(mod.fc_weight[k * D:(k + 1) * D], ref_sd[p + "fc.weight"])
            assert torch.equal(mod.feat_weight[k], ref_sd[p + "feat_fc.weight"])
            assert torch.equal(mod.attn_weight[k:k + 1], ref_sd[p + "attn_fc.weight"])
            if mod.feat_bias is not None:
                assert torch.equal(mod.feat_bias[k], ref_sd[p + "feat_fc.bias"])
    # and a checkpoint written by this build restores into a fresh model
    m2 = _model(cls)
    m2.load_state_dict(back)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, back[k]), k
