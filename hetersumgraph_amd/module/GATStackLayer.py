"""Multi-head wrapper (reference: module/GATStackLayer.py:46-63).

The reference keeps one module per head, loops over heads in Python (each head a
full DGL pass on its own dropout of the input) and ``torch.cat``s the results.
Here all heads run as one fused HIP pass, and their parameters live in fused
tensors so no per-forward concatenation or per-head gradient bookkeeping is
needed:

    fc_weight   [H*D, in]   rows k*D..(k+1)*D-1 = heads.k.fc.weight
    attn_weight [H, 3*D]    row k = heads.k.attn_fc.weight
    feat_weight [H, D, F]   heads.k.feat_fc.weight
    feat_bias   [H, D]      heads.k.feat_fc.bias        (SWGATLayer only)

``state_dict()`` / ``load_state_dict()`` still speak the reference's per-head keys
(``heads.{k}.fc.weight`` ...) through state-dict hooks, and the
per-head tensors they expose are views of the fused storage.  The head modules
are created first (so a given ``torch.manual_seed`` reproduces the reference's
initial values) and then emptied.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .GATLayer import SGATLayer, fused_heads, sgat_heads

_FUSED = ("fc_weight", "attn_weight", "feat_weight", "feat_bias")


class MultiHeadLayer(nn.Module):
    def __init__(self, in_dim, out_dim, num_heads, attn_drop_out, feat_embed_size, layer, merge="cat"):
        super().__init__()
        if merge != "cat":
            # GATStackLayer.py:60-62 'mean' branch is never constructed by WSWGAT
            raise NotImplementedError("only merge='cat' is used by WSWGAT (GAT.py:35-37)")
        heads = [layer(in_dim, out_dim, feat_embed_size) for _ in range(num_heads)]
        self.merge = merge
        self.dropout = nn.Dropout(attn_drop_out)
        self.kind = layer.kind
        self.num_heads, self.head_dim = num_heads, out_dim
        with torch.no_grad():
            self.fc_weight = nn.Parameter(torch.cat([h.fc.weight for h in heads], 0).clone())
            self.attn_weight = nn.Parameter(torch.cat([h.attn_fc.weight for h in heads], 0).clone())
            self.feat_weight = nn.Parameter(torch.stack([h.feat_fc.weight for h in heads], 0).clone())
            if heads[0].feat_fc.bias is not None:
                self.feat_bias = nn.Parameter(torch.stack([h.feat_fc.bias for h in heads], 0).clone())
            else:
                self.register_parameter("feat_bias", None)
        for k, h in enumerate(heads):
            h.bind(self, k)
        self.heads = nn.ModuleList(heads)
        self._register_state_dict_hook(_to_reference_keys)
        self._register_load_state_dict_pre_hook(_from_reference_keys, with_module=True)

    def head_views(self, k):
        """Per-head tensors (views of the fused parameters) under reference names, in
        the reference's registration order (fc, feat_fc, attn_fc: GATLayer.py:84-87 /
        123-126), so state_dict() lists keys exactly as the reference does."""
        D = self.head_dim
        out = {"fc.weight": self.fc_weight[k * D:(k + 1) * D],
               "feat_fc.weight": self.feat_weight[k]}
        if self.feat_bias is not None:
            out["feat_fc.bias"] = self.feat_bias[k]
        out["attn_fc.weight"] = self.attn_weight[k:k + 1]
        return out

    def reference_named_grads(self, prefix=""):
        """(reference key, grad view) pairs -- what ``named_parameters`` of the
        reference module would report as ``.grad``."""
        D = self.head_dim
        for k in range(self.num_heads):
            g = {"fc.weight": self.fc_weight.grad[k * D:(k + 1) * D] if self.fc_weight.grad is not None else None,
                 "feat_fc.weight": self.feat_weight.grad[k] if self.feat_weight.grad is not None else None,
                 "attn_fc.weight": self.attn_weight.grad[k:k + 1] if self.attn_weight.grad is not None else None}
            if self.feat_bias is not None:
                g["feat_fc.bias"] = self.feat_bias.grad[k] if self.feat_bias.grad is not None else None
            for n, v in g.items():
                yield f"{prefix}heads.{k}.{n}", v

    def fused_params(self):
        return self.fc_weight, self.attn_weight, self.feat_weight, self.feat_bias

    def forward(self, g, h, origin=None):
        """[n_dst, H*out_dim] head concat; with ``origin`` the ELU + residual of
        GAT.py:56-57 is fused in (returns elu(heads) + origin)."""
        return fused_heads(g, h, self, self.kind, origin=origin, dropout=self.dropout)


class MultiHeadSGATLayer(nn.Module):
    """Multi-head S2S wrapper (reference: module/GATStackLayer.py:27-44), fused like
    :class:`MultiHeadLayer`: ``fc_weight`` [H*D, in] and ``attn_weight`` [H, 2D]
    (row k = heads.k.attn_fc.weight over [z_src, z_dst]); state_dict speaks the
    reference's per-head keys ``heads.{k}.fc.weight`` / ``heads.{k}.attn_fc.weight``."""

    kind = "S2S"

    def __init__(self, in_dim, out_dim, num_heads, attn_drop_out, merge="cat"):
        super().__init__()
        if merge != "cat":
            raise NotImplementedError("only merge='cat' is used by WSWGAT (GAT.py:38)")
        heads = [SGATLayer(in_dim, out_dim) for _ in range(num_heads)]
        self.merge = merge
        self.dropout = nn.Dropout(attn_drop_out)
        self.num_heads, self.head_dim = num_heads, out_dim
        with torch.no_grad():
            self.fc_weight = nn.Parameter(torch.cat([h.fc.weight for h in heads], 0).clone())
            self.attn_weight = nn.Parameter(torch.cat([h.attn_fc.weight for h in heads], 0).clone())
        self.register_parameter("feat_weight", None)
        self.register_parameter("feat_bias", None)
        for k, h in enumerate(heads):
            h.bind(self, k)
        self.heads = nn.ModuleList(heads)
        self._register_state_dict_hook(_to_reference_keys)
        self._register_load_state_dict_pre_hook(_from_reference_keys, with_module=True)

    def head_views(self, k):
        D = self.head_dim
        return {"fc.weight": self.fc_weight[k * D:(k + 1) * D], "attn_fc.weight": self.attn_weight[k:k + 1]}

    def reference_named_grads(self, prefix=""):
        D = self.head_dim
        g = lambda p, sl: p.grad[sl] if p.grad is not None else None
        for k in range(self.num_heads):
            yield f"{prefix}heads.{k}.fc.weight", g(self.fc_weight, slice(k * D, (k + 1) * D))
            yield f"{prefix}heads.{k}.attn_fc.weight", g(self.attn_weight, slice(k, k + 1))

    def fused_params(self):
        return self.fc_weight, self.attn_weight, None, None

    def forward(self, g, h, origin=None):
        """[n_unit1, H*out_dim] head concat; with ``origin`` elu(heads) + origin."""
        return sgat_heads(g, h, self, origin=origin, dropout=self.dropout)


def _to_reference_keys(module, state_dict, prefix, local_metadata):
    for name in _FUSED:
        state_dict.pop(prefix + name, None)
    for k in range(module.num_heads):
        for n, v in module.head_views(k).items():
            state_dict[f"{prefix}heads.{k}.{n}"] = v if v.requires_grad is False else v.detach()
    return state_dict


def _from_reference_keys(module, state_dict, prefix, local_metadata, strict, missing_keys,
                         unexpected_keys, error_msgs):
    key = lambda k, n: f"{prefix}heads.{k}.{n}"
    H, D = module.num_heads, module.head_dim
    if key(0, "fc.weight") not in state_dict:
        return
    state_dict[prefix + "fc_weight"] = torch.cat([state_dict.pop(key(k, "fc.weight")) for k in range(H)], 0)
    state_dict[prefix + "attn_weight"] = torch.cat([state_dict.pop(key(k, "attn_fc.weight")) for k in range(H)], 0)
    if module.feat_weight is not None:
        state_dict[prefix + "feat_weight"] = torch.stack([state_dict.pop(key(k, "feat_fc.weight")) for k in range(H)])
    if module.feat_bias is not None:
        state_dict[prefix + "feat_bias"] = torch.stack([state_dict.pop(key(k, "feat_fc.bias")) for k in range(H)])


def reference_named_grads(model):
    """(reference parameter name, .grad) for every parameter of ``model``, with the
    fused head tensors split back into the reference's per-head names -- i.e. what
    ``named_parameters()`` + ``.grad`` gives on the reference model."""
    fused_ids = set()
    out = []
    for mname, mod in model.named_modules():
        if isinstance(mod, (MultiHeadLayer, MultiHeadSGATLayer)):
            out.extend(mod.reference_named_grads(mname + "." if mname else ""))
            fused_ids |= {id(p) for p in mod.fused_params() if p is not None}
    for n, p in model.named_parameters():
        if id(p) not in fused_ids:
            out.append((n, p.grad))
    return out
