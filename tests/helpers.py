"""Shared fixtures: a small encoded Intrusion-schema table and an autograd oracle of one step."""
from __future__ import annotations

import torch
import torch.nn.functional as F

# (the table fixture lives in the package: __graft_entry__.smoke() uses it too)
from fed_tgan_amd.data.demo import small_table  # noqa: F401


def d_forward_masked(X, Ws, bs, masks, v, e, slope=0.2):
    """Packed D forward with explicit dropout keep-masks (values 0 / 2)."""
    h = X
    for W, b, M in zip(Ws, bs, masks):
        h = F.leaky_relu(h @ W.t() + b, slope) * M
    return h @ v.view(-1, 1) + e


def keep_mask_from_ms(ms, pre, slope=0.2):
    s = torch.where(pre > 0, torch.ones_like(pre), torch.full_like(pre, slope))
    return ms / s
