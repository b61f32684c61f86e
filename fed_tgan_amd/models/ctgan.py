"""CTGAN model family as ``torch.nn`` modules — the eager *oracle* path.

These modules re-state the reference model core (`Server/dtds/synthesizers/ctgan.py`)
with reference-compatible ``state_dict`` keys so checkpoints and weight exchange look
the same.  The production training path is :class:`fed_tgan_amd.models.engine.CTGANEngine`
(flat buffers, explicit backward, fused HIP kernels, hipGraph replay); this file is what
the engine is tested against.

Parity map:
* ``Residual`` / ``Generator``  — `ctgan.py:33-64` (Linear -> BN -> ReLU, output
  ``cat([out, input])``; final Linear to ``data_dim``).
* ``Discriminator``             — `ctgan.py:15-30` (PacGAN pack=10, LeakyReLU 0.2,
  Dropout 0.5, no BN).
* ``apply_activate``            — `ctgan.py:67-82` (tanh / Gumbel-softmax tau=0.2).
* ``cond_loss``                 — `ctgan.py:174-194` (cross-entropy on every softmax span,
  masked to the sampled span).
* ``slerp`` / ``calc_gradient_penalty`` — `ctgan.py:231-258` (spherical interpolation with a
  per-row alpha, lambda=10, pack-wise gradient norm, double backward).
"""
from __future__ import annotations

from typing import Sequence

import torch
import torch.nn.functional as F
from torch import nn

from ..features.transformer import SOFTMAX, TANH

PACK = 10
GUMBEL_TAU = 0.2
LRELU_SLOPE = 0.2
DROPOUT_P = 0.5
GP_LAMBDA = 10.0


class Residual(nn.Module):
    def __init__(self, i: int, o: int):
        super().__init__()
        self.fc = nn.Linear(i, o)
        self.bn = nn.BatchNorm1d(o)
        self.relu = nn.ReLU()

    def forward(self, x):
        return torch.cat([self.relu(self.bn(self.fc(x))), x], dim=1)


class Generator(nn.Module):
    def __init__(self, embedding_dim: int, gen_dims: Sequence[int], data_dim: int):
        super().__init__()
        layers = []
        dim = embedding_dim
        for h in gen_dims:
            layers.append(Residual(dim, h))
            dim += h
        layers.append(nn.Linear(dim, data_dim))
        self.seq = nn.Sequential(*layers)

    def forward(self, x):
        return self.seq(x)


class Discriminator(nn.Module):
    def __init__(self, input_dim: int, dis_dims: Sequence[int], pack: int = PACK):
        super().__init__()
        self.pack = pack
        self.packdim = input_dim * pack
        layers = []
        dim = self.packdim
        for h in dis_dims:
            layers += [nn.Linear(dim, h), nn.LeakyReLU(LRELU_SLOPE), nn.Dropout(DROPOUT_P)]
            dim = h
        layers.append(nn.Linear(dim, 1))
        self.seq = nn.Sequential(*layers)

    def forward(self, x):
        if x.size(0) % self.pack != 0:
            raise ValueError(f"batch {x.size(0)} is not a multiple of pack {self.pack}")
        return self.seq(x.reshape(-1, self.packdim))


def _spans(output_info):
    pos = 0
    for w, kind in output_info:
        yield pos, pos + int(w), kind
        pos += int(w)


def apply_activate(data: torch.Tensor, output_info, tau: float = GUMBEL_TAU) -> torch.Tensor:
    parts = []
    for a, b, kind in _spans(output_info):
        if kind == TANH:
            parts.append(torch.tanh(data[:, a:b]))
        elif kind == SOFTMAX:
            parts.append(F.gumbel_softmax(data[:, a:b], tau=tau))
        else:
            raise ValueError(kind)
    return torch.cat(parts, dim=1)


def cond_loss(data: torch.Tensor, output_info, c: torch.Tensor, m: torch.Tensor) -> torch.Tensor:
    losses = []
    opt = 0
    for a, b, kind in _spans(output_info):
        if kind != SOFTMAX:
            continue
        w = b - a
        target = c[:, opt:opt + w].argmax(dim=1)
        losses.append(F.cross_entropy(data[:, a:b], target, reduction="none"))
        opt += w
    return (torch.stack(losses, dim=1) * m).sum() / data.size(0)


def slerp(val: torch.Tensor, low: torch.Tensor, high: torch.Tensor) -> torch.Tensor:
    lo = low / low.norm(dim=1, keepdim=True)
    hi = high / high.norm(dim=1, keepdim=True)
    omega = torch.acos((lo * hi).sum(1)).view(val.size(0), 1)
    so = torch.sin(omega)
    return (torch.sin((1.0 - val) * omega) / so) * low + (torch.sin(val * omega) / so) * high


def calc_gradient_penalty(netD: nn.Module, real: torch.Tensor, fake: torch.Tensor, pac: int = PACK,
                          lambda_: float = GP_LAMBDA, alpha: torch.Tensor | None = None) -> torch.Tensor:
    if alpha is None:
        alpha = torch.rand(real.size(0), 1, device=real.device)
    x = slerp(alpha, real, fake)
    if not x.requires_grad:
        x.requires_grad_(True)
    y = netD(x)
    grads = torch.autograd.grad(outputs=y, inputs=x, grad_outputs=torch.ones_like(y), create_graph=True,
                                retain_graph=True, only_inputs=True)[0]
    return ((grads.reshape(-1, pac * real.size(1)).norm(2, dim=1) - 1) ** 2).mean() * lambda_
