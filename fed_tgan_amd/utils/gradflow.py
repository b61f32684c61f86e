"""Gradient-flow diagnostics: mean |grad| per parameter tensor of G and D over training.

Parity with the reference's `update_grad_flow` / `plot_grad_flow`
(`Server/dtds/synthesizers/ctgan.py:261-306`; its call sites are commented out, `:432, 438`).
- The reference reads `p.grad` of every named parameter after a backward, and plots with
  matplotlib's TkAgg backend.
- Here the engine keeps every gradient in two flat buffers, so one snapshot is one batched
  reduction on the device plus one host copy per network. The plot uses the headless Agg
  backend, and the raw series is also written as CSV.
"""
from __future__ import annotations

import csv
import os
from typing import Dict, List

import torch


class GradFlow:
    def __init__(self):
        self.ave: Dict[str, List[List[float]]] = {"G": [], "D": []}
        self.layers: Dict[str, List[str]] = {"G": [], "D": []}

    def update(self, engine) -> None:
        """Record one snapshot of the engine's current G and D gradients (reference layer names)."""
        for net, keymap in (("G", engine.g_key_map()), ("D", engine.d_key_map())):
            names = [(k, n) for k, n in keymap if n in engine.g]
            self.layers[net] = [k for k, _ in names]
            vals = torch.stack([engine.g[n].abs().mean() for _, n in names]).cpu().tolist()
            self.ave[net].append([float(v) for v in vals])

    def save_csv(self, path: str) -> None:
        with open(path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["net", "snapshot", "layer", "mean_abs_grad"])
            for net in ("G", "D"):
                for i, row in enumerate(self.ave[net]):
                    for name, v in zip(self.layers[net], row):
                        w.writerow([net, i, name, v])

    def plot(self, save_dir: str) -> str | None:
        """grad_flow.png (D left, G right; colour runs from the first to the last snapshot)."""
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
        except Exception:
            return None
        os.makedirs(save_dir, exist_ok=True)
        fig, ax = plt.subplots(1, 2, figsize=(12, 6))
        n = max(len(self.ave["G"]), 1)
        cmap = plt.get_cmap("winter")
        for p, net in enumerate(("D", "G")):
            for i, row in enumerate(self.ave[net]):
                ax[p].plot(range(len(row)), row, alpha=0.5, color=cmap(i / max(n - 1, 1)))
            ax[p].set_xticks(range(len(self.layers[net])))
            ax[p].set_xticklabels(self.layers[net], rotation=30, ha="right", fontsize=7)
            ax[p].set_xlabel(f"Layers {net}")
        ax[0].set_ylabel("Average gradient")
        fig.suptitle("Gradient flow")
        fig.tight_layout()
        path = os.path.join(save_dir, "grad_flow.png")
        fig.savefig(path)
        plt.close(fig)
        return path
