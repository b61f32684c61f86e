"""Activation kernels on wide rows: one workgroup per 1-4 rows vs one 512-thread workgroup per row.

    python tools/act_bench.py [--dim 7000] [--rows 1000]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def layout(dim, seed=0):
    """tanh + softmax spans shaped like the wide synthetic schema (mostly 2-20 options)."""
    rng = np.random.default_rng(seed)
    spans, cond, pos = [], [], 0
    while pos < dim:
        spans.append((pos, 1, 0))
        pos += 1
        w = int(rng.choice([2, 3, 5, 8, 10, 13, 20, 40]))
        spans.append((pos, w, 1))
        cond.append((pos, w))
        pos += w
    return spans, cond, pos


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=7000)
    ap.add_argument("--rows", type=int, default=1000)
    args = ap.parse_args()
    from fed_tgan_amd.ops.hip import HipOps
    dev = torch.device("cuda:0")
    o = HipOps(dev)
    spans, cond, D = layout(args.dim)
    R, nc = args.rows, 256
    logits = torch.randn(R, D, device=dev)
    fake = torch.zeros(R, D + nc, device=dev)
    real = torch.randn(R, D + nc, device=dev)
    interp = torch.zeros(R // 2, D + nc, device=dev)
    dact = torch.randn(R, D, device=dev)
    col = (torch.arange(R, device=dev) % len(cond)).to(torch.int32)
    opt = torch.zeros(R, dtype=torch.int32, device=dev)
    d = torch.zeros_like(logits)
    loss = torch.zeros(R, device=dev)
    mb = R * D * 4 / 1e6
    print(f"rows {R} x data_dim {D}, {len(spans)} spans ({mb:.1f} MB per [rows, D] fp32 tensor)")
    for mode in (0, 1, 0, 1):
        prev = torch.ops.fedtgan.set_tuning("act_row_mode", mode)
        t_a = timed(lambda: o.activate(logits, fake[:, :D], spans, 0.2))
        t_s = timed(lambda: o.activate(logits, fake[:, :D], spans, 0.2, slerp=(real[:R // 2], fake, interp, 3)))
        t_b = timed(lambda: o.act_bwd_ce(dact, fake[:, :D], logits, spans, cond, col, opt, d, loss, 0.2))
        torch.ops.fedtgan.set_tuning("act_row_mode", prev)
        tag = "row per workgroup" if mode else "rows per wave    "
        print(f"{tag}: activate {t_a:7.1f} us  activate+slerp {t_s:7.1f} us  act_bwd_ce {t_b:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
