"""Probe of the wide table's generator output GEMM (1000 x 7,018, dense K = 640 + a one-hot condition block;
profiles/wide_r5.md: 58 us against a 9 us byte bound).  Times the launch in isolation with variants that take one
ingredient away at a time -- one-hot gather, input-major (TB = false) weights, tile size, bias -- plus torch's
library GEMM of the same product, so the over-bound part can be attributed.

    python tools/gout_probe.py [--reps 50]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timed(fn, reps):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--M", type=int, default=1000)
    ap.add_argument("--N", type=int, default=7018)
    ap.add_argument("--K", type=int, default=640)
    ap.add_argument("--C", type=int, default=6762)
    args = ap.parse_args()
    from fed_tgan_amd.ops.hip import HipOps
    dev = torch.device("cuda:0")
    o = HipOps(dev, seed=1, precision="bf16")
    M, N, K, C = args.M, args.N, args.K, args.C
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, K, generator=g).to(dev)
    Wst = (torch.randn(K + C, N, generator=g) * 0.02).to(dev)      # input-major storage [in, out]
    W = Wst.t()                                                      # logical [out, in] (transposed view)
    Wd = Wst[:K].t().contiguous()                                    # dense part as [out, K] rows (TB = true)
    b = torch.randn(N, generator=g).to(dev)
    out = torch.empty(M, N, device=dev)
    col = torch.randint(0, 8, (M,), generator=g, dtype=torch.int32).to(dev)
    opt = torch.randint(0, 4, (M,), generator=g, dtype=torch.int32).to(dev)
    off = (torch.arange(8, dtype=torch.int32) * (C // 8)).to(dev)
    oh = (W[:, K:], col, opt, off)
    res = {}
    for tile in (None, 64, 128):
        tag = f"tile{tile or 'auto'}"
        res[f"inmajor_onehot_bias_{tag}"] = timed(
            lambda: o.gemm(x, W[:, :K], out, tb=True, bias=b, onehot=oh, tile=tile), args.reps)
        res[f"inmajor_bias_{tag}"] = timed(lambda: o.gemm(x, W[:, :K], out, tb=True, bias=b, tile=tile), args.reps)
        res[f"inmajor_plain_{tag}"] = timed(lambda: o.gemm(x, W[:, :K], out, tb=True, tile=tile), args.reps)
        res[f"rowmajor_plain_{tag}"] = timed(lambda: o.gemm(x, Wd, out, tb=True, tile=tile), args.reps)
    xb, wb = x.bfloat16(), Wst[:K].bfloat16()
    res["torch_mm_fp32"] = timed(lambda: torch.mm(x, Wst[:K], out=out), args.reps)
    ob = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    res["torch_mm_bf16"] = timed(lambda: torch.mm(xb, wb, out=ob), args.reps)
    res["copy_out_28MB"] = timed(lambda: out.fill_(1.0), args.reps)
    for k, v in res.items():
        print(f"{k:36s} {v:8.2f} us", flush=True)
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
