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
    ap.add_argument("--k1", type=int, default=137800, help="packed D input width (pac x row width)")
    ap.add_argument("--only-gout", action="store_true", help="just the engine-layout G.out launch (counter runs)")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE", help="native set_tuning knob")
    args = ap.parse_args()
    from fed_tgan_amd.ops.hip import HipOps
    from fed_tgan_amd.ops import native
    for kv in args.tuning:
        k, v = kv.split("=", 1)
        native.require().set_tuning(k, int(v))
    dev = torch.device("cuda:0")
    o = HipOps(dev, seed=1, precision="bf16")
    M, N, K, C = args.M, args.N, args.K, args.C
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(M, K, generator=g).to(dev)
    Np = -(-N // 4) * 4                                              # rows padded to 16 B, as the engine's flat buffer
    Wst = (torch.randn(K + C, Np, generator=g) * 0.02).to(dev)[:, :N]   # input-major storage [in, out]
    W = Wst.t()                                                      # logical [out, in] (transposed view)
    Wd = Wst[:K].t().contiguous()                                    # dense part as [out, K] rows (TB = true)
    b = torch.randn(N, generator=g).to(dev)
    out = torch.empty(M, N, device=dev)
    col = torch.randint(0, 8, (M,), generator=g, dtype=torch.int32).to(dev)
    opt = torch.randint(0, 4, (M,), generator=g, dtype=torch.int32).to(dev)
    off = (torch.arange(8, dtype=torch.int32) * (C // 8)).to(dev)
    oh = (W[:, K:], col, opt, off)
    res = {}
    if args.only_gout:
        res["gout_engine_layout"] = timed(lambda: o.gemm(x, W[:, :K], out, tb=True, bias=b, onehot=oh), args.reps)
        print(json.dumps(res))
        return
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
    del Wst, W, Wd, xb, wb, ob, out
    # the two long-K / short-K discriminator GEMMs of the same step: dW0 = A0^T X (K = 150 rows) and the D-phase
    # D0 forward X W0^T (150 x 256, K = 137,800)
    K1, R, H = args.k1, 150, 256
    X = torch.randn(R, K1, generator=g).to(dev)
    A0 = torch.randn(R, H, generator=g).to(dev)
    W0 = (torch.randn(H, K1, generator=g) * 0.01).to(dev)
    dW = torch.empty(H, K1, device=dev)
    res["dW0_shortk"] = timed(lambda: o.gemm(A0, X, dW, ta=True), args.reps)
    ref = dW.clone()
    prev = torch.ops.fedtgan.set_tuning("gemm_shortk", 0)
    for tile in (None, 64, 128):
        tag = f"tile{tile or 'auto'}"
        res[f"dW0_{tag}"] = timed(lambda: o.gemm(A0, X, dW, ta=True, tile=tile), args.reps)
    torch.ops.fedtgan.set_tuning("gemm_shortk", prev)
    res["dW0_shortk_vs_tile_maxdiff"] = float((dW - ref).abs().max())
    res["dW0_torch_fp32"] = timed(lambda: torch.mm(A0.t(), X, out=dW), args.reps)
    res["dW0_torch_bf16"] = timed(lambda: torch.mm(A0.t().bfloat16(), X.bfloat16()), args.reps)
    res["fill_141MB"] = timed(lambda: dW.fill_(1.0), args.reps)
    d0 = torch.empty(R, H, device=dev)
    res["D0fwd_auto"] = timed(lambda: o.gemm(X, W0, d0, tb=True), args.reps)
    for sk in (8, 16, 32, 64):
        res[f"D0fwd_sk{sk}"] = timed(lambda: o.gemm(X, W0, d0, tb=True, splitk=sk), args.reps)
    for t, sk in ((128, 32), (128, 64), (64, 48), (64, 64)):
        res[f"D0fwd_t{t}_sk{sk}"] = timed(lambda: o.gemm(X, W0, d0, tb=True, tile=t, splitk=sk), args.reps)
    res["D0fwd_torch_fp32"] = timed(lambda: torch.mm(X, W0.t(), out=d0), args.reps)
    res["read_W0_X"] = timed(lambda: (W0.sum(), X.sum()), args.reps)
    for k, v in res.items():
        print(f"{k:36s} {v:10.4f}", flush=True)
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
