"""Large GEMMs of the wide-table config (TFLOP/s), through the HIP GEMM with the planner's tile.

    python tools/gemm_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    from fed_tgan_amd.ops.hip import HipOps
    dev = torch.device("cuda:0")
    o = HipOps(dev)
    def padded(rows, cols):   # [rows, cols] view of rows padded to 4 floats (the engine's storage)
        return torch.randn(rows, -(-cols // 4) * 4, device=dev)[:, :cols]

    cases = {
        "G out fwd 1000x7018x7402 NT": ((1000, 7402), (7018, 7402), (1000, 7018), False, True),
        "dW out 7018x7402x500 TN": ((500, 7018), (500, 7402), (7018, 7402), True, False),
        "G out fwd gen 40960x325x943 NT": ((40960, 943), (325, 943), (40960, 325), False, True),
        "G0 fwd gen 40960x256x431 NT": ((40960, 431), (256, 431), (40960, 256), False, True),
        "G1 fwd gen 40960x256x687 NT": ((40960, 687), (256, 687), (40960, 256), False, True),
    }
    tiles = [int(x) for x in os.environ.get("GEMM_TILES", "0").split(",")]
    for name, (sa, sb, sc, ta, tb) in cases.items():
        a, b, c = padded(*sa), padded(*sb), padded(*sc)
        M = a.shape[1] if ta else a.shape[0]
        K = a.shape[0] if ta else a.shape[1]
        N = b.shape[0] if tb else b.shape[1]
        for tile in tiles:   # 0 = the planner's tile
            o.tile_override = tile or None
            t = timed(lambda: o.gemm(a, b, c, ta=ta, tb=tb))
            print(f"{name:34s} tile {tile or 'plan':>4} {t:8.1f} us  {2 * M * N * K / t / 1e6:7.1f} TFLOP/s",
                  flush=True)
        o.tile_override = None


if __name__ == "__main__":
    main()
