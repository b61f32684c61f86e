"""Adam at wide-table sizes: plain vs folded launch, per store policy (HBM-bound: 28 B/param).

    python tools/adam_bench.py [--n 19500000]
"""
import argparse
import os
import sys

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=19_500_000)
    args = ap.parse_args()
    from fed_tgan_amd.ops.hip import HipOps
    dev = torch.device("cuda:0")
    o = HipOps(dev)
    n = args.n // 16 * 16
    p, g, m, v = (torch.randn(n, device=dev) for _ in range(4))
    v.abs_()
    step = torch.ones(1, device=dev)
    src = torch.randn(500, 256, device=dev)
    jobs = ([src], [g[1024:1280]], [None], [None])
    gb = n * 28 / 1e9
    for aux in (0, 2, 16):
        prev = torch.ops.fedtgan.set_tuning("adam_store", aux)
        for cap in (65535, 4096, 1024):
            pc = torch.ops.fedtgan.set_tuning("adam_max_blocks", cap)
            t0 = timed(lambda: o.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 0.0))
            t1 = timed(lambda: o.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 0.0, jobs=jobs))
            torch.ops.fedtgan.set_tuning("adam_max_blocks", pc)
            print(f"store={aux:2d} max_blocks={cap:5d}: plain {t0:8.1f} us ({gb / t0 * 1e3:5.2f} TB/s)   "
                  f"folded {t1:8.1f} us ({gb / t1 * 1e3:5.2f} TB/s)", flush=True)
        torch.ops.fedtgan.set_tuning("adam_store", prev)


if __name__ == "__main__":
    main()
