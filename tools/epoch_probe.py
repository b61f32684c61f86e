"""Per-step time of whole captured epochs on the bench's own runtime data (vs the microbench)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.parallel.comm import Comm
    dev = torch.device("cuda:0")
    cfg = FedConfig(spec=intrusion_spec(), epochs=1, out_dir="/tmp/ep_probe", verbose=False)
    rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
    rt.initialize()
    eng = rt.engine
    print("layout", eng.Dd, eng.C, "steps/epoch", eng.steps_per_epoch, flush=True)
    for unroll in (1, 8):
        eng.cfg.graph_unroll = unroll
        eng.train_epoch()
        torch.cuda.synchronize()
        for rep in range(3):
            t = time.perf_counter()
            eng.train_epoch()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            print(f"unroll {unroll}: epoch {dt * 1e3:.2f} ms = {dt / eng.steps_per_epoch * 1e6:.1f} us/step", flush=True)
    # back-to-back epochs without a sync in between
    t = time.perf_counter()
    for _ in range(5):
        eng.train_epoch()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 5
    print(f"5 epochs back to back: {dt * 1e3:.2f} ms/epoch = {dt / eng.steps_per_epoch * 1e6:.1f} us/step")


if __name__ == "__main__":
    main()
