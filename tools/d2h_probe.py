"""First-use costs of the epoch table's device-to-host path on the box: pinned allocation + async copy
(utils/devsync.PendingHost) and a pageable .cpu(), first vs later calls (ms)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from fed_tgan_amd.utils.devsync import PendingHost  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    x = torch.randn(40000, 42, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    rec = {}
    for i in range(3):
        t = time.perf_counter()
        p = PendingHost(x, s)
        t1 = time.perf_counter()
        p.get()
        rec[f"pinned_{i}"] = [round((t1 - t) * 1e3, 2), round((time.perf_counter() - t1) * 1e3, 2)]
    for i in range(2):
        t = time.perf_counter()
        x.cpu()
        rec[f"pageable_{i}"] = round((time.perf_counter() - t) * 1e3, 2)
    t = time.perf_counter()
    h = torch.empty(40000, 42, dtype=torch.float64, pin_memory=True)
    rec["pin_alloc_new"] = round((time.perf_counter() - t) * 1e3, 2)
    del h
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
