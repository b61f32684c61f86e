"""Time the epoch-CSV write of a real generated Intrusion table (40,000 rows) by thread count.

    python tools/csv_probe.py
"""
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.parallel.comm import Comm
    from fed_tgan_amd.utils import csvio
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    out = tempfile.mkdtemp()
    cfg = FedConfig(spec=intrusion_spec(), epochs=2, synthetic_rows=40000, out_dir=out, n_sample=40000,
                    gmm_backend="torch", seed=0, verbose=False, async_csv=False)
    rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
    rt.initialize()
    rt.run_round(0)
    vals = rt.engine.generate_decoded(40000).cpu().numpy()
    lay = rt.csv_cols
    path = os.path.join(out, "probe.csv")
    print(f"cpus {os.cpu_count()} affinity {len(os.sched_getaffinity(0))}")
    for th in (1, 2, 4, 8, 16, 0, 0):
        t0 = time.perf_counter()
        csvio.write_layout(path, vals, lay, threads=th)
        dt = time.perf_counter() - t0
        print(f"threads={th:2d}: {dt * 1e3:7.2f} ms  ({os.path.getsize(path) / 1e6:.1f} MB)", flush=True)
    # the same formatting with the bytes going nowhere: formatting cost vs file-write cost
    for th in (16, 0):
        t0 = time.perf_counter()
        csvio.write_layout(os.devnull, vals, lay, threads=th)
        print(f"threads={th:2d} -> /dev/null: {(time.perf_counter() - t0) * 1e3:7.2f} ms", flush=True)
    import numpy as np
    t0 = time.perf_counter()
    for _ in range(10):
        np.array(vals, dtype=np.float64, copy=True)
    print(f"host copy of the table: {(time.perf_counter() - t0) * 100:7.2f} ms", flush=True)


if __name__ == "__main__":
    main()
