"""Time the batched VGM fit: HIP data passes vs torch passes (GPU), on a wide-table-like batch."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from fed_tgan_amd.features.vgm_fit import fit_vgm_torch  # noqa: E402


def main(n_cols=256, n_rows=100000):
    rng = np.random.default_rng(0)
    cols = [rng.normal((i % 4) * 3.0, 0.5 + 0.25 * (i % 3), n_rows) + 3.0 * rng.integers(0, 1 + i % 4, n_rows)
            for i in range(n_cols)]
    dev = torch.device("cuda:0")
    fit_vgm_torch(cols[:4], seed=0, device=dev, use_hip=True)    # warm up
    for use_hip in (True, False):
        torch.cuda.synchronize()
        t = time.perf_counter()
        fit_vgm_torch(cols, seed=0, device=dev, use_hip=use_hip)
        torch.cuda.synchronize()
        print(f"{'hip' if use_hip else 'torch'} passes: {n_cols} cols x {n_rows} rows: {time.perf_counter() - t:.2f} s",
              flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
