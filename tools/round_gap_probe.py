"""Where does a multi-client round spend the time its phases do not account for?

K emulated clients on one GPU (threads, one HIP stream each), Intrusion schema, synthetic rows.
Per configuration: mean round time over rounds 2..E-1 and the federator's mean phase times:
  * csv=async: the epoch CSV written on the background writer (default);
  * csv=sync : written inside the round;
  * csv=off  : no CSV (FedConfig.write_csv = False).

    python tools/round_gap_probe.py [--clients 8] [--epochs 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=8)
    args = ap.parse_args()
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.local import run_local_emulation
    from fed_tgan_amd.fed.runtime import FedConfig
    dev = torch.device("cuda:0")
    for mode in ("async", "sync", "off"):
        cfg = FedConfig(spec=intrusion_spec(), epochs=args.epochs, synthetic_rows=40000, n_sample=40000,
                        out_dir=f"/tmp/gap_{mode}", backend="hip", verbose=False, async_csv=mode == "async",
                        write_csv=mode != "off")
        rt = run_local_emulation(cfg, args.clients, backend="hip", device=dev)
        rs = rt.round_times[2:]
        print(json.dumps({"csv": mode, "clients": args.clients, "round_ms": round(1e3 * float(np.mean(rs)), 2),
                          "rounds_ms": [round(1e3 * x, 1) for x in rt.round_times],
                          "phase_ms_total": {k: round(1e3 * v / args.epochs, 2) for k, v in rt.timer.totals.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
