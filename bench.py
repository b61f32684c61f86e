"""Headline benchmark: sec/epoch (+ Avg_JSD / Avg_WD) of federated CTGAN on Intrusion.

Metric (BASELINE.json): one full federated round — every client trains one local epoch
(rows // 500 WGAN-GP steps), weighted aggregation, sampling + decoding the 40,000-row
synthetic table and writing its CSV — exactly the span the reference times into
``timestamp_experiment.csv`` (`Server/dtds/distributed.py:795-825`).

Config: the Intrusion (KDD-99) 42-column schema; every client holds its own 40,000-row
synthetic shard (weak scaling: per-GPU work fixed as N grows); random-init weights;
batch 500, embedding 128, G/D (256, 256), pack 10.  One rank per GPU; the data plane is
RCCL (``nccl``) for N > 1.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

"steps" are federated rounds (epochs).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_SEC_PER_EPOCH = 24.2   # README.md:53-54 (2 clients, epoch 1); BASELINE.md


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed federated rounds")
    ap.add_argument("--warmup", type=int, default=2, help="untimed rounds")
    ap.add_argument("--rows", type=int, default=40000, help="rows per client")
    ap.add_argument("--n-sample", type=int, default=40000)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--gmm", default="torch")
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--sync-csv", action="store_true", help="write each epoch CSV inside its round")
    args = ap.parse_args()

    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.parallel.comm import Comm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    comm = Comm.from_env("auto", device)
    out = args.out or os.path.join(tempfile.gettempdir(), f"fedtgan_bench_{os.getpid()}_{rank}")
    if world > 1:
        out = comm.broadcast_object(out, src=0)
    os.makedirs(out, exist_ok=True)
    spec = intrusion_spec()
    cfg = FedConfig(spec=spec, epochs=args.warmup + args.steps, synthetic_rows=args.rows, out_dir=out,
                    n_sample=args.n_sample, backend=args.backend, gmm_backend=args.gmm, seed=0,
                    verbose=not args.quiet, async_csv=not args.sync_csv)
    rt = FedRuntime(cfg, comm, device)
    rt.initialize()
    for ep in range(args.warmup):
        rt.run_round(ep)
    rt.flush_writes()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for ep in range(args.warmup, args.warmup + args.steps):
        rt.round_times.append(rt.run_round(ep))
    rt.flush_writes()       # every timed round's CSV is on disk inside the timed region
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = comm.max_float(elapsed)
    sec_per_epoch = elapsed / max(args.steps, 1)

    avg_jsd = avg_wd = None
    if rank == 0 and not args.no_eval:
        from fed_tgan_amd.data.synthetic import generate
        from fed_tgan_amd.eval.similarity import stat_sim
        import pandas as pd
        last = os.path.join(out, f"{spec.name}_result", f"{spec.name}_synthesis_epoch_{cfg.epochs - 1}.csv")
        if os.path.exists(last):
            real = pd.concat([generate(spec, args.rows, seed=i) for i in range(max(world, 1))])
            avg_jsd, avg_wd = stat_sim(real, pd.read_csv(last), spec.categorical_list)
    if rank == 0:
        rec = {
            "metric": "sec_per_epoch", "value": round(sec_per_epoch, 6), "unit": "s/epoch", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(sec_per_epoch * 1000.0, 3),
            "higher_is_better": False, "scaling": "weak",
            "vs_baseline": round(sec_per_epoch / BASELINE_SEC_PER_EPOCH, 6),
            "dtype": cfg.engine.precision if rt.engine.ops.name == "hip" else "fp32",
            "data": f"synthetic (Intrusion schema, {args.rows} rows per client; random-init weights)",
            "config": {"model": "Fed-TGAN CTGAN (G 256x256 residual+BN, D 256x256 pack10, WGAN-GP slerp)",
                       "global_batch": 500 * world, "seq_len": None, "parallelism": f"fed{world}",
                       "rows_per_client": args.rows, "n_sample": args.n_sample,
                       "steps_per_epoch": args.rows // 500, "backend": rt.engine.ops.name},
            "avg_jsd": avg_jsd, "avg_wd": avg_wd, "epochs_trained": cfg.epochs,
            "phase_s": {k: round(v / max(cfg.epochs, 1), 6) for k, v in rt.timer.totals.items()},
        }
        print(json.dumps(rec), flush=True)
    comm.destroy()


if __name__ == "__main__":
    main()
