"""Serving throughput of a trained generator (the `python -m dtds.sample` path).

Trains a 1-client Intrusion-schema federation for one round on the GPU, which writes
models/Intrusion_generator.pt. It then loads that file the way `dtds.sample` does
(weights only, a fresh HIP engine) and times, per request size:

  * `sample(n)`: sample, eval G, decode, device-to-host copy (float64 table);
  * `write_csv(path, n)`: the same plus the native CSV formatter and the file write.

    python tools/serve_bench.py [--sizes 40000 200000 1000000] [--out-dir /tmp/serve]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[40000, 200000, 1000000])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out-dir", default="/tmp/serve")
    args = ap.parse_args()
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.models.engine import EngineConfig
    from fed_tgan_amd.models.generator_io import load_generator
    from fed_tgan_amd.parallel.comm import Comm
    dev = torch.device("cuda:0")
    cfg = FedConfig(spec=intrusion_spec(), epochs=1, synthetic_rows=40000, n_sample=1000, out_dir=args.out_dir,
                    backend="hip", gmm_backend="torch", engine=EngineConfig(), verbose=False)
    rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
    rt.initialize()
    rt.fit()
    rt.flush_writes()
    path = os.path.join(args.out_dir, "models", "Intrusion_generator.pt")
    t0 = time.perf_counter()
    gen = load_generator(path, dev, backend="hip", seed=1)
    t_load = time.perf_counter() - t0
    print(json.dumps({"model": path, "load_s": round(t_load, 3), "gen_bf16": gen.engine.gen16}), flush=True)
    for n in args.sizes:
        gen.sample(n)                       # captures the generation graph for this size
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(args.reps):
            gen.engine.generate_decoded(n)
        torch.cuda.synchronize(dev)
        t_dev = (time.perf_counter() - t) / args.reps
        t = time.perf_counter()
        for _ in range(args.reps):
            v = gen.sample(n)
        t_host = (time.perf_counter() - t) / args.reps
        csv = os.path.join(args.out_dir, f"serve_{n}.csv")
        gen.write_csv(csv, n)
        t = time.perf_counter()
        for _ in range(max(1, args.reps // 2)):
            gen.write_csv(csv, n)
        t_csv = (time.perf_counter() - t) / max(1, args.reps // 2)
        rec = {"rows": n, "cols": int(v.shape[1]), "device_ms": round(t_dev * 1e3, 3),
               "device_rows_per_s": round(n / t_dev), "to_host_ms": round(t_host * 1e3, 3),
               "to_host_rows_per_s": round(n / t_host), "csv_ms": round(t_csv * 1e3, 2),
               "csv_rows_per_s": round(n / t_csv), "csv_mb": round(os.path.getsize(csv) / 2**20, 1)}
        print(json.dumps(rec), flush=True)
        os.remove(csv)


if __name__ == "__main__":
    main()
