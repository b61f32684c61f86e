"""Run one BASELINE.json config end to end and report sec/epoch + Avg_JSD / Avg_WD per epoch.

    python tools/run_config.py --spec intrusion --clients 1 --epochs 10
    python tools/run_config.py --spec adult --clients 8 --shard dirichlet --alpha 0.3 --epochs 5
    python tools/run_config.py --spec wide --rows 100000 --clients 1 --epochs 3 --n-sample 10000

K > 1 clients run as the in-process emulation on one device (fed/local.py: K engines, one
thread each, weighted aggregation through the ThreadComm); the 8-GPU node runs the same code
one rank per GPU.  The real table for the similarity metrics is the union of the client shards,
as in `Server/similarity_analysis.py`.  One JSON line per epoch, plus a summary line.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import pandas as pd
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def _engine_cfg(ecfg, overrides):
    for kv in overrides:
        k, v = kv.split("=", 1)
        cur = getattr(ecfg, k)
        if isinstance(cur, bool) or (cur is None and v.lower() in ("0", "1", "true", "false", "yes", "no")):
            setattr(ecfg, k, v.lower() in ("1", "true", "yes"))
        else:
            setattr(ecfg, k, v if cur is None else type(cur)(v))
    return ecfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="intrusion")
    ap.add_argument("--rows", type=int, default=40000, help="rows per client")
    ap.add_argument("--clients", type=int, default=1)
    ap.add_argument("--shard", default="independent", help="independent | iid | dirichlet | skew")
    ap.add_argument("--alpha", type=float, default=0.3)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--n-sample", type=int, default=40000)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--aggregation", default="weighted")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--json", default=None, help="append the JSON lines to this file")
    ap.add_argument("--one-stream", action="store_true", help="emulated clients share one HIP stream")
    ap.add_argument("--batched", default="auto", choices=["auto", "on", "off"],
                    help="emulated clients as one batched engine (FedConfig.batched_clients) or one engine per thread")
    ap.add_argument("--engine", action="append", default=[], metavar="KEY=VALUE",
                    help="EngineConfig override for A/B runs, e.g. --engine g_wt=1")
    ap.add_argument("--fed", action="append", default=[], metavar="KEY=VALUE",
                    help="FedConfig override for A/B runs, e.g. --fed label_encoders_early=0")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE",
                    help="native set_tuning knob for A/B runs, e.g. --tuning gemm_pairs=0")
    ap.add_argument("--plan", action="append", default=[], metavar="KEY=VALUE",
                    help="GEMM planner knob of fed_tgan_amd.ops.hip (module constant), e.g. --plan WAVE_FILL_64=1")
    args = ap.parse_args()
    if args.plan:
        from fed_tgan_amd.ops import hip as hip_ops
        for kv in args.plan:
            key, val = kv.split("=", 1)
            getattr(hip_ops, key)
            setattr(hip_ops, key, bool(int(val)) if isinstance(getattr(hip_ops, key), bool) else int(val))
    if args.tuning:     # (before round 6 this loop sat under `if args.plan:` -- tuning alone was silently ignored)
        from fed_tgan_amd.ops import native
        for kv in args.tuning:
            key, val = kv.split("=", 1)
            native.require().set_tuning(key, int(val))

    from fed_tgan_amd.data.schema import get_spec
    from fed_tgan_amd.data.synthetic import generate, shard
    from fed_tgan_amd.eval.similarity import stat_sim
    from fed_tgan_amd.fed.local import run_local_emulation
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.models.engine import EngineConfig
    from fed_tgan_amd.parallel.comm import Comm
    from fed_tgan_amd.utils.metrics import cpu_quota

    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    spec = get_spec(args.spec)
    out = args.out or tempfile.mkdtemp(prefix=f"fedtgan_{spec.name}_")
    cfg = FedConfig(spec=spec, epochs=args.epochs, synthetic_rows=args.rows, shard_mode=args.shard,
                    dirichlet_alpha=args.alpha, out_dir=out, n_sample=args.n_sample, backend=args.backend,
                    gmm_backend="torch", aggregation=args.aggregation, seed=args.seed,
                    engine=_engine_cfg(EngineConfig(precision=args.precision), args.engine), verbose=True,
                    client_streams=not args.one_stream, batched_clients=args.batched)
    _engine_cfg(cfg, args.fed)
    t0 = time.time()
    if args.clients == 1:
        rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
        rt.initialize()
        rt.fit()
    else:
        rt = run_local_emulation(cfg, args.clients, backend=args.backend, device=dev)
    wall = time.time() - t0
    # the real table: union of the client shards (what the evaluators compare against)
    k = args.clients
    if args.shard == "independent":
        real = pd.concat([generate(spec, args.rows, seed=args.seed * 1000 + i) for i in range(k)])
    else:
        real = pd.concat(shard(generate(spec, args.rows * k, seed=args.seed), k, args.shard, seed=args.seed,
                               target=spec.target_column, alpha=args.alpha))
    real = real[spec.selected_variables]
    lines = []
    res = os.path.join(out, f"{spec.name}_result")
    for ep in range(args.epochs):
        fake = pd.read_csv(os.path.join(res, f"{spec.name}_synthesis_epoch_{ep}.csv"))
        jsd, wd = stat_sim(real, fake, spec.categorical_list)
        rec = {"spec": spec.name, "clients": k, "shard": args.shard, "precision": args.precision, "epoch": ep,
               "backend": rt.engine.ops.name, "seed": args.seed,
               "sec": round(rt.round_times[ep], 4), "avg_jsd": round(jsd, 5), "avg_wd": round(wd, 5)}
        lines.append(rec)
        print(json.dumps(rec), flush=True)
    summ = {"spec": spec.name, "clients": k, "shard": args.shard, "precision": args.precision,
            "batched": bool(getattr(rt, "batched", False)),
            "rows_per_client": args.rows, "epochs": args.epochs, "weights": [round(float(w), 4) for w in rt.weights],
            "mean_sec_per_epoch_after_first": round(sum(rt.round_times[1:]) / max(len(rt.round_times) - 1, 1), 4),
            "wall_s_incl_init": round(wall, 2),
            "init_s": {k: round(v, 3) for k, v in getattr(rt, "init_times", {}).items()},
            "final_avg_jsd": lines[-1]["avg_jsd"], "final_avg_wd": lines[-1]["avg_wd"], "cpu": cpu_quota()}
    if args.engine:
        summ["engine_overrides"] = args.engine
    if args.tuning:
        summ["tuning"] = args.tuning
    if args.plan:
        summ["plan"] = args.plan
    if args.fed:
        summ["fed_overrides"] = args.fed
    print(json.dumps(summ), flush=True)
    if args.json:
        with open(args.json, "a") as f:
            for r in lines + [summ]:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
