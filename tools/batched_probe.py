"""Epoch time of K clients on one GPU: the batched engine (one launch per kernel for all K clients)
against one plain engine, and against K plain engines on K streams (the thread emulation's layout).

    python tools/batched_probe.py [--rows 40000] [--ks 1 2 4 8] [--reps 5]
"""
import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--ks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--streams", action="store_true", help="also K plain engines on K streams")
    ap.add_argument("--plan", default="on", choices=["on", "off", "both"],
                    help="HipOps.batch_plan: split-K / tile planning over clients x tiles (on) or per client (off)")
    ap.add_argument("--profile-k", type=int, default=0, help="only run the batched engine with this K (profiling)")
    ap.add_argument("--engine", action="append", default=[], metavar="KEY=VALUE",
                    help="EngineConfig override (repeatable), e.g. --engine chain_d1=0")
    ap.add_argument("--ops", action="append", default=[], metavar="KEY=VALUE",
                    help="HipOps attribute of the issuing engine (repeatable), e.g. --ops bn_fused=1")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE",
                    help="native set_tuning knob (repeatable), e.g. --tuning bn_cols=16")
    ap.add_argument("--module", action="append", default=[], metavar="KEY=VALUE",
                    help="boolean fed_tgan_amd.ops.hip module flag, e.g. --module LONG_K_64=0")
    ap.add_argument("--skip-plain", action="store_true")
    ap.add_argument("--groups", type=int, nargs="*", default=[],
                    help="also K clients as G batched groups of K/G clients on G streams (one entry per G)")
    args = ap.parse_args()
    import numpy as np
    import torch
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.data.synthetic import generate
    from fed_tgan_amd.data.table import TablePreprocessor
    from fed_tgan_amd.features.transformer import VGMTransformer
    from fed_tgan_amd.fed.stats import merge_categorical_metas
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    dev = torch.device("cuda:0")
    spec = intrusion_spec()
    df = generate(spec, args.rows, seed=0)
    tp = TablePreprocessor(df, "Intrusion", spec.problem_type, spec.target_column, spec.categorical_list,
                           spec.nonnegative_list)
    meta, vocabs, _ = merge_categorical_metas([tp.local_meta()])
    enc = tp.encode(vocabs)
    cat = tp.categorical_indices()
    tr = VGMTransformer().fit(enc, cat, (), seed=0, backend="torch", device=dev)
    tr.refit(enc, meta, vocabs, cat, (), tr.bank, tr.components)
    X = tr.transform(enc, np.random.default_rng(0))
    rng = np.random.default_rng(1)
    cfg = EngineConfig()
    for kv in args.engine:
        key, val = kv.split("=", 1)
        cur = getattr(cfg, key)
        setattr(cfg, key, (val.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(val))

    from fed_tgan_amd.ops import native
    for kv in args.tuning:
        key, val = kv.split("=", 1)
        native.require().set_tuning(key, int(val))

    import fed_tgan_amd.ops.hip as hipmod
    for kv in args.module:
        key, val = kv.split("=", 1)
        setattr(hipmod, key, val.lower() in ("1", "true", "yes"))

    def set_ops(bc):
        for kv in args.ops:
            key, val = kv.split("=", 1)
            for e in bc.engines:
                cur = getattr(e.ops, key)
                setattr(e.ops, key, (val.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(val))

    def timed(fn, reps):
        fn()                       # capture / warm-up
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    if args.profile_k:
        bc = BatchedClients(tr.layout, cfg, dev, [100 + c for c in range(args.profile_k)], n_rows=len(X))
        bc.engines[0].ops.batch_plan = args.plan != "off"
        set_ops(bc)
        for c, e in enumerate(bc.engines):
            e.set_training_data(X if c == 0 else X[rng.permutation(len(X))])
        for _ in range(args.reps):
            bc.train_epoch()
        torch.cuda.synchronize()
        return
    plain = CTGANEngine(tr.layout, cfg, dev, backend="hip", seed=0)
    plain.set_training_data(X)
    steps = plain.steps_per_epoch
    t1 = timed(plain.train_epoch, args.reps) if not args.skip_plain else float("nan")
    print(json.dumps({"mode": "plain", "k": 1, "epoch_ms": round(t1 * 1e3, 3), "engine": args.engine,
                      "step_us": round(t1 / steps * 1e6, 1)}), flush=True)
    plans = {"on": [True], "off": [False], "both": [False, True]}[args.plan]
    for k in args.ks:
        for plan in plans:
            bc = BatchedClients(tr.layout, cfg, dev, [100 + c for c in range(k)], n_rows=len(X))
            bc.engines[0].ops.batch_plan = plan
            set_ops(bc)
            for c, e in enumerate(bc.engines):
                e.set_training_data(X if c == 0 else X[rng.permutation(len(X))])
            tk = timed(bc.train_epoch, args.reps)
            tagg = timed(lambda: bc.weighted_average([1.0 / k] * k), args.reps)
            print(json.dumps({"mode": "batched", "k": k, "batch_plan": plan, "engine": args.engine, "ops": args.ops,
                              "tuning": args.tuning,
                              "epoch_ms": round(tk * 1e3, 3),
                              "step_us": round(tk / steps * 1e6, 1), "vs_one_client": round(tk / t1, 3),
                              "fedavg_us": round(tagg * 1e6, 1)}), flush=True)
            del bc
            gc.collect()
            torch.cuda.synchronize()
        for G in args.groups:
            if k % G or G <= 1:
                continue
            m = k // G
            groups, streams = [], []
            for j in range(G):
                bc = BatchedClients(tr.layout, cfg, dev, [300 + 10 * j + c for c in range(m)], n_rows=len(X))
                for e in bc.engines:
                    e.set_training_data(X[rng.permutation(len(X))])
                    e.capture_mode = "thread_local"
                groups.append(bc)
                streams.append(torch.cuda.Stream(dev))

            def run_groups():
                for bc, s in zip(groups, streams):
                    s.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(s):
                        bc.train_epoch()
                for s in streams:
                    torch.cuda.current_stream(dev).wait_stream(s)
            tg = timed(run_groups, args.reps)
            print(json.dumps({"mode": f"{G} groups x {m}", "k": k, "engine": args.engine, "epoch_ms": round(tg * 1e3, 3),
                              "vs_one_client": round(tg / t1, 3)}), flush=True)
            del groups
            gc.collect()
            torch.cuda.synchronize()
        if args.streams and k > 1:
            engines, streams = [], []
            for c in range(k):
                e = CTGANEngine(tr.layout, cfg, dev, backend="hip", seed=200 + c)
                e.set_training_data(X)
                e.capture_mode = "thread_local"
                engines.append(e)
                streams.append(torch.cuda.Stream(dev))

            def run_streams():
                for e, s in zip(engines, streams):
                    s.wait_stream(torch.cuda.current_stream(dev))
                    with torch.cuda.stream(s):
                        e.train_epoch()
                for s in streams:
                    torch.cuda.current_stream(dev).wait_stream(s)
            ts = timed(run_streams, args.reps)
            print(json.dumps({"mode": "streams", "k": k, "epoch_ms": round(ts * 1e3, 3),
                              "vs_one_client": round(ts / t1, 3)}), flush=True)
            del engines
            gc.collect()
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
