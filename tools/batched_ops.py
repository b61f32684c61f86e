"""Per-GEMM cost of the batched K-client step under other tiles / split-K factors.

Records every ``ops.gemm`` call of one batched step (eager, inside the batched launch context), then times
each call alone -- as a plain launch (no pairing, no chain, no fused Adam) captured 20x in a hipGraph --
with the planner's tile / split-K and with forced alternatives.  The table says how far the planner's
choice is from the best single-launch variant at this client count:

    python tools/batched_ops.py [--k 8] [--rows 40000] [--tiles 32 64 128] [--splits 0 1 2 4 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--spec", default="intrusion", help="dataset schema (intrusion, wide, ...)")
    ap.add_argument("--only", type=int, nargs="*", default=None, help="only these call indices")
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--tiles", type=int, nargs="+", default=[32, 64, 128])
    ap.add_argument("--splits", type=int, nargs="+", default=[0, 1, 2, 4, 8], help="0 = the planner's split-K")
    ap.add_argument("--n", type=int, default=20, help="launches per graph")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE", help="native set_tuning knob")
    ap.add_argument("--only-planner", action="store_true", help="time only the planner's variant of each GEMM")
    args = ap.parse_args()
    import numpy as np
    import torch
    from fed_tgan_amd.data.schema import get_spec
    from fed_tgan_amd.data.synthetic import generate
    from fed_tgan_amd.data.table import TablePreprocessor
    from fed_tgan_amd.features.transformer import VGMTransformer
    from fed_tgan_amd.fed.stats import merge_categorical_metas
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.models.engine import EngineConfig
    from fed_tgan_amd.ops import hip as hipmod
    from fed_tgan_amd.ops import native
    for kv in args.tuning:
        key, val = kv.split("=", 1)
        native.require().set_tuning(key, int(val))
    dev = torch.device("cuda:0")
    spec = get_spec(args.spec)
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
    bc = BatchedClients(tr.layout, EngineConfig(), dev, [100 + c for c in range(args.k)], n_rows=len(X))
    for c, e in enumerate(bc.engines):
        e.set_training_data(X if c == 0 else X[rng.permutation(len(X))])
    e0 = bc.engines[0]
    ops = e0.ops
    calls = []
    orig = hipmod.HipOps.gemm

    def rec(self, a, b, c, **kw):
        calls.append((a, b, c, dict(kw)))
        return orig(self, a, b, c, **kw)
    hipmod.HipOps.gemm = rec
    bc.train_steps(1, use_graph=False)
    hipmod.HipOps.gemm = orig
    torch.cuda.synchronize()

    def per_call(fn):
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(args.n):
                fn()
        g.replay()
        torch.cuda.synchronize(dev)
        best = 1e9
        for _ in range(3):
            t = time.perf_counter()
            for _ in range(args.reps):
                g.replay()
            torch.cuda.synchronize(dev)
            best = min(best, (time.perf_counter() - t) / (args.reps * args.n) * 1e6)
        return best

    with bc._batched():
        for i, (a, b, c, kw) in enumerate(calls):
            if args.only is not None and i not in args.only:
                continue
            kw = dict(kw)
            kw["group"] = 0
            kw.pop("chain", None)
            ta, tb = kw.get("ta", False), kw.get("tb", False)
            a2, ta2 = hipmod._rowmajor(a, ta)
            b2, tb2 = hipmod._rowmajor(b, tb)
            M = a2.shape[1] if ta2 else a2.shape[0]
            K = a2.shape[0] if ta2 else a2.shape[1]
            N = b2.shape[0] if tb2 else b2.shape[1]
            kc = 64 if ops.f32 else 128
            tile_p, sk_p = hipmod._plan(M, N, K, kc, ops._plan_clients())
            res = {"i": i, "M": M, "N": N, "K": K, "ta": bool(ta), "tb": bool(tb), "epi": kw.get("epi", 0),
                   "onehot": kw.get("onehot") is not None, "plan": [tile_p, sk_p], "us": {}}
            for tile in ([] if args.only_planner else args.tiles):
                for sk in args.splits:
                    if tile == 128 and (M < 128 or sk not in (0, 1)):
                        continue
                    ops.tile_override = tile
                    ops.split_override = sk or None
                    try:
                        t = per_call(lambda: ops.gemm(a, b, c, **kw))
                    except Exception as ex:     # noqa: BLE001 - an unsupported variant
                        t = float("nan")
                        res.setdefault("errors", []).append(f"{tile}/{sk}: {str(ex)[:80]}")
                    res["us"][f"{tile}/{sk or 'p'}"] = round(t, 2)
            ops.tile_override = None
            ops.split_override = None
            res["us"]["planner"] = round(per_call(lambda: ops.gemm(a, b, c, **kw)), 2)
            good = {k: v for k, v in res["us"].items() if v == v}
            res["best"] = min(good, key=good.get)
            res["tuning"] = args.tuning
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
