"""Debug aid: where does a batched client's step first differ from a plain single-client engine?

Runs one step phase by phase (prepare, D update, G update) on a BatchedClients group and on plain
engines with the same seeds / weights / data, and prints the first buffers that differ.

    python tools/batched_diff.py [--k 2] [--precision bf16]
"""
import argparse
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--engine", action="append", default=[], metavar="KEY=VALUE",
                    help="EngineConfig override (repeatable), e.g. --engine bn_colown=1")
    args = ap.parse_args()
    import numpy as np
    import torch
    from fed_tgan_amd.data.demo import small_table
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    dev = torch.device("cuda:0")
    _, _, _, _, _, _, tr, X = small_table(2000, 0)
    cfg = EngineConfig(batch_size=500, precision=args.precision)
    for kv in args.engine:
        key, val = kv.split("=", 1)
        cur = getattr(cfg, key)
        setattr(cfg, key, (val.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(val))
    k = args.k
    seeds = [1000 + c for c in range(k)]
    rng = np.random.default_rng(7)
    data = [X if c == 0 else X[rng.permutation(len(X))] for c in range(k)]
    bc = BatchedClients(tr.layout, cfg, dev, seeds, n_rows=len(X))
    bc.engines[0].ops.batch_plan = False      # per-client split-K planning: bit-identical sums
    for e, Xc in zip(bc.engines, data):
        e.set_training_data(Xc)
    plain = []
    for s, e, Xc in zip(seeds, bc.engines, data):
        # (the batched step neither chains D1 nor fuses D1's weight gradient into the Adam launch)
        p = CTGANEngine(tr.layout, dataclasses.replace(cfg, chain_d1=False, fuse_d_adam=False), dev, backend="hip",
                        seed=s)
        p.flat.copy_(e.flat)
        p.set_training_data(Xc)
        plain.append(p)
    bc.freeze()
    names = ["H2", "logits2", "Xall", "col2", "opt2", "gbuf", "gradD", "gradG", "flat", "mD", "vD", "mG",
             "vG", "stepD", "stepG", "dlogits", "dH", "pen_rows", "ce_rows"]
    lists = ["abuf2", "nhat2", "bn_mean2", "bn_invstd2", "dl", "ms", "A", "da"]

    def compare(tag):
        torch.cuda.synchronize()
        bad = []
        for c, (e, p) in enumerate(zip(bc.engines, plain)):
            for n in names:
                a, b = getattr(e, n), getattr(p, n)
                if not torch.equal(a, b):
                    d = (a.double() - b.double()).abs().max().item()
                    bad.append(f"client {c} {n}: max |diff| {d:.3g}")
            for n in lists:
                for i, (a, b) in enumerate(zip(getattr(e, n), getattr(p, n))):
                    if not torch.equal(a, b):
                        d = (a.double() - b.double()).abs().max().item()
                        bad.append(f"client {c} {n}[{i}]: max |diff| {d:.3g}")
            if not torch.equal(e.ops.ctr, p.ops.ctr):
                bad.append(f"client {c} ctr {e.ops.ctr.item()} vs {p.ops.ctr.item()}")
        print(f"== {tag}: {'identical' if not bad else str(len(bad)) + ' differ'}")
        for b in bad[:40]:
            print("   ", b)
        return not bad

    compare("initial")
    e0 = bc.engines[0]
    for phase in ("_prepare_paired", "_d_update", "_g_update"):
        with bc._batched():
            e0.ops.begin_step(e0)
            getattr(e0, phase)()
        for p in plain:
            if phase == "_prepare_paired":
                p.ops.begin_step(p)
            getattr(p, phase)()
        if not compare(phase):
            break
    # then whole steps: eager, and graph-captured (8 per graph, then single-step graphs)
    for tag, n, graph in (("eager x2", 2, False), ("graph x8", 8, True), ("graph x3", 3, True), ("graph x8 again", 8, True)):
        bc.train_steps(n, use_graph=graph)
        for p in plain:
            p.train_steps(n, use_graph=graph)
        if not compare(tag):
            break


if __name__ == "__main__":
    main()
