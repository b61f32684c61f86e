"""Per-op device cost inside hipGraphs: capture N back-to-back calls of one op, replay, time.

Reports microseconds per call (including the kernel-boundary cost inside a graph), which is
what a captured training step actually pays per launch.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def per_call(fn, dev, n=50, reps=20):
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t) / (reps * n) * 1e6


def step_only(eng, dev, epochs_only=False):
    # the engine's own epoch path: its graph_unroll-step graphs (multi-step sampler draw, EngineConfig.multi_draw)
    eng.train_steps(eng.steps_per_epoch)
    torch.cuda.synchronize(dev)
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(5):
            eng.train_steps(eng.steps_per_epoch)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t) / (5 * eng.steps_per_epoch) * 1e6
        print(f"engine epoch graphs (unroll {eng.cfg.graph_unroll}, multi_draw {eng._multi}): {dt:8.2f} us/step",
              flush=True)
    if epochs_only:
        return
    for _ in range(2):
        a = per_call(eng._one_step, dev, n=5, reps=20)
        lanes, eng.lanes = eng.lanes, None
        b = per_call(eng._one_step, dev, n=5, reps=20)
        eng.lanes = lanes
        print(f"full step: side lanes {a:8.2f} us   one stream {b:8.2f} us")


def onehot_ab(eng, tr, X, dev):
    """EngineConfig.onehot A/B: full captured step and generate_decoded(40000), dense K vs gathered c."""
    from fed_tgan_amd.models.samplers import CondTables
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    for rep in range(2):
        for oh, tr_ in ((False, False), (True, False), (True, True)):
            eng.use_onehot = oh
            eng.cfg.onehot_trans = tr_
            eng._gen_graphs = {}
            t_step = per_call(eng._one_step, dev, n=5, reps=20)
            eng.generate_decoded(40000)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for _ in range(20):
                eng.generate_decoded(40000)
            torch.cuda.synchronize(dev)
            t_gen = (time.perf_counter() - t) / 20 * 1e6
            print(f"onehot={int(oh)} train_transposed={int(tr_)}: full step {t_step:8.2f} us   "
                  f"generate_decoded(40000) {t_gen:8.1f} us", flush=True)


def gwt_ab(tr, X, dev, precision, key="g_wt", base=None):
    """A/B of a boolean EngineConfig field (default g_wt: generator weights stored [out, in] vs
    input-major); full captured step and generate_decoded(40000), two engines from the same initial
    weights, alternating."""
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from fed_tgan_amd.models.samplers import CondTables
    engs = {}
    for g_wt in (False, True):
        import dataclasses
        cfg = dataclasses.replace(base, **{key: g_wt}) if base is not None else EngineConfig(precision=precision, **{key: g_wt})
        e = CTGANEngine(tr.layout, cfg, dev, backend="hip", seed=1)
        e.set_training_data(X)
        e.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
        engs[g_wt] = e
    engs[True].load_g_state_dict(engs[False].g_state_dict())
    for rep in range(3):
        for g_wt, e in engs.items():
            t_step = per_call(e._one_step, dev, n=5, reps=20)
            e.generate_decoded(40000)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for _ in range(20):
                e.generate_decoded(40000)
            torch.cuda.synchronize(dev)
            t_gen = (time.perf_counter() - t) / 20 * 1e6
            print(f"{key}={int(g_wt)}: full step {t_step:8.2f} us   generate_decoded(40000) {t_gen:8.1f} us", flush=True)


def fork_probe(eng, dev):
    """Cost of a forked branch inside the captured step: the one-stream step vs the same step with a
    second sampler launch (into scratch buffers) on a side stream, forked after the G phase's dlogits
    and joined at the end of the step (what hiding step t+1's sampler behind step t's G backward
    would look like)."""
    o, B = eng.ops, eng.B
    side = torch.cuda.Stream(dev)
    H2s, Xs, Xr = eng.H2.clone(), eng.Xall[2 * B:4 * B].clone(), eng.X_real.clone()
    col, opt = eng.col2.clone(), eng.opt2.clone()
    sD, sG, met = eng.stepD.clone(), eng.stepG.clone(), eng.metrics.clone()
    ctr_s = torch.zeros(1, dtype=torch.int64, device=dev)

    def forked(work: bool):
        def step():
            cur = torch.cuda.current_stream(dev)
            eng._prepare_paired()
            eng._d_update()
            eng._g_dlogits()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                if work:
                    o.sample_train(eng.tables, H2s, eng.z_cols, eng.c_cols, Xs, Xr, eng.Dd, col, opt,
                                   step_counter=(sD, sG), metrics=met, zero_metrics=True, stream_id=1)
                else:
                    o.L.rng_bump(ctr_s)
            eng._g_adam(eng._g_backward(fold_colsum=True))
            cur.wait_stream(side)
        return step

    for _ in range(3):
        base = per_call(eng._one_step, dev, n=5, reps=20)
        f0 = per_call(forked(False), dev, n=5, reps=20)
        f1 = per_call(forked(True), dev, n=5, reps=20)
        print(f"one stream {base:8.2f} us   fork+join (1-thread kernel) {f0:8.2f} us   "
              f"fork+join (concurrent sampler) {f1:8.2f} us", flush=True)


def bn_ab(eng, dev):
    """BN(train) from GEMM partials (bn_relu_apply) vs the separate full-reduction BN kernel."""
    for rep in range(3):
        for fused in (False, True):
            eng.ops.bn_fused = fused
            print(f"bn_fused={int(fused)}: full step {per_call(eng._one_step, dev, n=5, reps=20):8.2f} us", flush=True)


def colown_ab(eng, dev):
    """Generator Linear -> BN(train) -> ReLU: tile GEMM + BN kernel (two launches) vs one launch by column
    ownership (EngineConfig.bn_colown) -- each paired layer alone, then the full captured step."""
    def layer(i):
        a, b_ = eng.off[i], eng.off[i + 1]
        x, W, oh = eng._g_in(eng.H2, a, eng.p[f"G.{i}.W"], (eng.col2, eng.opt2, eng.cfg.onehot_trans))
        return lambda: eng.ops.linear_bn_relu(
            x, W, eng.p[f"G.{i}.b"], eng.p[f"G.{i}.gamma"], eng.p[f"G.{i}.beta"], eng.H2[:, b_:a], eng.abuf2[i],
            eng.nhat2[i], eng.bn_mean2[i], eng.bn_invstd2[i], eng.p[f"G.{i}.rm"], eng.p[f"G.{i}.rv"], True,
            eng.cfg.bn_momentum, eng.cfg.bn_eps, groups=2, onehot=oh)
    eng._prepare_paired()
    if os.environ.get("COLOWN_DBG"):
        # phase costs of the one-launch kernel (results wrong while a bit is set): 1 no GEMM, 2 no
        # staging, 4 no output stores
        eng.ops.bn_colown = True
        for dbg in (0, 1, 2, 4, 7):
            torch.ops.fedtgan.set_tuning("colown_dbg", dbg)
            row = [per_call(layer(i), dev) for i in range(len(eng.gdims))]
            print(f"colown_dbg={dbg}: " + "  ".join(f"G{i} paired {v:6.2f} us" for i, v in enumerate(row)), flush=True)
        torch.ops.fedtgan.set_tuning("colown_dbg", 0)
    for rep in range(3):
        for on in (False, True):
            eng.ops.bn_colown = on
            row = [per_call(layer(i), dev) for i in range(len(eng.gdims))]
            t_step = per_call(eng._one_step, dev, n=5, reps=20)
            print(f"bn_colown={int(on)}: " + "  ".join(f"G{i} paired {v:6.2f} us" for i, v in enumerate(row)) +
                  f"   full step {t_step:8.2f} us", flush=True)


def dw0_tile_ab(eng, dev):
    """D0 weight-gradient GEMM (paired with R0): planner tile vs 128x128 (fewer, fatter workgroups)."""
    for rep in range(3):
        for t in (0, 128):
            eng.cfg.dw0_tile = t
            print(f"dw0_tile={t}: full step {per_call(eng._one_step, dev, n=5, reps=20):8.2f} us", flush=True)


def inlaunch_ab(eng, dev):
    """Split-K reduction: separate gemm_splitk_epilogue launch vs the last-arriving K-slice workgroup
    (tile counters) -- the step's split GEMMs alone, then the full captured step."""
    from fed_tgan_amd.ops.hip import EPI_LRELU_DROPOUT
    o, nP = eng.ops, eng.nP
    X = eng.X
    shapes = {
        "D0 fwd 3nP x256 xDin lrelu+drop": (X, eng.p["D.0.W"], eng.dl[0], dict(tb=True, bias=eng.p["D.0.b"],
                                                                              epi=EPI_LRELU_DROPOUT, ms=eng.ms[0])),
        "D0 fwd nP x256 xDin (G phase)": (X[:nP], eng.p["D.0.W"], eng.dl[0][:nP], dict(tb=True)),
    }
    for rep in range(2):
        for inl in (False, True):
            o.splitk_inlaunch = inl
            row = [per_call(lambda: o.gemm(a, b, c, **kw), dev) for a, b, c, kw in shapes.values()]
            t_step = per_call(eng._one_step, dev, n=5, reps=20)
            print(f"splitk_inlaunch={int(inl)}: " + "  ".join(f"{k} {v:6.2f} us" for k, v in zip(shapes, row)) +
                  f"   full step {t_step:8.2f} us", flush=True)
    o.splitk_inlaunch = False


def gen_only(eng, tr, X, dev):
    """generate_decoded(40000): eager vs hipGraph, chunk 8192 vs one chunk (wall time per call)."""
    from fed_tgan_amd.models.samplers import CondTables
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    for chunk in (8192, 40000):
        eng.cfg.gen_chunk = chunk
        eng._gen_bufs, eng._gen_graphs = None, {}
        for graph in (False, True):
            eng.generate_decoded(40000, use_graph=graph)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for _ in range(10):
                v = eng.generate_decoded(40000, use_graph=graph)
            torch.cuda.synchronize(dev)
            us = (time.perf_counter() - t) / 10 * 1e6
            t = time.perf_counter()
            for _ in range(10):
                h = v.cpu()
            d2h = (time.perf_counter() - t) / 10 * 1e6
            print(f"generate_decoded(40000) chunk={chunk:6d} graph={graph!s:5}: {us:9.1f} us   "
                  f"(D2H pageable copy {d2h:8.1f} us)", flush=True)
    # decode kernel alone on one 40000-row chunk: one thread per cell vs one wave per row
    logits = torch.randn(40000, X.shape[1], device=dev) * 3
    out = torch.zeros(40000, len(tr.meta), dtype=torch.float64, device=dev)
    for mode in (0, 1, 2):
        prev = torch.ops.fedtgan.set_tuning("decode_rows", mode)
        try:
            us = per_call(lambda: eng.ops.sample_decode(logits, out, eng.gen_tables), dev, n=20, reps=10)
        finally:
            torch.ops.fedtgan.set_tuning("decode_rows", prev)
        print(f"sample_decode 40000 rows, decode_rows={mode}: {us:9.1f} us", flush=True)
    # whole captured pass vs the GEMM tile order (the 40k-row GEMMs are K = 431 / 687 / 943)
    eng.cfg.gen_chunk = 40960
    for remap in (0, 1, 2, 1, 0, 2):
        prev = torch.ops.fedtgan.set_tuning("gemm_xcd_remap", remap)
        try:
            eng._gen_bufs, eng._gen_graphs = None, {}
            eng.generate_decoded(40000)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for _ in range(20):
                eng.generate_decoded(40000)
            torch.cuda.synchronize(dev)
            us = (time.perf_counter() - t) / 20 * 1e6
        finally:
            torch.ops.fedtgan.set_tuning("gemm_xcd_remap", prev)
        print(f"generate_decoded(40000) graph, gemm_xcd_remap={remap}: {us:9.1f} us", flush=True)


def unroll_sweep(eng, dev):
    """Wall time of one 80-step local epoch for several steps-per-graph settings."""
    for U in (1, 2, 4, 8, 16, 40, 80):
        eng.cfg.graph_unroll = U
        eng.graphs = {}
        eng.train_steps(80)
        torch.cuda.synchronize(dev)
        best = 1e9
        for _ in range(5):
            t = time.perf_counter()
            eng.train_steps(80)
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t)
        print(f"graph_unroll={U:3d}: epoch of 80 steps {best * 1e3:8.3f} ms  ({best / 80 * 1e6:7.1f} us/step)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--init-rng", default=None, help="EngineConfig.init_rng (engine | global)")
    ap.add_argument("--engine", action="append", default=[], metavar="KEY=VALUE",
                    help="EngineConfig override for A/B runs, e.g. --engine chain_d1=0")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE",
                    help="native set_tuning knob for A/B runs, e.g. --tuning bn_cols=16")
    ap.add_argument("--split-sweep", action="store_true", help="time every GEMM shape at each split-K factor")
    ap.add_argument("--step-only", action="store_true", help="time only the full captured step")
    ap.add_argument("--epochs-only", action="store_true", help="with --step-only: only the engine's own epoch graphs")
    ap.add_argument("--gen", action="store_true", help="time the generation pass (eager / graph, chunk sizes)")
    ap.add_argument("--unroll", action="store_true", help="epoch time vs training steps captured per graph")
    ap.add_argument("--xcd-sweep", action="store_true", help="each step GEMM: dispatch vs XCD-contiguous tile order")
    ap.add_argument("--adam-sweep", action="store_true", help="Adam store policy: plain / nt / sc1")
    ap.add_argument("--store-sweep", action="store_true", help="GEMM output stores: plain / write-through")
    ap.add_argument("--fold-sweep", action="store_true", help="column sums: own launch / folded into Adam")
    ap.add_argument("--pair-sweep", action="store_true", help="independent GEMM pairs: two launches / one")
    ap.add_argument("--onehot-ab", action="store_true", help="step + generation: dense c block vs one-hot gather")
    ap.add_argument("--bn-ab", action="store_true", help="step: BN from GEMM partials vs full-reduction BN kernel")
    ap.add_argument("--colown-ab", action="store_true", help="step: G layers as tile GEMM + BN vs one colown launch")
    ap.add_argument("--dw0-ab", action="store_true", help="step: D0 weight-gradient tile 64 vs 128")
    ap.add_argument("--inlaunch-ab", action="store_true", help="split-K: epilogue launch vs in-launch reduction")
    ap.add_argument("--gwt-ab", action="store_true", help="step + generation: generator weights [out, in] vs input-major")
    ap.add_argument("--cfg-ab", default=None, metavar="FIELD", help="step + generation: a boolean EngineConfig field off / on")
    ap.add_argument("--fork-probe", action="store_true", help="step: cost of a forked side-stream branch in the graph")
    args = ap.parse_args()
    if args.tuning:
        from fed_tgan_amd.ops import native as _nat
        for kv in args.tuning:
            k_, v_ = kv.split("=", 1)
            _nat.require().set_tuning(k_, int(v_))
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from helpers import small_table
    dev = torch.device("cuda:0")
    _, _, _, _, _, _, tr, X = small_table(40000, 0)
    cfg = EngineConfig(precision=args.precision)
    for kv in args.engine:
        k_, v_ = kv.split("=", 1)
        cur = getattr(cfg, k_)
        setattr(cfg, k_, (v_.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v_))
    if args.init_rng:
        cfg.init_rng = args.init_rng
    eng = CTGANEngine(tr.layout, cfg, dev, backend="hip", seed=1)
    eng.set_training_data(X)
    o = eng.ops
    nP, B = eng.nP, eng.B
    res = {}
    if args.step_only:
        return step_only(eng, dev, args.epochs_only)
    if args.fork_probe:
        return fork_probe(eng, dev)
    if args.gwt_ab:
        return gwt_ab(tr, X, dev, args.precision)
    if args.cfg_ab:
        return gwt_ab(tr, X, dev, args.precision, key=args.cfg_ab, base=cfg)
    if args.gen:
        return gen_only(eng, tr, X, dev)
    if args.onehot_ab:
        return onehot_ab(eng, tr, X, dev)
    if args.bn_ab:
        return bn_ab(eng, dev)
    if args.colown_ab:
        return colown_ab(eng, dev)
    if args.dw0_ab:
        return dw0_tile_ab(eng, dev)
    if args.inlaunch_ab:
        return inlaunch_ab(eng, dev)
    if args.unroll:
        return unroll_sweep(eng, dev)
    res["rng_bump (1 thread)"] = per_call(lambda: o.L.rng_bump(o.ctr), dev)
    shapes = {
        "G0 fwd 500x256x(E+C) NT": (*eng._kpad(eng.H, eng.off[0], eng.p["G.0.W"]), eng.abuf[0], False, True),
        "G0 fwd paired 1000x256x(E+C) NT": (*eng._kpad(eng.H2, eng.off[0], eng.p["G.0.W"]), eng.abuf2[0], False, True),
        "G1 fwd paired 1000x256x(E+C+256) NT": (*eng._kpad(eng.H2, eng.off[1], eng.p["G.1.W"]), eng.abuf2[1], False,
                                                 True),
        "Gout fwd paired 1000xDdxHw NT": (*eng._kpad(eng.H2, 0, eng.p["G.out.W"]), eng.logits2, False, True),
        "G1 fwd 500x256x(E+C+256) NT": (*eng._kpad(eng.H, eng.off[1], eng.p["G.1.W"]), eng.abuf[1], False, True),
        "Gout fwd 500xDdxHw NT": (*eng._kpad(eng.H, 0, eng.p["G.out.W"]), eng.logits, False, True),
        "D0 fwd 150x256xK1 NT": (eng.X, eng.p["D.0.W"], eng.dl[0], False, True),
        "D1 fwd 150x256x256 NT": (eng.dl[0], eng.p["D.1.W"], eng.dl[1], False, True),
        "A chain 150x256x256 NN": (eng.A[1], eng.p["D.1.W"], eng.A[0], False, False),
        "gp g 50xK1x256 NN": (eng.A[0][:nP], eng.p["D.0.W"], eng.gbuf, False, False),
        "dV0 256xK1x150 TN": (eng.A[0], eng.X, eng.g["D.0.W"], True, False),
        "dWout DdxHwx500 TN": (eng.dlogits, *eng._kpad(eng.H, 0, eng.g["G.out.W"]), True, False),
        "dH 500x512xDd NN": (eng.dlogits, eng.p["G.out.W"][:, :eng.off[0]], eng.dH[:, :eng.off[0]], False, False),
        "R0 50x256xK1 NT": (eng.X[eng.rows_i], eng.p["D.0.W"], eng.dl[0][eng.rows_i], False, True),
        "dW1 256x(E+C+256)x500 TN": (eng.da[1], *eng._kpad(eng.H, eng.off[1], eng.g["G.1.W"]), True, False),
    }
    if args.split_sweep:
        for name, (a, b, c, ta, tb) in shapes.items():
            K = a.shape[0] if ta else a.shape[1]
            kc = 64 if o.f32 else 128
            bursts = -(-K // kc)
            for tile in (64, 32):
                o.tile_override = tile
                row = []
                for sk in [0, 1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48]:
                    if sk > bursts:
                        break
                    o.split_override = sk or None
                    us = per_call(lambda a=a, b=b, c=c, ta=ta, tb=tb: o.gemm(a, b, c, ta=ta, tb=tb), dev)
                    row.append(f"{'auto' if sk == 0 else sk}:{us:.1f}")
                print(f"{name:28s} t{tile} " + "  ".join(row), flush=True)
            o.split_override = None
            o.tile_override = None
        return
    if args.pair_sweep:
        for pr in (0, 1, 0, 1):
            prev = torch.ops.fedtgan.set_tuning("gemm_pairs", pr)
            print(f"gemm_pairs={pr}: full step {per_call(eng._one_step, dev, n=5, reps=20):8.2f} us", flush=True)
            torch.ops.fedtgan.set_tuning("gemm_pairs", prev)
        return
    if args.fold_sweep:
        for rep in range(2):
            for tag, fl, p_, g_, m_, v_, st, wd, jobs in (
                    ("D", eng.flatD, eng.flatD, eng.gradD, eng.mD, eng.vD, eng.stepD, 0.0, eng._d_colsum_jobs()),
                    ("G", eng.flatG, eng.flatG, eng.gradG, eng.mG, eng.vG, eng.stepG, 1e-6, eng._g_colsum_jobs())):
                t_cs = per_call(lambda: o.colsum_many(*jobs), dev)
                t_ad = per_call(lambda: o.adam(p_, g_, m_, v_, st, 2e-4, 0.5, 0.9, 1e-8, wd), dev)
                t_two = per_call(lambda: (o.colsum_many(*jobs), o.adam(p_, g_, m_, v_, st, 2e-4, 0.5, 0.9, 1e-8, wd)),
                                 dev)
                t_f = per_call(lambda: o.adam(p_, g_, m_, v_, st, 2e-4, 0.5, 0.9, 1e-8, wd, jobs=jobs), dev)
                print(f"{tag}: colsum {t_cs:6.2f}  adam {t_ad:6.2f}  colsum+adam {t_two:6.2f}  folded {t_f:6.2f} us",
                      flush=True)
        return
    if args.store_sweep:
        for wt in (0, 1, 0, 1):
            prev = torch.ops.fedtgan.set_tuning("gemm_store_wt", wt)
            row = [per_call(lambda a=a, b=b, c=c, ta=ta, tb=tb: o.gemm(a, b, c, ta=ta, tb=tb), dev)
                   for (a, b, c, ta, tb) in shapes.values()]
            t_step = per_call(eng._one_step, dev, n=5, reps=20)
            torch.ops.fedtgan.set_tuning("gemm_store_wt", prev)
            print(f"gemm_store_wt={wt}: GEMMs " + " ".join(f"{x:5.2f}" for x in row) + f"   full step {t_step:8.2f} us",
                  flush=True)
        return
    if args.adam_sweep:
        for aux in (0, 2, 16, 0, 2, 16):
            prev = torch.ops.fedtgan.set_tuning("adam_store", aux)
            t_adam = per_call(lambda: o.adam(eng.flatD, eng.gradD, eng.mD, eng.vD, eng.stepD, 2e-4, 0.5, 0.9, 1e-8,
                                             0.0), dev)
            t_step = per_call(eng._one_step, dev, n=5, reps=20)
            torch.ops.fedtgan.set_tuning("adam_store", prev)
            print(f"adam_store={aux:2d}: adam D {t_adam:7.2f} us   full step {t_step:8.2f} us", flush=True)
        for nb in (512, 1024, 2048, 65535):
            prev = torch.ops.fedtgan.set_tuning("adam_max_blocks", nb)
            t_adam = per_call(lambda: o.adam(eng.flatD, eng.gradD, eng.mD, eng.vD, eng.stepD, 2e-4, 0.5, 0.9, 1e-8,
                                             0.0), dev)
            torch.ops.fedtgan.set_tuning("adam_max_blocks", prev)
            print(f"adam_max_blocks={nb:5d}: adam D {t_adam:7.2f} us", flush=True)
        return
    if args.xcd_sweep:
        for name, (a, b, c, ta, tb) in shapes.items():
            row = []
            for rm in (0, 2):
                prev = torch.ops.fedtgan.set_tuning("gemm_xcd_remap", rm)
                row.append(per_call(lambda a=a, b=b, c=c, ta=ta, tb=tb: o.gemm(a, b, c, ta=ta, tb=tb), dev))
                torch.ops.fedtgan.set_tuning("gemm_xcd_remap", prev)
            print(f"{name:36s} dispatch order {row[0]:7.2f} us   XCD-contiguous {row[1]:7.2f} us", flush=True)
        for rm in (0, 1, 2, 0, 1, 2):
            prev = torch.ops.fedtgan.set_tuning("gemm_xcd_remap", rm)
            print(f"full step xcd_remap={rm}: {per_call(eng._one_step, dev, n=5, reps=20):8.2f} us", flush=True)
            torch.ops.fedtgan.set_tuning("gemm_xcd_remap", prev)
        return
    for name, (a, b, c, ta, tb) in shapes.items():
        res[name] = per_call(lambda a=a, b=b, c=c, ta=ta, tb=tb: o.gemm(a, b, c, ta=ta, tb=tb), dev)
    t = eng.tables
    res["sample_train D"] = per_call(lambda: o.sample_train(t, eng.H, eng.z_cols, eng.c_cols, eng.X_fake,
                                                            eng.X_real, eng.Dd, eng.col, eng.opt), dev)
    res["sample_train G"] = per_call(lambda: o.sample_train(t, eng.H, eng.z_cols, eng.c_cols, eng.Xg, None,
                                                            eng.Dd, eng.col, eng.opt), dev)
    res["sample_train paired (D+G)"] = per_call(lambda: o.sample_train(t, eng.H2, eng.z_cols, eng.c_cols,
                                                                        eng.Xall[2 * B:], eng.X_real, eng.Dd, eng.col2,
                                                                        eng.opt2), dev)
    res["activate"] = per_call(lambda: o.activate(eng.logits, eng.Xg[:, :eng.Dd], eng.spans), dev)
    res["activate + slerp"] = per_call(lambda: o.activate(eng.logits, eng.X_fake[:, :eng.Dd], eng.spans,
                                                          slerp=(eng.X_real, eng.X_fake, eng.X_interp, 3)), dev)
    res["activate paired + slerp"] = per_call(lambda: o.activate(eng.logits2, eng.Xall[2 * B:, :eng.Dd], eng.spans,
                                                                 slerp=(eng.X_real, eng.X_fake, eng.X_interp, 3)), dev)
    res["act_bwd_ce"] = per_call(lambda: o.act_bwd_ce(eng.gbuf.view(B, eng.Din)[:, :eng.Dd], eng.Xg[:, :eng.Dd],
                                                      eng.logits, eng.spans, eng.cond_spans, eng.col, eng.opt,
                                                      eng.dlogits, eng.ce_rows), dev)
    res["bn_relu_train"] = per_call(lambda: o.bn_relu_fwd(eng.abuf[0], eng.p["G.0.gamma"], eng.p["G.0.beta"],
                                                          eng.H[:, eng.off[1]:eng.off[0]], eng.nhat[0], eng.bn_mean[0],
                                                          eng.bn_invstd[0], eng.p["G.0.rm"], eng.p["G.0.rv"]), dev)
    res["bn_relu_train paired"] = per_call(lambda: o.bn_relu_fwd(eng.abuf2[0], eng.p["G.0.gamma"], eng.p["G.0.beta"],
                                                                 eng.H2[:, eng.off[1]:eng.off[0]], eng.nhat2[0],
                                                                 eng.bn_mean2[0], eng.bn_invstd2[0], eng.p["G.0.rm"],
                                                                 eng.p["G.0.rv"], groups=2), dev)
    for bc in (4, 8, 16):
        prev = torch.ops.fedtgan.set_tuning("bn_cols", bc)
        res[f"bn_relu_train paired cols={bc}"] = per_call(
            lambda: o.bn_relu_fwd(eng.abuf2[0], eng.p["G.0.gamma"], eng.p["G.0.beta"], eng.H2[:, eng.off[1]:eng.off[0]],
                                  eng.nhat2[0], eng.bn_mean2[0], eng.bn_invstd2[0], eng.p["G.0.rm"], eng.p["G.0.rv"],
                                  groups=2), dev)
        res[f"bn_relu_bwd cols={bc}"] = per_call(
            lambda: o.bn_relu_bwd(eng.dH[:, eng.off[1]:eng.off[0]], eng.H[:, eng.off[1]:eng.off[0]], eng.nhat[0],
                                  eng.p["G.0.gamma"], eng.bn_invstd[0], eng.da[0], eng.g["G.0.gamma"],
                                  eng.g["G.0.beta"], eng.g["G.0.b"]), dev)
        torch.ops.fedtgan.set_tuning("bn_cols", prev)
    res["adam D"] = per_call(lambda: o.adam(eng.flatD, eng.gradD, eng.mD, eng.vD, eng.stepD, 2e-4, 0.5, 0.9, 1e-8, 0.0),
                             dev)
    res["slerp"] = per_call(lambda: o.slerp(eng.X_real, eng.X_fake, eng.X_interp), dev)
    res["gp_scale"] = per_call(lambda: o.gp_scale(eng.gbuf, eng.X[eng.rows_i], 10.0, eng.pen_rows), dev)
    eng.cfg.paired = False
    res["full step (graph, per-phase prepare)"] = per_call(eng._one_step, dev, n=5, reps=20)
    eng.cfg.paired = True
    res["full step (graph, paired prepare)"] = per_call(eng._one_step, dev, n=5, reps=20)
    for k, v in res.items():
        print(f"{v:9.2f} us  {k}")


if __name__ == "__main__":
    main()
