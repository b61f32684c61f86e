"""Generation at 40,000 rows: each launch of the pass timed alone inside a hipGraph (fp32 storage vs
bf16 storage, EngineConfig.gen_bf16; planner / 64 / 128 output tiles), then the whole captured
generate_decoded(40000).

    python tools/gen_probe.py [--rows 40000]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

from microbench import per_call  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--g0", action="store_true", help="G0 variants only")
    args = ap.parse_args()
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from fed_tgan_amd.models.samplers import CondTables
    from helpers import small_table
    dev = torch.device("cuda:0")
    _, _, _, _, _, _, tr, X = small_table(40000, 0)
    eng = CTGANEngine(tr.layout, EngineConfig(gen_chunk=max(args.rows, 40960)), dev, backend="hip", seed=1)
    eng.set_training_data(X)
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    n = args.rows
    o = eng.ops
    p = eng.p
    c0 = eng.c_cols[0]

    def layers_for(bf16):
        eng.cfg.gen_bf16 = bf16
        eng._gen_graphs, eng._gen_bufs = {}, None
        eng.generate_decoded(n)
        _, H, lg, out, col, opt = eng._gen_graphs[n]
        w16 = eng._gen_weights16()[0] if bf16 else None
        res = []
        for i, g in enumerate(eng.gdims):
            a, b_ = eng.off[i], eng.off[i + 1]
            W = p[f"G.{i}.W"]
            oh = (W[:, c0 - a:].t().contiguous(), col, opt, eng._cond_off, True)
            x, Wd = (H[:, a:c0], w16[i]) if bf16 else (H[:, a:c0], W[:, :c0 - a])
            res.append((f"G{i} K{c0 - a}",
                        lambda x=x, Wd=Wd, oh=oh, i=i, a=a, b_=b_, H=H: o.linear_bn_relu(
                            x, Wd, p[f"G.{i}.b"], p[f"G.{i}.gamma"], p[f"G.{i}.beta"], H[:, b_:a], None, None, None,
                            None, p[f"G.{i}.rm"], p[f"G.{i}.rv"], False, onehot=oh)))
        W = p["G.out.W"]
        oh = (W[:, c0:].t().contiguous(), col, opt, eng._cond_off, True)
        x, Wd = (H[:, :c0], w16[-1]) if bf16 else (H[:, :c0], W[:, :c0])
        res.append((f"Gout N{W.shape[0]} K{c0}", lambda x=x, Wd=Wd, oh=oh: o.gemm(x, Wd, lg, tb=True, bias=p["G.out.b"],
                                                                                 onehot=oh)))
        res.append(("sample", lambda H=H, col=col, opt=opt: o.sample_gen(eng.gen_cond, H, eng.c_cols, eng.z_cols,
                                                                         col_out=col, opt_out=opt, stream_id=21)))
        res.append(("decode", lambda: o.sample_decode(lg, out, eng.gen_tables)))
        if bf16:
            res.append(("weights->bf16", eng._gen_weights16))

        def decode_mode(mode):
            prev = torch.ops.fedtgan.set_tuning("decode_rows", mode)
            try:
                o.sample_decode(lg, out, eng.gen_tables)
            finally:
                torch.ops.fedtgan.set_tuning("decode_rows", prev)
        res.append(("decode(row)", lambda: decode_mode(1)))
        return res

    if args.g0:
        # G0 variants: what does its time depend on (one-hot gather, BN epilogue, output dtype, tile)?
        from fed_tgan_amd.ops.hip import EPI_BN_EVAL_RELU
        layers_for(True)
        _, H, lg, out, col, opt = eng._gen_graphs[n]
        w16 = eng._gen_weights16()[0]
        a, b_ = eng.off[0], eng.off[1]
        W = p["G.0.W"]
        oh = (W[:, c0 - a:].t().contiguous(), col, opt, eng._cond_off, True)
        x = H[:, a:c0]
        o32 = torch.zeros(n, W.shape[0], device=dev)
        bn = (p["G.0.gamma"], p["G.0.beta"], p["G.0.rm"], p["G.0.rv"])
        cases = {
            "onehot+bn, bf16 out": lambda: o.gemm(x, w16[0], H[:, b_:a], tb=True, bias=p["G.0.b"], epi=EPI_BN_EVAL_RELU,
                                                  bn=bn, onehot=oh),
            "bn, bf16 out": lambda: o.gemm(x, w16[0], H[:, b_:a], tb=True, bias=p["G.0.b"], epi=EPI_BN_EVAL_RELU, bn=bn),
            "onehot, bf16 out": lambda: o.gemm(x, w16[0], H[:, b_:a], tb=True, bias=p["G.0.b"], onehot=oh),
            "plain, bf16 out": lambda: o.gemm(x, w16[0], H[:, b_:a], tb=True),
            "plain, fp32 out": lambda: o.gemm(x, w16[0], o32, tb=True),
            "onehot+bn, fp32 out": lambda: o.gemm(x, w16[0], o32, tb=True, bias=p["G.0.b"], epi=EPI_BN_EVAL_RELU, bn=bn,
                                                  onehot=oh),
        }
        for tile in (None, 32, 128):
            o.tile_override = tile
            print(f"tile={tile}: " + "  ".join(f"{k}: {per_call(fn, dev, n=10, reps=10):6.1f}" for k, fn in cases.items()),
                  flush=True)
        o.tile_override = None
        return
    for rep in range(2):
        for bf16, tile in ((False, None), (True, None), (True, 64), (True, 128)):
            layers = layers_for(bf16)
            o.tile_override = tile
            row = [per_call(fn, dev, n=10, reps=10) for _, fn in layers]
            eng._gen_graphs = {}
            eng.generate_decoded(n)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            for _ in range(20):
                eng.generate_decoded(n)
            torch.cuda.synchronize(dev)
            tot = (time.perf_counter() - t) / 20 * 1e6
            o.tile_override = None
            print(f"gen_bf16={int(bf16)} tile={tile}: " + "  ".join(f"{k}: {v:6.1f}" for (k, _), v in zip(layers, row)) +
                  f"  | generate_decoded({n}) {tot:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
