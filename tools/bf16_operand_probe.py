"""Per-launch A/B for bf16 operand storage in training: the TB GEMMs that read D0's
weight -- D forward (D phase, 3 nP rows; G phase, nP rows) and the penalty's R0 product -- with fp32
operands (rounded to bf16 while staging, the training path) against bf16 operands (GemmArgs::bin, the
generation path: half the operand bytes, 16-B loads of 8 values).  Same epilogues, no D1 chain on
either side (the bf16 path has none).  Each variant: 64 launches captured in one hipGraph, best of 7.

    python tools/bf16_operand_probe.py [--rows 40000] [--reps 7]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def bf16_copy(t):
    import torch
    ld = -(-t.shape[1] // 8) * 8
    s = torch.zeros(t.shape[0], ld, dtype=torch.bfloat16, device=t.device)
    s[:, :t.shape[1]] = t
    return s[:, :t.shape[1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--n", type=int, default=64, help="launches per graph")
    args = ap.parse_args()
    import torch
    from fed_tgan_amd.data.demo import small_table
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from fed_tgan_amd.ops.hip import EPI_LRELU_DROPOUT, EPI_MASK
    dev = torch.device("cuda:0")
    _, _, _, _, _, _, tr, X = small_table(args.rows, 0)
    e = CTGANEngine(tr.layout, EngineConfig(), dev, backend="hip", seed=0)
    e.set_training_data(X)
    e.train_steps(4, use_graph=False)           # realistic activations / masks
    torch.cuda.synchronize()
    o, nP = e.ops, e.nP
    W = e.p["D.0.W"]
    W16 = bf16_copy(W)
    Xs = e.X.clone()
    X16 = bf16_copy(Xs)
    cases = {
        "D fwd, D phase (3nP rows)": dict(rows=slice(0, 3 * nP), epi=EPI_LRELU_DROPOUT, bias=True),
        "D fwd, G phase (nP rows)": dict(rows=slice(0, nP), epi=EPI_LRELU_DROPOUT, bias=True),
        "R0 = X_I W0^T . MS (nP rows)": dict(rows=slice(0, nP), epi=EPI_MASK, bias=False),
    }
    out = []
    for name, c in cases.items():
        r = c["rows"]
        m = Xs[r].shape[0]
        dst = torch.zeros(m, W.shape[0], device=dev)
        ms = e.ms[0][r].clone()
        kw = dict(tb=True, epi=c["epi"], ms=ms, slope=0.2, p_drop=0.5, stream_id=9)
        if c["bias"]:
            kw["bias"] = e.p["D.0.b"]
        res = {"case": name, "M": m, "N": W.shape[0], "K": W.shape[1]}
        ref = None
        for tag, (a, b) in (("fp32_operands", (Xs[r], W)), ("bf16_operands", (X16[r], W16))):
            o.gemm(a, b, dst, **kw)                # sizes the split-K workspace before capture
            torch.cuda.synchronize()
            if ref is None:
                ref = dst.clone()
            else:
                res["max_abs_diff"] = float((dst - ref).abs().max())
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for _ in range(args.n):
                        o.gemm(a, b, dst, **kw)
            torch.cuda.current_stream(dev).wait_stream(s)
            best = 1e9
            for _ in range(args.reps):
                t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0.record()
                g.replay()
                t1.record()
                t1.synchronize()
                best = min(best, t0.elapsed_time(t1) * 1e3 / args.n)
            res[f"{tag}_us"] = round(best, 3)
            del g
        res["saving_us"] = round(res["fp32_operands_us"] - res["bf16_operands_us"], 3)
        out.append(res)
        print(json.dumps(res), flush=True)
    # what the shadow costs: Adam writing a bf16 copy of W0 = 2 B per weight more traffic in a
    # bandwidth-bound launch (p, g, m, v read + p, m, v written = 28 B per weight now)
    n = W.numel()
    print(json.dumps({"adam_extra_bytes": 2 * n, "adam_bytes_now": 28 * n,
                      "extra_fraction": round(2 / 28, 4)}), flush=True)


if __name__ == "__main__":
    main()
