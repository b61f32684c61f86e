"""First-use cost of the torch GPU kernels federated initialisation touches (each distinct kernel's first launch
loads its code object), issued from one thread or spread over several.

    python tools/cold_probe.py --threads 1|4 [--json out.jsonl]

Run it as the first GPU process of a fresh box for the cold numbers.  Prints the HIP context time, then the wall
time of the warm-up set (and, with one thread, each op's own first-call time).
"""
import argparse
import json
import threading
import time

import torch


def _ops(dev):
    """(name, thunk) of the first-use kernels seen in a cold FedRuntime.initialize cProfile (round 5)."""
    f32 = torch.rand(40000, 34, device=dev)
    f64 = f32.double()
    i64 = torch.randint(0, 100, (40000,), device=dev)
    return [
        ("sort_f32", lambda: torch.sort(f32.reshape(-1))),
        ("sort_f64_dim0", lambda: torch.sort(f64, dim=0)),
        ("argsort_i64", lambda: torch.argsort(i64, stable=True)),
        ("isfinite", lambda: torch.isfinite(f64).all()),
        ("floor", lambda: torch.floor(f64)),
        ("sum_dim", lambda: f64.sum(0)),
        ("any", lambda: (f32 > 2).any()),
        ("cumsum", lambda: f64.cumsum(0)),
        ("searchsorted", lambda: torch.searchsorted(torch.sort(f64[:, 0]).values, f64[:100, 0].contiguous())),
        ("gather", lambda: torch.gather(f64, 0, i64.clamp(max=39999)[:, None].expand(-1, 34))),
        ("where", lambda: torch.where(f32 > 0.5, f32, 0.0)),
        ("exp_log", lambda: torch.log(torch.exp(f32) + 1)),
        ("max_dim", lambda: f64.max(dim=1)),
        ("to_cpu", lambda: f64[:10].cpu()),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    t = time.perf_counter()
    torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    rec = {"threads": args.threads, "hip_context_s": round(time.perf_counter() - t, 3)}
    ops = _ops(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if args.threads <= 1:
        per = {}
        for name, fn in ops:
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            per[name] = round(time.perf_counter() - t, 4)
        rec["per_op_s"] = per
    else:
        def run(chunk):
            torch.cuda.set_device(dev)
            for _, fn in chunk:
                fn()
            torch.cuda.synchronize()
        ths = [threading.Thread(target=run, args=(ops[i::args.threads],)) for i in range(args.threads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
    rec["warm_set_s"] = round(time.perf_counter() - t0, 3)
    print(json.dumps(rec), flush=True)
    if args.json:
        with open(args.json, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
