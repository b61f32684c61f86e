"""Where does FedRuntime.initialize spend its time?  cProfile of one single-client initialisation
(Intrusion schema, 40k rows), top functions by cumulative time.

    python tools/init_profile.py [--rows 40000] [--top 30] [--cuda-first]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--cuda-first", action="store_true", help="initialise the HIP context before timing")
    args = ap.parse_args()
    import torch
    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.parallel.comm import Comm
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    if args.cuda_first and dev.type == "cuda":
        t = time.time()
        torch.zeros(1, device=dev)
        torch.cuda.synchronize()
        print(f"hip context: {time.time() - t:.3f}s", flush=True)
    out = tempfile.mkdtemp()
    cfg = FedConfig(spec=intrusion_spec(), epochs=1, synthetic_rows=args.rows, out_dir=out, seed=0,
                    backend="hip" if dev.type == "cuda" else "torch", verbose=False)
    rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
    pr = cProfile.Profile()
    t = time.time()
    pr.enable()
    rt.initialize()
    pr.disable()
    print(f"initialize: {time.time() - t:.3f}s  stages {rt.init_times}", flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(args.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(args.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
