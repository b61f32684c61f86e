"""``python -m dtds.sample`` -- generate rows from a trained federated generator.

    python -m dtds.sample -model models/Intrusion_generator.pt -n 40000 -out Intrusion_synthetic.csv

The federator writes ``models/{name}_generator.pt`` after the last round (see
:mod:`fed_tgan_amd.models.generator_io`); the reference only had an unused ``save_model``
(`Server/dtds/distributed.py:560-563`).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    p = argparse.ArgumentParser(prog="python -m dtds.sample")
    p.add_argument("-model", required=True, help="models/{name}_generator.pt written by the federator")
    p.add_argument("-n", type=int, default=40000, help="rows to generate")
    p.add_argument("-out", default=None, help="CSV path (default {name}_synthetic.csv)")
    p.add_argument("-backend", default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("-seed", type=int, default=0)
    args = p.parse_args(argv)
    import torch
    from fed_tgan_amd.models.generator_io import load_generator
    dev = torch.device("cuda", 0) if (torch.cuda.is_available() and args.backend != "torch") else torch.device("cpu")
    gen = load_generator(args.model, dev, backend=args.backend, seed=args.seed)
    out = args.out or f"{gen.name}_synthetic.csv"
    t0 = time.time()
    gen.write_csv(out, args.n)
    print(f"{args.n} rows -> {out} ({time.time() - t0:.3f} s, {gen.engine.ops.name} on {dev})", flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
