"""Quick GPU timing probe of the engine: eager vs hipGraph step time, generation, decode."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))

from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig  # noqa: E402
from fed_tgan_amd.models.samplers import CondTables  # noqa: E402
from helpers import small_table  # noqa: E402


def timeit(fn, n, dev):
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="torch")
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--precision", default="bf16")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    _, _, _, _, _, _, tr, X = small_table(args.rows, 0)
    print("layout data_dim", tr.layout.data_dim, "n_opt", tr.layout.n_opt, flush=True)
    eng = CTGANEngine(tr.layout, EngineConfig(precision=args.precision), dev, backend=args.backend, seed=1)
    eng.set_training_data(X)
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    t_eager = timeit(lambda: eng.train_steps(1, use_graph=False), args.steps, dev)
    print(f"eager step: {t_eager * 1e3:.3f} ms", flush=True)
    eng.train_steps(1, use_graph=True)
    t_graph = timeit(lambda: eng.train_steps(1, use_graph=True), args.steps, dev)
    print(f"graph step: {t_graph * 1e3:.3f} ms  -> epoch(80) {t_graph * 80 * 1e3:.1f} ms", flush=True)
    t_gen = timeit(lambda: eng.generate_decoded(40000), 3, dev)
    print(f"generate+decode 40000: {t_gen * 1e3:.2f} ms", flush=True)
    out = eng.generate_decoded(40000)
    t_d2h = timeit(lambda: out.cpu(), 3, dev)
    print(f"D2H 40000x{out.shape[1]} f64: {t_d2h * 1e3:.2f} ms", flush=True)
    print("losses", eng.losses())


if __name__ == "__main__":
    main()
