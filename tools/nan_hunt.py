"""Find the first engine op that produces a non-finite value (eager, op-by-op checks)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


class Checked:
    def __init__(self, ops, eng):
        self._ops = ops
        self._eng = eng
        self.calls = 0

    def __getattr__(self, name):
        f = getattr(self._ops, name)
        if not callable(f) or name.startswith("_"):
            return f

        def wrapped(*args, **kw):
            out = f(*args, **kw)
            torch.cuda.synchronize()
            self.calls += 1
            for i, a in enumerate(list(args) + list(kw.values())):
                if isinstance(a, torch.Tensor) and a.is_floating_point() and not bool(torch.isfinite(a).all()):
                    raise RuntimeError(f"non-finite after call #{self.calls} {name} (arg {i}, shape {tuple(a.shape)})")
            return out
        return wrapped


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=800)
    ap.add_argument("--precision", default="bf16")
    args = ap.parse_args()
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from helpers import small_table
    dev = torch.device("cuda:0")
    _, _, _, _, _, _, tr, X = small_table(40000, 0)
    eng = CTGANEngine(tr.layout, EngineConfig(precision=args.precision), dev, backend="hip", seed=1)
    eng.set_training_data(X)
    eng.ops = Checked(eng.ops, eng)
    for s in range(args.steps):
        try:
            eng._one_step()
        except RuntimeError as e:
            print(f"step {s}: {e}")
            m = eng.metrics.cpu().tolist()
            print("metrics", m, "gbuf max", eng.gbuf.abs().max().item(), "flat finite", bool(torch.isfinite(eng.flat).all()))
            for n, t in eng.p.items():
                if not bool(torch.isfinite(t).all()):
                    print("  non-finite param", n)
            return
        if s % 100 == 0:
            print("step", s, "losses", eng.losses(), flush=True)
    print("no non-finite values in", args.steps, "steps")


if __name__ == "__main__":
    main()
