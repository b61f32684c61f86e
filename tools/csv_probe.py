"""Native CSV writer on the box: wall time of consecutive 40,000-row writes (first vs later) and how far a
Python thread spinning next to a background write gets (GIL / CPU starvation check).

    python tools/csv_probe.py --threads 0 --rows 40000
"""
import argparse
import json
import os
import tempfile
import threading
import time

import numpy as np

sys_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
import sys  # noqa: E402
sys.path.insert(0, sys_path)

from fed_tgan_amd.data.decode import KIND_FLOAT, KIND_VOCAB, CsvLayout
from fed_tgan_amd.utils import csvio


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--warm-rows", type=int, default=0, help="a devnull write of this many rows first")
    args = ap.parse_args()
    names = [f"c{i}" for i in range(42)]
    kinds = [KIND_VOCAB if i % 3 == 0 else KIND_FLOAT for i in range(42)]
    vocabs = [[f"v{j}" for j in range(20)] if k == KIND_VOCAB else [] for k in kinds]
    lay = CsvLayout(names=names, kinds=kinds, vocabs=vocabs, src=list(range(42)))
    rng = np.random.default_rng(0)
    v = rng.random((args.rows, 42)) * 100
    v[:, ::3] = np.floor(rng.random((args.rows, 14)) * 20)
    out = tempfile.mkdtemp()
    from fed_tgan_amd.ops import native
    native.require()                  # (the library load is not the writer's cost)
    rec = {"threads": args.threads, "rows": args.rows, "cpus": len(os.sched_getaffinity(0))}
    if args.warm_rows:
        t = time.perf_counter()
        csvio.write_layout(os.devnull, v[:args.warm_rows], lay, threads=args.threads)
        rec["warm_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    rec["write_ms"] = []
    for i in range(4):
        t = time.perf_counter()
        csvio.write_layout(os.path.join(out, f"t{i}.csv"), v, lay, threads=args.threads)
        rec["write_ms"].append(round((time.perf_counter() - t) * 1e3, 2))

    def spin(dur):
        n, t = 0, time.perf_counter()
        while time.perf_counter() - t < dur:
            n += 1
        return n
    alone = spin(0.05)
    th = threading.Thread(target=lambda: csvio.write_layout(os.path.join(out, "bg.csv"), v, lay, threads=args.threads))
    th.start()
    beside = spin(0.05)
    th.join()
    rec["spin_ratio_beside_write"] = round(beside / max(alone, 1), 3)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
