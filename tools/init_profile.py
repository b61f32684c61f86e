"""Where does FedRuntime.initialize spend its time?  One single-client initialisation, stage times
(``init_times``: cumulative seconds at the end of each stage) and, with ``--cprofile``, the top functions.

    python tools/init_profile.py [--spec intrusion|wide] [--rows 40000] [--source synthetic|csv] [--reader auto]
                                 [--cprofile --top 30] [--cuda-first] [--json out.jsonl]

``--source synthetic``: the client generates its synthetic shard inside stage A (reported separately as
``generate_s``, measured by a second generation of the same shard before the timed run); ``--source csv``:
the shard is written to a CSV first (untimed) and the timed initialisation reads it -- the reference's path,
CSV read -> meta -> VGM fits -> encode (`Server/dtds/distributed.py:592-765`, `file_generator.py:59-231`).
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import tempfile
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="intrusion")
    ap.add_argument("--rows", type=int, default=40000)
    ap.add_argument("--source", default="synthetic", choices=["synthetic", "csv"])
    ap.add_argument("--reader", default="auto", help="FedConfig.table_reader for --source csv")
    ap.add_argument("--cprofile", action="store_true")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--cuda-first", action="store_true", help="initialise the HIP context before timing")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import torch
    from fed_tgan_amd.data.schema import get_spec
    from fed_tgan_amd.data.synthetic import generate
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.parallel.comm import Comm
    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    rec = {"spec": args.spec, "rows": args.rows, "source": args.source, "device": str(dev)}
    if args.cuda_first and dev.type == "cuda":
        t = time.time()
        torch.zeros(1, device=dev)
        torch.cuda.synchronize()
        rec["hip_context_s"] = round(time.time() - t, 3)
    spec = get_spec(args.spec)
    out = tempfile.mkdtemp()
    t = time.time()
    frame = generate(spec, args.rows, seed=0, as_category=True)
    rec["generate_s"] = round(time.time() - t, 3)
    datapath = None
    if args.source == "csv":
        datapath = os.path.join(out, "client0.csv")
        frame.to_csv(datapath, index=False)
        rec["csv_mb"] = round(os.path.getsize(datapath) / 1e6, 1)
        rec["reader"] = args.reader
    del frame
    cfg = FedConfig(spec=spec, epochs=1, synthetic_rows=args.rows, out_dir=out, seed=0, datapath=datapath,
                    backend="hip" if dev.type == "cuda" else "torch", verbose=False, table_reader=args.reader)
    rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
    pr = cProfile.Profile() if args.cprofile else None
    t = time.time()
    if pr:
        pr.enable()
    rt.initialize()
    if pr:
        pr.disable()
    rec["initialize_s"] = round(time.time() - t, 3)
    stages, prev = {}, 0.0
    for k, v in rt.init_times.items():           # cumulative -> per stage
        if k == "total":
            continue
        stages[k] = round(v - prev, 3)
        prev = v
    rec["stage_s"] = stages
    if args.source == "synthetic":
        rec["initialize_minus_generate_s"] = round(rec["initialize_s"] - rec["generate_s"], 3)
    print(json.dumps(rec), flush=True)
    if args.json:
        with open(args.json, "a") as f:
            f.write(json.dumps(rec) + "\n")
    if pr:
        for key in ("cumulative", "tottime"):
            s = io.StringIO()
            pstats.Stats(pr, stream=s).sort_stats(key).print_stats(args.top)
            print(s.getvalue())


if __name__ == "__main__":
    main()
