"""Run a federation in the reference's launch topology -- rank 0 a dataless federator, ranks 1..K the clients
(`R/README.md:7-25`) -- as K+1 local processes, and report what each rank ended with.

    python tools/topology_probe.py [--world-size 2] [--epochs 5] [--colocated] [--out DIR] [--rows 4000]

The parent only starts the rank processes (it never touches the GPU).  Each rank runs
``fed_tgan_amd.cli.run_rank`` and, after the last round, writes its data plane, data-group size, round times
and final flat buffer; the parent prints one JSON line: ``data_backend`` / ``data_world_size`` per rank,
``flat_equal`` (every rank holds the same aggregate -- the federator received it), the steady-state round time.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _child(a):
    import torch
    from fed_tgan_amd.cli import build_parser, run_rank
    argv = ["-rank", str(a.rank), "-world_size", str(a.world_size), "-epochs", str(a.epochs), "-port", str(a.port),
            "-synthetic_rows", str(a.rows), "-n_sample", str(a.n_sample), "-out_dir", a.out, "-quiet"]
    if a.colocated:
        argv.append("-colocated")
    args = build_parser().parse_args(argv + a.extra)

    def done(rt, comm):
        info = {"rank": a.rank, "data_backend": comm.data_backend, "data_world_size": comm.data_world_size()
                if comm.is_client else 0, "round_s": list(rt.round_times), "is_client": comm.is_client}
        if rt.engine.flat.is_cuda:
            torch.cuda.synchronize(rt.engine.flat.device)
        torch.save(rt.engine.flat.detach().cpu(), os.path.join(a.scratch, f"flat{a.rank}.pt"))
        with open(os.path.join(a.scratch, f"info{a.rank}.json"), "w") as f:
            json.dump(info, f)
    run_rank(a.rank, args, on_done=done)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world-size", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--rows", type=int, default=4000)
    ap.add_argument("--n-sample", type=int, default=3000)
    ap.add_argument("--colocated", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--port", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--scratch", default=None, help=argparse.SUPPRESS)
    ap.add_argument("extra", nargs="*", help="more dtds.distributed flags (after --)")
    a = ap.parse_args()
    if a.rank >= 0:
        return _child(a)
    out = a.out or tempfile.mkdtemp(prefix="topology_")
    scratch = tempfile.mkdtemp(prefix="topology_ranks_")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.setdefault("GPU_MAX_HW_QUEUES", "2")      # ranks share the GPU (fed_tgan_amd/cli.py cap_shared_queues)
    cmd = [sys.executable, os.path.abspath(__file__), "--world-size", str(a.world_size), "--epochs", str(a.epochs),
           "--rows", str(a.rows), "--n-sample", str(a.n_sample), "--out", out, "--port", str(port),
           "--scratch", scratch] + (["--colocated"] if a.colocated else [])
    procs = [subprocess.Popen(cmd + ["--rank", str(r)] + (["--"] + a.extra if a.extra else []), env=env, cwd=ROOT)
             for r in range(a.world_size)]
    codes = [p.wait() for p in procs]
    if any(codes):
        raise SystemExit(f"rank exit codes {codes}")
    import torch
    flats = [torch.load(os.path.join(scratch, f"flat{r}.pt"), weights_only=True) for r in range(a.world_size)]
    infos = [json.load(open(os.path.join(scratch, f"info{r}.json"))) for r in range(a.world_size)]
    rounds = infos[-1]["round_s"]
    steady = rounds[1:] if len(rounds) > 1 else rounds
    print(json.dumps({"world_size": a.world_size, "colocated": a.colocated, "epochs": len(rounds),
                      "data_backend": [i["data_backend"] for i in infos],
                      "data_world_size": [i["data_world_size"] for i in infos],
                      "flat_equal": all(torch.equal(f, flats[0]) for f in flats[1:]),
                      "round_ms_steady": 1e3 * sum(steady) / max(len(steady), 1),
                      "round_ms": [round(1e3 * r, 2) for r in rounds]}), flush=True)


if __name__ == "__main__":
    main()
