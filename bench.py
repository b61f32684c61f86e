"""Headline benchmark: sec/epoch (+ Avg_JSD / Avg_WD) of federated CTGAN on Intrusion.

Metric (BASELINE.json): one full federated round — every client trains one local epoch
(rows // 500 WGAN-GP steps), weighted aggregation, sampling + decoding the 40,000-row
synthetic table and writing its CSV — exactly the span the reference times into
``timestamp_experiment.csv`` (`Server/dtds/distributed.py:795-825`).

Config: the Intrusion (KDD-99) 42-column schema; every client holds its own 40,000-row
synthetic shard (weak scaling: per-GPU work fixed as N grows); random-init weights;
batch 500, embedding 128, G/D (256, 256), pack 10.  One rank per GPU; the data plane is
RCCL (``nccl``) for N > 1.

    python bench.py --gpus N --steps K --warmup W
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Without ``WORLD_SIZE`` in the environment and ``--gpus N > 1`` the script is its own launcher
(the reference's intended one-command single-node fan-out, `Server/dtds/distributed.py:956-971`):
the parent starts N fresh rank processes before anything touches the GPU, waits for them and
exits with the first failing rank's code; rank 0 prints the JSON line.

"steps" are federated rounds (epochs).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_SEC_PER_EPOCH = 24.2   # README.md:53-54 (2 clients, epoch 1); BASELINE.md


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed federated rounds")
    ap.add_argument("--warmup", type=int, default=2, help="untimed rounds")
    ap.add_argument("--rows", type=int, default=40000, help="rows per client")
    ap.add_argument("--n-sample", type=int, default=40000)
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--gmm", default="torch")
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--sync-csv", action="store_true", help="write each epoch CSV inside its round")
    ap.add_argument("--device-reset-at-exit", action="store_true",
                    help="tear the HIP device down (hipDeviceReset) before interpreter exit: a run under rocprofv3 "
                         "otherwise segfaults in libamdhip64's exit-time destructor (profiles/exit_r6.txt)")
    ap.add_argument("--check", action=argparse.BooleanOptionalAction, default=None,
                    help="after the timed rounds: assert every rank holds a bit-identical aggregate and the "
                         "last epoch CSV has n_sample rows (reported as 'consistency'); default on for N > 1")
    ap.add_argument("--engine", action="append", default=[], metavar="KEY=VALUE",
                    help="EngineConfig override for A/B measurements, e.g. --engine onehot=0")
    ap.add_argument("--fed", action="append", default=[], metavar="KEY=VALUE",
                    help="FedConfig override for A/B measurements, e.g. --fed csv_threads=8")
    ap.add_argument("--tuning", action="append", default=[], metavar="KEY=VALUE",
                    help="native set_tuning knob for A/B measurements, e.g. --tuning gemm_xcd_remap=0")
    ap.add_argument("--phase-timer", default="events", choices=["events", "sync"],
                    help="phase timers: HIP events (no host sync) or stream-synchronised wall time")
    ap.add_argument("--native-rccl", action="store_true",
                    help="the weight all-reduce through the native RCCL plane (csrc/comm; the default)")
    ap.add_argument("--torch-rccl", action="store_true",
                    help="the weight all-reduce through torch.distributed's RCCL ProcessGroup instead")
    ap.add_argument("--force-dist", action="store_true",
                    help="build real process groups even for one rank (1 GPU: the aggregation runs as an "
                         "RCCL all-reduce on a one-rank communicator)")
    return ap


# ----------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _visible_gpus() -> int:
    # from the kernel driver's topology, without loading HIP: the parent stays alive for the whole
    # run and must not hold a GPU context (or queues) of its own
    from fed_tgan_amd.utils.gpus import visible_gpu_count
    return visible_gpu_count()


def launch(n: int, argv) -> int:
    """Start N rank processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set), wait, return the exit code."""
    ngpu = _visible_gpus()
    if ngpu > 0 and n > ngpu:
        print(f"bench.py: --gpus {n} but only {ngpu} GPU(s) are visible", file=sys.stderr, flush=True)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if ngpu == 0:   # CPU ranks share the host: do not oversubscribe the cores
            env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 8) // n)))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      start_new_session=True))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in live:     # one rank died: the others would block in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


# ----------------------------------------------------------------------------- transport record
def _rccl_log_setup() -> str | None:
    """Ask RCCL for its init / connection log in side files (one per rank): the channel lines name the
    transport every ring / tree link uses (P2P/IPC over xGMI, SHM, NET).  Logged at communicator setup
    only (the warm-up collectives), never per call.  A user-set NCCL_DEBUG_FILE is left alone (no record);
    a quieter NCCL_DEBUG level (e.g. WARN from the environment) is raised to INFO for the side file."""
    if os.environ.get("NCCL_DEBUG_FILE"):
        return None
    d = os.path.join(tempfile.gettempdir(), f"fedtgan_rccl_{os.environ.get('MASTER_PORT', '0')}")
    os.makedirs(d, exist_ok=True)
    if os.environ.get("NCCL_DEBUG", "").upper() not in ("INFO", "TRACE"):
        os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,P2P,SHM,NET")
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "rccl.%h.%p.log")
    return d


def _rccl_transport(d: str | None) -> dict:
    """Transport counts over every rank's connection lines ('... via P2P/IPC ...') + the version line."""
    import glob
    import re
    out = {"links": {}, "files": 0, "nccl_debug": os.environ.get("NCCL_DEBUG")}
    if not d:
        return out
    pat = re.compile(r"\bvia (\S+)")
    for f in glob.glob(os.path.join(d, "rccl.*.log")):
        out["files"] += 1
        with open(f, errors="replace") as fh:
            for line in fh:
                m = pat.search(line)
                if m and ("->" in line or "Channel" in line):
                    k = m.group(1).rstrip(",")
                    out["links"][k] = out["links"].get(k, 0) + 1
                if "version" not in out and ("RCCL version" in line or "NCCL version" in line):
                    out["version"] = line.split("INFO", 1)[-1].strip()
    return out


# ----------------------------------------------------------------------------- one rank
def run_rank(args) -> None:
    import torch

    from fed_tgan_amd.data.schema import intrusion_spec
    from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
    from fed_tgan_amd.parallel.comm import Comm

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
        if world > 1:
            torch.set_num_threads(max(1, (os.cpu_count() or 8) // world))
    if args.force_dist and world == 1:
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    rccl_dir = _rccl_log_setup() if (device.type == "cuda" and (world > 1 or args.force_dist)) else None
    if args.native_rccl:
        os.environ["FEDTGAN_NATIVE_RCCL"] = "1"
    if args.torch_rccl:
        os.environ["FEDTGAN_NATIVE_RCCL"] = "0"
    comm = Comm.from_env("auto", device, force_dist=args.force_dist)
    n_data = comm.data_world_size()
    if n_data != world:
        raise SystemExit(f"bench.py: data plane has {n_data} ranks, expected {world}")
    out = args.out or os.path.join(tempfile.gettempdir(), f"fedtgan_bench_{os.getpid()}_{rank}")
    if world > 1:
        out = comm.broadcast_object(out, src=0)
    os.makedirs(out, exist_ok=True)
    spec = intrusion_spec()
    from fed_tgan_amd.models.engine import EngineConfig
    ecfg = EngineConfig()
    for kv in args.engine:
        k, v = kv.split("=", 1)
        cur = getattr(ecfg, k)
        setattr(ecfg, k, (v.lower() in ("1", "true", "yes")) if isinstance(cur, bool) else type(cur)(v))
    cfg = FedConfig(spec=spec, epochs=args.warmup + args.steps, synthetic_rows=args.rows, out_dir=out,
                    n_sample=args.n_sample, backend=args.backend, gmm_backend=args.gmm, seed=0,
                    verbose=not args.quiet, async_csv=not args.sync_csv, engine=ecfg, phase_timer=args.phase_timer)
    for kv in args.fed:
        k, v = kv.split("=", 1)
        cur = getattr(cfg, k)
        if isinstance(cur, bool) or (cur is None and v.lower() in ("0", "1", "true", "false", "yes", "no")):
            setattr(cfg, k, v.lower() in ("1", "true", "yes"))
        else:
            setattr(cfg, k, v if cur is None else type(cur)(v))
    if args.tuning:
        from fed_tgan_amd.ops import native
        for kv in args.tuning:
            k, v = kv.split("=", 1)
            native.require().set_tuning(k, int(v))
    rt = FedRuntime(cfg, comm, device)
    rt.initialize()
    for ep in range(args.warmup):
        rt.run_round(ep)
    rt.flush_writes()
    rt.timer.reset()                 # phase breakdown over the timed rounds only
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for ep in range(args.warmup, args.warmup + args.steps):
        rt.round_times.append(rt.run_round(ep))
    rt.flush_writes()       # every timed round's CSV is on disk inside the timed region
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = comm.max_float(elapsed)
    sec_per_epoch = elapsed / max(args.steps, 1)
    last = os.path.join(out, f"{spec.name}_result", f"{spec.name}_synthesis_epoch_{cfg.epochs - 1}.csv")

    rt.timer.resolve(block=True)
    check = args.check if args.check is not None else world > 1
    consistency = None
    if check:
        digest = hashlib.sha256(rt.engine.flat.detach().cpu().numpy().tobytes()).hexdigest()
        digests = comm.all_gather_object(digest)
        consistency = {"flat_identical": len(set(digests)) == 1, "ranks": len(digests)}
        if rank == 0:
            with open(last) as f:
                consistency["csv_rows"] = sum(1 for _ in f) - 1
        if not consistency["flat_identical"]:
            raise SystemExit(f"bench.py: ranks disagree on the aggregate: {digests}")

    avg_jsd = avg_wd = None
    if rank == 0 and not args.no_eval:
        from fed_tgan_amd.data.synthetic import generate
        from fed_tgan_amd.eval.similarity import stat_sim
        import pandas as pd
        if os.path.exists(last):
            real = pd.concat([generate(spec, args.rows, seed=i) for i in range(max(world, 1))])
            avg_jsd, avg_wd = stat_sim(real, pd.read_csv(last), spec.categorical_list)
    if rank == 0:
        rec = {
            "metric": "sec_per_epoch", "value": round(sec_per_epoch, 6), "unit": "s/epoch", "n_gpus": n_data,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(sec_per_epoch * 1000.0, 3),
            "higher_is_better": False, "scaling": "weak",
            "vs_baseline": round(sec_per_epoch / BASELINE_SEC_PER_EPOCH, 6),
            "dtype": cfg.engine.precision if rt.engine.ops.name == "hip" else "fp32",
            "data": f"synthetic (Intrusion schema, {args.rows} rows per client; random-init weights)",
            "config": {"model": "Fed-TGAN CTGAN (G 256x256 residual+BN, D 256x256 pack10, WGAN-GP slerp)",
                       "global_batch": 500 * world, "seq_len": None, "parallelism": f"fed{world}",
                       "rows_per_client": args.rows, "n_sample": args.n_sample,
                       "steps_per_epoch": args.rows // 500, "backend": rt.engine.ops.name,
                       "data_plane": comm.data_backend if comm.dist_active else "none"},
            "avg_jsd": avg_jsd, "avg_wd": avg_wd, "epochs_trained": cfg.epochs,
            "phase_s": {k: round(v / max(args.steps, 1), 6) for k, v in rt.timer.totals.items()},
            "init_s": {k: round(v, 3) for k, v in rt.init_times.items()},    # cumulative, untimed
        }
        if consistency is not None:
            rec["consistency"] = consistency
        if comm.dist_active:
            import torch.distributed as dist
            ver = None
            if device.type == "cuda":
                try:
                    ver = ".".join(str(x) for x in torch.cuda.nccl.version())
                except Exception:   # pragma: no cover - build without RCCL
                    ver = None
            rec["comm"] = {"data_world_size": dist.get_world_size(comm.data), "data_backend": comm.data_backend,
                           "all_reduce_plane": "native" if getattr(comm, "_native", None) is not None else "torch",
                           "rccl_version": ver, "transport": _rccl_transport(rccl_dir)}
        if args.engine:
            rec["engine_overrides"] = args.engine
        if args.tuning:
            rec["tuning"] = args.tuning
        print(json.dumps(rec), flush=True)
    rt.close()           # writers joined, graphs released, communicators destroyed -- before interpreter exit
    if args.device_reset_at_exit and device.type == "cuda":
        from fed_tgan_amd.ops import native
        native.require().device_reset()
    maps = os.environ.get("FEDTGAN_DUMP_MAPS")
    if maps:             # (diagnostics: the loaded libraries' address ranges, to symbolise a crash in exit())
        with open("/proc/self/maps") as src, open(f"{maps}.{rank}", "w") as dst:
            dst.write(src.read())


def main():
    argv = sys.argv[1:]
    args = build_parser().parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch(args.gpus, argv))
    run_rank(args)


if __name__ == "__main__":
    main()
