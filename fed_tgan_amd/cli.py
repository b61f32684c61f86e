"""Command-line entry point, flag-compatible with the reference ``python -m dtds.distributed``.

Reference flags (`Server/dtds/distributed.py:895-934`, `R/README.md:10-23`) keep their meaning:

    -rank R            this process' rank; 0 = federator, 1..K = clients (world_size = K + 1)
    -ip / -port        rendezvous address of the federator (default 127.0.0.1:7788)
    -world_size W      clients + 1
    -epochs / -epoch   federated rounds
    -datapath P        each client's local CSV ('{client}' / '{rank}' are substituted);
                       a missing file means "generate a synthetic shard of the dataset schema"
    -name -E_interval -report -problem_type -target_column -selected_variables
    -categorical_list -nonnegative_list -date_dic
    (list flags take comma-separated values; -date_dic takes JSON)

Without ``-rank`` the whole federation is launched locally (the reference's intended but broken
``mp.spawn`` path, `Server/dtds/distributed.py:956-971`): one federator + (world_size-1) clients,
or with ``-colocated`` one process per client where rank 0 is also the federator (the MI355X
layout: one process per GPU, RCCL data plane).

New flags: -config (dataset spec JSON or builtin name), -backend {auto,hip,torch},
-precision {bf16,fp32}, -data_backend {auto,gloo,nccl}, -synthetic_rows, -shard
{independent,iid,dirichlet,skew}, -alpha, -n_sample, -aggregation {weighted,uniform}, -gmm
{torch,sklearn}, -seed, -out_dir, -ckpt_every, -resume, -local_clients K (K clients per process,
as threads sharing its GPU; with -world_size N: N*K clients over N ranks), -drop_client_prob (fault
injection), -metrics_log, -mode {fedavg,mdgan},
-init {independent,broadcast} (initial weights; independent = the reference's per-client init).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
from typing import List, Optional

import torch

from .data.schema import DatasetSpec, get_spec


def _csv_list(s: str) -> List[str]:
    return [x.strip() for x in s.split(",") if x.strip()]


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m dtds.distributed", allow_abbrev=True,
                                description="Federated CTGAN (Fed-TGAN) on MI355X")
    p.add_argument("-rank", type=int, default=None)
    p.add_argument("-ip", type=str, default="127.0.0.1")
    p.add_argument("-port", type=int, default=7788)
    p.add_argument("-name", type=str, default=None)
    p.add_argument("-datapath", type=str, default="data/raw/Intrusion_train.csv")
    p.add_argument("-epochs", type=int, default=10)
    p.add_argument("-E_interval", type=int, default=1)
    p.add_argument("-world_size", type=int, default=None, help="processes (default 2; 1 with -local_clients)")
    p.add_argument("-report", action="store_true")
    p.add_argument("-problem_type", type=str, default=None)
    p.add_argument("-target_column", type=str, default=None)
    p.add_argument("-selected_variables", type=_csv_list, default=None)
    p.add_argument("-categorical_list", type=_csv_list, default=None)
    p.add_argument("-nonnegative_list", type=_csv_list, default=None)
    p.add_argument("-date_dic", type=json.loads, default=None)
    # new
    p.add_argument("-config", type=str, default="intrusion")
    p.add_argument("-colocated", action="store_true")
    p.add_argument("-backend", type=str, default="auto", choices=["auto", "hip", "torch"])
    p.add_argument("-precision", type=str, default="bf16", choices=["bf16", "fp32"])
    p.add_argument("-data_backend", type=str, default="auto", choices=["auto", "gloo", "nccl"])
    p.add_argument("-synthetic_rows", type=int, default=40000)
    p.add_argument("-shard", type=str, default="independent", choices=["independent", "iid", "dirichlet", "skew"])
    p.add_argument("-alpha", type=float, default=0.5)
    p.add_argument("-n_sample", type=int, default=None)
    p.add_argument("-aggregation", type=str, default="weighted", choices=["weighted", "uniform"])
    p.add_argument("-gmm", type=str, default="torch", choices=["torch", "sklearn"])
    p.add_argument("-gmm_pool_cap", type=int, default=0)
    p.add_argument("-seed", type=int, default=0)
    p.add_argument("-out_dir", type=str, default=".")
    p.add_argument("-ckpt_every", type=int, default=0)
    p.add_argument("-resume", action="store_true")
    p.add_argument("-local_clients", type=int, default=0)
    p.add_argument("-drop_client_prob", type=float, default=0.0)
    p.add_argument("-metrics_log", type=str, default=None)
    p.add_argument("-mode", type=str, default="fedavg", choices=["fedavg", "mdgan"])
    p.add_argument("-batch_size", type=int, default=500)
    p.add_argument("-timeout", type=float, default=600.0)
    p.add_argument("-dump_real", action="store_true", help="write the synthetic client shards under out_dir/data/raw")
    p.add_argument("-heartbeat", type=float, default=0.0,
                   help="per-round monitored barrier: fail fast (naming the dead ranks) after this many seconds")
    p.add_argument("-profile_dir", default=None, help="export a torch.profiler Chrome trace of round 1 here")
    p.add_argument("-grad_flow", action="store_true", help="write reports/grad_flow.{csv,png} (client 0)")
    p.add_argument("-sync_csv", action="store_true",
                   help="write each epoch CSV inside its round (reference timing) instead of in the background")
    p.add_argument("-init", type=str, default="independent", choices=["independent", "broadcast"],
                   help="initial G/D weights: each client its own random init (reference) or client 0's on every rank")
    p.add_argument("-batched_clients", default="auto", choices=["auto", "on", "off"],
                   help="-local_clients K: the K clients as one batched launch sequence (on) or one engine and HIP "
                        "stream per client thread (off; what auto picks, see FedConfig.batched_clients)")
    p.add_argument("-native_rccl", action="store_true",
                   help="the weight all-reduce through the native RCCL plane (csrc/comm; the default, kept for "
                        "compatibility)")
    p.add_argument("-torch_rccl", action="store_true",
                   help="the weight all-reduce through torch.distributed's RCCL ProcessGroup instead of the native plane")
    p.add_argument("-pipeline_sample", default="auto", choices=["auto", "on", "off"],
                   help="generate round r's table on a side stream after a model snapshot (FedConfig.pipeline_sample)")
    p.add_argument("-table_reader", default="auto", choices=["auto", "pandas", "arrow"],
                   help="client CSV reader (pyarrow from 32 MiB up with auto)")
    p.add_argument("-quiet", action="store_true")
    return p


def spec_from_args(args) -> DatasetSpec:
    spec = get_spec(args.config)
    if args.name:
        spec.name = args.name.replace("_train", "") if args.name.endswith("_train") else args.name
    for flag, field in (("selected_variables", "selected_variables"), ("categorical_list", "categorical_list"),
                        ("nonnegative_list", "nonnegative_list"), ("date_dic", "date_dic"),
                        ("target_column", "target_column"), ("problem_type", "problem_type")):
        v = getattr(args, flag)
        if v is not None:
            setattr(spec, field, v)
    if args.n_sample:
        spec.n_sample = args.n_sample
    return spec


def fed_config_from_args(args):
    from .fed.runtime import FedConfig
    from .models.engine import EngineConfig
    return FedConfig(spec=spec_from_args(args), epochs=args.epochs, datapath=args.datapath,
                     synthetic_rows=args.synthetic_rows, shard_mode=args.shard, dirichlet_alpha=args.alpha,
                     out_dir=args.out_dir, n_sample=args.n_sample, aggregation=args.aggregation,
                     gmm_backend=args.gmm, gmm_pool_cap=args.gmm_pool_cap, backend=args.backend, seed=args.seed,
                     engine=EngineConfig(batch_size=args.batch_size, precision=args.precision),
                     ckpt_every=args.ckpt_every, resume=args.resume, verbose=not args.quiet,
                     metrics_log=args.metrics_log, drop_client_prob=args.drop_client_prob, mode=args.mode,
                     e_interval=args.E_interval, grad_flow=args.grad_flow, profile_dir=args.profile_dir,
                     heartbeat_s=args.heartbeat,
                     dump_real=args.dump_real, async_csv=not args.sync_csv, init=args.init,
                     batched_clients=args.batched_clients, table_reader=args.table_reader,
                     pipeline_sample={"auto": None, "on": True, "off": False}[args.pipeline_sample])


def pick_device(rank: int, colocated: bool, backend: str, mode: str = "fedavg") -> torch.device:
    if backend == "torch" or not torch.cuda.is_available():
        return torch.device("cpu")
    n = torch.cuda.device_count()
    # dedicated federator: it shares GPU 0 with client 1, except in MD-GAN mode where it runs the
    # generator for every client and gets a GPU of its own (RCCL needs one rank per device)
    idx = device_index(int(os.environ.get("LOCAL_RANK", rank)), n, colocated, mode)
    torch.cuda.set_device(idx)
    return torch.device("cuda", idx)


def device_index(local: int, ngpu: int, colocated: bool, mode: str = "fedavg") -> int:
    """The GPU of the rank with node-local index ``local`` (see pick_device): one per rank when
    co-located (or MD-GAN), else the dedicated federator shares GPU 0 with client 1."""
    return local % ngpu if (colocated or mode == "mdgan") else max(local - 1, 0) % ngpu


def gpus_shared(world: int, colocated: bool, mode: str = "fedavg") -> bool:
    """Will several ranks of this node run on one GPU (a dedicated federator next to client 1, or
    more clients than GPUs)?"""
    from .utils.gpus import visible_gpu_count
    ngpu = visible_gpu_count()      # (no HIP here: a launcher parent must not hold a GPU context)
    if not ngpu:
        return False
    idx = [device_index(r, ngpu, colocated, mode) for r in range(world)]
    return len(set(idx)) < len(idx)


# Ranks sharing a GPU run with at most 2 HIP hardware queues each.  With HIP's default of 4 per
# process, three processes oversubscribe the GPU's hardware queue slots and are time-sliced:
# measured on one MI355X (world_size 3, dedicated federator) 69.9 ms per round with 4 queues against
# 26.3 ms with 1 or 2 (`tools/gpu_recipes/topologies_queues.sh`).  HIP reads the variable when the
# library loads, so the launcher sets it for its children; ranks started by hand need it in their
# environment (run_rank prints a hint).
SHARED_GPU_QUEUES = "2"


def cap_shared_queues() -> None:
    """Lower GPU_MAX_HW_QUEUES to FEDTGAN_SHARED_HW_QUEUES (default 2) for ranks that share a GPU; a
    lower value already in the environment is kept (boxes often export HIP's default, 4)."""
    target = int(os.environ.get("FEDTGAN_SHARED_HW_QUEUES", SHARED_GPU_QUEUES))
    cur = os.environ.get("GPU_MAX_HW_QUEUES")
    try:
        keep = cur is not None and int(cur) <= target
    except ValueError:
        keep = False
    if not keep:
        os.environ["GPU_MAX_HW_QUEUES"] = str(target)


def run_rank(rank: int, args, on_done=None) -> None:
    """One process of the federation (the reference ``run()``, `Server/dtds/distributed.py:838-891`).
    ``on_done(runtime, comm)`` (probes, tests) runs after the last round, before the process groups close."""
    from .fed.runtime import FedRuntime
    from .fed.mdgan import MDGANRuntime
    from .parallel.comm import Comm
    world = args.world_size
    colocated = args.colocated
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) > int(SHARED_GPU_QUEUES) and args.backend != "torch" \
            and gpus_shared(world, colocated, args.mode):
        print(f"[rank {rank}] several ranks share a GPU: export GPU_MAX_HW_QUEUES={SHARED_GPU_QUEUES} before "
              "starting each rank (HIP's default 4 queues per process get time-sliced)", flush=True)
    device = pick_device(rank, colocated, args.backend, args.mode)
    if not args.quiet:
        print(f"[rank {rank}] device {device}, GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')}",
              flush=True)
    if device.type == "cpu":   # several ranks on one host: do not oversubscribe the cores
        torch.set_num_threads(max(1, (os.cpu_count() or 4) // max(world * max(args.local_clients, 1), 1)))
    client_ranks = list(range(world)) if colocated else list(range(1, world))
    data_backend = args.data_backend
    if data_backend == "auto":
        # agreed by every rank over the gloo control plane (Comm._vote_data_backend): RCCL among the client
        # ranks (MD-GAN: among all ranks) when each of them has a GPU of its own, gloo everywhere otherwise.  A
        # dedicated federator stays outside the RCCL group and receives the aggregate from the first client
        # (Comm.share_with_federator)
        data_backend = "auto_all" if args.mode == "mdgan" else "auto"
    comm = Comm(rank, world, client_ranks, data_backend, args.ip, args.port, timeout_s=args.timeout, device=device,
                native_rccl=False if args.torch_rccl else (True if args.native_rccl else None))
    if not args.quiet:
        print(f"[rank {rank}] data plane {comm.data_backend} over client ranks {client_ranks}", flush=True)
    try:
        if args.local_clients:      # K clients as threads of this rank: clients rank*K .. rank*K+K-1
            from .fed.local import run_local_emulation
            run_local_emulation(fed_config_from_args(args), args.local_clients, backend=args.backend, device=device,
                                outer=comm)
            comm.barrier()
            return
        cls = MDGANRuntime if args.mode == "mdgan" else FedRuntime
        rt = cls(fed_config_from_args(args), comm, device, federator=0)
        rt.initialize()
        rt.fit()
        if on_done is not None:
            on_done(rt, comm)
        comm.barrier()
        rt.close()          # writers joined, graphs released, communicators destroyed (before interpreter exit)
    finally:
        comm.destroy()


def _spawn_entry(rank: int, args) -> None:
    run_rank(rank, args)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(argv: Optional[List[str]] = None) -> None:
    args = build_parser().parse_args(argv)
    if args.world_size is None:
        args.world_size = 1 if args.local_clients else 2
    if args.local_clients:
        if args.mode == "mdgan":
            raise SystemExit("-local_clients: the MD-GAN split mode runs one client per process")
        if args.rank is None and args.world_size <= 1:
            from .fed.local import run_local_emulation
            run_local_emulation(fed_config_from_args(args), args.local_clients, backend=args.backend)
            return
        # N processes x K clients each: every process runs clients, rank 0 hosts the federator
        args.colocated = True
    if args.rank is not None:
        run_rank(args.rank, args)
        return
    # no rank given: launch the whole federation on this node
    if args.world_size <= 1 or (args.world_size == 1 and not args.colocated):
        args.colocated = True
    if args.port == 7788:
        args.port = free_port()
    shared = args.backend != "torch" and gpus_shared(args.world_size, args.colocated, args.mode)
    if shared:
        cap_shared_queues()       # inherited by the spawned ranks
    if not args.quiet:
        print(f"[launch] {args.world_size} ranks, GPUs shared: {shared}", flush=True)
    import torch.multiprocessing as mp
    mp.spawn(_spawn_entry, args=(args,), nprocs=args.world_size, join=True)


if __name__ == "__main__":
    main(sys.argv[1:])
