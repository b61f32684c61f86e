"""Execute the RCCL (``nccl``) branches of :class:`fed_tgan_amd.parallel.comm.Comm` on one GPU.

A single-GPU box cannot host two RCCL ranks, but a ONE-rank RCCL communicator still runs the real
collective kernels.  ``force_dist=True`` builds the gloo control plane and the RCCL data plane for
world size 1, so the aggregation (`Server/dtds/distributed.py:86-106` -> weighted all-reduce), the
sharded-sample gather and the MD-GAN point-to-point exchange take their nccl code paths instead of
the world-size-1 short-circuits.  Prints one JSON line with the checks; exit code 0 = all passed.

    python tools/rccl_selftest.py            (NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=COLL shows the ops)
"""
from __future__ import annotations

import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def hier_check(comm, dev, g) -> dict:
    """``-world_size N -local_clients K`` on this box (N = 1, K = 2): two client threads, one HIP stream
    each, combine on the GPU and thread 0 runs the process-level RCCL all-reduce / gather (HierComm)."""
    import threading

    import torch

    from fed_tgan_amd.fed.local import HierComm, LocalGroup
    group = LocalGroup(2)
    bufs = [torch.randn(1_000_003, generator=g).to(dev) for _ in range(2)]
    ws = [0.25, 0.75]
    want = torch.zeros_like(bufs[0])
    for b, w in zip(bufs, ws):
        want.add_(b, alpha=w)
    got, errors = [None, None], []

    def worker(t):
        try:
            torch.cuda.set_device(dev)
            with torch.cuda.stream(torch.cuda.Stream(dev)):
                hc = HierComm(group, t, dev, comm)
                f = bufs[t].clone()
                hc.weighted_all_reduce(f, ws[t])
                rows = torch.full((100 + t, 42), float(t + 1), device=dev)
                out = hc.gather_rows(rows, [100, 101], [0, 1], dst=0, to_host=False)
                torch.cuda.current_stream(dev).synchronize()
                got[t] = (f, out)
        except BaseException as e:   # surfaced in the result
            errors.append(repr(e))
            group.failed.set()
            group.barrier.abort()
    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        return {"hier_allreduce_ok": False, "hier_gather_ok": False, "hier_error": errors[0]}
    ar = all(torch.equal(f, want) for f, _ in got)
    out0, out1 = got[0][1], got[1][1]
    ga = out1 is None and out0 is not None and tuple(out0.shape) == (201, 42) and \
        bool((out0[:100] == 1).all()) and bool((out0[100:] == 2).all())
    return {"hier_allreduce_ok": bool(ar), "hier_gather_ok": bool(ga)}


def main() -> int:
    import torch
    import torch.distributed as dist

    from fed_tgan_amd.parallel.comm import Comm

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm(0, 1, [0], "nccl", "127.0.0.1", _port(), timeout_s=60, device=dev, force_dist=True)
    res = {"data_backend": dist.get_backend(comm.data), "data_ranks": comm.data_world_size()}
    g = torch.Generator(device="cpu").manual_seed(0)
    # weighted FedAvg: flat <- w * flat summed over the (one) client
    flat = torch.randn(2_130_000, generator=g).to(dev)
    want = flat * 0.375
    comm.weighted_all_reduce(flat, 0.375)
    torch.cuda.synchronize()
    res["allreduce_ok"] = bool(torch.equal(flat, want))
    # sharded generation gather (padded rows, rank order)
    rows = torch.randn(1234, 42, generator=g).to(dev)
    out = comm.gather_rows(rows, [1234], [0], dst=0, to_host=False)
    res["gather_ok"] = bool(out.device.type == "cuda" and torch.equal(out, rows))
    # MD-GAN batched point-to-point over the RCCL p2p group (send to / receive from self)
    comm.init_p2p()
    src = torch.randn(500, 128, generator=g).to(dev)
    dst = torch.empty_like(src)
    comm.exchange(sends=[(src, 0)], recvs=[(dst, 0)])
    torch.cuda.synchronize()
    res["exchange_ok"] = bool(torch.equal(src, dst))
    res.update(hier_check(comm, dev, g))
    comm.destroy()
    ok = res["data_backend"] == "nccl" and res["allreduce_ok"] and res["gather_ok"] and res["exchange_ok"] and \
        res["hier_allreduce_ok"] and res["hier_gather_ok"]
    res["ok"] = bool(ok)
    print(json.dumps(res), flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
