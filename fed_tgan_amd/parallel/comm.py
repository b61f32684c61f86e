"""Process groups for the federation: a gloo control plane and an RCCL data plane.

The reference moves everything — meta dicts, sklearn objects, whole ``nn.Module``s and
8.5 MB of state_dicts per client per round — as pickled PyTorch-RPC messages over the
Gloo/TCP ``PROCESS_GROUP`` agent (`Server/dtds/distributed.py:838-891`, survey §2-E
M1-M12), serialising the push-back client by client (`:821-823`).

Here the same exchanges are collectives:

* control plane (all ranks, gloo over TCP, keeps the reference ``-ip/-port/-rank/
  -world_size`` rendezvous): ``all_gather_object`` / ``broadcast_object`` of metadata and
  GMM parameters (M2-M5), barriers with timeouts (failure detection);
* data plane (client ranks, ``nccl`` = RCCL over xGMI when every client owns a GPU,
  otherwise gloo): the per-round aggregation is ONE ``all_reduce(SUM)`` of the flat,
  pre-scaled ``w_i * [theta_G | theta_D | BN stats]`` buffer — which replaces the
  reference's gather (M9) + weighted average + serial broadcast (M10).  Every client then
  holds the aggregate, so there is no push-back step at all.

``Comm`` also works without ``torch.distributed`` (world size 1) so the single-client
path and the CLI need no rendezvous.
"""
from __future__ import annotations

import datetime
import os
from typing import Any, List, Optional, Sequence

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank: int = 0, world_size: int = 1, client_ranks: Sequence[int] = (0,),
                 data_backend: str = "gloo", ip: str = "127.0.0.1", port: int = 7788, timeout_s: float = 600.0,
                 device: torch.device | None = None, init: bool = True, force_dist: bool = False,
                 native_rccl: bool | None = None):
        self.rank = rank
        self.world_size = world_size
        self.client_ranks = list(client_ranks)
        # "auto" / "auto_all": agreed over the control plane at init (_vote_data_backend)
        self.data_backend = data_backend
        self.device = device or torch.device("cpu")
        self.timeout = datetime.timedelta(seconds=timeout_s)
        self.ctrl = None
        self.data = None
        self.p2p = None
        self.share_pg = {}          # dedicated federator rank -> gloo pair group {first client, federator}
        self._share = None          # first client: (pinned buffer, side stream, executor, pending send)
        self.initialized = False
        # RCCL data plane: fold the client weight into the all-reduce (pre-multiplied sum) instead of scaling the
        # buffer first (tools/premul_probe.py checks it against x * w on the box)
        self.premul_sum = True
        # the weight all-reduce through the native RCCL plane (parallel/rccl.py, csrc/comm) instead of
        # torch.distributed's ProcessGroup.  None: on unless FEDTGAN_NATIVE_RCCL=0 -- the default since round 6: a
        # one-rank RCCL round costs plain + 0.0-0.04 ms with it, + 0.1-0.3 ms through the ProcessGroup (whose
        # all-reduce holds the next round's generation back, profiles/sync_r6.txt); bitwise the same aggregate and
        # tables (tests/test_gpu_federation.py::test_gpu_one_rank_rccl_pipelined_gather_matches_unpipelined)
        self.native_rccl = (os.environ.get("FEDTGAN_NATIVE_RCCL", "1") == "1") if native_rccl is None else native_rccl
        self._native = None
        # ``force_dist``: build real process groups even for one rank, so the collective branches
        # (RCCL all-reduce / gather / send-recv) execute on a single-GPU box instead of the
        # world-size-1 short-circuits
        self.dist_active = (world_size > 1 or force_dist) and init
        if self.dist_active:
            self._init(ip, port)
        elif self.data_backend in ("auto", "auto_all"):
            self.data_backend = "nccl" if self.device.type == "cuda" else "gloo"

    def _init(self, ip: str, port: int):
        os.environ.setdefault("MASTER_ADDR", ip)
        os.environ.setdefault("MASTER_PORT", str(port))
        if not dist.is_initialized():
            dist.init_process_group("gloo", init_method=f"tcp://{ip}:{port}", rank=self.rank,
                                    world_size=self.world_size, timeout=self.timeout)
        self.initialized = True
        self.ctrl = dist.group.WORLD
        if self.data_backend in ("auto", "auto_all"):
            self.data_backend = self._vote_data_backend(self.data_backend == "auto_all")
        if self.data_backend == "nccl":
            # every rank must call new_group, members or not
            self.data = dist.new_group(ranks=self.client_ranks, backend="nccl", timeout=self.timeout)
            # a dedicated federator sits outside the RCCL group (it shares a GPU with a client, and RCCL
            # takes one rank per device): the first client hands it the aggregate over a gloo pair group of
            # its own, so those transfers never interleave with the control plane's collectives
            for f in range(self.world_size):
                if f not in self.client_ranks:
                    pg = dist.new_group(ranks=sorted({self.client_ranks[0], f}), backend="gloo", timeout=self.timeout)
                    self.share_pg[f] = pg
            if self.native_rccl:
                self._init_native()
        else:
            # gloo data plane: reduce over every rank; a dedicated federator contributes zeros
            self.data = self.ctrl

    def _init_native(self):
        """The client ranks' native RCCL communicator: the first client's unique id travels over the control
        plane (every rank takes part in that collective; only client ranks join the communicator)."""
        from .rccl import NativeRccl
        first = self.client_ranks[0]
        ids = [None] * self.world_size
        uid = None
        if self.rank == first:
            from ..ops import native
            from .rccl import rccl_library_path
            L = native.require()
            L.rccl_load(rccl_library_path())
            uid = L.rccl_unique_id().tolist()
        dist.all_gather_object(ids, uid, group=self.ctrl)
        if self.rank in self.client_ranks:
            shared = torch.tensor(ids[first], dtype=torch.uint8)
            self._native = NativeRccl(self.client_ranks.index(self.rank), len(self.client_ranks), self.device,
                                      share_id=lambda _uid: shared)

    def _vote_data_backend(self, all_ranks: bool) -> str:
        """Collective (control plane): every rank reaches the SAME data-plane choice.  RCCL when each rank
        that joins it (the client ranks; every rank for ``all_ranks``, the MD-GAN point-to-point group) has
        a GPU of its own -- no two such ranks on one (host, device) -- and gloo on every rank otherwise.
        Deciding from each rank's local device count alone let ranks disagree (a CPU-only dedicated
        federator picking gloo while a GPU client created an RCCL group: init hung until the timeout)."""
        import socket
        me = (self.rank in self.client_ranks or all_ranks, self.device.type, socket.gethostname(),
              self.device.index if self.device.type == "cuda" else -1)
        views = [None] * self.world_size
        dist.all_gather_object(views, me, group=self.ctrl)
        return self.pick_data_backend(views)

    @staticmethod
    def pick_data_backend(views) -> str:
        """views: one (joins the data plane, device type, host, device index) per rank."""
        members = [v for v in views if v[0]]
        ok = bool(members) and all(v[1] == "cuda" for v in members) and \
            len({(v[2], v[3]) for v in members}) == len(members)
        return "nccl" if ok else "gloo"

    @classmethod
    def from_env(cls, data_backend: str = "auto", device: torch.device | None = None,
                 force_dist: bool = False) -> "Comm":
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        ip = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        if data_backend == "auto" and not (ws > 1 or force_dist):
            data_backend = "nccl" if (device is not None and device.type == "cuda") else "gloo"
        return cls(rank, ws, list(range(ws)), data_backend, ip, port, device=device, force_dist=force_dist)

    def data_world_size(self) -> int:
        """Ranks in the data-plane group (the clients that take part in the all-reduce)."""
        if not self.dist_active or self.data is None:
            return 1
        return dist.get_world_size(self.data)

    # ------------------------------------------------------------------ properties
    @property
    def is_client(self) -> bool:
        return self.rank in self.client_ranks

    @property
    def n_clients(self) -> int:
        return len(self.client_ranks)

    @property
    def client_index(self) -> int:
        return self.client_ranks.index(self.rank) if self.is_client else -1

    # ------------------------------------------------------------------ control plane
    def all_gather_object(self, obj: Any) -> List[Any]:
        if not self.dist_active:
            return [obj]
        out: List[Any] = [None] * self.world_size
        dist.all_gather_object(out, obj, group=self.ctrl)
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.dist_active:
            return obj
        box = [obj if self.rank == src else None]
        dist.broadcast_object_list(box, src=src, group=self.ctrl)
        return box[0]

    def barrier(self):
        if self.dist_active:
            dist.barrier(group=self.ctrl)

    def heartbeat(self, timeout_s: float):
        """Failure detection: a monitored gloo barrier over the control plane.  If a rank does not
        arrive within ``timeout_s`` every live rank raises, naming the missing ranks (instead of
        hanging until the process-group timeout)."""
        if self.dist_active:
            dist.monitored_barrier(group=self.ctrl, timeout=datetime.timedelta(seconds=timeout_s),
                                   wait_all_ranks=True)

    def broadcast_tensor(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        """Broadcast a tensor over the control plane (device tensors are staged through host memory)."""
        if not self.dist_active:
            return t
        host = t.detach().to("cpu", copy=True) if t.device.type != "cpu" else t
        dist.broadcast(host, src=src, group=self.ctrl)
        if host is not t:
            t.copy_(host)
        return t

    def all_reduce_cpu(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if self.dist_active:
            dist.all_reduce(t, op=op, group=self.ctrl)
        return t

    def max_float(self, x: float) -> float:
        if not self.dist_active:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.ctrl)
        return float(t.item())

    def gather_bytes(self, payload: bytes, dst: int = 0) -> Optional[List[bytes]]:
        if not self.dist_active:
            return [payload]
        out = [None] * self.world_size if self.rank == dst else None
        dist.gather_object(payload, out, dst=dst, group=self.ctrl)
        return out

    # ------------------------------------------------------------------ data plane
    def gather_rows(self, t: torch.Tensor, counts: Sequence[int], ranks: Sequence[int], dst: int = 0,
                    to_host: bool = True):
        """Row-concatenate the [counts[i], C] tensors of ``ranks`` (in order) on ``dst``.

        With an RCCL data plane the device tensors move GPU to GPU over xGMI (padded to the
        largest share, one ``gather``) and ``dst`` copies the result to the host once (or, with
        ``to_host=False``, keeps it on the device for an asynchronous copy); the gloo path gathers
        host tensors.  Returns the tensor on ``dst``, None elsewhere."""
        if not self.dist_active:
            return t.cpu() if to_host else t
        nccl = self.data_backend == "nccl"
        width = t.shape[1]
        m = max(counts)
        if nccl and t.shape[0] == m and t.is_contiguous():
            buf = t                     # a full share: sent as it is (no padded copy, no fill)
        else:
            buf = torch.zeros(m, width, dtype=t.dtype, device=t.device if nccl else "cpu")
            buf[:t.shape[0]] = t if nccl else t.cpu()
        group = self.data if nccl else self.ctrl
        nw = dist.get_world_size(group)
        whole = gl = None
        if self.rank == dst:
            # the receive slots are views of ONE buffer: with equal shares in group order it already is the table
            whole = torch.empty(nw, m, width, dtype=buf.dtype, device=buf.device)
            gl = list(whole.unbind(0))
        dist.gather(buf, gl, dst=dst, group=group)
        if self.rank != dst:
            return None
        order = dist.get_process_group_ranks(group) if group is not dist.group.WORLD else list(range(self.world_size))
        if list(ranks) == list(order) and all(int(n) == m for n in counts):
            out = whole.view(nw * m, width)
        else:
            parts = {r: g for r, g in zip(order, gl)}
            out = torch.cat([parts[r][:n] for r, n in zip(ranks, counts)])
        return out.cpu() if to_host else out

    def weighted_all_reduce(self, flat: torch.Tensor, weight: float) -> torch.Tensor:
        """flat <- sum_i w_i * flat_i over the data group (in place).

        Non-client ranks (a dedicated federator) contribute zeros and receive the sum too
        when the data plane spans every rank (gloo).
        """
        if not self.dist_active:
            if weight != 1.0:
                flat.mul_(weight)
            return flat
        if self.data_backend == "nccl":
            if self._native is not None:        # client ranks: the native plane, on the current stream
                self._native.all_reduce(flat, weight)
                return flat
            if self.is_client:
                if weight != 1.0 and self.premul_sum and hasattr(dist, "_make_nccl_premul_sum"):
                    # the client weight rides in the collective (RCCL's pre-multiplied sum: each rank's input is
                    # scaled as it is loaded), so no separate scaling launch precedes the all-reduce
                    dist.all_reduce(flat, op=dist._make_nccl_premul_sum(float(weight)), group=self.data)
                    return flat
                if weight != 1.0:
                    flat.mul_(weight)
                dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.data)
            return flat
        # gloo: reduce on host memory
        host = flat.detach().to("cpu", copy=True) if flat.device.type != "cpu" else flat
        if self.is_client:
            host.mul_(weight)
        else:
            host.zero_()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.data)
        if host is not flat:
            flat.copy_(host)
        return flat

    def share_with_federator(self, flat: torch.Tensor, federator: int = 0, extra: Optional[torch.Tensor] = None):
        """After an RCCL reduce among the clients, hand the aggregate to a dataless federator rank
        (the reference's server holds the averaged model to sample from, `Server/dtds/distributed.py:
        809-820`).  The first client copies it to pinned host memory on a side stream and a helper thread
        sends it over the pair group once the copy lands, so the clients go on with the next round at
        once (only the copy, ~0.2 ms for 8.5 MB, is ordered before the next round's kernels); the
        federator receives it and copies it to its device.  ``extra`` (a small device tensor every client
        holds, e.g. the client-averaged losses) rides along in the same message and lands in the
        federator's ``extra``.  Returns True on EVERY rank when the hand-off took place this round (the
        decision depends only on state all ranks share), so callers that branch on it stay collective."""
        if not self.dist_active or self.data_backend != "nccl" or federator in self.client_ranks:
            return False
        src = self.client_ranks[0]
        pg = self.share_pg.get(federator)
        parts = [flat] + ([extra] if extra is not None else [])
        if self.rank == src:
            self._share_send(parts, federator, pg)
        elif self.rank == federator:
            host = self._share_buffer(parts)[0]
            dist.recv(host, src=src, group=pg)
            off = 0
            for t in parts:
                n = t.numel()
                t.view(-1).copy_(host[off:off + n], non_blocking=t.is_cuda)
                off += n
            if flat.is_cuda:            # the pinned buffer is received into again next round
                torch.cuda.current_stream(flat.device).synchronize()
        # the other clients take no part in the transfer, but the hand-off happened for them too: every
        # client already holds ``extra`` (client_mean), so nothing else needs a control collective
        return True

    def _share_buffer(self, parts):
        n = sum(t.numel() for t in parts)
        if self._share is None or self._share[0].numel() != n:
            cuda = parts[0].is_cuda
            host = torch.empty(n, dtype=parts[0].dtype, pin_memory=cuda)
            stream = torch.cuda.Stream(parts[0].device) if cuda else None
            from concurrent.futures import ThreadPoolExecutor
            self._share = [host, stream, ThreadPoolExecutor(1), None]
        return self._share

    def _share_send(self, parts, dst: int, pg) -> None:
        host, stream, pool, pending = self._share_buffer(parts)
        if pending is not None:
            pending.result()            # the previous round's send has left the buffer
        flat = parts[0]
        if flat.is_cuda:
            cur = torch.cuda.current_stream(flat.device)
            stream.wait_stream(cur)
            with torch.cuda.stream(stream):
                off = 0
                for t in parts:
                    host[off:off + t.numel()].copy_(t.view(-1), non_blocking=True)
                    off += t.numel()
                ev = torch.cuda.Event()
                ev.record(stream)
            cur.wait_stream(stream)     # the next round's updates of flat wait for the copy, not for the send
        else:
            off = 0
            for t in parts:
                host[off:off + t.numel()].copy_(t.view(-1))
                off += t.numel()
            ev = None

        def send():
            if ev is not None:
                ev.synchronize()
            dist.send(host, dst=dst, group=pg)
        self._share[3] = pool.submit(send)

    def client_mean(self, t: torch.Tensor) -> torch.Tensor:
        """t <- mean of t over the client ranks, in place, on the RCCL data plane (device-side: no host
        wait).  Only meaningful where ``data_backend == "nccl"`` and this rank is a client."""
        if self.dist_active and self.data_backend == "nccl" and self.is_client:
            t.div_(self.n_clients)
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.data)
        return t

    def share_wait(self) -> None:
        """Block until this rank's last hand-off to the federator has been sent."""
        if self._share is not None and self._share[3] is not None:
            self._share[3].result()
            self._share[3] = None

    # ------------------------------------------------------------------ point to point (MD-GAN)
    def init_p2p(self):
        """Collective (every rank): the point-to-point group of the split (MD-GAN) mode -- RCCL over
        all ranks when the data plane is RCCL, else the gloo control plane."""
        if not self.dist_active:
            self.p2p = None
        elif self.data_backend == "nccl":
            self.p2p = dist.new_group(ranks=list(range(self.world_size)), backend="nccl", timeout=self.timeout)
        else:
            self.p2p = self.ctrl
        return self.p2p

    def exchange(self, sends: Sequence[tuple] = (), recvs: Sequence[tuple] = ()):
        """Batched point-to-point: ``sends`` = [(tensor, dst)], ``recvs`` = [(tensor, src)]; all
        posted together, returns when every transfer is complete.  Over gloo, device tensors are
        staged through host memory; over RCCL they move GPU to GPU (xGMI)."""
        if not sends and not recvs:
            return
        nccl = self.data_backend == "nccl"
        host = (lambda t: t) if nccl else (lambda t: t.detach().to("cpu", copy=True) if t.device.type != "cpu" else t)
        s_bufs = [(host(t.contiguous()), d) for t, d in sends]
        r_bufs = [(t if (nccl or t.device.type == "cpu") and t.is_contiguous() else
                   torch.empty(t.shape, dtype=t.dtype, device=t.device if nccl else "cpu"), t, src)
                  for t, src in recvs]
        ops = [dist.P2POp(dist.isend, b, d, group=self.p2p) for b, d in s_bufs]
        ops += [dist.P2POp(dist.irecv, b, src, group=self.p2p) for b, _, src in r_bufs]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for b, t, _ in r_bufs:
            if b is not t:
                t.copy_(b)

    def warmup(self, width: int = 4, dst: int = 0, gather: bool = True):
        """Run each data-plane collective once with tiny tensors (collective: every rank).  RCCL sets
        up its communicator and point-to-point connections lazily at the first all-reduce / gather;
        doing it here keeps that one-off cost (~1 s) out of the first training round."""
        if not self.dist_active or self.data_backend != "nccl":
            return
        t = torch.zeros(8, dtype=torch.float32, device=self.device)
        if self.is_client:
            dist.all_reduce(t, group=self.data)
        ranks = self.client_ranks
        rows = torch.zeros(1, width, dtype=torch.float64, device=self.device)
        if gather and self.rank in ranks:
            self.gather_rows(rows, [1] * len(ranks), ranks, dst=dst, to_host=False)
        torch.cuda.synchronize(self.device)

    def destroy(self):
        self.share_wait()
        if self._native is not None:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)      # (no collective of this communicator in flight)
            self._native.destroy()
            self._native = None
        if self.initialized and dist.is_initialized():
            dist.destroy_process_group()
            self.initialized = False
