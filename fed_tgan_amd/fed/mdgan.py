"""MD-GAN split mode: ONE generator on the federator, one discriminator per client.

The reference ships this mode dormant and incomplete.
- Clients register a generator RRef (`Client/.../dtds/distributed.py:87-93`).
- `train_D` queries the remote generator for every batch (`:292-333`).
- `loss_G` only *returns summed losses*: there is no distributed autograd, so no gradient ever
  reaches G (`:335-377`).
- No server driver calls any of it.

This module completes the mode along the lines of MD-GAN (Hardy et al., 2019), keeping the
reference's per-batch exchange shapes (survey M11: a `[B, E + n_opt]` generator input goes up,
`[B, data_dim]` logits come back down). Every step does the following.

D step:
- each client draws its conditional vectors, noise and real rows on its GPU;
- it sends the generator input `[z | c]` to the server;
- the server runs G for every client batch (train-mode BN per batch, as the reference's
  per-RPC forward does) and sends back the logits;
- the client applies the Gumbel / tanh activation and slerp, then runs its WGAN-GP D update
  (the same kernels as the federated engine).

G step:
- clients draw fresh `[z | c]` and the server returns the logits;
- each client back-propagates `-mean D(fake) + cond CE` through its discriminator and
  activation down to the logits, and returns `dL/dlogits`;
- the server back-propagates every client's `dL/dlogits` through the saved G activations,
  averages the gradients with the federation weights (JSD/WD weights or uniform) and takes one
  Adam step.

Every `e_interval` (`-E_interval`) epochs the clients pass their discriminators (plus Adam state) one step
around a ring (MD-GAN §3 "discriminator swapping").

Transport: batched point-to-point transfers (`Comm.exchange`). These are RCCL send/recv over
xGMI when every rank has a GPU, else gloo. Transfers for all K clients are posted together, so
the server never serialises clients.

Requirements: a dedicated federator (`world_size = K + 1`, not co-located), and the same
`steps = min_k(rows_k) // batch` per epoch on every rank (lockstep).

Timers: like the reference's `time_train_d` / `time_loss_g`
(`Client/.../dtds/distributed.py:301-309, 353-360, 379-386`), each client records the wall time
of its G round trip per step and writes `time_train_d_client{i}.csv` and
`time_loss_g_client{i}.csv` at the end.
"""
from __future__ import annotations

import csv
import os
import time
from typing import List

import numpy as np
import torch

from .runtime import FedRuntime, _log
from ..utils.devsync import device_sync


class MDGANRuntime(FedRuntime):
    def initialize(self):
        super().initialize()
        c = self.comm
        if self.federator in c.client_ranks:
            raise ValueError("MD-GAN mode needs a dedicated generator rank (world_size = clients + 1)")
        c.init_p2p()
        eng = self.engine
        self.md_steps = int(min(self.steps)) if self.steps else 0
        self.in_cols = eng.E + eng.C
        self.time_train_d: List[float] = []
        self.time_loss_g: List[float] = []
        if self.is_fed:
            K = c.n_clients
            self.gbufs = [eng.new_g_buffers() for _ in range(K)]
            self.gsum = torch.zeros_like(eng.gradG)
            self.w = torch.as_tensor(np.asarray(self.weights, dtype=np.float64), dtype=torch.float32)
        _log(self.cfg, self.rank, f"[mdgan] {c.n_clients} discriminators, generator on rank {self.federator}, "
                                  f"{self.md_steps} lockstep steps/epoch")

    # ------------------------------------------------------------------ server side
    def _server_forward(self, training: bool = True):
        """Receive every client's [z | c], run G per client batch, send the logits back."""
        c, eng = self.comm, self.engine
        ins = [eng.g_input_view(b["H"]) for b in self.gbufs]
        staged = [torch.empty(eng.B, self.in_cols, device=self.device) for _ in ins]
        c.exchange(recvs=[(t, r) for t, r in zip(staged, c.client_ranks)])
        for k, b in enumerate(self.gbufs):
            ins[k].copy_(staged[k])
            with eng.use_g_buffers(b):
                eng._g_forward(eng.H, eng.logits, training=training)
        c.exchange(sends=[(b["logits"], r) for b, r in zip(self.gbufs, c.client_ranks)])

    def _server_step(self):
        c, eng = self.comm, self.engine
        self._server_forward()                       # D step of every client
        self._server_forward()                       # G step: forward ...
        c.exchange(recvs=[(b["dlogits"], r) for b, r in zip(self.gbufs, c.client_ranks)])
        self.gsum.zero_()
        for k, b in enumerate(self.gbufs):           # ... and backward per client batch
            with eng.use_g_buffers(b):
                eng._g_backward()
            self.gsum.add_(eng.gradG, alpha=float(self.w[k]))
        eng.gradG.copy_(self.gsum)
        if not eng.ops.adam_counts_steps:           # (in the fused step the G sampler bumps it)
            eng.stepG += 1
        eng._g_adam()

    # ------------------------------------------------------------------ client side
    def _remote_logits(self) -> float:
        c, eng = self.comm, self.engine
        t0 = time.perf_counter()
        c.exchange(sends=[(eng.g_input_view(), self.federator)])
        c.exchange(recvs=[(eng.logits, self.federator)])
        if self.device.type == "cuda":
            device_sync(self.device)
        return time.perf_counter() - t0

    def _client_step(self):
        eng, o, B = self.engine, self.engine.ops, self.engine.B
        # D step: local batch, remote generator, local D update
        o.sample_train(eng.tables, eng.H, eng.z_cols, eng.c_cols, eng.X_fake, eng.X_real, eng.Dd, eng.col,
                       eng.opt, step_counter=eng.stepD, metrics=eng.metrics, zero_metrics=True, stream_id=1)
        self.time_train_d.append(self._remote_logits())
        o.activate(eng.logits, eng.X_fake[:, :eng.Dd], eng.spans, eng.cfg.tau, stream_id=2)
        o.slerp(eng.X_real, eng.X_fake, eng.X_interp, stream_id=3)
        eng._d_update()
        # G step: feedback dL/dlogits for the server
        o.sample_train(eng.tables, eng.H, eng.z_cols, eng.c_cols, eng.Xg, None, eng.Dd, eng.col, eng.opt,
                       step_counter=eng.stepG, stream_id=11)
        self.time_loss_g.append(self._remote_logits())
        o.activate(eng.logits, eng.Xg[:, :eng.Dd], eng.spans, eng.cfg.tau, stream_id=12)
        eng._g_dlogits()
        self.comm.exchange(sends=[(eng.dlogits, self.federator)])
        eng._g_loss_metric()
        if hasattr(o, "ctr"):
            o.L.rng_bump(o.ctr)                      # fresh Philox streams for the next step

    def _swap_discriminators(self):
        """Ring-pass each client's discriminator + Adam state to the next client."""
        c, eng = self.comm, self.engine
        K = c.n_clients
        if K < 2 or not self.is_client:
            return
        i = c.client_index
        nxt, prv = c.client_ranks[(i + 1) % K], c.client_ranks[(i - 1) % K]
        out = torch.cat([eng.flatD, eng.mD, eng.vD, eng.stepD])
        inc = torch.empty_like(out)
        c.exchange(sends=[(out, nxt)], recvs=[(inc, prv)])
        n = eng.flatD.numel()
        eng.flatD.copy_(inc[:n])
        eng.mD.copy_(inc[n:2 * n])
        eng.vD.copy_(inc[2 * n:3 * n])
        eng.stepD.copy_(inc[3 * n:])

    # ------------------------------------------------------------------ rounds
    def run_round(self, epoch: int) -> float:
        dt = self._run_round(epoch)
        self._sync_losses()
        return dt

    def _run_round(self, epoch: int) -> float:
        t0 = time.time()
        with self.timer.phase("train", self.device):
            for _ in range(self.md_steps):
                if self.is_fed:
                    self._server_step()
                elif self.is_client:
                    self._client_step()
        self._epoch_done = epoch + 1
        self.engine.bn_batches += 2 * self.comm.n_clients * self.md_steps
        iv = max(int(self.cfg.e_interval), 0)
        with self.timer.phase("aggregate", self.device):
            if iv and (epoch + 1) % iv == 0:
                self._swap_discriminators()
        with self.timer.phase("sample_dump", self.device):
            self.sample_round(epoch)
        if self.device.type == "cuda":
            device_sync(self.device)
        return time.time() - t0

    def fit(self):
        super().fit()
        if self.is_client:
            d = self.cfg.out_dir
            i = self.comm.client_index
            for name, vals in (("time_train_d", self.time_train_d), ("time_loss_g", self.time_loss_g)):
                with open(os.path.join(d, f"{name}_client{i}.csv"), "w", newline="") as f:
                    csv.writer(f).writerows([[v] for v in vals])
