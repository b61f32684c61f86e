"""MD-GAN split mode: the generator on a server, one discriminator per client.

1. With one client, a split step reproduces the federated engine's fused step exactly. The
   server's G parameters and BN statistics match, and so do the client's D parameters. The
   two roles run in two threads over an in-process point-to-point transport, and the engine
   RNG is drawn only by the client, in the same order as in the fused step.
2. The CLI runs the mode end to end as three gloo processes (server + 2 clients).
"""
import os
import queue
import subprocess
import sys
import threading

import numpy as np
import pandas as pd
import pytest
import torch

from fed_tgan_amd.fed.mdgan import MDGANRuntime
from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig

from helpers import small_table

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class QueueP2P:
    """Point-to-point transport between threads (the shape of parallel.comm.Comm.exchange)."""

    def __init__(self, qs, rank, client_ranks):
        self.qs, self.rank, self.client_ranks = qs, rank, list(client_ranks)

    @property
    def n_clients(self):
        return len(self.client_ranks)

    @property
    def client_index(self):
        return self.client_ranks.index(self.rank) if self.rank in self.client_ranks else -1

    def exchange(self, sends=(), recvs=()):
        for t, dst in sends:
            self.qs[(self.rank, dst)].put(t.detach().clone().contiguous())
        for t, src in recvs:
            t.copy_(self.qs[(src, self.rank)].get(timeout=120))


def _engine(tr, X=None):
    torch.manual_seed(0)
    # per-phase step order: the split mode draws each phase's batch when it runs, and the fused
    # reference must consume torch's global RNG in that same order.  The split server receives only
    # [z | c] (no row conditions), so its generator multiplies c densely: the fused reference does too
    eng = CTGANEngine(tr.layout, EngineConfig(batch_size=100, paired=False, onehot=False), "cpu", backend="torch",
                      seed=3)
    if X is not None:
        eng.set_training_data(X)
    return eng


def _runtime(eng, comm, is_fed, weights=(1.0,)):
    rt = object.__new__(MDGANRuntime)
    rt.comm, rt.engine, rt.federator, rt.device = comm, eng, 0, torch.device("cpu")
    rt.is_fed, rt.is_client = is_fed, not is_fed
    rt.in_cols = eng.E + eng.C
    rt.time_train_d, rt.time_loss_g = [], []
    if is_fed:
        rt.gbufs = [eng.new_g_buffers() for _ in comm.client_ranks]
        rt.gsum = torch.zeros_like(eng.gradG)
        rt.w = torch.tensor(weights, dtype=torch.float32)
    return rt


def test_split_step_equals_fused_step():
    _, _, _, _, _, _, tr, X = small_table()
    ref = _engine(tr, X)
    client = _engine(tr, X)
    server = _engine(tr)
    assert torch.equal(server.flat, client.flat)
    qs = {(0, 1): queue.Queue(), (1, 0): queue.Queue()}
    rs = _runtime(server, QueueP2P(qs, 0, [1]), True)
    rc = _runtime(client, QueueP2P(qs, 1, [1]), False)
    for step in range(2):
        th = threading.Thread(target=rs._server_step)
        th.start()
        torch.manual_seed(100 + step)
        rc._client_step()
        th.join()
        torch.manual_seed(100 + step)
        ref._one_step()
    gA, gB = ref.group_range["G"]
    dA, dB = ref.group_range["D"]
    sA, sB = ref.group_range["S"]
    assert torch.allclose(server.flat[gA:gB], ref.flat[gA:gB], rtol=0, atol=1e-6)
    assert torch.allclose(server.flat[sA:sB], ref.flat[sA:sB], rtol=0, atol=1e-6)   # BN running stats (server)
    assert torch.allclose(client.flat[dA:dB], ref.flat[dA:dB], rtol=0, atol=1e-6)
    assert not torch.allclose(server.flat[gA:gB], client.flat[gA:gB])              # G lives on the server
    assert np.allclose(client.losses(), ref.losses(), atol=1e-5)
    assert len(rc.time_train_d) == 2 and len(rc.time_loss_g) == 2


def test_two_clients_weighted_generator_update():
    """Server G gradient = sum_k w_k * (client k's G gradient)."""
    _, _, _, _, _, _, tr, X = small_table()
    server = _engine(tr)
    clients = [_engine(tr, X[:600]), _engine(tr, X[600:])]
    qs = {(a, b): queue.Queue() for a in range(3) for b in range(3)}
    rs = _runtime(server, QueueP2P(qs, 0, [1, 2]), True, weights=(0.25, 0.75))
    rcs = [_runtime(e, QueueP2P(qs, r, [1, 2]), False) for e, r in zip(clients, (1, 2))]
    # capture the per-client dL/dlogits the server receives, to rebuild the expected gradient
    ths = [threading.Thread(target=r._client_step) for r in rcs]
    before = server.flat.clone()
    [t.start() for t in ths]
    rs._server_step()
    [t.join() for t in ths]
    expect = torch.zeros_like(server.gradG)
    probe = _engine(tr)
    probe.flat.copy_(before)
    for k, (w, b) in enumerate(zip((0.25, 0.75), rs.gbufs)):
        with probe.use_g_buffers(b):
            # re-run the G step forward for client k's input (same params, train-mode BN) and its backward
            probe._g_forward(probe.H, probe.logits, training=True)
            probe._g_backward()
        expect.add_(probe.gradG, alpha=w)
    assert torch.allclose(server.gradG, expect, atol=1e-6)
    assert not torch.equal(server.flat, before)


@pytest.mark.slow
def test_cli_mdgan_gloo(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "dtds.distributed", "-world_size", "3", "-mode", "mdgan", "-epochs", "2",
                        "-backend", "torch", "-synthetic_rows", "1000", "-n_sample", "400", "-batch_size", "100",
                        "-E_interval", "1", "-out_dir", str(tmp_path), "-quiet"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    df = pd.read_csv(tmp_path / "Intrusion_result" / "Intrusion_synthesis_epoch_1.csv")
    assert df.shape[0] == 400
    for i in range(2):
        t = pd.read_csv(tmp_path / f"time_train_d_client{i}.csv", header=None)
        assert len(t) == 2 * 10
