"""Several clients per process over several processes (``-world_size N -local_clients K``).

``HierComm`` runs every collective in two levels (threads of a process, then one process-level
gloo / RCCL collective from thread 0).  Checked here on the CPU with 2 gloo processes x 3 threads
against the flat 6-client semantics, and end to end through the CLI (2 processes x 2 clients).
"""
import os
import subprocess
import sys
import threading

import pandas as pd
import pytest
import torch
import torch.multiprocessing as mp

from fed_tgan_amd.cli import free_port
from fed_tgan_amd.fed.local import HierComm, LocalGroup
from fed_tgan_amd.parallel.comm import Comm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, K = 2, 3


def _client_data(i):
    g = torch.Generator().manual_seed(100 + i)
    return torch.randn(257, generator=g), 0.05 + 0.1 * i


def _worker(rank, port):
    torch.set_num_threads(1)
    outer = Comm(rank, N, list(range(N)), "gloo", port=port, device=torch.device("cpu"))
    group = LocalGroup(K)
    errors = []
    world = N * K
    weights = [_client_data(i)[1] for i in range(world)]
    expect = sum(w * _client_data(i)[0] for i, w in enumerate(weights))
    counts = [3, 0, 5, 2, 4, 1]

    def client(t):
        try:
            c = HierComm(group, t, torch.device("cpu"), outer)
            i = c.rank
            assert i == rank * K + t and c.world_size == world and c.client_index == i
            assert c.all_gather_object(("id", i)) == [("id", j) for j in range(world)]
            assert c.broadcast_object(f"from{i}", src=4) == "from4"
            x, w = _client_data(i)
            c.weighted_all_reduce(x, w)
            assert torch.allclose(x, expect, atol=1e-5)
            v = torch.full((3,), float(i))
            c.all_reduce_cpu(v)
            assert torch.equal(v, torch.full((3,), float(sum(range(world)))))
            assert c.max_float(float(i)) == world - 1
            b = torch.full((4,), float(i))
            c.broadcast_tensor(b, src=3)
            assert torch.equal(b, torch.full((4,), 3.0))
            rows = torch.arange(counts[i] * 2, dtype=torch.float64).reshape(-1, 2) + 100 * i
            pad = torch.cat([rows, torch.full((2, 2), -1.0, dtype=torch.float64)])     # callers may over-allocate
            got = c.gather_rows(pad, counts, list(range(world)), dst=0)
            if i == 0:
                ref = torch.cat([torch.arange(n * 2, dtype=torch.float64).reshape(-1, 2) + 100 * j
                                 for j, n in enumerate(counts)])
                assert torch.equal(got, ref)
            else:
                assert got is None
            c.barrier()
        except BaseException as e:  # pragma: no cover - re-raised below
            errors.append(e)
            group.failed.set()
            group.barrier.abort()

    ts = [threading.Thread(target=client, args=(t,)) for t in range(K)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    outer.destroy()
    if errors:
        raise errors[0]


def test_hier_collectives_match_flat_semantics():
    mp.spawn(_worker, args=(free_port(),), nprocs=N, join=True)


def test_hier_rejects_dedicated_federator():
    outer = Comm(0, 1, [0], "gloo", init=False)
    outer.client_ranks = [1]
    try:
        HierComm(LocalGroup(2), 0, torch.device("cpu"), outer)
    except ValueError:
        return
    raise AssertionError("expected a ValueError")


@pytest.mark.parametrize("k,extra", [(2, []), (4, ["-shard", "dirichlet", "-alpha", "0.5"])])
def test_cli_two_ranks_k_clients_each(tmp_path, k, extra):
    """2 processes x k clients; k = 4 with Dirichlet shards (clients with different row counts)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "dtds.distributed", "-world_size", "2", "-local_clients", str(k),
                        "-epochs", "2", "-backend", "torch", "-synthetic_rows", "800", "-n_sample", "503",
                        "-batch_size", "100", "-out_dir", str(tmp_path), "-dump_real", "-quiet"] + extra, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-3000:]
    raw = tmp_path / "data" / "raw"
    assert sorted(p.name for p in raw.glob("Intrusion_train_client*.csv")) == \
        [f"Intrusion_train_client{i}.csv" for i in range(2 * k)]
    if extra:
        sizes = [len(pd.read_csv(raw / f"Intrusion_train_client{i}.csv")) for i in range(2 * k)]
        assert len(set(sizes)) > 1
    df = pd.read_csv(tmp_path / "Intrusion_result" / "Intrusion_synthesis_epoch_1.csv")
    assert df.shape == (503, 42)
    assert len(pd.read_csv(tmp_path / "timestamp_experiment.csv", header=None)) == 2
