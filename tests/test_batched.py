"""Batched multi-client engine (models/batched.py): K clients' steps issued once, client = blockIdx.z.

Every client's trajectory must be bit-identical to a single-client engine with the same seed, initial
weights and data -- the batched launches only add a per-client pointer offset and seed step.
"""
import dataclasses

import numpy as np
import pytest
import torch

from fed_tgan_amd.data.demo import small_table
from fed_tgan_amd.models.arena import Arena
from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig

DEV = torch.device("cuda:0")


def _twin_cfg(cfg):
    """A single-client engine issuing the batched engine's launch sequence: the batched step never chains
    D1 into D0's reduction launch nor fuses D1's weight gradient into the D Adam (models/engine.py,
    batch_k > 1) -- fp32 epilogue paths that are close to, not bitwise equal to, the bf16-operand GEMMs."""
    return dataclasses.replace(cfg, chain_d1=False, fuse_d_adam=False)


def _client_tables(X, k):
    rng = np.random.default_rng(7)
    return [X[rng.permutation(len(X))] if c else X for c in range(k)]


def test_arena_slabs_mirror_and_refuse_divergent_layouts():
    """CPU: slab allocators give identical offsets for identical sequences; freeze() rejects others."""
    a = Arena(3, 1 << 20, "cpu")
    views = []
    for c in range(3):
        s = a.slab(c)
        views.append((s.zeros(10, 7), s.zeros(5, dtype=torch.int64), s.tensor(np.arange(4, dtype=np.int32))))
    a.freeze()
    for c in range(1, 3):
        assert views[c][0].data_ptr() - views[0][0].data_ptr() == c * a.stride
        assert torch.equal(a.client_view(views[0][2], c), views[c][2])
    b = Arena(2, 1 << 20, "cpu")
    b.slab(0).zeros(10)
    b.slab(1).zeros(11)
    with pytest.raises(RuntimeError, match="do not mirror"):
        b.freeze()
    # after the freeze, allocations outside a batched launch are plain memory; inside one, every slab
    t = a.slab(1).zeros(3)
    assert not (a.base <= t.data_ptr() < a.base + 3 * a.stride)
    a.batch_active = True
    g = a.slab(0).tensor(np.full(6, 5, dtype=np.int32))
    a.batch_active = False
    for c in range(3):
        assert torch.equal(a.client_view(g, c), torch.full((6,), 5, dtype=torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_batched_clients_bit_identical_to_single_engines(precision):
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table(2000, 0)
    k = 3
    cfg = EngineConfig(batch_size=500, precision=precision)
    seeds = [1000 + c for c in range(k)]
    data = _client_tables(X, k)
    bc = BatchedClients(tr.layout, cfg, DEV, seeds, n_rows=len(X))
    # (per-client GEMM planning: the same split-K factors as the single-client engines -> bit-identical sums;
    # the default plans over clients x tiles, see test_batched_plan_close_to_single_engines)
    bc.engines[0].ops.batch_plan = False
    for e, Xc in zip(bc.engines, data):
        e.set_training_data(Xc)
    plain = []
    for s, e, Xc in zip(seeds, bc.engines, data):
        p = CTGANEngine(tr.layout, _twin_cfg(cfg), DEV, backend="hip", seed=s)
        p.flat.copy_(e.flat)
        p.set_training_data(Xc)
        plain.append(p)
    # eager steps, then graph-captured ones (8 per graph + a remainder), then an aggregation
    bc.train_steps(2, use_graph=False)
    for p in plain:
        p.train_steps(2, use_graph=False)
    bc.train_steps(11)
    for p in plain:
        p.train_steps(11)
    torch.cuda.synchronize()
    for c, (e, p) in enumerate(zip(bc.engines, plain)):
        for name in ("flat", "mG", "vG", "mD", "vD", "stepG", "stepD"):
            assert torch.equal(getattr(e, name), getattr(p, name)), (c, name)
        assert torch.equal(e.ops.ctr, p.ops.ctr)
        torch.testing.assert_close(e.metrics, p.metrics, rtol=1e-5, atol=1e-6)
        assert e.bn_batches == p.bn_batches == 26
    # the clients really differ (different data / seeds), and the FedAvg reduces over the arena
    assert not torch.equal(bc.engines[0].flat, bc.engines[1].flat)
    w = [0.2, 0.3, 0.5]
    want = sum(wi * p.flat.double() for wi, p in zip(w, plain)).float()
    bc.weighted_average(w)
    torch.cuda.synchronize()
    for e in bc.engines:
        torch.testing.assert_close(e.flat, want, rtol=1e-6, atol=1e-7)
        assert torch.equal(e.flat, bc.engines[0].flat)


@pytest.mark.gpu
def test_batched_plan_close_to_single_engines():
    """Default planning (split-K / tiles chosen for clients x tiles): the same math with other K splits, so
    each client stays within fp32-reassociation distance of its single-client twin over a few steps."""
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table(2000, 0)
    k = 8
    cfg = EngineConfig(batch_size=500, precision="fp32")
    seeds = [2000 + c for c in range(k)]
    data = _client_tables(X, k)
    bc = BatchedClients(tr.layout, cfg, DEV, seeds, n_rows=len(X))
    assert bc.engines[0].ops.batch_plan
    for e, Xc in zip(bc.engines, data):
        e.set_training_data(Xc)
    plain = []
    for s, e, Xc in zip(seeds, bc.engines, data):
        p = CTGANEngine(tr.layout, _twin_cfg(cfg), DEV, backend="hip", seed=s)
        p.flat.copy_(e.flat)
        p.set_training_data(Xc)
        plain.append(p)
    bc.train_steps(3, use_graph=False)
    for p in plain:
        p.train_steps(3, use_graph=False)
    torch.cuda.synchronize()
    steps, lr = 3, cfg.lr
    for c, (e, p) in enumerate(zip(bc.engines, plain)):
        assert torch.equal(e.stepD, p.stepD) and torch.equal(e.ops.ctr, p.ops.ctr)
        # Adam normalises each element's step: where a gradient is reassociation noise around 0 the twins may
        # step +-lr in either direction (up to 2 lr per step per element); the tensors as a whole agree
        d = (e.flat - p.flat).abs()
        assert d.max().item() <= 2 * steps * lr + 1e-6, (c, d.max().item())
        rel = ((e.flat - p.flat).norm() / p.flat.norm()).item()
        assert rel < 1e-3, (c, rel)


@pytest.mark.gpu
def test_batched_launch_refuses_buffers_outside_the_arena():
    """A batched launch handed a tensor outside client 0's slab fails loudly (no silent aliasing)."""
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table(2000, 0)
    bc = BatchedClients(tr.layout, EngineConfig(batch_size=500), DEV, [5, 6], n_rows=len(X))
    for e in bc.engines:
        e.set_training_data(X)
    bc.freeze()
    e0 = bc.engines[0]
    stray = torch.zeros(500, e0.gdims[0], device=DEV)
    with bc._batched():
        with pytest.raises(RuntimeError, match="slab"):
            e0.ops.gemm(e0.H[:, :e0.gdims[0]], e0.p["G.0.W"][:, :e0.gdims[0]], stray, tb=True)
    e0.ops.reset_held()
    bc.train_steps(1, use_graph=False)      # the context is restored: training still works


@pytest.mark.gpu
def test_batched_clients_refuse_misordered_or_oversized_tables():
    """Slabs must hold the clients in non-increasing order of steps per epoch, and no client may hold more
    rows than the arena's row tables were sized for (n_rows)."""
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table(2000, 0)
    bc = BatchedClients(tr.layout, EngineConfig(batch_size=500), DEV, [5, 6], n_rows=len(X))
    bc.engines[0].set_training_data(X[:1500])
    bc.engines[1].set_training_data(X)
    with pytest.raises(RuntimeError, match="non-increasing"):
        bc.train_steps(1, use_graph=False)
    bc = BatchedClients(tr.layout, EngineConfig(batch_size=500), DEV, [5, 6], n_rows=1500)
    bc.engines[0].set_training_data(X)
    bc.engines[1].set_training_data(X[:1500])
    with pytest.raises(RuntimeError, match="mirror"):
        bc.train_steps(1, use_graph=False)


@pytest.mark.gpu
def test_batched_ragged_clients_bit_identical_to_single_engines():
    """Clients with different row counts (non-IID shards) in one batched engine: each trains its own
    len(rows) // batch steps per epoch (`Client/.../dtds/distributed.py:155, 186`) and ends every epoch
    bit-identical to a single engine with its own row count.  Epoch segments here: 3 clients x 2 steps
    (one-step graphs), 2 x 8 (an 8-step graph), then the largest client alone for 8 (plain launches)."""
    from fed_tgan_amd.models.batched import BatchedClients
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table(4000, 0)
    rng = np.random.default_rng(11)
    rows = [9000, 5000, 1000]
    data = [X[rng.integers(0, len(X), n)] for n in rows]
    # no D1 chain / fused D Adam: the launch sequence of one client alone (k = 1) is then the batched one
    cfg = EngineConfig(batch_size=500, chain_d1=False, fuse_d_adam=False)
    seeds = [3000 + c for c in range(3)]
    bc = BatchedClients(tr.layout, cfg, DEV, seeds, n_rows=max(rows))
    bc.engines[0].ops.batch_plan = False
    for e, Xc in zip(bc.engines, data):
        e.set_training_data(Xc)
    assert bc.steps() == [18, 10, 2] and bc._segments() == [(3, 2), (2, 8), (1, 8)]
    plain = []
    for s, e, Xc in zip(seeds, bc.engines, data):
        p = CTGANEngine(tr.layout, cfg, DEV, backend="hip", seed=s)
        p.flat.copy_(e.flat)
        p.set_training_data(Xc)
        plain.append(p)
    for _ in range(2):
        bc.train_epoch()
        for p in plain:
            p.train_epoch()
    torch.cuda.synchronize()
    for c, (e, p) in enumerate(zip(bc.engines, plain)):
        for name in ("flat", "mG", "vG", "mD", "vD", "stepG", "stepD"):
            assert torch.equal(getattr(e, name), getattr(p, name)), (c, name)
        assert torch.equal(e.ops.ctr, p.ops.ctr), c
        assert e.bn_batches == p.bn_batches == 4 * p.steps_per_epoch
        assert float(e.stepD) == 2 * p.steps_per_epoch
    assert set(bc.engines[0].graphs) == {(1, 3), (8, 2), 8}
