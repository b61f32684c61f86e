"""GPU tests of the engine: eager torch ops on the device, hipGraph capture, HIP backend."""
import numpy as np
import pytest
import torch

from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
from fed_tgan_amd.models.samplers import CondTables

from helpers import small_table

pytestmark = pytest.mark.gpu


def _engine(backend, batch=500):
    _, _, _, _, _, _, tr, X = small_table()
    torch.manual_seed(0)
    eng = CTGANEngine(tr.layout, EngineConfig(batch_size=batch), torch.device("cuda:0"), backend=backend, seed=3)
    eng.set_training_data(X)
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    return eng, tr


@pytest.mark.parametrize("backend", ["torch", "hip"])
def test_graph_replay_trains(backend):
    eng, _ = _engine(backend)
    eng.train_steps(3, use_graph=True)
    torch.cuda.synchronize()
    ld, lg = eng.losses()
    assert np.isfinite(ld) and np.isfinite(lg)
    assert bool(torch.isfinite(eng.flat).all())
    out = eng.generate_decoded(2000)
    assert bool(torch.isfinite(out).all())


def test_hip_step_matches_torch_step():
    """Same parameters + deterministic inputs: one HIP D step equals the torch-ops D step within fp32 noise
    on the deterministic parts (forward of fixed rows)."""
    from fed_tgan_amd.ops import native
    native.require()
    eng_t, tr = _engine("torch", batch=100)
    eng_h, _ = _engine("hip", batch=100)
    eng_h.flat.copy_(eng_t.flat)
    x = torch.randn(eng_t.B, eng_t.Hw, device="cuda:0")
    eng_t.H.copy_(x)
    eng_h.H.copy_(x)
    eng_t._g_forward(eng_t.H, eng_t.logits, training=True)
    eng_h._g_forward(eng_h.H, eng_h.logits, training=True)
    torch.cuda.synchronize()
    assert torch.allclose(eng_t.logits, eng_h.logits, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("batch", [100, 500])
def test_hip_paired_forward_matches_torch(batch):
    """The paired generator pass (2B rows, per-batch BN) on the HIP kernels equals the torch ops:
    logits of both batches, per-batch normalised activations and statistics, running statistics."""
    from fed_tgan_amd.ops import native
    native.require()
    eng_t, tr = _engine("torch", batch=batch)
    eng_h, _ = _engine("hip", batch=batch)
    eng_h.flat.copy_(eng_t.flat)
    x = torch.randn(2 * eng_t.B, eng_t.Hw, device="cuda:0")
    x[batch:] = 0.5 * x[batch:] + 1.0       # the two batches have different statistics
    eng_t.H2.copy_(x)
    eng_h.H2.copy_(x)
    eng_t._g_forward(eng_t.H2, eng_t.logits2, training=True, paired=True)
    eng_h._g_forward(eng_h.H2, eng_h.logits2, training=True, paired=True)
    torch.cuda.synchronize()
    assert torch.allclose(eng_t.logits2, eng_h.logits2, rtol=3e-2, atol=3e-2)
    for i in range(len(eng_t.gdims)):
        assert torch.allclose(eng_t.bn_mean2[i], eng_h.bn_mean2[i], rtol=1e-2, atol=1e-2)
        assert torch.allclose(eng_t.bn_invstd2[i], eng_h.bn_invstd2[i], rtol=2e-2, atol=1e-3)
        assert torch.allclose(eng_t.nhat2[i], eng_h.nhat2[i], rtol=3e-2, atol=3e-2)
    sA, sB = eng_t.group_range["S"]
    assert torch.allclose(eng_t.flat[sA:sB], eng_h.flat[sA:sB], rtol=1e-2, atol=1e-2)


def test_hip_paired_prepare_fills_d_inputs():
    """One paired sampler + generator launch sequence: conditions of both batches, real rows for
    the D batch only, interpolates on the slerp arc, step counters of both optimizers bumped."""
    from fed_tgan_amd.ops import native
    native.require()
    eng, tr = _engine("hip", batch=500)
    B, Dd = eng.B, eng.Dd
    sd, sg = float(eng.stepD), float(eng.stepG)
    eng._prepare_paired()
    torch.cuda.synchronize()
    assert float(eng.stepD) == sd + 1 and float(eng.stepG) == sg + 1
    c = eng.c_cols
    assert torch.equal(eng.X_fake[:, Dd:], eng.H2[:B, c[0]:c[1]])
    assert torch.equal(eng.Xg[:, Dd:], eng.H2[B:, c[0]:c[1]])
    assert torch.equal(eng.H2[:, c[0]:c[1]].sum(1), torch.ones(2 * B, device="cuda:0"))
    assert torch.equal(eng.X_real[:, Dd:].sum(0), eng.X_fake[:, Dd:].sum(0))
    # G-phase col/opt select the G batch's hot condition columns
    offs = torch.as_tensor(tr.layout.cond_offset, device="cuda:0").long()
    hot = offs[eng.col.long()] + eng.opt.long()
    assert torch.equal(eng.H2[B:, c[0]:c[1]].argmax(1), hot)
    # interpolates lie in span{real, fake} of their row (slerp weights), non-degenerate
    r, f, i = (t.double() for t in (eng.X_real, eng.X_fake, eng.X_interp))
    G = torch.stack([torch.stack([(r * r).sum(1), (r * f).sum(1)], 1),
                     torch.stack([(r * f).sum(1), (f * f).sum(1)], 1)], 1)
    rhs = torch.stack([(r * i).sum(1), (f * i).sum(1)], 1)
    w = torch.linalg.solve(G + 1e-9 * torch.eye(2, dtype=G.dtype, device=G.device), rhs)
    resid = (i - w[:, :1] * r - w[:, 1:] * f).norm(dim=1) / i.norm(dim=1).clamp_min(1e-12)
    assert float(resid.max()) < 1e-3
    assert bool(torch.isfinite(eng.Xall).all())


def test_generation_graph_replays_fresh_rows():
    """The captured generation pass returns fresh rows each replay (device RNG counter advances),
    with the eager pass's shape and value ranges, and its output is a private copy."""
    eng, tr = _engine("hip")
    a = eng.generate_decoded(3000, use_graph=True)
    b = eng.generate_decoded(3000, use_graph=True)
    e = eng.generate_decoded(3000, use_graph=False)
    torch.cuda.synchronize()
    assert a.shape == b.shape == e.shape == (3000, len(tr.meta))
    assert bool(torch.isfinite(a).all()) and not torch.equal(a, b)
    assert a.data_ptr() != b.data_ptr()
    for j, m in enumerate(tr.meta):
        if m["type"] != "continuous":     # category codes inside the vocabulary in both paths
            hi = float(max(m["i2s"])) if len(m["i2s"]) else 0.0
            assert float(a[:, j].max()) <= hi and float(e[:, j].max()) <= hi
