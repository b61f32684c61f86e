"""EngineConfig.bn_fold stated in torch (ops/ref.py: per-tile partials, BatchNorm-on-load, materialisation): the
folded generator forward equals the GEMM + BatchNorm forward -- the CPU oracle of the HIP path's plumbing (the
pre-BN rows Hp beside H, the sampler's z columns there, the ranges each GEMM stages, who publishes the batch and
running statistics).  The HIP kernels are checked against this path's semantics in test_hip_engine.py."""
import pytest
import torch

from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
from fed_tgan_amd.ops.ref import TorchOps

from helpers import small_table


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("gen_dims", [(256, 256), (128,)])
def test_bn_fold_torch_oracle_matches_bn_path(monkeypatch, gen_dims):
    monkeypatch.setattr(TorchOps, "bn_fold_capable", True)
    _, _, _, _, _, _, tr, X = small_table()
    engs = []
    for fold in (False, True):
        torch.manual_seed(0)
        e = CTGANEngine(tr.layout, EngineConfig(batch_size=500, bn_fold=fold, gen_dims=gen_dims), "cpu",
                        backend="torch", seed=3)
        e.set_training_data(X)
        engs.append(e)
    a, b = engs
    b.flat.copy_(a.flat)
    assert not a._fold_on() and b._fold_on()
    for e in engs:
        torch.manual_seed(7)
        e._prepare_paired()
    c0 = a.c_cols[0]
    for i in range(len(a.gdims)):
        for x, y in ((b.bn_mean2[i], a.bn_mean2[i]), (b.bn_invstd2[i], a.bn_invstd2[i]), (b.nhat2[i], a.nhat2[i]),
                     (b.p[f"G.{i}.rm"], a.p[f"G.{i}.rm"]), (b.p[f"G.{i}.rv"], a.p[f"G.{i}.rv"])):
            assert _rel(x, y) < 1e-5, i
    assert _rel(b.H2[:, :c0], a.H2[:, :c0]) < 1e-5
    assert torch.equal(b.H2[:, c0:], a.H2[:, c0:])
    assert _rel(b.logits2, a.logits2) < 1e-5
    for e in engs:            # a whole step through the folded forward
        torch.manual_seed(11)
        e.train_steps(1, use_graph=False)
    assert _rel(b.flat, a.flat) < 1e-4
