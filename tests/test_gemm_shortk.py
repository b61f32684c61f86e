"""Short-K weight-gradient GEMM (csrc/kernels/gemm.hip gemm_shortk_kernel: C = A^T B, K <= 160, M <= 256, persistent
64-column strips, operands read with ds_read_b64_tr_b16) against a float64 product of the same bf16-rounded operands,
and against the tile GEMM it replaces (the wide table's dW0, `Server/dtds/synthesizers/ctgan.py:15-30` D's first
Linear).  The HIP path is forced on small shapes by lowering gemm_shortk_min_n."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _tuning(key, value):
    return torch.ops.fedtgan.set_tuning(key, int(value))


@pytest.mark.parametrize("M,K,N,pad", [(256, 150, 137800, 0), (256, 150, 20004, 12), (128, 7, 4100, 0),
                                       (100, 160, 8192, 4), (256, 33, 65536, 0)])
def test_shortk_matches_bf16_reference_and_tile_gemm(M, K, N, pad):
    from fed_tgan_amd.ops import native
    from fed_tgan_amd.ops.hip import HipOps
    native.require()
    o = HipOps(DEV, seed=1, precision="bf16")
    g = torch.Generator(device="cpu").manual_seed(M + K + N)
    A = torch.randn(K, M + pad, generator=g).to(DEV)[:, :M]
    B = torch.randn(K, N + pad, generator=g).to(DEV)[:, :N]
    C = torch.full((M, N + pad), float("nan"), device=DEV)[:, :N]
    prev = _tuning("gemm_shortk_min_n", 4)
    try:
        o.gemm(A, B, C, ta=True)
        torch.cuda.synchronize()
        ref = A.bfloat16().double().t() @ B.bfloat16().double()
        err = (C.double() - ref).abs().max().item()
        assert err <= 1e-4 * max(1.0, ref.abs().max().item()), err
        C2 = torch.zeros_like(C)
        old = _tuning("gemm_shortk", 0)
        try:
            o.gemm(A, B, C2, ta=True)
        finally:
            _tuning("gemm_shortk", old)
        torch.cuda.synchronize()
        torch.testing.assert_close(C, C2, rtol=1e-5, atol=1e-4)
        C3 = torch.zeros_like(C)
        o.gemm(A, B, C3, ta=True)
        torch.cuda.synchronize()
        assert torch.equal(C, C3)                     # deterministic
    finally:
        _tuning("gemm_shortk_min_n", prev)


def test_shortk_leaves_other_shapes_to_the_tile_gemm():
    """Shapes outside the kernel's contract (K > 160, an epilogue, fp32 operands) still produce the plain product."""
    from fed_tgan_amd.ops import native
    from fed_tgan_amd.ops.hip import HipOps
    native.require()
    prev = _tuning("gemm_shortk_min_n", 4)
    try:
        for prec, K in (("bf16", 200), ("fp32", 150)):
            o = HipOps(DEV, seed=1, precision=prec)
            A = torch.randn(K, 64, device=DEV)
            B = torch.randn(K, 4096, device=DEV)
            C = torch.empty(64, 4096, device=DEV)
            o.gemm(A, B, C, ta=True)
            torch.cuda.synchronize()
            torch.testing.assert_close(C, A.t() @ B, rtol=2e-2, atol=2e-1 if prec == "bf16" else 1e-3)
    finally:
        _tuning("gemm_shortk_min_n", prev)


@pytest.mark.parametrize("keep_grad", [False, True])
def test_d0_shortk_adam_matches_unfused_step(keep_grad):
    """EngineConfig.fuse_d0_shortk: D0's weight gradient applying Adam in the short-K kernel's epilogue just before
    the optimizer launch (which skips its range) trains bitwise like the gradient-then-Adam schedule, on the reduced
    wide table with the short-K thresholds lowered so its packed rows take the kernel.  keep_grad: the fused
    epilogue also stores the gradient (EngineConfig.keep_grads: gemm(..., group=7)), equal to the unfused one."""
    from fed_tgan_amd.data.demo import wide_table
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from fed_tgan_amd.ops import native
    from fed_tgan_amd.ops.hip import HipOps
    native.require()
    _, _, _, _, _, _, tr, X = wide_table(device="cuda:0")
    prev = (_tuning("gemm_shortk_min_n", 4), HipOps.shortk_min_n)
    HipOps.shortk_min_n = 4
    try:
        out = []
        for fused in (False, True):
            torch.manual_seed(0)
            cfg = EngineConfig(batch_size=500, fuse_d0_shortk=fused, keep_grads=keep_grad)
            eng = CTGANEngine(tr.layout, cfg, DEV, backend="hip", seed=9)
            assert eng.ops.shortk_ok(eng.ddims[0], eng.K1, 3 * eng.nP)
            eng.set_training_data(X)
            eng.train_steps(3, use_graph=False)
            torch.cuda.synchronize()
            out.append((eng.flat.clone(), eng.mD.clone(), eng.vD.clone(), eng.g["D.0.W"].clone()))
        for k, name in enumerate(("flat", "mD", "vD")):
            assert torch.equal(out[0][k], out[1][k]), name
        if keep_grad:
            assert torch.equal(out[0][3], out[1][3])
    finally:
        _tuning("gemm_shortk_min_n", prev[0])
        HipOps.shortk_min_n = prev[1]
