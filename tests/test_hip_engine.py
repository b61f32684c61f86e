"""HIP engine step vs the torch-autograd oracle of the reference math (bf16-MFMA tolerances).

The batch is drawn by the HIP sampler; the oracle reuses the drawn rows, the Gumbel noise
recovered from the kernel's own softmax output (g = tau*log(y) - logits, exact up to a
per-span constant that softmax ignores) and the dropout masks recovered from the saved
mask*slope buffers.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fed_tgan_amd.models.ctgan import Generator, cond_loss
from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig

from helpers import d_forward_masked, keep_mask_from_ms, small_table

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _engine(precision="bf16", g_wt=False, wide=False):
    """wide: the reduced wide table (fed_tgan_amd.data.demo.wide_table) with the scattered one-hot weight
    gradients forced on -- the step takes every kernel path that only the 100k x 512 config takes by
    default (activation row kernels, chunk-split gradient-penalty scale, deep split-K D GEMMs)."""
    from fed_tgan_amd.ops import native
    native.require()
    if wide:
        from fed_tgan_amd.data.demo import wide_table
        _, _, _, _, _, _, tr, X = wide_table(device="cuda:0")
    else:
        _, _, _, _, _, _, tr, X = small_table()
    torch.manual_seed(0)
    cfg = EngineConfig(batch_size=500, precision=precision, g_wt=g_wt or wide, keep_grads=True)
    if wide:
        cfg.onehot_wgrad_min = 1
    eng = CTGANEngine(tr.layout, cfg, DEV, backend="hip", seed=11)
    eng.set_training_data(X)
    return eng, tr


def _masks(eng, rows, P, X):
    masks, h = [], X
    for i in range(len(eng.ddims)):
        pre = h @ P[f"D.{i}.W"].t() + P[f"D.{i}.b"]
        M = keep_mask_from_ms(eng.ms[i][rows], pre)
        M = torch.where(M > 1.0, torch.full_like(M, 2.0), torch.zeros_like(M))   # snap rounding-level noise
        masks.append(M)
        h = F.leaky_relu(pre, 0.2) * M
    return masks


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


TOL = {"bf16": 5e-2, "fp32": 2e-3}


@pytest.mark.parametrize("precision,wide", [("bf16", False), ("fp32", False), ("bf16", True), ("fp32", True)])
def test_hip_d_update_matches_autograd(precision, wide):
    eng, tr = _engine(precision, wide=wide)
    if wide:
        assert eng.K1 > 8192 and eng.Dd > 512       # chunk-split GP scale, activation row kernels
    B, nP = eng.B, eng.nP
    eng._d_prepare()
    torch.cuda.synchronize()
    Xf = eng.X_fake.reshape(nP, eng.K1).clone()
    Xr = eng.X_real.reshape(nP, eng.K1).clone()
    Xi0 = eng.X_interp.reshape(nP, eng.K1).clone()
    P = {n: t.detach().clone() for n, t in eng.p.items() if n.startswith("D.")}
    eng._d_update()
    torch.cuda.synchronize()
    L = len(eng.ddims)
    Q = {n: t.clone().requires_grad_(True) for n, t in P.items()}
    Ws = [Q[f"D.{i}.W"] for i in range(L)]
    bs = [Q[f"D.{i}.b"] for i in range(L)]
    Xi = Xi0.clone().requires_grad_(True)
    yf = d_forward_masked(Xf, Ws, bs, _masks(eng, slice(2 * nP, 3 * nP), P, Xf), Q["D.out.W"], Q["D.out.b"])
    yr = d_forward_masked(Xr, Ws, bs, _masks(eng, slice(nP, 2 * nP), P, Xr), Q["D.out.W"], Q["D.out.b"])
    yi = d_forward_masked(Xi, Ws, bs, _masks(eng, slice(0, nP), P, Xi0), Q["D.out.W"], Q["D.out.b"])
    g = torch.autograd.grad(yi.sum(), Xi, create_graph=True)[0]
    pen = ((g.norm(2, dim=1) - 1) ** 2).mean() * 10.0
    loss = yf.mean() - yr.mean()
    (loss + pen).backward()
    assert abs(eng.metrics[0].item() - loss.item()) < 2e-2 * (1 + abs(loss.item()))
    assert abs(eng.metrics[1].item() - pen.item()) < 2e-2 * (1 + abs(pen.item()))
    for n, t in Q.items():
        if n == "D.out.b":
            assert eng.g[n].abs().max().item() == 0.0
            continue
        assert _rel(eng.g[n], t.grad) < TOL[precision], (n, _rel(eng.g[n], t.grad))


@pytest.mark.parametrize("precision,g_wt,wide,row_mode", [
    ("bf16", False, False, None), ("fp32", False, False, None), ("bf16", True, False, None), ("fp32", True, False, None),
    ("bf16", True, True, None), ("fp32", True, True, None), ("fp32", True, True, 1)])
def test_hip_g_update_matches_autograd(precision, g_wt, wide, row_mode):
    prev = torch.ops.fedtgan.set_tuning("act_row_mode", row_mode) if row_mode is not None else None
    try:
        _g_update_vs_autograd(precision, g_wt, wide)
    finally:
        if prev is not None:
            torch.ops.fedtgan.set_tuning("act_row_mode", prev)


def _g_update_vs_autograd(precision, g_wt, wide):
    eng, tr = _engine(precision, g_wt, wide)
    if wide:
        assert eng._onehot_w_ok(eng.p["G.out.W"])   # the scattered one-hot weight gradients run
    B, nP, Dd = eng.B, eng.nP, eng.Dd
    eng._d_step()
    before = {n: t.detach().clone() for n, t in eng.p.items()}
    eng._g_prepare()
    torch.cuda.synchronize()
    x0 = eng.H[:, eng.off[0]:].clone()
    act_k = eng.Xg[:, :Dd].clone()
    logits_k = eng.logits.clone()
    snap = []
    if wide:
        # the scattered one-hot gradient rows are cleared right after the Adam step: keep a copy to compare
        real = eng.ops.onehot_wgrad

        def spy(dys, ws, *a, zero=False, **k):
            if zero:
                snap.extend((w, w.clone()) for w in ws)
            return real(dys, ws, *a, zero=zero, **k)
        eng.ops.onehot_wgrad = spy
    try:
        eng._g_update()
    finally:
        if wide:
            del eng.ops.onehot_wgrad
    torch.cuda.synchronize()
    assert len(snap) == (len(eng.gdims) + 1 if wide else 0)
    for w, saved in snap:
        w.copy_(saved)
    G = Generator(eng.E + eng.C, eng.gdims, Dd).to(DEV)
    sd = {k: before[n] for k, n in eng.g_key_map()}
    for i in range(len(eng.gdims)):
        sd[f"seq.{i}.bn.num_batches_tracked"] = torch.tensor(0)
    G.load_state_dict(sd)
    G.train()
    logits = G(x0)
    assert _rel(logits, logits_k) < (2e-2 if precision == "bf16" else 1e-4)
    acts = []
    for s, w, k in eng.spans:
        x = logits[:, s:s + w]
        if k == 0:
            acts.append(torch.tanh(x))
        else:
            gn = (0.2 * torch.log(act_k[:, s:s + w].clamp_min(1e-30)) - logits_k[:, s:s + w]).detach()
            acts.append(torch.softmax((x + gn) / 0.2, dim=1))
    c1 = x0[:, eng.E:]
    fake = torch.cat(acts + [c1], dim=1).reshape(nP, eng.K1)
    L = len(eng.ddims)
    P = {n: before[n] for n in before if n.startswith("D.")}
    masks = _masks(eng, slice(0, nP), P, fake.detach())
    y = d_forward_masked(fake, [P[f"D.{i}.W"] for i in range(L)], [P[f"D.{i}.b"] for i in range(L)], masks,
                         P["D.out.W"], P["D.out.b"])
    m1 = torch.zeros(B, eng.layout.n_col, device=DEV)
    m1[torch.arange(B), eng.col.long()] = 1.0
    ce = cond_loss(logits, tr.output_info, c1, m1)
    (-y.mean() + ce).backward()
    assert abs(eng.metrics[3].item() - ce.item()) < 2e-2 * (1 + ce.item())
    gsd = dict(G.named_parameters())
    for k, n in eng.g_key_map():
        if k in gsd and not k.endswith("fc.bias"):
            tol = 8e-2 if precision == "bf16" else 5e-3
            assert _rel(eng.g[n], gsd[k].grad) < tol, (k, _rel(eng.g[n], gsd[k].grad))


def test_side_stream_overlap_is_race_free():
    """The multi-lane step (G prepare || D update, weight-grad GEMMs on side lanes) replays to the
    bitwise-same parameters and optimizer state as the single-stream step."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    out = []
    for streams in (False, True):
        torch.manual_seed(0)
        # (both per-phase: the lanes path draws each phase's batch separately; both with R1 as its own GEMM,
        # as the lanes path does not ride it on R0's reduction launch)
        # (bn_pair off: the lanes path keeps each weight gradient beside its layer's dH product, and only the
        # same GEMM launches give bitwise the same sums)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, streams=streams, paired=False, fuse_d_adam=False,
                                                  bn_pair=False),
                          DEV, backend="hip", seed=5)
        eng.set_training_data(X)
        eng.train_steps(6, use_graph=True)
        torch.cuda.synchronize()
        out.append((eng.flat.clone(), eng.mG.clone(), eng.vD.clone()))
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("batch", [600, 2500])
def test_large_batches_train(batch):
    """Batches past the register-resident BN kernels (paired 2B = 1200 / 5000 rows take the streaming
    BN kernels at 5000): the paired generator pass matches per-batch BatchNorm of its own GEMM output,
    and a few captured steps stay finite."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    torch.manual_seed(0)
    eng = CTGANEngine(tr.layout, EngineConfig(batch_size=batch), DEV, backend="hip", seed=3)
    eng.set_training_data(X)
    rm0 = eng.p["G.0.rm"].clone()
    eng._prepare_paired()
    torch.cuda.synchronize()
    B, g0 = eng.B, eng.gdims[0]
    a = eng.abuf2[0]          # the layer's pre-BN output (the GEMM's scratch)
    out = eng.H2[:, eng.off[1]:eng.off[0]]
    for h in (slice(0, B), slice(B, 2 * B)):
        ref = torch.relu(F.batch_norm(a[h], None, None, eng.p["G.0.gamma"], eng.p["G.0.beta"], True, 0.1, 1e-5))
        assert torch.allclose(out[h], ref, atol=2e-4, rtol=2e-4)
    m0, m1 = a[:B].mean(0), a[B:].mean(0)
    want = 0.81 * rm0 + 0.09 * m0 + 0.1 * m1
    assert torch.allclose(eng.p["G.0.rm"], want, atol=1e-5)
    eng.train_steps(3, use_graph=True)
    torch.cuda.synchronize()
    assert np.isfinite(eng.losses()).all() and bool(torch.isfinite(eng.flat).all())
    assert g0 == out.shape[1]


def test_onehot_generator_matches_dense():
    """EngineConfig.onehot: the generator's conditional block applied as a gather gives the same
    paired forward (logits, BN statistics) and the same generation tables as the dense K range."""
    from fed_tgan_amd.models.samplers import CondTables
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    outs = []
    for oh in (True, False):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, precision="fp32", onehot=oh), DEV, backend="hip",
                          seed=9)
        eng.set_training_data(X)
        eng._prepare_paired()
        eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
        enc = eng.generate_encoded(3000)
        torch.cuda.synchronize()
        outs.append((eng.logits2.clone(), eng.bn_mean2[0].clone(), eng.p["G.1.rv"].clone(), enc))
    (la, ma, va, ea), (lb, mb, vb, eb) = outs
    assert torch.allclose(la, lb, atol=1e-4, rtol=1e-4)
    assert torch.allclose(ma, mb, atol=1e-5, rtol=1e-5) and torch.allclose(va, vb, atol=1e-5, rtol=1e-5)
    assert torch.allclose(ea, eb, atol=1e-3)     # same Philox draws: identical up to GEMM rounding


@pytest.mark.parametrize("n", [40000, 3000, 77])
def test_bf16_generation_is_bit_identical(n):
    """EngineConfig.gen_bf16: generation on a bf16 activation buffer with bf16 weight copies gives
    exactly the fp32-storage path's table (the GEMMs round their staged operands to bf16 either way),
    graph-replayed and eager, including after a weight update (the copies refresh every pass)."""
    from fed_tgan_amd.models.samplers import CondTables
    eng, tr = _engine()
    _, _, _, _, _, _, _, X = small_table()
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    ctr0 = eng.ops.ctr.clone()

    def run(bf16, graph):
        eng.cfg.gen_bf16 = bf16
        eng._gen_graphs, eng._gen_bufs = {}, None
        eng.ops.ctr.copy_(ctr0)
        out = [eng.generate_decoded(n, use_graph=graph) for _ in range(2)]
        assert eng.gen16 == bf16
        return out

    for graph in (True, False):
        ref, got = run(False, graph), run(True, graph)
        for r, g in zip(ref, got):
            assert torch.equal(r, g)
    eng.train_steps(2)       # new weights: a replayed bf16 graph must pick them up
    ref, got = run(False, True), run(True, True)
    assert torch.equal(ref[0], got[0])
    eng.cfg.gen_bf16 = True


def test_input_major_generator_weights_match_row_major():
    """EngineConfig.g_wt: the generator weights stored input-major ([in, out] rows; transposed views
    into the GEMMs, one-hot gathers from contiguous rows) train like the [out, in] layout from the same
    initial weights and Philox draws, and generate bit-identical tables from the same weights (the
    generation copies are built from the same logical values)."""
    from fed_tgan_amd.models.samplers import CondTables
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    cond = CondTables.from_encoded(X, tr.layout)
    engs = []
    for g_wt in (False, True):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, precision="fp32", g_wt=g_wt), DEV, backend="hip",
                          seed=4)
        eng.set_training_data(X)
        eng.set_generation_tables(cond, tr)
        engs.append(eng)
    a, b = engs
    b.load_g_state_dict(a.g_state_dict())
    b.load_d_state_dict(a.d_state_dict())
    assert torch.equal(b.p["G.out.W"], a.p["G.out.W"]) and b.p["G.out.W"].stride(0) == 1
    ga, gb = a.generate_decoded(4000), b.generate_decoded(4000)
    assert torch.equal(ga, gb)
    for e in engs:
        e._prepare_paired()
    torch.cuda.synchronize()
    assert torch.allclose(a.logits2, b.logits2, atol=1e-4, rtol=1e-4)
    for e in engs:       # one step: the layouts differ by GEMM rounding only
        e.train_steps(1, use_graph=False)
    torch.cuda.synchronize()
    lr = a.cfg.lr
    for n in a.p:
        # Adam normalises each element's step: where a gradient is rounding noise around 0 (a hidden
        # Linear's bias before BatchNorm, rarely drawn conditions) the two layouts may step +-lr in
        # either direction, so elements may differ by up to 2 lr per step; the tensors as a whole agree
        assert (a.p[n] - b.p[n]).abs().max() <= 8 * lr + 1e-6, n
        if n.endswith(".W"):     # (vectors that start at 0 / 1 -- biases, BN affine -- moved by ~4 lr only)
            assert _rel(b.p[n], a.p[n]) < 2e-3, (n, _rel(b.p[n], a.p[n]))
    for n in ("G.out.W", "G.0.W", "G.1.W"):
        assert _rel(b.g[n], a.g[n]) < 2e-3, (n, _rel(b.g[n], a.g[n]))
    la, lb = a.losses(), b.losses()
    assert np.allclose(la, lb, rtol=1e-3, atol=1e-4), (la, lb)
    for e in engs:       # a few captured steps: the trajectories stay together (GAN training is chaotic,
        e.train_steps(4, use_graph=True)        # so only loosely)
    torch.cuda.synchronize()
    for n in ("G.out.W", "G.0.W", "G.1.W", "D.0.W"):
        assert _rel(b.p[n], a.p[n]) < 2e-2, (n, _rel(b.p[n], a.p[n]))


@pytest.mark.parametrize("knob", ["fuse_g_adam", "fuse_d_adam", "chain_d1"])
def test_fused_adam_launches_match_separate_launches(knob):
    """EngineConfig.fuse_g_adam: the generator's first-layer weight gradient and the generator's Adam
    in one launch (the GEMM's tiles update their own outputs) give the same gradients, parameters and
    moments as the separate launches (one Adam expression everywhere: bitwise).  fuse_d_adam: the same
    for D1's weight gradient and the D Adam, with R1 computed in fp32 in R0's reduction launch (instead
    of a bf16-operand GEMM): close, not bitwise.  chain_d1: D1's forward in D0's reduction launch (fp32,
    the same Philox dropout masks): close."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    engs = []
    for fuse in (False, True):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, **{knob: fuse}), DEV, backend="hip", seed=6)
        eng.set_training_data(X)
        engs.append(eng)
    a, b = engs
    b.flat.copy_(a.flat)
    for e in engs:
        e.train_steps(1, use_graph=False)
    torch.cuda.synchronize()
    if knob == "fuse_g_adam":
        assert torch.equal(a.g["G.0.W"], b.g["G.0.W"]) and torch.equal(a.g["D.0.W"], b.g["D.0.W"])
        for buf in ("flat", "mG", "vG", "mD", "vD"):       # one Adam expression (adam_elem) in both kernels
            x, y = getattr(a, buf), getattr(b, buf)
            assert torch.equal(x, y), (buf, float((x - y).abs().max()))
    else:
        I = a.rows_i
        assert _rel(b.dl[1][I], a.dl[1][I]) < 1e-2            # R1: fp32 dot products vs bf16 MFMA
        for n in ("D.0.W", "D.1.W", "D.out.W", "D.0.b", "D.1.b"):    # bf16-operand GEMM tolerance (TOL)
            assert _rel(b.g[n], a.g[n]) < TOL["bf16"], (n, _rel(b.g[n], a.g[n]))
        assert torch.equal(a.g["D.0.W"][:, :0], b.g["D.0.W"][:, :0])
        assert (a.flat - b.flat).abs().max() <= 2 * a.cfg.lr + 1e-6
    for e in engs:
        e.train_steps(8, use_graph=True)
    torch.cuda.synchronize()
    assert np.isfinite(b.losses()).all() and bool(torch.isfinite(b.flat).all())


def test_interrupted_hold_does_not_poison_next_step():
    """a raise between gemm(group=3 / 4 / 1) and its consumer must not leave the hold behind."""
    eng, _ = _engine()
    eng.train_steps(1, use_graph=False)
    o = eng.ops
    # hold a weight gradient for the Adam launch and a chain tail, then "fail" before their consumers
    g0 = eng.gdims[0]
    o.gemm(eng.da[0], eng.H[:, :g0], torch.zeros(g0, g0, device=DEV), ta=True, group=3)
    with pytest.raises(RuntimeError):
        o.gemm(eng.A[0], eng.X, eng.g["D.0.W"], ta=True, group=3)     # a second hold is refused
    assert o.reset_held() == 1
    assert o.reset_held() == 0

    def boom(*a, **k):
        raise RuntimeError("injected failure after the hold")
    real_adam = o.adam
    o.adam = boom
    try:
        with pytest.raises(RuntimeError, match="injected"):
            eng.train_steps(1, use_graph=False)
    finally:
        del o.adam
    assert o.adam == real_adam
    assert o.reset_held() == 0          # the engine dropped the hold on the way out
    eng.train_steps(2, use_graph=False)
    eng.train_steps(8)                  # and graph capture still works
    ld, lg = eng.losses()
    assert np.isfinite(ld) and np.isfinite(lg)


def test_onehot_wgrad_matches_dense_gemm():
    """EngineConfig.onehot_wgrad_min: the generator weight gradients' one-hot condition blocks as scattered
    rows (ops.onehot_wgrad) train like the dense GEMMs over the one-hot columns (fp32: same gradients up to
    summation order), and the blocks are all-zero again after every step (the invariant the scatter relies on)."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    engs = []
    for lim in (0, 1):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, precision="fp32", g_wt=True, onehot_wgrad_min=lim),
                          DEV, backend="hip", seed=12)
        eng.set_training_data(X)
        engs.append(eng)
    a, b = engs
    b.flat.copy_(a.flat)
    assert not a._onehot_w_ok(a.g["G.out.W"]) and b._onehot_w_ok(b.g["G.out.W"])
    for e in engs:
        e.train_steps(1, use_graph=False)
    torch.cuda.synchronize()
    C, c0 = b.C, b.c_cols[0]
    for i, n in enumerate(("G.out.W", "G.0.W", "G.1.W")):
        a_ = 0 if n == "G.out.W" else b.off[int(n[2])]
        kd = c0 - a_
        assert b.g[n][:, kd:].abs().max().item() == 0.0, n          # cleared after the Adam step
        assert torch.allclose(b.g[n][:, :kd], a.g[n][:, :kd], atol=1e-6, rtol=1e-4), n
    lr = a.cfg.lr
    for n in a.p:
        assert (a.p[n] - b.p[n]).abs().max() <= 8 * lr + 1e-6, n
    for e in engs:
        e.train_steps(8, use_graph=True)
    torch.cuda.synchronize()
    for n in ("G.out.W", "G.0.W", "G.1.W", "D.0.W"):
        assert _rel(b.p[n], a.p[n]) < 2e-2, (n, _rel(b.p[n], a.p[n]))
    for n in ("G.out.W", "G.0.W", "G.1.W"):
        a_ = 0 if n == "G.out.W" else b.off[int(n[2])]
        assert b.g[n][:, c0 - a_:].abs().max().item() == 0.0, n


def test_chain_tail_coalesced_matches_row_per_lane():
    """set_tuning("chain_coalesced"): the chained tail GEMM (D1 forward / R1 link in D0's / R0's reduction launch)
    with lane-contiguous weight rows + wave sums gives the same outputs as one weight row per lane (fp32 dot
    products in a different order: close), and a step with it trains the same parameters within rounding."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    res = []
    for co in (0, 1):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, precision="fp32"), DEV, backend="hip", seed=14)
        eng.set_training_data(X)
        prev = torch.ops.fedtgan.set_tuning("chain_coalesced", co)
        try:
            eng.train_steps(1, use_graph=False)
            torch.cuda.synchronize()
            res.append((eng.dl[1].clone(), eng.flat.clone()))
            eng.train_steps(8, use_graph=True)
            torch.cuda.synchronize()
            assert bool(torch.isfinite(eng.flat).all())
        finally:
            torch.ops.fedtgan.set_tuning("chain_coalesced", prev)
    (d0, f0), (d1, f1) = res
    assert torch.allclose(d0, d1, atol=1e-5, rtol=1e-4), float((d0 - d1).abs().max())
    assert (f0 - f1).abs().max().item() <= 2 * 2e-4 + 1e-6


@pytest.mark.parametrize("batch", [500, 510])
def test_chain_tail_prefetch_matches_plain(batch):
    """set_tuning("chain_pre" / "chain_rows"): the chained tail with its weights prefetched before the slab
    reduction, one head row per workgroup (the 50-row G-phase / R chains) or two (the 150-row D phase; batch 510:
    153 rows, an odd last pair), gives the outputs of the plain tail (same products, same order: bitwise) and a
    step with it trains the same parameters."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    res = []
    for pre, rows in ((0, 1), (1, 1), (1, 2), (2, 1)):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=batch, precision="fp32"), DEV, backend="hip", seed=14)
        eng.set_training_data(X)
        p0 = torch.ops.fedtgan.set_tuning("chain_pre", pre)
        r0 = torch.ops.fedtgan.set_tuning("chain_rows", rows)
        try:
            eng.train_steps(1, use_graph=False)
            torch.cuda.synchronize()
            res.append((eng.dl[1].clone(), eng.flat.clone()))
            eng.train_steps(8, use_graph=True)
            torch.cuda.synchronize()
            assert bool(torch.isfinite(eng.flat).all())
        finally:
            torch.ops.fedtgan.set_tuning("chain_pre", p0)
            torch.ops.fedtgan.set_tuning("chain_rows", r0)
    d0, f0 = res[0]
    for d, f in res[1:]:
        assert torch.equal(d, d0), float((d - d0).abs().max())
        assert torch.equal(f, f0), float((f - f0).abs().max())


def test_pending_achain_is_checked_and_dropped():
    """gemm_achain_next refuses operands the kernel cannot use, and a pending configuration is consumed by the next
    chain tail or dropped by reset_held -- never applied to a later, unrelated GEMM."""
    from fed_tgan_amd.ops import native
    L = native.require()
    f = lambda *s: torch.zeros(*s, device=DEV)  # noqa: E731
    cnt = torch.zeros(10, dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError):
        L.gemm_achain_next(f(10, 256), f(4 * 10 * 256), cnt.float())       # counters must be int32
    L.gemm_achain_next(f(10, 256), f(4 * 10 * 256), cnt)
    from fed_tgan_amd.ops.hip import HipOps
    with pytest.raises(RuntimeError):
        HipOps(DEV).gemm(f(10, 8), f(4, 8), f(10, 4), tb=True)    # not a chain tail: refused, still pending
    assert L.reset_held() == 1 and L.reset_held() == 0


@pytest.mark.gpu
def test_multi_draw_matches_per_step_sampler():
    """EngineConfig.multi_draw: the step graph's one sampler launch for all graph_unroll steps (buffer set k, RNG
    step ctr + k, per-step optimizer counters) trains bitwise like a sampler launch per step -- over two graph
    replays plus a leftover single step, with the canonical counters and last-step losses where the per-step path
    leaves them."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    out = []
    for multi in (False, True):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, multi_draw=multi, graph_unroll=4), DEV,
                          backend="hip", seed=7)
        assert eng._multi == multi
        eng.set_training_data(X)
        eng.train_steps(9, use_graph=True)      # 2 x 4-step graph + 1 single step
        eng.train_steps(1, use_graph=False)     # and one eager step on the canonical binding
        torch.cuda.synchronize()
        out.append((eng.flat.clone(), eng.mG.clone(), eng.vD.clone(), eng.stepD.clone(), eng.stepG.clone(),
                    eng.metrics.clone(), eng.ops.ctr.clone()))
    for name, a, b in zip(("flat", "mG", "vD", "stepD", "stepG", "metrics", "ctr"), *out):
        if name == "metrics":     # (the WGAN terms are float atomics across workgroups: order-dependent last bits)
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
        else:
            assert torch.equal(a, b), name
    assert float(out[1][3]) == 10.0 and float(out[1][4]) == 10.0


@pytest.mark.gpu
def test_bn_pair_matches_unpaired():
    """EngineConfig.bn_pair (BN backward + the weight gradient of the layer above in one launch, csrc
    gemm_bnbwd_kernel) computes the same G update as the default schedule (fp32: to summation order)."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    out = []
    for bp in (False, True):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, precision="fp32", bn_pair=bp), DEV, backend="hip",
                          seed=4)
        eng.set_training_data(X)
        eng.train_steps(2, use_graph=False)
        torch.cuda.synchronize()
        out.append((eng.flat.clone(), eng.gradG.clone()))
    torch.testing.assert_close(out[1][1], out[0][1], rtol=1e-4, atol=1e-6)
    torch.testing.assert_close(out[1][0], out[0][0], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_fused_achain_matches_gemm_chain():
    """EngineConfig.fuse_achain (A0 = (A1 W1) . MS0 formed in D0's chain launch from per-slab partials,
    csrc/kernels/gemm.hip chain_epilogue_kernel<..., ACH>) gives the D and G updates of the separate A-chain GEMM
    (fp32: to summation order), and is deterministic (slabs summed in a fixed order)."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    out = []
    for fa in (False, True, True):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, precision="fp32", fuse_achain=fa), DEV,
                          backend="hip", seed=5)
        assert bool(eng._ach) == fa
        eng.set_training_data(X)
        eng.train_steps(3, use_graph=False)
        torch.cuda.synchronize()
        out.append((eng.flat.clone(), eng.gradD.clone(), eng.gradG.clone(), eng.A[0].clone()))
    for k in range(4):
        torch.testing.assert_close(out[1][k], out[0][k], rtol=1e-4, atol=1e-5 if k == 0 else 1e-6)
        assert torch.equal(out[1][k], out[2][k]), k


@pytest.mark.gpu
def test_multi_block_graph_matches_block_graphs():
    """EngineConfig.graph_blocks: B blocks of graph_unroll steps captured in ONE hipGraph (each block with its own
    multi-step sampler launch) train bitwise like one graph per block -- over a 2-block graph, a leftover block and
    leftover single steps."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    out = []
    for blocks in (1, 2):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, graph_unroll=4, graph_blocks=blocks), DEV,
                          backend="hip", seed=7)
        eng.set_training_data(X)
        assert eng._graph_blocks() == blocks
        eng.train_steps(14, use_graph=True)      # 8 (one 2-block graph or two block graphs) + 4 + 2 single
        torch.cuda.synchronize()
        assert (8 in eng.graphs) == (blocks == 2)
        out.append((eng.flat.clone(), eng.mD.clone(), eng.vG.clone(), eng.stepD.clone(), eng.ops.ctr.clone()))
    for name, a, b in zip(("flat", "mD", "vG", "stepD", "ctr"), *out):
        assert torch.equal(a, b), name
    assert float(out[1][3]) == 14.0


def test_lead_event_marks_before_last_blocks():
    """train_steps(..., lead=N) (FedConfig.sync_lead_blocks): an event recorded before the last N graph blocks;
    the training itself is bitwise the same as without it."""
    from fed_tgan_amd.ops import native
    native.require()
    _, _, _, _, _, _, tr, X = small_table()
    out = []
    for lead in (0, 1):
        torch.manual_seed(0)
        eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500, graph_unroll=4), DEV, backend="hip", seed=7)
        eng.set_training_data(X)
        eng.train_steps(12, use_graph=True, lead=lead)
        assert (eng.lead_event is not None) == (lead > 0)
        if lead:
            eng.lead_event.synchronize()
        torch.cuda.synchronize()
        out.append((eng.flat.clone(), eng.ops.ctr.clone()))
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
