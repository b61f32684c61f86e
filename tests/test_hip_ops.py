"""Numerics of every HIP kernel against the eager-PyTorch fp32 reference (TorchOps) of the same op."""
import math

import numpy as np
import pytest
import torch

from fed_tgan_amd.ops.ref import TorchOps

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def hip():
    from fed_tgan_amd.ops import native
    from fed_tgan_amd.ops.hip import HipOps
    native.require()
    return HipOps(DEV, seed=1234)


REF = TorchOps()


def bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def mat(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(DEV)


@pytest.fixture(scope="module")
def hip32():
    from fed_tgan_amd.ops.hip import HipOps
    return HipOps(DEV, seed=1234, precision="fp32")


@pytest.mark.parametrize("tile", [128, 64, 32])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(150, 256, 6240), (50, 6240, 256), (500, 323, 941), (7, 5, 3), (256, 430, 500),
                                   (500, 256, 432)])
def test_gemm_layouts(hip, hip32, ta, tb, M, N, K, tile):
    hip.tile_override = hip32.tile_override = tile
    a = mat(*((K, M) if ta else (M, K)), seed=1)
    b = mat(*((N, K) if tb else (K, N)), seed=2)
    bias = mat(N, seed=3)
    ref32 = (a.double().t() if ta else a.double()) @ (b.double().t() if tb else b.double()) + bias.double()
    # bf16 operands: equal to the fp32 product of the bf16-rounded inputs
    c = torch.zeros(M, N, device=DEV)
    hip.gemm(a, b, c, ta=ta, tb=tb, bias=bias)
    A = bf(a).t() if ta else bf(a)
    B = bf(b).t() if tb else bf(b)
    ref = A @ B + bias
    torch.cuda.synchronize()
    assert (c - ref).abs().max().item() <= 1e-4 * math.sqrt(K) * 10 + 1e-5
    assert (c.double() - ref32).abs().max().item() < 4e-3 * math.sqrt(K) * 6 + 1e-3   # bf16 input rounding
    # exact-fp32 MFMA path: fp32 rounding only
    c32 = torch.zeros(M, N, device=DEV)
    hip32.gemm(a, b, c32, ta=ta, tb=tb, bias=bias)
    torch.cuda.synchronize()
    hip.tile_override = hip32.tile_override = None
    assert (c32.double() - ref32).abs().max().item() < 2e-6 * K + 1e-5


def test_gemm_strided_views_alpha_beta_mask(hip):
    big_a = mat(200, 900, seed=4)
    a = big_a[:, 100:600]                      # column slice, ld = 900
    b = mat(64, 500, seed=5)
    cbuf = mat(200, 80, seed=6)
    c = cbuf[:, 8:72]
    ms = (torch.rand(200, 64, device=DEV) > 0.5).float() * 2.0
    c0 = c.clone()
    hip.gemm(a, b, c, tb=True, alpha=0.5, beta=1.0, epi=2, ms=ms)
    ref = (0.5 * (bf(a) @ bf(b).t()) + c0) * ms
    torch.cuda.synchronize()
    assert torch.allclose(c, ref, atol=2e-3, rtol=1e-4)
    assert torch.equal(cbuf[:, :8], mat(200, 80, seed=6)[:, :8])      # untouched outside the view


def test_gemm_lrelu_dropout(hip):
    a = mat(150, 600, seed=7)
    b = mat(256, 600, seed=8)
    bias = mat(256, seed=9)
    c = torch.zeros(150, 256, device=DEV)
    ms = torch.zeros_like(c)
    hip.gemm(a, b, c, tb=True, bias=bias, epi=1, ms=ms, slope=0.2, p_drop=0.5)
    pre = bf(a) @ bf(b).t() + bias
    torch.cuda.synchronize()
    s = torch.where(pre > 0, torch.ones_like(pre), torch.full_like(pre, 0.2))
    keep = ms / s
    ok = (keep.sub(0).abs() < 1e-6) | (keep.sub(2).abs() < 1e-5)
    # sign of pre-activation can differ from the kernel's only for |pre| ~ rounding noise
    assert ok.float().mean().item() > 0.999
    frac = (ms != 0).float().mean().item()
    assert 0.45 < frac < 0.55
    assert torch.allclose(c, pre * ms, atol=3e-3, rtol=1e-3)


def test_gemm_bn_eval_relu(hip):
    x = mat(300, 200, seed=10)
    W = mat(64, 200, seed=11)
    b = mat(64, seed=12)
    gamma, beta = torch.rand(64, device=DEV) + 0.5, mat(64, seed=13)
    rm, rv = mat(64, seed=14), torch.rand(64, device=DEV) + 0.5
    out = torch.zeros(300, 64, device=DEV)
    hip.linear_bn_relu(x, W, b, gamma, beta, out, None, None, None, None, rm, rv, training=False)
    ref = torch.relu((bf(x) @ bf(W).t() + b - rm) * torch.rsqrt(rv + 1e-5) * gamma + beta)
    torch.cuda.synchronize()
    assert torch.allclose(out, ref, atol=2e-3, rtol=1e-3)


@pytest.mark.parametrize("rows,scale,offset,threads", [(500, 3.0, 1.0, 512), (37, 3.0, 1.0, 512), (500, 0.05, 50.0, 512),
                                                      (5000, 3.0, 1.0, 512), (1000, 3.0, 1.0, 1024), (500, 0.05, 50.0, 1024)])
def test_bn_relu_train_and_bwd(hip, rows, scale, offset, threads):
    # the (0.05, 50) case: tiny spread around a large mean -- the one-pass shifted statistics
    # must not lose the variance to cancellation.  threads: the BN workgroup size (set_tuning("bn_threads"))
    prev_t = torch.ops.fedtgan.set_tuning("bn_threads", threads)
    try:
        _bn_train_and_bwd(hip, rows, scale, offset)
    finally:
        torch.ops.fedtgan.set_tuning("bn_threads", prev_t)


def _bn_train_and_bwd(hip, rows, scale, offset):
    a = mat(rows, 300, seed=15) * scale + offset
    gamma, beta = torch.rand(300, device=DEV) + 0.5, mat(300, seed=16)
    fwd = {}
    for name, ops in (("hip", hip), ("ref", REF)):
        out = torch.zeros(rows, 300, device=DEV)
        nhat = torch.zeros_like(out)
        mean, inv = torch.zeros(300, device=DEV), torch.zeros(300, device=DEV)
        rm, rv = torch.zeros(300, device=DEV), torch.ones(300, device=DEV)
        ops.bn_relu_fwd(a, gamma, beta, out, nhat, mean, inv, rm, rv, True, 0.1, 1e-5)
        fwd[name] = (out, nhat, mean, inv, rm, rv)
    # the backward of both runs on the SAME (reference) forward tensors: a forward output within
    # rounding of 0 may sit on either side of the ReLU and flip its mask
    out, nhat, _, inv, _, _ = fwd["ref"]
    bwd = {}
    for name, ops in (("hip", hip), ("ref", REF)):
        dr = mat(rows, 300, seed=17)
        da = torch.zeros_like(out)
        dg, db, dbias = torch.zeros(300, device=DEV), torch.zeros(300, device=DEV), torch.zeros(300, device=DEV)
        ops.bn_relu_bwd(dr, out, nhat, gamma, inv, da, dg, db, dbias)
        bwd[name] = (da, dg, db, dbias)
    torch.cuda.synchronize()
    names = ("out", "nhat", "mean", "inv", "rm", "rv", "da", "dg", "db", "dbias")
    for nm, x, y in zip(names, fwd["hip"] + bwd["hip"], fwd["ref"] + bwd["ref"]):
        if offset < 10:
            assert torch.allclose(x, y, atol=2e-4, rtol=2e-4), nm
        else:
            # ill-conditioned input (inv std ~20 amplifies fp32 rounding of x ~ 50 in both
            # implementations): compare against each tensor's own scale
            # (dbias = sum_r da is ~0 by construction -- rounding noise -- so it is measured on
            # the scale of da itself)
            scale = (bwd["ref"][0] if nm == "dbias" else y).abs().max().clamp_min(1e-6)
            err = float((x - y).abs().max() / scale)
            assert err < 2e-3, (nm, err)


def test_adam_matches_torch(hip):
    n = 1003
    p = mat(n, seed=18)
    g = mat(n, seed=19)
    tp = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([tp], lr=2e-4, betas=(0.5, 0.9), weight_decay=1e-6)
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    step = torch.zeros(1, device=DEV)
    for it in range(3):
        gi = g * (it + 1)
        step += 1
        hip.adam(p, gi, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 1e-6)
        tp.grad = gi.clone()
        opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, tp.detach(), atol=1e-6, rtol=1e-5)


def test_gp_scale_dhead_colsum(hip):
    g = mat(50, 6240, seed=20) * 0.01
    o1, o2 = torch.zeros_like(g), torch.zeros_like(g)
    l1, l2 = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    hip.gp_scale(g, o1, 10.0, l1)
    REF.gp_scale(g, o2, 10.0, l2)
    d = mat(150, 256, seed=21)
    ms = (torch.rand(150, 256, device=DEV) > 0.5).float() * 2
    v, e = mat(256, seed=22), mat(1, seed=23)
    coef = torch.cat([torch.full((50,), 0.02), torch.full((50,), -0.02), torch.ones(50)]).to(DEV)
    wl = torch.cat([torch.full((50,), 0.02), torch.full((50,), -0.02), torch.zeros(50)]).to(DEV)
    y1, y2 = torch.zeros(150, device=DEV), torch.zeros(150, device=DEV)
    a1, a2 = torch.zeros_like(d), torch.zeros_like(d)
    m1, m2 = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    hip.d_head(d, ms, v, e, coef, wl, y1, a1, m1)
    REF.d_head(d, ms, v, e, coef, wl, y2, a2, m2)
    c1, c2 = torch.zeros(256, device=DEV), torch.zeros(256, device=DEV)
    hip.colsum_many([d[:100]], [c1])
    REF.colsum_many([d[:100]], [c2])
    torch.cuda.synchronize()
    assert torch.allclose(o1, o2, atol=1e-6, rtol=1e-4) and torch.allclose(l1, l2, rtol=1e-4)
    assert torch.allclose(y1, y2, atol=1e-4) and torch.allclose(a1, a2) and torch.allclose(m1, m2, atol=1e-4)
    assert torch.allclose(c1, c2, atol=1e-4)


def _spans():
    from helpers import small_table
    _, _, _, _, _, _, tr, X = small_table()
    spans = [(int(s), int(w), int(k)) for s, w, k in zip(tr.layout.start, tr.layout.width, tr.layout.kind)]
    cond = [(int(s), int(w)) for s, w in zip(tr.layout.cond_start, tr.layout.cond_width)]
    return tr, X, spans, cond


def test_activate_statistics(hip):
    tr, X, spans, cond = _spans()
    rows = 20000
    base = mat(1, tr.layout.data_dim, seed=24) * 2
    logits = base.repeat(rows, 1)
    o1, o2 = torch.zeros_like(logits), torch.zeros_like(logits)
    hip.activate(logits, o1, spans, 0.2)
    REF.activate(logits, o2, spans, 0.2)
    torch.cuda.synchronize()
    for s, w, k in spans:
        if k == 0:
            assert torch.allclose(o1[:, s], torch.tanh(logits[:, s]), atol=1e-6)
        else:
            assert torch.allclose(o1[:, s:s + w].sum(1), torch.ones(rows, device=DEV), atol=1e-5)
            # Gumbel-softmax mean vector agrees between kernel and torch.rand-based reference
            assert (o1[:, s:s + w].mean(0) - o2[:, s:s + w].mean(0)).abs().max().item() < 0.02


def test_act_bwd_ce_matches_reference(hip):
    tr, X, spans, cond = _spans()
    B = 500
    logits = mat(B, tr.layout.data_dim, seed=25)
    act = torch.zeros_like(logits)
    REF.activate(logits, act, spans, 0.2)
    dact = mat(B, tr.layout.data_dim, seed=26)
    col = torch.randint(0, len(cond), (B,), device=DEV, dtype=torch.int32)
    w = torch.tensor([w for _, w in cond], device=DEV)[col.long()]
    opt = (torch.rand(B, device=DEV) * w).floor().to(torch.int32)
    d1, d2 = torch.zeros_like(logits), torch.zeros_like(logits)
    l1, l2 = torch.zeros(1, device=DEV), torch.zeros(1, device=DEV)
    hip.act_bwd_ce(dact, act, logits, spans, cond, col, opt, d1, l1, 0.2)
    REF.act_bwd_ce(dact, act, logits, spans, cond, col, opt, d2, l2, 0.2)
    torch.cuda.synchronize()
    assert torch.allclose(d1, d2, atol=1e-5, rtol=1e-4)
    assert torch.allclose(l1, l2, rtol=1e-4)


def test_slerp_on_arc(hip):
    real = mat(300, 620, seed=27)
    fake = mat(300, 620, seed=28)
    out = torch.zeros_like(real)
    hip.slerp(real, fake, out)
    torch.cuda.synchronize()
    r, f, o = real.double(), fake.double(), out.double()
    # solve out = wa*real + wb*fake per row and check the slerp relation for some alpha in [0,1]
    A = torch.stack([r, f], 2)
    sol = torch.linalg.lstsq(A, o.unsqueeze(2)).solution.squeeze(2)
    cos = (r / r.norm(dim=1, keepdim=True) * f / f.norm(dim=1, keepdim=True)).sum(1).clamp(-1, 1)
    om = torch.acos(cos)
    # on the arc: wa = sin((1-a)om)/sin(om), wb = sin(a om)/sin(om)  <=>  (wa + wb cos om, wb sin om) is the
    # unit vector at angle a*om, so its norm is 1 and its angle gives a
    wa, wb = sol[:, 0], sol[:, 1]
    u, v = wa + wb * torch.cos(om), wb * torch.sin(om)
    assert torch.allclose(u * u + v * v, torch.ones_like(u), atol=2e-3)
    alpha = torch.atan2(v, u) / om
    assert (alpha >= -1e-3).all() and (alpha <= 1 + 1e-3).all()
    assert 0.35 < alpha.mean().item() < 0.65


def test_sampler_statistics(hip):
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    tr, X, spans, cond = _spans()
    eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500), DEV, backend="hip", seed=5)
    eng.set_training_data(X)
    B, Dd, C = eng.B, eng.Dd, eng.C
    counts = np.zeros((tr.layout.n_col, eng.tables["cdf_log"].shape[1]))
    for it in range(40):
        eng.ops.sample_train(eng.tables, eng.H, eng.z_cols, eng.c_cols, eng.X_fake, eng.X_real, Dd, eng.col,
                             eng.opt, stream_id=1)
        eng.ops.L.rng_bump(eng.ops.ctr)
        torch.cuda.synchronize()
        col, opt = eng.col.cpu().numpy(), eng.opt.cpu().numpy()
        np.add.at(counts, (col, opt), 1)
        c1 = eng.H[:, eng.c_cols[0]:eng.c_cols[1]]
        assert torch.equal(c1.sum(1), torch.ones(B, device=DEV))
        assert torch.equal(eng.X_fake[:, Dd:], c1)
        # real rows carry the permuted condition and agree with it
        c2 = eng.X_real[:, Dd:]
        assert torch.equal(c2.sum(0), c1.sum(0))
        hot = c2.argmax(1).cpu().numpy()
        real = eng.X_real[:, :Dd].cpu().numpy()
        offs = tr.layout.cond_offset
        for b in range(0, B, 7):
            cc = np.searchsorted(offs, hot[b], side="right") - 1
            o = hot[b] - offs[cc]
            assert real[b, tr.layout.cond_start[cc] + o] == 1.0
    z = eng.H[:, eng.z_cols[0]:eng.z_cols[1]]
    assert abs(z.mean().item()) < 0.05 and abs(z.std().item() - 1) < 0.05
    # option frequencies follow the log-frequency CDF (chi-square-ish tolerance)
    p = np.diff(np.concatenate([np.zeros((counts.shape[0], 1)), eng.tables["cdf_log"].cpu().numpy()], 1), axis=1)
    tot = counts.sum(1, keepdims=True)
    assert np.abs(tot.ravel() / tot.sum() - 1.0 / len(tot)).max() < 0.01
    assert np.abs(counts / np.maximum(tot, 1) - p).max() < 0.08


def test_sample_decode_deterministic_argmax(hip):
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from fed_tgan_amd.models.samplers import CondTables
    tr, X, spans, cond = _spans()
    eng = CTGANEngine(tr.layout, EngineConfig(), DEV, backend="hip", seed=5)
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    rows = 64
    enc = torch.as_tensor(X[:rows], device=DEV)
    logits = torch.where(enc > 0.5, torch.full_like(enc, 60.0), torch.zeros_like(enc))
    # tanh units: set logit = atanh(alpha)
    for s, w, k in spans:
        if k == 0:
            logits[:, s] = torch.atanh(enc[:, s].clamp(-0.99, 0.99))
    out = torch.zeros(rows, len(tr.meta), dtype=torch.float64, device=DEV)
    eng.ops.sample_decode(logits, out, eng.gen_tables)
    torch.cuda.synchronize()
    ref = tr.inverse_transform(X[:rows])
    assert np.allclose(out.cpu().numpy(), ref, rtol=1e-4, atol=1e-3)


def test_vgm_encode_matches_host(hip):
    """HIP VGM encode vs the numpy transform: exact categorical one-hots, exact alpha for the
    drawn mode, mode frequencies = mean posterior, and device row lists = host RowIndex."""
    from fed_tgan_amd.features.encode_gpu import encode_on_device
    from fed_tgan_amd.features.transformer import CONTINUOUS
    from fed_tgan_amd.models.samplers import CondTables, RowIndex
    from helpers import small_table
    _, _, _, _, _, enc, tr, X = small_table(4000, 3)
    d = encode_on_device(tr, enc, DEV, seed=7)
    torch.cuda.synchronize()
    D = d.data.cpu().numpy()
    assert D.shape == X.shape
    probs = tr.mode_probs(enc)                                 # [N, n_cont, K]
    pos, c = 0, 0
    for j, m in enumerate(tr.meta):
        if m["type"] == CONTINUOUS:
            valid = np.nonzero(tr.components[c])[0]
            nv = len(valid)
            oh = D[:, pos + 1:pos + 1 + nv]
            assert np.all(oh.sum(1) == 1.0)
            k = valid[oh.argmax(1)]
            mu, sd = tr.bank.means[c][k], tr.bank.stds[c][k]
            alpha = np.clip((enc[:, j] - mu) / (4 * sd), -0.99, 0.99)
            assert np.allclose(D[:, pos], alpha, atol=2e-5)
            freq = oh.mean(0)
            expect = probs[:, c, valid].mean(0)
            assert np.abs(freq - expect).max() < 0.03, (j, freq, expect)
            pos += 1 + nv
            c += 1
        else:
            w = int(m["size"])
            assert np.array_equal(D[:, pos:pos + w], X[:, pos:pos + w])
            pos += w
    host_rows = RowIndex(D, tr.layout)
    assert np.array_equal(d.rows["row_count"].cpu().numpy(), host_rows.count)
    assert np.array_equal(d.rows["row_offset"].cpu().numpy(), host_rows.offset)
    assert np.array_equal(d.rows["rows"].cpu().numpy(), host_rows.rows)
    assert np.array_equal(d.counts, CondTables.span_counts(D, tr.layout))


def test_vgm_fit_hip_passes_match_torch(hip):
    """The HIP E-step / k-means passes give the same fit as the torch passes (same seeding)."""
    from fed_tgan_amd.features.vgm_fit import fit_vgm_torch
    rng = np.random.default_rng(0)
    cols = [np.concatenate([rng.normal(0, 1, 3000), rng.normal(8, 0.5, 2000)]), rng.exponential(3, 4500),
            rng.normal(100, 10, 5000), np.round(rng.lognormal(2, 1, 4000))]
    a = fit_vgm_torch(cols, seed=1, device=DEV, use_hip=True, fused=False)
    b = fit_vgm_torch(cols, seed=1, device=DEV, use_hip=False)
    for f in ("wc_a", "wc_b", "mean_precision", "means", "dof", "covariances"):
        np.testing.assert_allclose(getattr(a, f), getattr(b, f), rtol=1e-5, atol=1e-7, err_msg=f)
    np.testing.assert_allclose(a.weights, b.weights, atol=1e-6)
    # the fused whole-fit kernel from the same k-means centres: the same EM trajectory on the device
    cen = np.stack([np.sort(np.quantile(c, np.linspace(0.05, 0.95, 10))) + 1e-3 * np.arange(10) for c in cols])
    f = fit_vgm_torch(cols, seed=1, device=DEV, init_centers=cen)
    t = fit_vgm_torch(cols, seed=1, device="cpu", init_centers=cen)
    for fld in ("wc_a", "wc_b", "mean_precision", "means", "dof", "covariances"):
        np.testing.assert_allclose(getattr(f, fld), getattr(t, fld), rtol=1e-5, atol=1e-7, err_msg=fld)
    # and from its own device k-means++ seeding: a converged, valid fit
    own = fit_vgm_torch(cols, seed=1, device=DEV)
    assert np.isfinite(own.means).all() and (own.covariances > 0).all()
    assert np.allclose(own.weights.sum(1), 1.0)


def test_gemm_head_seed_and_weighted_colsum(hip):
    """The D head folded into other launches: the last layer's LeakyReLU+dropout epilogue writes
    A_{L-1} = coef v^T * MS, and the bias-gradient launch computes weighted column sums and the
    WGAN value sum_r w_r (d_r . v + e)."""
    M, N, K = 150, 256, 300
    a, b = mat(M, K, seed=40), mat(N, K, seed=41)
    bias = mat(1, N, seed=42).view(-1).contiguous()
    coef = mat(M, 1, seed=43).view(-1).contiguous()
    v = mat(N, 1, seed=44).view(-1).contiguous()
    out, ms, A = (torch.zeros(M, N, device=DEV) for _ in range(3))
    hip.gemm(a, b, out, tb=True, bias=bias, epi=1, ms=ms, head=(coef, v, A))
    torch.cuda.synchronize()
    assert torch.allclose(A, coef.view(-1, 1) * v.view(1, -1) * ms, atol=1e-6, rtol=1e-6)
    w = mat(M, 1, seed=45).view(-1).contiguous()
    e = torch.tensor([0.3], device=DEV)
    loss = torch.zeros(1, device=DEV)
    og = torch.zeros(N, device=DEV)
    plain = torch.zeros(N, device=DEV)
    hip.colsum_many([out, out, out], [og, None, plain], weights=[w, w, None], dots=[None, (v, e, loss), None])
    torch.cuda.synchronize()
    s = (out.double() * w.double().view(-1, 1)).sum(0)
    assert torch.allclose(og.double(), s, atol=1e-3, rtol=1e-4)
    assert torch.allclose(plain.double(), out.double().sum(0), atol=1e-3, rtol=1e-4)
    ref = (s * v.double()).sum() + 0.3 * w.double().sum()
    assert abs(loss.item() - ref.item()) < 1e-3 * (1 + abs(ref.item()))


def test_activate_with_fused_slerp_matches_standalone(hip):
    """The slerp fused onto the fake rows' activation = activation, then the standalone slerp
    kernel (same Philox stream, same weights)."""
    tr, X, spans, cond = _spans()
    B, Dd = 256, tr.layout.data_dim
    Din = Dd + 40
    logits = mat(B, Dd, seed=50)
    xd = mat(3 * B, Din, seed=51)          # [fake | real | interp] blocks; fake cond columns random
    fake, real, interp = xd[0:B], xd[B:2 * B], xd[2 * B:]
    xd2 = xd.clone()
    hip.activate(logits, fake[:, :Dd], spans, 0.2, stream_id=2, slerp=(real, fake, interp, 3))
    hip.activate(logits, xd2[0:B, :Dd], spans, 0.2, stream_id=2)
    hip.slerp(xd2[B:2 * B], xd2[0:B], xd2[2 * B:], stream_id=3)
    torch.cuda.synchronize()
    assert torch.equal(fake, xd2[0:B])
    assert torch.allclose(interp, xd2[2 * B:], atol=2e-6, rtol=1e-5)


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(500, 325, 943), (150, 254, 6263), (37, 61, 150)])
def test_gemm_padded_views_use_vector_loads(hip, ta, tb, M, N, K):
    """Operands that are column views of 4-padded storage (odd logical widths, as the engine's
    padded buffers are) take the 16-B load path; the padding must never leak into the result."""
    def padded(r, c, seed):
        base = torch.full((r, (c + 3) // 4 * 4), float("nan"), device=DEV)   # poison the padding
        base[:, :c] = mat(r, c, seed=seed)
        return base[:, :c]
    a = padded(*((K, M) if ta else (M, K)), seed=61)
    b = padded(*((N, K) if tb else (K, N)), seed=62)
    c = torch.zeros(M, N, device=DEV)
    for tile in (32, 64):
        hip.tile_override = tile
        hip.gemm(a, b, c, ta=ta, tb=tb)
        torch.cuda.synchronize()
        A = bf(a).t() if ta else bf(a)
        B = bf(b).t() if tb else bf(b)
        assert torch.isfinite(c).all()
        assert (c - A @ B).abs().max().item() <= 1e-4 * math.sqrt(K) * 10 + 1e-5
    hip.tile_override = None


@pytest.mark.parametrize("cols,split,threads", [(6260, 1, 256), (6259, 1, 256), (40, 1, 256), (137800, 1, 256),
                                               (137800, 0, 256), (20004, 1, 256), (6280, 1, 1024), (40, 1, 1024)])
def test_gp_scale_per_row_terms(hip, cols, split, threads):
    """Vector (16-B, register-resident), scalar, one-workgroup-per-row wide and chunk-split wide (two launches,
    set_tuning("gp_split")) variants; per-pack loss terms sum to the penalty."""
    g = mat(50, cols, seed=30) * (0.02 if cols < 10000 else 0.004)
    o1, o2 = torch.zeros_like(g), torch.zeros_like(g)
    rows1 = torch.zeros(50, device=DEV)
    l2 = torch.zeros(1, device=DEV)
    prev = torch.ops.fedtgan.set_tuning("gp_split", split)
    prev_t = torch.ops.fedtgan.set_tuning("gp_threads", threads)
    try:
        hip.gp_scale(g, o1, 10.0, rows1)
    finally:
        torch.ops.fedtgan.set_tuning("gp_split", prev)
        torch.ops.fedtgan.set_tuning("gp_threads", prev_t)
    REF.gp_scale(g, o2, 10.0, l2)
    torch.cuda.synchronize()
    assert torch.allclose(o1, o2, atol=1e-6, rtol=1e-4)
    assert torch.allclose(rows1.sum(), l2[0], rtol=1e-4)


@pytest.mark.parametrize("splits", [2, 5, 8, 13, 16, 25, 40, 64, 100])
def test_gemm_split_counts(hip, splits):
    """Every split-K epilogue variant (register-held slabs: <= 8 / 16 / 32 / 64 splits; requests
    above 64 are capped) reduces all slabs and applies the epilogue."""
    a, b = mat(50, 9000, seed=40) * 0.1, mat(256, 9000, seed=41) * 0.1
    bias = mat(256, seed=42)
    c = torch.zeros(50, 256, device=DEV)
    hip.split_override = splits
    try:
        hip.gemm(a, b, c, tb=True, bias=bias, epi=3)    # EPI_RELU
    finally:
        hip.split_override = None
    torch.cuda.synchronize()
    ref = torch.relu(a.double() @ b.double().t() + bias.double()).float()
    assert ((c - ref).norm() / ref.norm()).item() < 1e-2


def _wide_spans(D_min=1500, seed=0):
    """Synthetic layout wider than the register-prefetch path (D > 512): tanh + softmax spans,
    some wider than a wave."""
    rng = np.random.default_rng(seed)
    spans, cond, pos = [], [], 0
    while pos < D_min:
        spans.append((pos, 1, 0))
        pos += 1
        w = int(rng.choice([2, 3, 7, 13, 70, 130]))
        spans.append((pos, w, 1))
        cond.append((pos, w))
        pos += w
    return spans, cond, pos


def test_wide_activation_and_backward(hip):
    spans, cond, D = _wide_spans()
    rows = 3000
    logits = mat(rows, D, seed=50) * 2
    o1, o2 = torch.zeros_like(logits), torch.zeros_like(logits)
    hip.activate(logits, o1, spans, 0.2)
    REF.activate(logits, o2, spans, 0.2)
    torch.cuda.synchronize()
    for s, w, k in spans:
        if k == 0:
            assert torch.allclose(o1[:, s], torch.tanh(logits[:, s]), atol=1e-6)
        else:
            assert torch.allclose(o1[:, s:s + w].sum(1), torch.ones(rows, device=DEV), atol=1e-4)
    # identical rows: Gumbel-softmax means agree with the torch reference.  Each column mean is
    # over 3000 draws (difference std <= sqrt(2 * 0.25 / 3000) ~ 0.013); the max over the wide
    # table's columns needs ~4.5 sigma.  Both draws are pinned: the torch reference by the seed, the
    # HIP Philox stream by a fresh counter (earlier tests in this module advance the fixture's)
    torch.manual_seed(1234)
    base = logits[:1].repeat(rows, 1)
    saved_ctr = hip.ctr.clone()
    hip.ctr.zero_()
    hip.activate(base, o1, spans, 0.2)
    hip.ctr.copy_(saved_ctr)
    REF.activate(base, o2, spans, 0.2)
    torch.cuda.synchronize()
    assert (o1.mean(0) - o2.mean(0)).abs().max().item() < 0.06
    # backward + cond CE against the reference, per-row loss terms
    B = 500
    lg = logits[:B].contiguous()
    act = torch.zeros_like(lg)
    REF.activate(lg, act, spans, 0.2)
    dact = mat(B, D, seed=51)
    col = torch.randint(0, len(cond), (B,), device=DEV, dtype=torch.int32)
    w = torch.tensor([w for _, w in cond], device=DEV)[col.long()]
    opt = (torch.rand(B, device=DEV) * w).floor().to(torch.int32)
    d1, d2 = torch.zeros_like(lg), torch.zeros_like(lg)
    rows1, l2 = torch.zeros(B, device=DEV), torch.zeros(1, device=DEV)
    hip.act_bwd_ce(dact, act, lg, spans, cond, col, opt, d1, rows1, 0.2)
    REF.act_bwd_ce(dact, act, lg, spans, cond, col, opt, d2, l2, 0.2)
    torch.cuda.synchronize()
    assert torch.allclose(d1, d2, atol=1e-5, rtol=1e-4)
    assert torch.allclose(rows1.sum(), l2[0], rtol=1e-4)


@pytest.mark.parametrize("aux", [0, 2, 16])
def test_adam_store_policies_match_torch(hip, aux):
    """Plain, non-temporal and write-through (sc1) buffer stores give the same Adam update."""
    n = 4 * 70001 + 3
    p = mat(n, seed=60)
    g = mat(n, seed=61)
    tp = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([tp], lr=2e-4, betas=(0.5, 0.9))
    m, v = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    step = torch.ones(1, device=DEV)
    prev = torch.ops.fedtgan.set_tuning("adam_store", aux)
    try:
        hip.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 0.0)
    finally:
        torch.ops.fedtgan.set_tuning("adam_store", prev)
    tp.grad = g.clone()
    opt.step()
    torch.cuda.synchronize()
    assert torch.allclose(p, tp.detach(), atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("case", ["dv_r64", "dv_r32", "dw_dh", "fallback"])
def test_gemm_pair_launch_matches_two_launches(hip, case):
    """Two independent GEMMs held + paired into one launch equal the same GEMMs launched one by one
    (including a split-K second GEMM and a pair with no fused instantiation)."""
    torch.manual_seed(3)
    if case == "dv_r64":      # weight gradient (64-tile) + split-K NT product with a mask epilogue
        A, X, W = mat(150, 256, seed=70), mat(150, 6280, seed=71), mat(256, 6280, seed=72)
        ms = (torch.rand(50, 256, device=DEV) > 0.5).float() * 2
        jobs = [dict(a=A, b=X, c=torch.zeros(256, 6280, device=DEV), ta=True),
                dict(a=X[:50], b=W, c=torch.zeros(50, 256, device=DEV), tb=True, epi=2, ms=ms)]
    elif case == "dv_r32":
        A, D0, W = mat(150, 256, seed=73), mat(150, 256, seed=74), mat(256, 256, seed=75)
        jobs = [dict(a=A, b=D0, c=torch.zeros(256, 256, device=DEV), ta=True),
                dict(a=D0[:50], b=W, c=torch.zeros(50, 256, device=DEV), tb=True)]
    elif case == "dw_dh":     # weight gradient + NN product accumulating into its output (beta = 1)
        G, H, W = mat(500, 325, seed=76), mat(500, 943, seed=77), mat(325, 512, seed=78)
        jobs = [dict(a=G, b=H, c=torch.zeros(325, 943, device=DEV), ta=True),
                dict(a=G, b=W, c=mat(500, 512, seed=79), beta=1.0)]
    else:                     # NN first: no fused instantiation, runs as two launches
        P, Q = mat(200, 300, seed=80), mat(300, 100, seed=81)
        jobs = [dict(a=P, b=Q, c=torch.zeros(200, 100, device=DEV)),
                dict(a=P, b=Q, c=torch.zeros(200, 100, device=DEV), beta=1.0)]
    refs = []
    for j in jobs:
        j2 = dict(j)
        j2["c"] = j["c"].clone()
        hip.gemm(**j2)
        refs.append(j2["c"])
    hip.gemm(**jobs[0], group=1)
    hip.gemm(**jobs[1], group=2)
    torch.cuda.synchronize()
    for j, r in zip(jobs, refs):
        assert torch.allclose(j["c"], r, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("aux", [0, 16])
def test_adam_with_folded_colsum_matches_two_launches(hip, aux):
    """adam(jobs=...) == colsum_many + adam: bias sums written into the gradient buffer (a 325-wide
    one with padding, 4-aligned), a weighted dot job into a metric, a sum outside the buffer."""
    n = 4 * 5000
    p0, g0 = mat(n, seed=90), mat(n, seed=91)
    src1, src2, src3 = mat(500, 328, seed=92)[:, :325], mat(150, 256, seed=93), mat(150, 325, seed=94)[:, :256]
    src0 = mat(77, 37, seed=99)     # unaligned rows: the scalar-load path
    w3, dv, de = mat(150, seed=95), mat(256, seed=96), mat(1, seed=97)
    rows = mat(50, 1, seed=98)
    step = torch.full((1,), 3.0, device=DEV)
    res = []
    for fused in (False, True):
        p, g = p0.clone(), g0.clone()
        g[1000:1004] = 0.0
        g[1000 + 325:1000 + 328] = 0.0     # ceil4 padding of the 325-wide output
        g[8037:8040] = 0.0
        m, v = torch.full_like(p, 0.01), torch.full_like(p, 0.02)
        met = torch.zeros(4, device=DEV)
        jobs = ([src1, src2, src3, rows, src0], [g[1000:1325], g[4096:4352], None, met[1:2], g[8000:8037]],
                [None, None, w3, None, None], [None, None, (dv, de, met[0:1]), None, None])
        prev = torch.ops.fedtgan.set_tuning("adam_store", aux)
        try:
            if fused:
                hip.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 1e-6, jobs=jobs)
            else:
                hip.colsum_many(*jobs)
                hip.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 1e-6)
        finally:
            torch.ops.fedtgan.set_tuning("adam_store", prev)
        torch.cuda.synchronize()
        res.append((p, g, m, v, met))
    # (column sums in a different order: the gradient sums agree to fp32 rounding)
    for name, a, b, tol in zip("pgmvM", *res, (1e-6, 1e-4, 1e-6, 1e-6, 1e-3)):
        err = (a - b).abs().max().item()
        assert torch.allclose(a, b, atol=tol, rtol=1e-5), (name, err)
    assert torch.allclose(res[1][1][1000:1325], src1.sum(0), atol=1e-4, rtol=1e-5)
    assert torch.allclose(res[1][1][8000:8037], src0.sum(0), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize("d_min", [300, 2300, 7000])
def test_wide_row_kernels_match_per_wave_kernels(hip, d_min):
    """Rows wider than 512: the one-workgroup-per-row kernels (LDS row image, and register-resident with 2 or 4
    groups per wave) draw the same Philox words as the per-wave kernels, so activation (+ fused slerp) and its
    backward agree element for element."""
    spans, cond, D = _wide_spans(D_min=d_min, seed=4)
    rows, nc = 600, 45
    Din = D + nc
    logits = mat(rows, D, seed=52) * 2
    real = mat(rows, Din, seed=53)
    cond_cols = mat(rows, nc, seed=54)
    res = []
    # (act_rowreg_narrow: rows <= 512 on the row kernels with 2 waves (1) or one 64-column block per wave (2))
    for mode, narrow in ((0, 0), (1, 1), (2, 1), (2, 2)):
        fake = torch.zeros(rows, Din, device=DEV)
        fake[:, D:] = cond_cols
        interp = torch.zeros(rows // 3, Din, device=DEV)
        prev = torch.ops.fedtgan.set_tuning("act_row_mode", mode)
        prev_n = torch.ops.fedtgan.set_tuning("act_rowreg_narrow", narrow)
        try:
            hip.activate(logits, fake[:, :D], spans, 0.2, stream_id=2, slerp=(real[:rows // 3], fake, interp, 3))
            dact = mat(rows, D, seed=55)
            col = (torch.arange(rows, device=DEV) % len(cond)).to(torch.int32)
            w = torch.tensor([w for _, w in cond], device=DEV)[col.long()]
            opt = ((torch.arange(rows, device=DEV) * 7) % w).to(torch.int32)
            d = torch.zeros_like(logits)
            loss = torch.zeros(rows, device=DEV)
            hip.act_bwd_ce(dact, fake[:, :D], logits, spans, cond, col, opt, d, loss, 0.2)
        finally:
            torch.ops.fedtgan.set_tuning("act_row_mode", prev)
            torch.ops.fedtgan.set_tuning("act_rowreg_narrow", prev_n)
        torch.cuda.synchronize()
        res.append((fake, interp, d, loss))
    for other in res[1:]:
        for name, a, b in zip(("act", "slerp", "dlogits", "ce"), res[0], other):
            err = (a - b).abs().max().item()
            assert torch.allclose(a, b, atol=2e-5, rtol=1e-4), (name, err)



def test_adam_folded_dot_over_own_parameters_reads_pre_update_values(hip):
    """The D head job: gradient (row weights w) and the WGAN value (row weights u) in one job whose
    dot runs over the very parameters the launch updates -- the value uses the old weights."""
    n = 4 * 3000
    p0, g0 = mat(n, seed=100), mat(n, seed=101)
    src, w, u, e = mat(150, 256, seed=102), mat(150, seed=103), mat(150, seed=104), mat(1, seed=105)
    step = torch.full((1,), 2.0, device=DEV)
    res = []
    for fused in (False, True):
        p, g = p0.clone(), g0.clone()
        m, v = torch.full_like(p, 0.01), torch.full_like(p, 0.02)
        met = torch.zeros(2, device=DEV)
        jobs = ([src], [g[2048:2304]], [w], [(p[2048:2304], e, met[0:1], u)])
        if fused:
            hip.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 0.0, jobs=jobs)
        else:
            hip.colsum_many(*jobs)
            hip.adam(p, g, m, v, step, 2e-4, 0.5, 0.9, 1e-8, 0.0)
        torch.cuda.synchronize()
        res.append((p, g, met))
    want = (src * u[:, None]).sum(0) @ p0[2048:2304] + e[0] * u.sum()
    assert torch.allclose(res[1][2][0], want, rtol=1e-4, atol=1e-3)
    assert torch.allclose(res[0][2][0], want, rtol=1e-4, atol=1e-3)
    assert torch.allclose(res[1][1][2048:2304], (src * w[:, None]).sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(res[0][0], res[1][0], atol=1e-6, rtol=1e-5)


def test_sample_decode_row_kernel_matches_per_cell_kernel(hip):
    """One wave per row (LDS 64-bit max per column; element per lane, or one Philox quad per lane)
    draws the same Gumbel noise per logit as the one-thread-per-cell decode, so all three give the
    same table bit for bit."""
    from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
    from fed_tgan_amd.models.samplers import CondTables
    tr, X, spans, cond = _spans()
    eng = CTGANEngine(tr.layout, EngineConfig(), DEV, backend="hip", seed=5)
    eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
    rows = 1500
    logits = mat(rows, X.shape[1], seed=120) * 3
    logits[:7] = 0.0                      # flat spans: the choice is the Gumbel noise alone
    res = []
    for mode in (0, 1, 2):
        out = torch.zeros(rows, len(tr.meta), dtype=torch.float64, device=DEV)
        ctr0 = eng.ops.ctr.clone()
        prev = torch.ops.fedtgan.set_tuning("decode_rows", mode)
        try:
            eng.ops.sample_decode(logits, out, eng.gen_tables)
        finally:
            torch.ops.fedtgan.set_tuning("decode_rows", prev)
        eng.ops.ctr.copy_(ctr0)           # same counter for every kernel
        torch.cuda.synchronize()
        res.append(out)
    assert torch.equal(res[0], res[1]) and torch.equal(res[0], res[2])


@pytest.mark.parametrize("trans", [False, True])
@pytest.mark.parametrize("tile", [32, 64, 128])
@pytest.mark.parametrize("bn", [False, True])
def test_gemm_onehot_gather_matches_dense(hip32, tile, bn, trans):
    """The one-hot conditional block as an epilogue gather (GemmArgs::oh_w) equals the dense product
    over [dense | one-hot] columns, incl. the eval-BN epilogue and the 128-tile LDS epilogue."""
    M, Kd, N = 700, 200, 96
    widths = [3, 7, 1, 12, 5]
    C = sum(widths)
    off = torch.tensor(np.cumsum([0] + widths[:-1]), dtype=torch.int32, device=DEV)
    g = torch.Generator(device="cpu").manual_seed(5)
    col = torch.randint(0, len(widths), (M,), generator=g)
    opt = torch.tensor([int(torch.randint(0, widths[c], (1,), generator=g)) for c in col], dtype=torch.int32)
    H = torch.zeros(M, Kd + C, device=DEV)
    H[:, :Kd] = mat(M, Kd, seed=60)
    H[torch.arange(M), Kd + off.cpu()[col].long() + opt.long()] = 1.0
    W = mat(N, Kd + C, seed=61)
    bias = mat(N, seed=62)
    col, opt = col.to(torch.int32).to(DEV), opt.to(DEV)
    hip32.tile_override = tile
    kw = {}
    if bn:
        kw = dict(epi=4, bn=(torch.rand(N, device=DEV) + 0.5, mat(N, seed=63), mat(N, seed=64),
                             torch.rand(N, device=DEV) + 0.5))
    dense = torch.zeros(M, N, device=DEV)
    hip32.gemm(H, W, dense, tb=True, bias=bias, **kw)
    gath = torch.zeros(M, N, device=DEV)
    oh = (W[:, Kd:].t().contiguous(), col, opt, off, True) if trans else (W[:, Kd:], col, opt, off)
    hip32.gemm(H[:, :Kd], W[:, :Kd], gath, tb=True, bias=bias, onehot=oh, **kw)
    torch.cuda.synchronize()
    hip32.tile_override = None
    assert torch.allclose(gath, dense, atol=2e-4, rtol=1e-5)


@pytest.mark.parametrize("rows,groups,tile", [(1000, 2, 32), (500, 1, 32), (1000, 2, 64), (37, 1, 32), (1200, 2, 32)])
def test_linear_bn_relu_from_gemm_partials(hip32, rows, groups, tile):
    """BatchNorm(train) from the GEMM epilogue's per-tile (count, mean, M2) partials merged by
    bn_relu_apply equals the separate full-reduction BN kernel (both batches, running stats)."""
    K, N = 200, 256
    x = mat(rows, K, seed=70) * 2 + 3
    W = mat(N, K, seed=71) * 0.1
    bvec = mat(N, seed=72)
    gamma, beta = torch.rand(N, device=DEV) + 0.5, mat(N, seed=73)
    res = {}
    for fused in (True, False):
        hip32.bn_fused = fused
        hip32.tile_override = tile
        ab, out, nh = (torch.zeros(rows, N, device=DEV) for _ in range(3))
        mean, inv = torch.zeros(groups, N, device=DEV), torch.zeros(groups, N, device=DEV)
        rm, rv = torch.full((N,), 0.3, device=DEV), torch.full((N,), 1.7, device=DEV)
        hip32.linear_bn_relu(x, W, bvec, gamma, beta, out, ab, nh, mean, inv, rm, rv, True, 0.1, 1e-5, groups=groups)
        torch.cuda.synchronize()
        res[fused] = (out, nh, mean, inv, rm, rv)
    hip32.bn_fused, hip32.tile_override = False, None
    for name, a, b in zip(("out", "nhat", "mean", "invstd", "rm", "rv"), res[True], res[False]):
        assert torch.allclose(a, b, atol=1e-4, rtol=1e-4), name


@pytest.mark.parametrize("case", ["relu", "lrelu_head", "mask_beta", "onehot", "tile64", "pair"])
def test_gemm_splitk_inlaunch_matches_epilogue_kernel(hip, hip32, case):
    """Split-K reduced by the last-arriving K-slice workgroup (tile counters) gives bit-identical
    outputs to the separate gemm_splitk_epilogue launch -- same slab sum order, same epilogue --
    over repeated launches (the reducer re-zeroes the counters) and inside a replayed hipGraph."""
    ops = hip32 if case == "onehot" else hip

    def jobs():
        if case == "relu":
            return [dict(a=mat(50, 9000, seed=90) * 0.1, b=mat(256, 9000, seed=91) * 0.1, tb=True, bias=mat(256, seed=92),
                         epi=3, out=(50, 256))]
        if case == "lrelu_head":
            return [dict(a=mat(150, 6280, seed=93), b=mat(256, 6280, seed=94), tb=True, bias=mat(256, seed=95), epi=1,
                         ms=torch.zeros(150, 256, device=DEV), head=(mat(150, seed=96), mat(256, seed=97),
                                                                      torch.zeros(150, 256, device=DEV)),
                         out=(150, 256))]
        if case == "mask_beta":
            ms = (mat(50, 256, seed=98) > 0).float() * 2
            return [dict(a=mat(50, 6280, seed=99), b=mat(256, 6280, seed=100), tb=True, beta=1.0, epi=2, ms=ms,
                         c0=mat(50, 256, seed=101), out=(50, 256))]
        if case == "onehot":
            Wc = mat(256, 300, seed=102)
            col = torch.randint(0, 3, (60,), device=DEV, dtype=torch.int32)
            opt = torch.randint(0, 100, (60,), device=DEV, dtype=torch.int32)
            off = torch.tensor([0, 100, 200], device=DEV, dtype=torch.int32)
            return [dict(a=mat(60, 5000, seed=103), b=mat(256, 5000, seed=104), tb=True, bias=mat(256, seed=105),
                         onehot=(Wc, col, opt, off), out=(60, 256))]
        if case == "tile64":
            return [dict(a=mat(130, 7000, seed=106), b=mat(200, 7000, seed=107), tb=True, tile=64, out=(130, 200))]
        A, X, W = mat(150, 256, seed=108), mat(150, 6280, seed=109), mat(256, 6280, seed=110)
        ms = (mat(50, 256, seed=111) > 0).float() * 2
        return [dict(a=A, b=X, ta=True, out=(256, 6280), group=1),
                dict(a=X[:50], b=W, tb=True, epi=2, ms=ms, out=(50, 256), group=2)]

    def run(inlaunch, graph=False):
        torch.manual_seed(0)
        js = jobs()
        outs = [j.pop("c0").clone() if "c0" in j else torch.zeros(*j["out"], device=DEV) for j in js]
        for j in js:
            j.pop("out")
        ops.splitk_inlaunch = inlaunch
        saved = ops.ctr.clone()
        try:
            def launch():
                for j, c in zip(js, outs):
                    ops.gemm(c=c, **j)
            if case in ("relu", "mask_beta", "onehot", "tile64"):
                ops.split_override = 13
            launch()                              # sizes the workspace / counters
            for _ in range(2):
                launch()                          # counters must be back at zero
            if graph:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    launch()
                for _ in range(3):
                    g.replay()
        finally:
            ops.split_override = None
            ops.splitk_inlaunch = False
            ops.ctr.copy_(saved)
        torch.cuda.synchronize()
        extra = [j["ms"] for j in js if j.get("epi") == 1] + [j["head"][2] for j in js if j.get("head")]
        return outs + extra

    ref = run(False)
    got = run(True)
    for r, o in zip(ref, got):
        assert torch.equal(r, o)
    got_g = run(True, graph=True)
    ref_g = run(False, graph=True)
    for r, o in zip(ref_g, got_g):
        assert torch.equal(r, o)


def test_onehot_wgrad_scatter_and_clear(hip):
    """ops.onehot_wgrad: block row k = sum of the dy rows whose condition index is k (duplicates summed in batch
    order), the other rows untouched; zero=True clears exactly the touched rows."""
    B, n, ncol = 500, 301, 7
    widths = torch.tensor([3, 1, 40, 5, 9, 2, 60])
    cond_off = torch.cat([torch.zeros(1, dtype=torch.int64), widths.cumsum(0)[:-1]]).to(torch.int32).to(DEV)
    C = int(widths.sum())
    g = torch.Generator().manual_seed(3)
    col = torch.randint(0, ncol, (B,), generator=g)
    opt = (torch.rand(B, generator=g) * widths[col]).floor().long()
    col, opt = col.to(torch.int32).to(DEV), opt.to(torch.int32).to(DEV)
    dy = mat(B, n, seed=120)
    w = torch.zeros(C + 5, n + 3, device=DEV)[2:C + 2, :n]        # a strided view inside a larger buffer
    hip.onehot_wgrad([dy], [w], col, opt, cond_off)
    torch.cuda.synchronize()
    idx = (cond_off.long()[col.long()] + opt.long())
    ref = torch.zeros(C, n, dtype=torch.float64, device=DEV).index_add_(0, idx, dy.double())
    assert torch.allclose(w.double(), ref, atol=1e-5, rtol=1e-5)
    assert len(torch.unique(idx)) < B          # (duplicates were exercised)
    hip.onehot_wgrad([dy], [w], col, opt, cond_off, zero=True)
    torch.cuda.synchronize()
    assert w.abs().max().item() == 0.0
