"""The engine's explicit backward (incl. the hand-derived GP double backward) vs torch autograd.

The oracle re-runs one D step and one G step of the reference math
(`Server/dtds/synthesizers/ctgan.py:15-64, 174-258`, `Client/.../distributed.py:185-265`)
with torch autograd in float64-free fp32, using the exact random draws the engine made
(recorded Gumbel noise and slerp output; dropout keep-masks recovered from the saved
mask*slope buffers).
"""
import pytest
import torch
import torch.nn.functional as F

from fed_tgan_amd.models.ctgan import Generator, cond_loss
from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
from fed_tgan_amd.ops.ref import TorchOps

from helpers import d_forward_masked, keep_mask_from_ms, small_table


class RecordingOps(TorchOps):
    def __init__(self):
        self.rec = {}

    def activate(self, logits, out, spans, tau=0.2, stream_id=0):
        noise = []
        for s, w, k in spans:
            x = logits[:, s:s + w]
            if k == 0:
                out[:, s:s + w].copy_(torch.tanh(x))
                noise.append(None)
            else:
                u = torch.rand(x.shape).clamp_(1e-20, 1 - 1e-7)
                g = -torch.log(-torch.log(u))
                noise.append(g)
                out[:, s:s + w].copy_(torch.softmax((x + g) / tau, dim=1))
        self.rec.setdefault("gumbel", []).append(noise)

    def slerp(self, real, fake, out, stream_id=0):
        super().slerp(real, fake, out, stream_id)
        self.rec["interp"] = out.clone()


def _setup(gen_dims=(256, 256), dis_dims=(256, 256), batch=100, g_wt=False):
    _, _, _, _, _, _, tr, X = small_table()
    cfg = EngineConfig(gen_dims=gen_dims, dis_dims=dis_dims, batch_size=batch, g_wt=g_wt)
    torch.manual_seed(0)
    eng = CTGANEngine(tr.layout, cfg, "cpu", backend="torch")
    eng.ops = RecordingOps()
    eng.set_training_data(X)
    return eng, tr


def _d_params(eng, src):
    L = len(eng.ddims)
    names = [f"D.{i}.W" for i in range(L)] + [f"D.{i}.b" for i in range(L)] + ["D.out.W", "D.out.b"]
    out = {}
    for n in names:
        out[n] = src[n].detach().clone().requires_grad_(True)
    return out


def _masks(eng, rows, P, X):
    L = len(eng.ddims)
    masks = []
    h = X
    for i in range(L):
        pre = h @ P[f"D.{i}.W"].detach().t() + P[f"D.{i}.b"].detach()
        M = keep_mask_from_ms(eng.ms[i][rows], pre)
        masks.append(M)
        h = F.leaky_relu(pre, 0.2) * M
    return masks


def test_d_step_matches_autograd():
    eng, tr = _setup()
    B, nP, Dd = eng.B, eng.nP, eng.Dd
    before = {n: t.detach().clone() for n, t in eng.p.items()}
    eng._d_step()
    P = _d_params(eng, before)
    L = len(eng.ddims)
    Xf = eng.X_fake.reshape(nP, eng.K1).clone()
    Xr = eng.X_real.reshape(nP, eng.K1).clone()
    Xi = eng.ops.rec["interp"].reshape(nP, eng.K1).clone().requires_grad_(True)
    Ws = [P[f"D.{i}.W"] for i in range(L)]
    bs = [P[f"D.{i}.b"] for i in range(L)]
    mf = _masks(eng, slice(2 * nP, 3 * nP), P, Xf)
    mr = _masks(eng, slice(nP, 2 * nP), P, Xr)
    mi = _masks(eng, slice(0, nP), P, Xi.detach())
    yf = d_forward_masked(Xf, Ws, bs, mf, P["D.out.W"], P["D.out.b"])
    yr = d_forward_masked(Xr, Ws, bs, mr, P["D.out.W"], P["D.out.b"])
    yi = d_forward_masked(Xi, Ws, bs, mi, P["D.out.W"], P["D.out.b"])
    loss_d = -(yr.mean() - yf.mean())
    g = torch.autograd.grad(yi.sum(), Xi, create_graph=True)[0]
    pen = ((g.norm(2, dim=1) - 1) ** 2).mean() * 10.0
    (loss_d + pen).backward()
    m = eng.metrics
    assert torch.allclose(m[0], loss_d.detach(), rtol=1e-4, atol=1e-5)
    assert torch.allclose(m[1], pen.detach(), rtol=1e-4, atol=1e-5)
    for n, t in P.items():
        ref = t.grad if t.grad is not None else torch.zeros_like(t)
        got = eng.g[n]
        scale = ref.abs().max().clamp_min(1e-6)
        assert (got - ref).abs().max() / scale < 2e-4, n
    # Adam update of D equals torch.optim.Adam on the same gradients
    for n, t in P.items():
        t.grad = eng.g[n].clone()
    opt = torch.optim.Adam(list(P.values()), lr=2e-4, betas=(0.5, 0.9))
    opt.step()
    for n, t in P.items():
        assert torch.allclose(eng.p[n], t.detach(), rtol=1e-5, atol=1e-7), n


@pytest.mark.parametrize("g_wt", [False, True])
def test_g_step_matches_autograd(g_wt):
    """(g_wt: generator weights stored input-major; the logical views and the math are the same)"""
    eng, tr = _setup(g_wt=g_wt)
    B, nP, Dd = eng.B, eng.nP, eng.Dd
    eng._d_step()
    before = {n: t.detach().clone() for n, t in eng.p.items()}
    eng.ops.rec.clear()
    eng._g_step()
    G = Generator(eng.E + eng.C, eng.gdims, Dd)
    sd = {}
    for k, n in eng.g_key_map():
        sd[k] = before[n].clone()
    for i in range(len(eng.gdims)):
        sd[f"seq.{i}.bn.num_batches_tracked"] = torch.tensor(0)
    G.load_state_dict(sd)
    G.train()
    x0 = eng.H[:, eng.off[0]:].clone()
    logits = G(x0)
    noise = eng.ops.rec["gumbel"][0]
    acts = []
    for (s, w, k), gn in zip(eng.spans, noise):
        x = logits[:, s:s + w]
        acts.append(torch.tanh(x) if k == 0 else torch.softmax((x + gn) / 0.2, dim=1))
    c1 = x0[:, eng.E:]
    fake = torch.cat(acts + [c1], dim=1).reshape(nP, eng.K1)
    L = len(eng.ddims)
    P = {n: before[n] for n in before if n.startswith("D.")}
    masks = _masks(eng, slice(0, nP), P, fake.detach())
    y = d_forward_masked(fake, [P[f"D.{i}.W"] for i in range(L)], [P[f"D.{i}.b"] for i in range(L)], masks,
                         P["D.out.W"], P["D.out.b"])
    m1 = torch.zeros(B, eng.layout.n_col)
    m1[torch.arange(B), eng.col.long()] = 1.0
    ce = cond_loss(logits, tr.output_info, c1, m1)
    loss_g = -y.mean() + ce
    G.zero_grad()
    loss_g.backward()
    assert torch.allclose(eng.metrics[2] + eng.metrics[3], loss_g.detach(), rtol=1e-4, atol=1e-5)
    assert torch.allclose(eng.metrics[3], ce.detach(), rtol=1e-4, atol=1e-6)
    gsd = dict(G.named_parameters())
    for k, n in eng.g_key_map():
        if k not in gsd:
            continue
        ref = gsd[k].grad
        got = eng.g[n]
        scale = ref.abs().max().clamp_min(1e-6)
        assert (got - ref).abs().max() < 2e-4 * scale + 1e-7, (k, float((got - ref).abs().max()), float(scale))
    # running statistics follow the reference BN (momentum 0.1, unbiased running var)
    bsd = G.state_dict()
    for i in range(len(eng.gdims)):
        assert torch.allclose(eng.p[f"G.{i}.rm"], bsd[f"seq.{i}.bn.running_mean"], rtol=1e-5, atol=1e-6)
        assert torch.allclose(eng.p[f"G.{i}.rv"], bsd[f"seq.{i}.bn.running_var"], rtol=1e-5, atol=1e-6)
    # Adam with L2 weight decay 1e-6 on G
    for k, n in eng.g_key_map():
        if k in gsd:
            gsd[k].grad = eng.g[n].clone()
    opt = torch.optim.Adam(G.parameters(), lr=2e-4, betas=(0.5, 0.9), weight_decay=1e-6)
    opt.step()
    psd = dict(G.named_parameters())
    for k, n in eng.g_key_map():
        if k in psd:
            assert torch.allclose(eng.p[n], psd[k].detach(), rtol=1e-5, atol=1e-7), k


def test_deeper_discriminator_gp():
    """Three hidden D layers and one G layer: the generic A/R chains still match autograd."""
    eng, tr = _setup(gen_dims=(128,), dis_dims=(64, 32, 16), batch=50)
    B, nP = eng.B, eng.nP
    before = {n: t.detach().clone() for n, t in eng.p.items()}
    eng._d_step()
    P = _d_params(eng, before)
    L = len(eng.ddims)
    Xf = eng.X_fake.reshape(nP, eng.K1).clone()
    Xr = eng.X_real.reshape(nP, eng.K1).clone()
    Xi = eng.ops.rec["interp"].reshape(nP, eng.K1).clone().requires_grad_(True)
    Ws = [P[f"D.{i}.W"] for i in range(L)]
    bs = [P[f"D.{i}.b"] for i in range(L)]
    yf = d_forward_masked(Xf, Ws, bs, _masks(eng, slice(2 * nP, 3 * nP), P, Xf), P["D.out.W"], P["D.out.b"])
    yr = d_forward_masked(Xr, Ws, bs, _masks(eng, slice(nP, 2 * nP), P, Xr), P["D.out.W"], P["D.out.b"])
    yi = d_forward_masked(Xi, Ws, bs, _masks(eng, slice(0, nP), P, Xi.detach()), P["D.out.W"],
                          P["D.out.b"])
    g = torch.autograd.grad(yi.sum(), Xi, create_graph=True)[0]
    pen = ((g.norm(2, dim=1) - 1) ** 2).mean() * 10.0
    (yf.mean() - yr.mean() + pen).backward()
    for n, t in P.items():
        ref = t.grad if t.grad is not None else torch.zeros_like(t)
        scale = ref.abs().max().clamp_min(1e-6)
        assert (eng.g[n] - ref).abs().max() / scale < 2e-4, n


@pytest.mark.parametrize("g_wt", [False, True])
def test_padded_storage_stays_zero(g_wt):
    """Weights live in rows padded to 4 floats (16-B GEMM loads); the padding columns and the
    activation buffers' padding must stay exactly zero through training (they enter K sums).
    g_wt: input-major generator weights, padded to 4 along both dimensions."""
    from fed_tgan_amd.models.engine import _ceil4, _ext
    eng, _ = _setup(batch=100, g_wt=g_wt)
    eng.ops = type(eng.ops).__mro__[1]()       # plain TorchOps
    eng.train_steps(3, use_graph=False)
    padded = 0
    for n, t in list(eng.p.items()) + [("g." + k, v) for k, v in eng.g.items()]:
        if t.dim() == 2 and t.shape[1] % 4:
            padded += 1
            full = _ext(t, _ceil4(t.shape[1]))
            assert torch.count_nonzero(full[:, t.shape[1]:]) == 0, n
    assert padded > 0
    for buf in (eng.H, eng.dH, eng.logits):
        if buf.shape[1] % 4:
            assert torch.count_nonzero(_ext(buf, _ceil4(buf.shape[1]))[:, buf.shape[1]:]) == 0
    x, W = eng._kpad(eng.H, 0, eng.p["G.out.W"])
    assert x.shape[1] % 4 == 0 and W.shape[1] == x.shape[1]
    if g_wt:
        # every generator weight is a transposed view of [ceil4(in), ceil4(out)] storage, and the whole
        # storage block outside the logical [in, out] corner is zero
        for n in eng.wt_names:
            t = eng.p[n]
            assert t.stride(0) == 1 and t.stride(1) == _ceil4(t.shape[0])
            o = t.storage_offset()
            blk = eng.flat[o:o + _ceil4(t.shape[1]) * _ceil4(t.shape[0])].view(_ceil4(t.shape[1]), -1)
            assert torch.equal(blk[:t.shape[1], :t.shape[0]], t.t())
            assert torch.count_nonzero(blk) == torch.count_nonzero(t), n


def test_paired_prepare_equals_two_phase_forwards():
    """The paired prepare (both phases' batches through one 2B-row generator pass) equals two
    separate training-mode forwards: per-batch BN statistics, running stats updated D batch then
    G batch, and the D input blocks / G-phase views it fills are the ones the updates read."""
    eng, tr = _setup()
    B = eng.B
    ref = CTGANEngine(tr.layout, eng.cfg, "cpu", backend="torch")
    ref.flat.copy_(eng.flat)
    eng._prepare_paired()
    a0 = eng.off[0]
    for half in (slice(0, B), slice(B, 2 * B)):
        ref.H[:, a0:].copy_(eng.H2[half, a0:])
        ref._g_forward(ref.H, ref.logits, training=True)
        assert torch.allclose(ref.logits, eng.logits2[half], rtol=1e-5, atol=1e-5)
        for i in range(len(eng.gdims)):
            assert torch.allclose(ref.nhat[i], eng.nhat2[i][half], rtol=1e-5, atol=1e-5)
    # running statistics after both batches, in the reference's order (D batch first)
    sA, sB = eng.group_range["S"]
    assert torch.allclose(ref.flat[sA:sB], eng.flat[sA:sB], rtol=1e-6, atol=1e-6)
    # G-phase views and the G-phase batch's BN statistics
    for i in range(len(eng.gdims)):
        assert eng.bn_invstd[i].data_ptr() == eng.bn_invstd2[i][1].data_ptr()
        assert torch.allclose(ref.bn_invstd[i], eng.bn_invstd[i], rtol=1e-5)
    assert eng.H.data_ptr() == eng.H2[B:].data_ptr()
    # conditions: fake rows carry their batch's one-hot, real rows a permutation of the D batch's
    c = eng.c_cols
    assert torch.equal(eng.X_fake[:, eng.Dd:], eng.H2[:B, c[0]:c[1]])
    assert torch.equal(eng.Xg[:, eng.Dd:], eng.H2[B:, c[0]:c[1]])
    assert torch.equal(eng.X_real[:, eng.Dd:].sum(0), eng.X_fake[:, eng.Dd:].sum(0))
    assert torch.equal(eng.col, eng.col2[B:])
    assert torch.all(eng.X_interp.abs().sum(1) > 0)


def test_paired_step_trains():
    """A few paired steps run end to end and stay finite (both phases' metrics written)."""
    eng, _ = _setup()
    eng.ops = TorchOps()
    for _ in range(3):
        eng._one_step()
    m = eng.metrics
    assert bool(torch.isfinite(m).all()) and float(m[1]) > 0
