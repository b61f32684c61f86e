"""Eager-PyTorch reference implementations of every fused op the engine uses.

Each method here states the math of one fused HIP kernel in ``csrc/kernels`` with plain
PyTorch ops.  It is (a) the CPU execution path (gloo demos, CI without a GPU) and
(b) the numerics oracle the HIP kernels are tested against.  Signatures are shared with
:class:`fed_tgan_amd.ops.hip.HipOps`; outputs are written in place into (possibly
strided, column-sliced) views so that the engine's concat-free buffer layout works on
both paths.

Randomness comes from the global torch generator of the tensor's device (the HIP path
uses counter-based Philox streams instead, so the two paths agree in distribution, not
bitwise).
"""
from __future__ import annotations

import math

import torch

EPI_NONE = 0
EPI_LRELU_DROPOUT = 1   # out = lrelu(acc + bias, slope) * M, M in {0, 1/(1-p)}; ms = lrelu'(.) * M
EPI_MASK = 2            # out = acc * ms
EPI_RELU = 3


class TorchOps:
    adam_counts_steps = True     # eager Adam bumps its step counter (the HIP sampler does it there)
    name = "torch"

    # ------------------------------------------------------------------ GEMM
    def gemm_plan(self, M: int, N: int, K: int):
        return 32, 1

    @staticmethod
    def _bn_partials(v: torch.Tensor, part: torch.Tensor, rpg: int, tile: int):
        """Per row tile and batch: (count, mean, M2) of every column -- the GEMM epilogue's partials."""
        M, N = v.shape
        pv = part.view(-1, 2, 3, N)
        for t in range(-(-M // tile)):
            for b in range(2):
                lo, hi = max(t * tile, rpg if b else 0), min((t + 1) * tile, M if b else rpg)
                if hi <= lo:
                    pv[t, b].zero_()
                    continue
                x = v[lo:hi]
                mu = x.mean(0)
                pv[t, b, 0] = float(hi - lo)
                pv[t, b, 1] = mu
                pv[t, b, 2] = ((x - mu) ** 2).sum(0)

    def gemm(self, a, b, c, ta=False, tb=False, alpha=1.0, beta=0.0, bias=None, epi=EPI_NONE, ms=None,
             slope=0.2, p_drop=0.5, stream_id=0, head=None, group=0, onehot=None, bn_part=None, bn_rpg=0, tile=None,
             splitk=None, **_):
        """c = epi(alpha * op(a) @ op(b) + beta * c + bias [+ onehot]).

        onehot = (W_c [N, C], col [M], opt [M], cond_offset): a holds only the dense input columns and
        the one-hot conditional block adds W_c[:, cond_offset[col[m]] + opt[m]] to row m.
        bn_part (with bn_rpg, tile): also the per-tile BatchNorm partials of the stored output."""
        A = a.t() if ta else a
        B = b.t() if tb else b
        acc = torch.matmul(A, B)
        if alpha != 1.0:
            acc = acc * alpha
        if beta != 0.0:
            acc = acc + beta * c
        if bias is not None:
            acc = acc + bias
        if onehot is not None:
            w_c, col, opt, off = onehot[:4]
            if len(onehot) > 4 and onehot[4]:
                w_c = w_c.t()
            m = acc.shape[0]
            idx = (off.long()[col[:m].long()] + opt[:m].long())
            acc = acc + w_c[:, idx].t()
        if epi == EPI_LRELU_DROPOUT:
            keep = (torch.rand(acc.shape, device=acc.device) >= p_drop).to(acc.dtype) / (1.0 - p_drop)
            s = torch.where(acc > 0, torch.ones_like(acc), torch.full_like(acc, slope))
            ms.copy_(s * keep)
            acc = acc * ms
            if head is not None:      # D head seed: A_{L-1} = coef * v * MS_{L-1}
                coef, v, a_out = head
                a_out.copy_(coef.view(-1, 1) * v.view(1, -1) * ms)
        elif epi == EPI_MASK:
            acc = acc * ms
        elif epi == EPI_RELU:
            acc = torch.relu(acc)
        c.copy_(acc)
        if bn_part is not None:
            self._bn_partials(acc, bn_part, int(bn_rpg), int(tile or 32))

    # ------------------------------------------------------------------ samplers
    def sample_train(self, t, h, z_cols, c_cols, x_fake, x_real, Dd, col_out, opt_out, step_counter=None,
                     metrics=None, zero_metrics=False, stream_id=0):
        """Draw the training conditional batch, noise, permutation and real rows.

        h[:, z_cols] <- N(0,1); h[:, c_cols] <- c1; x_fake[:, Dd:] <- c1; x_real <- [data[row], c1[perm]].
        t: dict of device tables (cdf_log, cond_offset, cond_width, row_offset, row_count, rows, data).
        (step_counter / metrics are bookkeeping of the HIP backend; eager Adam counts its own steps.)
        When x_real covers only the leading rows, those rows are a D-phase batch and the rest a
        G-phase batch (no real rows) drawn in the same call.
        """
        if x_real is not None and x_real.shape[0] < h.shape[0]:
            n = x_real.shape[0]
            self.sample_train(t, h[:n], z_cols, c_cols, x_fake[:n], x_real, Dd, col_out[:n], opt_out[:n])
            self.sample_train(t, h[n:], z_cols, c_cols, x_fake[n:], None, Dd, col_out[n:], opt_out[n:])
            return
        dev = h.device
        B = h.shape[0]
        x_fake_c = x_fake[:, Dd:]
        n_col = t["cond_width"].numel()
        h[:, z_cols[0]:z_cols[1]].normal_()
        c1 = h[:, c_cols[0]:c_cols[1]]
        c1.zero_()
        if n_col == 0:
            if x_real is not None:
                idx = torch.randint(0, t["data"].shape[0], (B,), device=dev)
                x_real.copy_(t["data"][idx])
            return
        col = torch.randint(0, n_col, (B,), device=dev)
        u = torch.rand(B, 1, device=dev, dtype=t["cdf_log"].dtype)
        opt = (t["cdf_log"][col] > u).to(torch.int32).argmax(1)
        opt = torch.minimum(opt, t["cond_width"][col].long() - 1)
        c1.scatter_(1, (t["cond_offset"][col].long() + opt).view(-1, 1), 1.0)
        x_fake_c.copy_(c1)
        col_out.copy_(col.to(col_out.dtype))
        opt_out.copy_(opt.to(opt_out.dtype))
        if x_real is None:
            return
        perm = torch.argsort(torch.rand(B, device=dev))
        cp, op_ = col[perm], opt[perm]
        cnt = t["row_count"][cp, op_]
        pick = torch.floor(torch.rand(B, device=dev, dtype=torch.float64) * cnt.clamp_min(1)).long()
        pick = torch.minimum(pick, (cnt - 1).clamp_min(0))
        row = t["rows"][t["row_offset"][cp, op_] + pick]
        dd = t["data"].shape[1]
        x_real[:, :dd].copy_(t["data"][row])
        x_real[:, dd:].copy_(c1[perm])

    def sample_gen(self, t, h, c_cols, z_cols, col_out=None, opt_out=None, stream_id=0):
        """Generation draw (``sample_zero``): noise + c from the empirical option CDF."""
        dev = h.device
        B = h.shape[0]
        h[:, z_cols[0]:z_cols[1]].normal_()
        c = h[:, c_cols[0]:c_cols[1]]
        c.zero_()
        n_col = t["cond_width"].numel()
        if n_col == 0:
            return
        col = torch.randint(0, n_col, (B,), device=dev)
        u = torch.rand(B, 1, device=dev, dtype=t["cdf_emp"].dtype)
        opt = (t["cdf_emp"][col] > u).to(torch.int32).argmax(1)
        opt = torch.minimum(opt, t["cond_width"][col].long() - 1)
        c.scatter_(1, (t["cond_offset"][col].long() + opt).view(-1, 1), 1.0)
        if col_out is not None:
            col_out[:B].copy_(col.to(col_out.dtype))
            opt_out[:B].copy_(opt.to(opt_out.dtype))

    # ------------------------------------------------------------------ batch norm + relu
    def bn_relu_fwd(self, a, gamma, beta, out, nhat, mean, invstd, rmean, rvar, training=True, momentum=0.1,
                    eps=1e-5, groups=1):
        """groups > 1: the rows are that many consecutive batches, each normalised with its own
        statistics; running statistics are updated batch after batch; mean / invstd [groups, cols]."""
        if groups > 1:
            n = a.shape[0] // groups
            for g in range(groups):
                r = slice(g * n, (g + 1) * n)
                self.bn_relu_fwd(a[r], gamma, beta, out[r], None if nhat is None else nhat[r],
                                 None if mean is None else mean[g], None if invstd is None else invstd[g],
                                 rmean, rvar, training, momentum, eps)
            return
        if training:
            mu = a.mean(0)
            var = a.var(0, unbiased=False)
            n = a.shape[0]
            with torch.no_grad():
                rmean.mul_(1 - momentum).add_(momentum * mu)
                rvar.mul_(1 - momentum).add_(momentum * var * n / max(n - 1, 1))
        else:
            mu, var = rmean, rvar
        istd = torch.rsqrt(var + eps)
        nh = (a - mu) * istd
        if nhat is not None:
            nhat.copy_(nh)
            mean.copy_(mu)
            invstd.copy_(istd)
        out.copy_(torch.relu(nh * gamma + beta))

    def linear_bn_relu(self, x, W, b, gamma, beta, out, abuf, nhat, mean, invstd, rmean, rvar, training=True,
                       momentum=0.1, eps=1e-5, groups=1, onehot=None):
        """out = relu(BN(x @ W^T + b)); training mode uses batch statistics and updates running ones."""
        a = torch.addmm(b, x, W.t())
        if onehot is not None:
            w_c, col, opt, off = onehot[:4]
            if len(onehot) > 4 and onehot[4]:
                w_c = w_c.t()
            a = a + w_c[:, off.long()[col[:a.shape[0]].long()] + opt[:a.shape[0]].long()].t()
        self.bn_relu_fwd(a, gamma, beta, out, nhat, mean, invstd, rmean, rvar, training, momentum, eps, groups)

    def bn_relu_bwd(self, dr, r, nhat, gamma, invstd, da, dgamma, dbeta, dbias=None):
        dy = dr * (r > 0).to(dr.dtype)
        dg = (dy * nhat).sum(0)
        db = dy.sum(0)
        dgamma.copy_(dg)
        dbeta.copy_(db)
        n = dr.shape[0]
        da.copy_(gamma * invstd * (dy - db / n - nhat * (dg / n)))
        if dbias is not None:
            dbias.copy_(da.sum(0))

    # ------------------------------------------------------------------ activations
    def linear_activate(self, x, W, b, logits, out, spans, tau=0.2, stream_id=0, slerp=None, onehot=None, **kw):
        self.gemm(x, W, logits, tb=True, bias=b, onehot=onehot, **kw)
        self.activate(logits, out, spans, tau, stream_id=stream_id)
        if slerp is not None:
            real, fake_full, interp, sid = slerp
            self.slerp(real, fake_full, interp, stream_id=sid)

    def activate(self, logits, out, spans, tau=0.2, stream_id=0):
        """spans: list of (start, width, kind) host tuples (kind 0 tanh, 1 gumbel-softmax)."""
        for s, w, k in spans:
            x = logits[:, s:s + w]
            if k == 0:
                out[:, s:s + w].copy_(torch.tanh(x))
            else:
                u = torch.rand(x.shape, device=x.device, dtype=x.dtype).clamp_(1e-20, 1.0 - 1e-7)
                g = -torch.log(-torch.log(u))
                out[:, s:s + w].copy_(torch.softmax((x + g) / tau, dim=1))

    def act_bwd_ce(self, dact, act, logits, spans, cond_spans, col, opt, dlogits, loss_out, tau=0.2):
        """dlogits = d(act)/d(logits)^T dact + d(cond_loss)/d(logits); loss_out[0] <- cond_loss, or, when
        loss_out has one entry per row, the per-row terms (their sum is cond_loss)."""
        for s, w, k in spans:
            g = dact[:, s:s + w]
            y = act[:, s:s + w]
            if k == 0:
                dlogits[:, s:s + w].copy_(g * (1 - y * y))
            else:
                dlogits[:, s:s + w].copy_(y * (g - (g * y).sum(1, keepdim=True)) / tau)
        B = logits.shape[0]
        per_row = B > 1 and loss_out.numel() == B
        loss = torch.zeros(B if per_row else (), device=logits.device, dtype=logits.dtype)
        colL = col.long()
        optL = opt.long()
        for c, (s, w) in enumerate(cond_spans):
            sel = (colL == c).to(logits.dtype)
            x = logits[:, s:s + w]
            tgt = torch.clamp(optL, max=w - 1).view(-1, 1)
            lse = torch.logsumexp(x, dim=1)
            term = sel * (lse - x.gather(1, tgt).view(-1))
            loss = loss + (term if per_row else term.sum())
            sm = torch.softmax(x, dim=1)
            sm = sm - torch.zeros_like(sm).scatter_(1, tgt, 1.0)
            dlogits[:, s:s + w] += sm * (sel / B).view(-1, 1)
        if per_row:
            loss_out.copy_(loss / B)
        else:
            loss_out[0] = loss / B

    # ------------------------------------------------------------------ gradient penalty pieces
    def slerp(self, real, fake, out, stream_id=0):
        alpha = torch.rand(real.shape[0], 1, device=real.device, dtype=real.dtype)
        rn = real.norm(dim=1, keepdim=True)
        fn = fake.norm(dim=1, keepdim=True)
        cos = ((real / rn) * (fake / fn)).sum(1, keepdim=True).clamp(-1.0, 1.0)
        om = torch.acos(cos)
        so = torch.sin(om)
        lin = so < 1e-6
        wr = torch.where(lin, 1 - alpha, torch.sin((1 - alpha) * om) / torch.where(lin, torch.ones_like(so), so))
        wf = torch.where(lin, alpha, torch.sin(alpha * om) / torch.where(lin, torch.ones_like(so), so))
        out.copy_(wr * real + wf * fake)

    def gp_scale(self, g, out, lam, loss_out):
        n = g.norm(dim=1, keepdim=True)
        P = g.shape[0]
        if P > 1 and loss_out.numel() == P:       # per-pack terms (summed by a later column sum)
            loss_out.copy_(lam * ((n.view(-1) - 1) ** 2) / P)
        else:
            loss_out[0] = lam * ((n - 1) ** 2).mean()
        out.copy_(g * (lam * 2.0 * (n - 1) / (n.clamp_min(1e-30) * P)))

    # ------------------------------------------------------------------ discriminator head
    def d_head(self, d_last, ms_last, v, e, coef, wloss, y, a_last, loss_out):
        """y = d_last @ v + e;  a_last = coef[:,None] * v[None,:] * ms_last;  loss_out[0] = sum(wloss * y)."""
        y.copy_(d_last @ v + e)
        a_last.copy_(coef.view(-1, 1) * v.view(1, -1) * ms_last)
        loss_out[0] = (wloss * y).sum()

    def colsum(self, a, out, beta=0.0):
        if beta == 0.0:
            out.copy_(a.sum(0))
        else:
            out.mul_(beta).add_(a.sum(0))

    def colsum_many(self, srcs, outs, weights=None, dots=None):
        n = len(srcs)
        for a, o, w, d in zip(srcs, outs, weights or [None] * n, dots or [None] * n):
            s = (a * w.view(-1, 1)).sum(0) if w is not None else a.sum(0)
            if o is not None:
                o.copy_(s)
            if d is not None:
                v, e, loss = d[:3]
                u = d[3] if len(d) > 3 and d[3] is not None else w
                su = (a * u.view(-1, 1)).sum(0) if u is not None else a.sum(0)
                usum = u.sum() if u is not None else torch.tensor(float(a.shape[0]), device=a.device)
                loss.add_((su * v.view(-1)).sum() + e.view(-1)[0] * usum)

    # ------------------------------------------------------------------ optimizer
    def adam(self, p, g, m, v, step, lr, b1, b2, eps, wd, last_in_step=False, jobs=None):
        """torch.optim.Adam (L2 weight decay added to the gradient, not AdamW); step is a device counter.
        jobs: colsum_many arguments computed first (the HIP backend folds them into the launch)."""
        if jobs is not None:
            self.colsum_many(*jobs)
        step.add_(1)
        if wd != 0.0:
            g = g + wd * p
        m.mul_(b1).add_(g, alpha=1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        t = step.to(torch.float64)
        bc1 = 1 - torch.pow(torch.full_like(t, b1), t)
        bc2 = 1 - torch.pow(torch.full_like(t, b2), t)
        denom = (v.sqrt() / torch.sqrt(bc2).to(v.dtype)).add_(eps)
        p.sub_((lr / bc1).to(p.dtype) * (m / denom))

    # ------------------------------------------------------------------ generation decode
    def sample_decode(self, logits, out, tabs, stream_id=0):
        """Fused activate + VGM/categorical decode of generated rows.

        out: [N, n_cols] float64 (continuous columns: value; categorical: label code).
        tabs: dict with host lists 'cols' of (kind, data_start, width, j_cont, i2s_codes).
        """
        N = logits.shape[0]
        for j, (kind, s, w, c, codes) in enumerate(tabs["cols"]):
            if kind == 0:  # continuous: alpha = tanh(logit); mode = argmax(logits + gumbel)
                alpha = torch.tanh(logits[:, s]).clamp(-1, 1)
                x = logits[:, s + 1:s + 1 + w]
                u = torch.rand(x.shape, device=x.device, dtype=x.dtype).clamp_(1e-20, 1.0 - 1e-7)
                k = (x - torch.log(-torch.log(u))).argmax(1)
                mu = tabs["mu"][c][k]
                sd = tabs["sd"][c][k]
                out[:, j] = (alpha.double() * 4 * sd + mu)
            else:
                x = logits[:, s:s + w]
                u = torch.rand(x.shape, device=x.device, dtype=x.dtype).clamp_(1e-20, 1.0 - 1e-7)
                k = (x - torch.log(-torch.log(u))).argmax(1)
                out[:, j] = codes[k].double()
        return out
