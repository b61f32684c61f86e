"""HIP backend of the engine ops: thin dispatch onto ``torch.ops.fedtgan`` (csrc/).

Same method signatures as :class:`fed_tgan_amd.ops.ref.TorchOps`.  There is no silent
fallback: constructing :class:`HipOps` raises if the native library is not built or does not
load.  Host-side work per call is limited to picking split-K factors, caching int32 span
tables on the device and reusing one split-K workspace per stream lane, so the launch sequence of a step is
static and hipGraph-capturable.

RNG bookkeeping: one device int64 step counter per engine (``self.ctr``) addresses every
Philox stream; the generator's Adam launch (last kernel of a step) bumps it, as does each
generation chunk.  Optimizer step counters are bumped by the sampler launch of the matching
phase, so Adam itself only reads them.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch

from . import native

EPI_NONE, EPI_LRELU_DROPOUT, EPI_MASK, EPI_RELU, EPI_BN_EVAL_RELU = 0, 1, 2, 3, 4


LONG_K_64 = True    # _plan's long-K rule with 64x64 tiles when workgroups are plentiful (A/B knob)
# 128x128 tiles covering less than two waves of the 256 CUs give way to 64x64 tiles when those still number
# >= 1024 (the wide table's G-out forward: 440 128-tiles, 1.7 waves, with a short K of 640) (A/B knob)
WAVE_FILL_64 = False
# long-K GEMMs over 128..255 rows (the wide table's D0 forward: 150 x 256 x 137,800) with 128x128 tiles and deep
# split-K: the 150 rows are 2 row tiles instead of 3, so W0 (141 MB) streams twice instead of three times, and X
# (83 MB) twice instead of four times (A/B knob).  Measured slower, off: wide 0.2489 / 0.2504 -> 0.2541 / 0.2552
# s/epoch (profiles/wide_r5.md)
LONG_K_128 = False


def _plan(M: int, N: int, K: int, kc: int = 128, clients: int = 1) -> tuple:
    """(output tile, split-K factor) for the burst GEMM (one K-burst = ``kc`` values per row).

    Measured on MI355X (profiles/gemm_split_sweep_r1.txt): a split costs an epilogue launch
    (~4.6 us) and 64x64 tiles leave most CUs idle on these skinny shapes, so
      * >= 256 128x128 tiles (generation at M = 40k, wide tables): 128x128, no split -- small
        tiles re-read the fp32 operands from L2 so often that the GEMM becomes L2-bound;
      * >= 256 64x64 tiles: 64x64, no split (the grid already covers the chip);
      * short K (<= 8 bursts): 32x32 tiles, no split (4x the workgroups, no epilogue) --
        e.g. 500x256x432: 5.5 us vs 7.7 us for 64x64 split 4;
      * long K: 32x32 tiles split ~512 workgroups deep (one CU pulls only ~60-100 GB/s), and
        deeper where that would leave more than ~8 bursts per split (wide tables: D0's K is
        137,800 -- 83 serial bursts at 13 splits); at least 2 bursts per split, fp32 slabs
        capped at ~6 MB.  (Every Intrusion shape keeps its measured split.)
    clients: a batched multi-client launch (models/batched.py) runs every tile once per client, so the
    grid-filling thresholds count clients x tiles (8 clients' 40 tiles need far less split-K).  D0's weight
    gradient at 8 clients (256 x 6200 x 150, 784 128-tiles) takes 128x128 tiles: the 8-client step
    709 -> 677 us against 64x64 (profiles/batched_r3.md).
    """
    c = max(1, int(clients))
    t128 = -(-M // 128) * -(-N // 128) * c
    t64 = -(-M // 64) * -(-N // 64) * c
    t32 = -(-M // 32) * -(-N // 32) * c
    bursts = -(-K // kc)
    if t128 >= 256 and K >= 128 and M >= 128:    # (a 128-row tile over < 128 rows idles its MFMA rows)
        if WAVE_FILL_64 and c == 1 and t128 < 512 and t64 >= 1024:
            return 64, 1
        return 128, 1
    if t64 >= 256:
        return 64, 1
    if bursts <= 8:
        return 32, 1
    cap_ws = max(1, (6 << 20) // max(1, M * N * 4))
    want = max(-(-512 // t32), -(-bursts // 8))
    sk32 = int(max(1, min(want, -(-bursts // 2), cap_ws)))
    if LONG_K_128 and c == 1 and 128 <= M < 256 and N >= 128 and bursts >= 256:
        want = max(-(-256 // t128), -(-bursts // 16))
        return 128, int(max(1, min(want, GEMM_MAX_SPLITS, -(-bursts // 2))))
    if LONG_K_64 and c == 1 and t32 * min(sk32, 64) >= 768:
        # plenty of workgroups either way (the wide table's K = 137k): 64x64 tiles re-read the long operands half as
        # often (the 150-row D0 input by 4 instead of 8 column tiles, W0 by 3 instead of 5 row tiles).  Measured
        # (tools/batched_ops.py): the wide table's D0 forward 101.5 -> 72.3 us; the one-client Intrusion GEMMs stay
        # below the threshold.  (8 batched clients: 42.9 -> 37.7 us for D0's forward alone, but the step lost
        # 0.3 ms per epoch -- profiles/batched_r4.md -- so batched launches keep the 32-tile plan)
        want = max(-(-512 // t64), -(-bursts // 8))
        return 64, int(max(1, min(want, -(-bursts // 2), cap_ws)))
    return 32, sk32


def _is_transposed(t) -> bool:
    """A 2-D view whose rows are strided and whose columns are contiguous in memory (W.t() of a
    row-major W) -- the GEMM library takes row-major operands, so such a view is passed as W."""
    return t is not None and t.dim() == 2 and t.shape[0] > 1 and t.shape[1] > 1 and t.stride(0) == 1 \
        and t.stride(1) != 1


def _rowmajor(t, flag: bool):
    return (t.t(), not flag) if _is_transposed(t) else (t, flag)


GEMM_MAX_SPLITS = 64   # gemm.hip: the split-K epilogue keeps every slab value in registers


def _effective_splits(K: int, sk: int, kc: int) -> int:
    """The split count launch_gemm actually runs: at most GEMM_MAX_SPLITS, K slices rounded up to
    whole bursts."""
    sk = min(sk, GEMM_MAX_SPLITS)
    if sk <= 1:
        return 1
    kchunk = -(-max(K, 1) // sk)
    kchunk = -(-kchunk // kc) * kc
    return -(-max(K, 1) // kchunk)


class HipOps:
    name = "hip"
    adam_counts_steps = False    # step counters are bumped by the sampler launch of each phase
    gemm_adam = True             # gemm(..., group=3) + adam(jobs=...) run as one launch
    achain_capable = True        # EngineConfig.fuse_achain (gemm_achain_next)
    shortk_min_n = 16384         # mirrors the native gemm_shortk_min_n (set both to route narrower products)

    def __init__(self, device: torch.device, seed: int = 0, precision: str = "bf16", mem=None):
        self.L = native.require()
        if precision not in ("bf16", "fp32"):
            raise ValueError(f"precision must be bf16 or fp32, got {precision!r}")
        self.f32 = precision == "fp32"
        self.device = device
        # every operand a training step's launches touch comes from ``mem`` (models/arena.py): for the
        # batched multi-client engine that is a client slab, and the lazily sized workspaces below are then
        # created in every slab at once
        if mem is None:
            from ..models.arena import TorchAlloc
            mem = TorchAlloc(device)
        self.mem = mem
        self.seed = int(seed) & ((1 << 62) - 1)
        self.ctr = mem.zeros(1, dtype=torch.int64)
        self.split_override = None   # int: force the split-K factor (tuning / microbenchmarks)
        self.batch_k = 1             # clients of the batched launches being issued (set_client_batch)
        self.batch_plan = True       # plan tiles / split-K over clients x tiles in a batched launch (A/B knob)
        self.tile_override = None    # 32 | 64: force the output tile (tuning / microbenchmarks)
        self.lane = 0          # set by the engine while it issues work on a side stream
        self._ws: Dict[Tuple[int, bool], torch.Tensor] = {}
        self._cnt: Dict[Tuple[int, bool], torch.Tensor] = {}
        # split-K partial slabs reduced by the last-arriving K-slice workgroup inside the GEMM launch
        # (no gemm_splitk_epilogue launch).  A/B knob, default off: bit-identical but measured slower
        # (the G-phase D0 forward 9.4 -> 11.7 us, full step 228 -> 230 us: the reducer reads its tile's
        # 13-25 write-through slabs serially; profiles/splitk_inlaunch_ab_r2.txt)
        self.splitk_inlaunch = False
        self._spans: Dict[Tuple, Tuple[torch.Tensor, ...]] = {}
        self._dec: Dict[int, Tuple] = {}
        self._dummy_i32 = mem.zeros(1, dtype=torch.int32)
        # BatchNorm(train) from the GEMM's per-tile partial statistics (gemm epilogue + bn_relu_apply)
        # instead of a separate full reduction over the batch (bn_relu_train).  A/B knob, default off:
        # measured slower in the step (224.6 -> 231.4 us; bn_relu_apply 11.3 us vs bn_relu_train 7.8 us,
        # profiles/README.md "negative results")
        self.bn_fused = False
        self._bnp: Dict[int, torch.Tensor] = {}
        # Linear -> BatchNorm(train) -> ReLU as one launch by column ownership (kernels/bn_fused.hip);
        # bf16 only.  Set from EngineConfig.bn_colown.
        self.bn_colown = False
        self._colown: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}

    # ------------------------------------------------------------------ helpers
    def set_client_batch(self, k: int, stride: int = 0, seed_step: int = 0, base: int = 0) -> int:
        """This thread's launches from here on run K clients at once (csrc/kernels/launch.h ClientBatch);
        k = 1 restores plain launches.  Returns the previous k."""
        self.batch_k = int(k)
        return int(self.L.set_client_batch(int(k), int(stride), int(seed_step), int(base)))

    def _plan_clients(self) -> int:
        return self.batch_k if self.batch_plan else 1

    def reset_held(self) -> int:
        """Drop every GEMM this thread holds for pairing / a chain / the Adam launch (see gemm's
        ``group``), unlaunched; returns how many there were."""
        return int(self.L.reset_held())

    def begin_step(self, engine) -> None:
        """A step starts with no GEMM held: a previous step that raised between a hold and its consumer
        leaves nothing behind (a stale hold would refuse every later GEMM, or be launched with operand
        pointers that no longer belong to it)."""
        n = self.reset_held()
        if n:
            import warnings
            warnings.warn(f"dropped {n} GEMM hold(s) left by an interrupted step", RuntimeWarning)

    def check(self) -> None:
        """Checked native build (FEDTGAN_CHECKED=1): raise if a kernel flagged an out-of-range table
        index since the last check (synchronises).  Release build: nothing."""
        if native.CHECKED:
            native.check()

    def _workspace(self, n: int, held: bool = False) -> torch.Tensor:
        """Split-K slab of the current lane (concurrent lanes never share one; nor do the two GEMMs
        of a pair: ``held`` = the first of the pair)."""
        key = (self.lane, held)
        ws = self._ws.get(key)
        if ws is None or ws.numel() < n:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("split-K workspace must be sized before graph capture")
            ws = self.mem.zeros(max(1 << 20, int(n * 1.25)), dtype=torch.float32)
            self._ws[key] = ws
        return ws

    def _tile_counters(self, n: int, held: bool = False) -> torch.Tensor:
        """Arrival counters of the in-launch split-K reduction (per lane / pair slot like the
        workspace; zero between launches: the reducing workgroup re-zeroes its tile's counter)."""
        key = (self.lane, held)
        t = self._cnt.get(key)
        if t is None or t.numel() < n:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("split-K tile counters must be sized before graph capture")
            t = self.mem.zeros(max(n, 4096), dtype=torch.int32)
            self._cnt[key] = t
        return t

    def _bn_partials(self, n: int) -> torch.Tensor:
        """Per-tile BN partial-statistics buffer of the current lane (sized before graph capture)."""
        t = self._bnp.get(self.lane)
        if t is None or t.numel() < n:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("BN partials buffer must be sized before graph capture")
            t = self.mem.zeros(max(n, 1 << 16), dtype=torch.float32)
            self._bnp[self.lane] = t
        return t

    def _colown_bufs(self, n: int):
        """(stat, cnt) of the current lane for linear_bn_relu_colown: the batch-statistics hand-off and
        the per-column-block arrival counters (zero between launches; sized before graph capture)."""
        t = self._colown.get(self.lane)
        if t is None or t[0].numel() < 4 * n:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("colown buffers must be sized before graph capture")
            m = max(n, 1024)
            t = (self.mem.zeros(4 * m, dtype=torch.float32), self.mem.zeros(-(-m // 16), dtype=torch.int32))
            self._colown[self.lane] = t
        return t

    def _colown_ok(self, x, W, nhat, groups) -> bool:
        if not (self.bn_colown and not self.f32 and nhat is not None and groups in (1, 2)):
            return False
        rows, K = x.shape
        if rows % groups or rows // groups < 2 or x.stride(1) != 1:
            return False
        kp = -(-K // 32) * 32 + 8
        return 16 * kp * 2 + (rows // groups * 21 + 2052) * 4 <= 64 * 1024

    def _span_tables(self, spans, cond_spans=None):
        key = (tuple(spans), tuple(cond_spans or ()))
        t = self._spans.get(key)
        if t is None:
            cidx = []
            cpos = {s: i for i, (s, _w) in enumerate(cond_spans or [])}
            ci = 0
            for s, w, k in spans:
                if k == 1:
                    cidx.append(cpos.get(s, ci) if cond_spans else ci)
                    ci += 1
                else:
                    cidx.append(-1)
            elem = []      # data column -> span index, | 1 << 30 for softmax spans (kernel-side einfo)
            for i, (s, w, k) in enumerate(spans):
                elem.extend([i | ((1 << 30) if k != 0 else 0)] * w)
            st, wd, kd = [s for s, _, _ in spans], [w for _, w, _ in spans], [k for _, _, k in spans]
            # the LDS image the activation kernels stage: [elem | kind | start | width | cidx], padded to 4
            packed = elem + kd + st + wd + cidx
            packed += [0] * (-len(packed) % 4)
            mk = lambda v: self.mem.tensor(np.asarray(v, dtype=np.int32))  # noqa: E731
            t = (mk(st), mk(wd), mk(kd), mk(cidx), mk(packed))
            self._spans[key] = t
        return t

    # ------------------------------------------------------------------ GEMM
    def gemm(self, a, b, c, ta=False, tb=False, alpha=1.0, beta=0.0, bias=None, epi=EPI_NONE, ms=None,
             slope=0.2, p_drop=0.5, stream_id=0, bn=None, bn_eps=1e-5, head=None, group=0, onehot=None,
             bn_part=None, bn_rpg=0, tile=None, chain=False, splitk=None):
        """C = epi(alpha op(A) op(B) + beta C + bias [+ onehot]).  head = (coef [M], v [N], A_out [M, N]):
        with the LeakyReLU+dropout epilogue also A_out = coef v^T * mask-slopes (D's head seed).
        onehot = (W_c [N, C], col [M], opt [M], cond_offset[, transposed]): A holds only the dense input
        columns; the trailing one-hot block contributes W_c[n, cond_offset[col[m]] + opt[m]] (a gather, no
        MFMA).  transposed: W_c is given as [C, N] (contiguous rows: coalesced gathers).
        group 1 holds this GEMM, group 2 launches it together with the held one in ONE kernel (the
        two must be independent); group 3 holds a weight gradient (plain epilogue, inside an optimizer's
        gradient buffer) for the next adam(..., jobs=...), which then runs both in ONE kernel, the GEMM's
        tiles applying Adam to their outputs; 0 launches now.
        group 4 holds a chain tail C2 = epi2(C B2^T + bias2) whose A operand is the output C of the next
        gemm(..., chain=True): the tail is computed row by row (fp32 dots) in that GEMM's split-K
        reduction launch (the discriminator's second layer and its R-chain link: one launch each saved).
        Transposed views (unit row stride, e.g. the input-major generator weights of EngineConfig.g_wt)
        are passed as their row-major storage with the transposition flag flipped; a transposed C is
        computed as C^T = op(B)^T op(A)^T (plain epilogue only)."""
        a, ta = _rowmajor(a, ta)
        b, tb = _rowmajor(b, tb)
        if _is_transposed(c):
            if bias is not None or epi != EPI_NONE or onehot is not None or head is not None or bn is not None \
                    or bn_part is not None or chain:
                raise ValueError("gemm: a transposed output takes no bias / epilogue / one-hot term")
            a, b, ta, tb, c = b, a, not tb, not ta, c.t()
        if onehot is not None and _is_transposed(onehot[0]):
            if len(onehot) > 4 and onehot[4]:
                raise ValueError("gemm: one-hot block given transposed twice")
            onehot = (onehot[0].t(), onehot[1], onehot[2], onehot[3], True)
        M = a.shape[1] if ta else a.shape[0]
        K = a.shape[0] if ta else a.shape[1]
        N = b.shape[0] if tb else b.shape[1]
        kc = 64 if self.f32 else 128
        tile_p, sk = _plan(M, N, K, kc, self._plan_clients())
        tile = self.tile_override or tile or tile_p
        sk = _effective_splits(K, splitk or self.split_override or sk, kc)
        if c.dtype == torch.bfloat16:
            sk = 1          # a bf16 output is written by the GEMM's own epilogue
        ws = cnt = None
        if sk > 1:
            ws = self._workspace(sk * M * N, held=group == 1)
            if self.splitk_inlaunch:
                cnt = self._tile_counters(-(-M // tile) * -(-N // tile), held=group == 1)
        g = bn or (None, None, None, None)
        self.L.gemm(a, b, c, bool(ta), bool(tb), float(alpha), float(beta), bias, int(epi), ms, float(slope),
                    float(p_drop), ws, int(sk), self.seed, self.ctr, int(stream_id), g[0], g[1], g[2], g[3],
                    float(bn_eps), self.f32, *(head or (None, None, None)), int(tile), int(group),
                    *(onehot[:4] if onehot else (None, None, None, None)),
                    bool(onehot is not None and len(onehot) > 4 and onehot[4]), bn_part, int(bn_rpg), cnt,
                    bool(chain))

    def gemm_plan(self, M: int, N: int, K: int) -> Tuple[int, int]:
        """(output tile, split-K factor) gemm() picks for an M x N x K product on this backend."""
        kc = 64 if self.f32 else 128
        tile, sk = _plan(M, N, K, kc, self._plan_clients())
        return self.tile_override or tile, _effective_splits(K, self.split_override or sk, kc)

    def shortk_ok(self, M: int, N: int, K: int) -> bool:
        """Does C [M, N] = A^T B over K rows run as the short-K strip kernel (csrc gemm_shortk_kernel; the shape
        contract of gemm_shortk_ok for 16-B aligned row-major operands, default gemm_shortk_min_n)?"""
        return (not self.f32 and getattr(self, "batch_k", 1) == 1 and M <= 256 and M % 4 == 0 and 1 <= K <= 160
                and N % 4 == 0 and N >= self.shortk_min_n)

    def gemm_achain_next(self, out, ws, cnt):
        """The next chain tail (gemm(..., group=4) with a head seed) also forms the head's backward link
        out = (A1 W1) . MS0 in the chain launch (csrc/kernels/launch.h GemmArgs::ach_*, EngineConfig.fuse_achain)."""
        self.L.gemm_achain_next(out, ws, cnt)

    def linear_bn_relu(self, x, W, b, gamma, beta, out, abuf, nhat, mean, invstd, rmean, rvar, training=True,
                       momentum=0.1, eps=1e-5, groups=1, onehot=None):
        """groups = 2: the rows are two batches (BN statistics per batch, running stats updated
        batch after batch); mean / invstd are then [2, cols].  onehot: see gemm."""
        if training and self._colown_ok(x, W, nhat, groups):
            stat, cnt = self._colown_bufs(W.shape[0])
            oh = onehot or (None, None, None, None)
            self.L.linear_bn_relu_colown(x, W, b, gamma, beta, out, nhat, mean, invstd, rmean, rvar, float(momentum),
                                         float(eps), int(groups), oh[0], oh[1], oh[2], oh[3],
                                         bool(onehot is not None and len(onehot) > 4 and onehot[4]), stat, cnt)
            return
        if training:
            M, N, K = x.shape[0], W.shape[0], x.shape[1]
            kc = 64 if self.f32 else 128
            tile, sk = _plan(M, N, K, kc, self._plan_clients())
            tile = self.tile_override or tile
            sk = _effective_splits(K, self.split_override or sk, kc)
            if self.bn_fused and tile in (32, 64) and sk == 1 and -(-M // tile) <= 64:
                # the GEMM epilogue writes per-tile (count, mean, M2) per column and batch; the BN
                # kernel merges them (no reduction over the rows) and normalises many row blocks
                nt = -(-M // tile)
                part = self._bn_partials(nt * 6 * N)
                self.gemm(x, W, abuf, tb=True, bias=b, onehot=onehot, bn_part=part, bn_rpg=M // groups)
                self.L.bn_relu_apply(abuf, part, nt, gamma, beta, out, nhat, mean, invstd, rmean, rvar, float(momentum),
                                     float(eps), int(groups))
                return
            # (fusing the split-K reduction into this BN launch was measured slower: the BN grid
            # has only cols/16 workgroups to pull the slabs -- profiles/README.md)
            self.gemm(x, W, abuf, tb=True, bias=b, onehot=onehot)
            self.L.bn_relu_train(abuf, gamma, beta, out, nhat, mean, invstd, rmean, rvar, float(momentum), float(eps),
                                 int(groups))
        else:
            self.gemm(x, W, out, tb=True, bias=b, epi=EPI_BN_EVAL_RELU, bn=(gamma, beta, rmean, rvar), bn_eps=eps,
                      onehot=onehot)

    def bn_relu_fwd(self, a, gamma, beta, out, nhat, mean, invstd, rmean, rvar, training=True, momentum=0.1,
                    eps=1e-5, groups=1):
        if not training:
            raise NotImplementedError("eval-mode BN is fused into the GEMM epilogue on the HIP backend")
        self.L.bn_relu_train(a, gamma, beta, out, nhat, mean, invstd, rmean, rvar, float(momentum), float(eps),
                             int(groups))

    bn_pair_capable = True

    def bn_relu_bwd(self, dr, r, nhat, gamma, invstd, da, dgamma, dbeta, dbias=None, paired=False):
        """paired: the GEMM held with gemm(..., group=1) runs in the same launch (an independent weight gradient
        beside the BN backward's narrow column workgroups, csrc gemm_bnbwd_kernel)."""
        self.L.bn_relu_bwd(dr, r, nhat, gamma, invstd, da, dgamma, dbeta, dbias, bool(paired))

    # ------------------------------------------------------------------ samplers
    def sample_train(self, t, h, z_cols, c_cols, x_fake, x_real, Dd, col_out, opt_out, step_counter=None,
                     metrics=None, zero_metrics=False, stream_id=0, draws=1, strides=(0, 0, 0)):
        """x_real may cover only the leading x_real.shape[0] rows of h / x_fake: those rows are the
        D-phase batch, the rest a G-phase batch drawn by the same launch.  step_counter: a device
        counter or a pair of them, bumped by the launch.  draws > 1: the batches of that many consecutive
        steps (strides = element offsets between the draws' h / D-input / col-opt buffers; step_counter and
        metrics are then per-step arrays, see SampleArgs::draws)."""
        E = z_cols[1] - z_cols[0]
        sc = step_counter if isinstance(step_counter, (tuple, list)) else (step_counter, None)
        if x_real is not None:
            self.L.sample(h, z_cols[0], c_cols[0], E, x_fake, x_real, Dd, t["cdf_log"], t["cond_offset"],
                          t["cond_width"], t["row_offset"], t["row_count"], t["rows"], t["data"], col_out, opt_out,
                          sc[0], sc[1], metrics, bool(zero_metrics), self.seed, self.ctr, int(stream_id) * 16,
                          int(draws), *(int(x) for x in strides))
        else:
            self.L.sample(h, z_cols[0], c_cols[0], E, x_fake, None, Dd, t["cdf_log"], t["cond_offset"],
                          t["cond_width"], None, None, None, None, col_out, opt_out, sc[0], sc[1], metrics,
                          bool(zero_metrics), self.seed, self.ctr, int(stream_id) * 16)

    def sample_gen(self, t, h, c_cols, z_cols, col_out=None, opt_out=None, stream_id=0, ctr=None):
        """ctr: the step counter to key the draws on (default the engine's; the pipelined generation passes its
        snapshot)."""
        E = z_cols[1] - z_cols[0]
        self.L.sample(h, z_cols[0], c_cols[0], E, None, None, 0, t["cdf_emp"], t["cond_offset"], t["cond_width"],
                      None, None, None, None, col_out, opt_out, None, None, None, False, self.seed,
                      self.ctr if ctr is None else ctr, int(stream_id) * 16)

    # ------------------------------------------------------------------ activations
    def activate(self, logits, out, spans, tau=0.2, stream_id=0, slerp=None):
        """Per-span tanh / Gumbel-softmax.  slerp = (real, fake_full, interp, stream_id): also
        interp = slerp(real, fake_full) in the same launch (fake_full = out's rows continued by
        their conditional columns)."""
        st, w, k, ci, el = self._span_tables(spans)
        if slerp is None:
            sr, so, cols, ss = None, None, 0, 0
        else:
            sr, fake_full, so, sid = slerp
            cols, ss = int(fake_full.shape[1]), int(sid) * 16
        self.L.activate(logits, out, st, w, k, ci, el, float(tau), self.seed, self.ctr, int(stream_id) * 16, sr, so,
                        cols, ss)

    def linear_activate(self, x, W, b, logits, out, spans, tau=0.2, stream_id=0, slerp=None, onehot=None, tile=None,
                        splitk=None):
        """logits = x W^T + b; out = activate(logits) (optionally + the fused slerp)."""
        self.gemm(x, W, logits, tb=True, bias=b, onehot=onehot, tile=tile, splitk=splitk)
        self.activate(logits, out, spans, tau, stream_id, slerp=slerp)

    def act_bwd_ce(self, dact, act, logits, spans, cond_spans, col, opt, dlogits, loss_out, tau=0.2):
        st, w, k, ci, el = self._span_tables(spans, cond_spans)
        self.L.act_bwd_ce(dact, act, logits, st, w, k, ci, el, col, opt, dlogits, loss_out, float(tau))

    # ------------------------------------------------------------------ gradient penalty
    def slerp(self, real, fake, out, stream_id=0):
        self.L.slerp(real, fake, out, self.seed, self.ctr, int(stream_id) * 16)

    def gp_scale(self, g, out, lam, loss_out):
        ws = None
        if g.shape[1] > 8192:      # chunk partials of the split launch (csrc launch_gp_scale)
            n = g.shape[0] * -(-g.shape[1] // 8192)
            ws = self._gpws if getattr(self, "_gpws", None) is not None and self._gpws.numel() >= n else None
            if ws is None:
                if torch.cuda.is_current_stream_capturing():
                    raise RuntimeError("gp_scale workspace must be sized before graph capture")
                ws = self._gpws = self.mem.zeros(n, dtype=torch.float32)
        self.L.gp_scale(g, out, float(lam), loss_out, ws)

    # ------------------------------------------------------------------ one-hot input block weight gradients
    def onehot_wgrad(self, dys, ws, col, opt, cond_off, zero: bool = False):
        """ws[j][k] = sum of dys[j] rows r with cond_off[col[r]] + opt[r] == k (batch order); the other rows of
        ws[j] must be zero and stay untouched.  zero=True clears the rows this batch touched instead."""
        self.L.onehot_wgrad(list(dys), list(ws), col, opt, cond_off, 1 if zero else 0)

    def d_head(self, d_last, ms_last, v, e, coef, wloss, y, a_last, loss_out):
        self.L.d_head(d_last, ms_last, v, e, coef, wloss, y, a_last, loss_out)

    def colsum(self, a, out, beta=0.0):
        if beta != 0.0:
            raise NotImplementedError
        self.L.colsum([a], [out])

    @staticmethod
    def _dot_lists(dots, n):
        dots = dots or [None] * n
        return ([d[0] if d else None for d in dots], [d[1] if d else None for d in dots],
                [d[2] if d else None for d in dots], [d[3] if d and len(d) > 3 else None for d in dots])

    def colsum_many(self, srcs, outs, weights=None, dots=None):
        """out_i = sum_r w_i[r] src_i[r, :] (out_i may be None); dots[i] = (v, e, loss[, u]): loss +=
        sum_r u[r] (src_i[r] . v + e) in the same launch (the WGAN term of the D head), u = w_i
        unless given."""
        if weights is not None or dots is not None:
            n = len(srcs)
            weights = weights or [None] * n
            self.L.colsum_ex(list(srcs), list(outs), list(weights), *self._dot_lists(dots, n))
            return
        self.L.colsum(list(srcs), list(outs))

    # ------------------------------------------------------------------ optimizer
    def gemm_is_split(self, M: int, N: int, K: int) -> bool:
        """Does a GEMM of this shape get a split-K reduction launch (the launch a chain tail rides on)?"""
        kc = 64 if self.f32 else 128
        _, sk = _plan(M, N, K, kc, self._plan_clients())
        return _effective_splits(K, self.split_override or sk, kc) > 1 and not self.splitk_inlaunch

    def adam(self, p, g, m, v, step, lr, b1, b2, eps, wd, last_in_step=False, jobs=None):
        """Adam over a flat buffer.  jobs = (srcs, outs, weights, dots) as for colsum_many: the column
        sums run in the same launch, and outputs inside g get their Adam update from the sums."""
        bump = self.ctr if last_in_step else None
        if jobs is None:
            self.L.adam(p, g, m, v, step, float(lr), float(b1), float(b2), float(eps), float(wd), bump)
            return
        srcs, outs, weights, dots = jobs
        n = len(srcs)
        weights = weights or [None] * n
        self.L.adam_cs(p, g, m, v, step, float(lr), float(b1), float(b2), float(eps), float(wd), bump, list(srcs),
                       list(outs), list(weights), *self._dot_lists(dots, n))

    # ------------------------------------------------------------------ generation decode
    def _decode_tables(self, tabs):
        key = id(tabs)
        t = self._dec.get(key)
        if t is None:
            kind, start, width, cont, code_off, codes = [], [], [], [], [], []
            for kk, s, w, c, cd in tabs["cols"]:
                kind.append(kk)
                start.append(s)
                width.append(w)
                cont.append(max(c, 0))
                code_off.append(len(codes))
                if cd is not None:
                    codes.extend(cd.detach().cpu().tolist())
            mk = lambda v: torch.tensor(v, dtype=torch.int32, device=self.device)  # noqa: E731
            codes_t = torch.tensor(codes if codes else [0.0], dtype=torch.float64, device=self.device)
            mu = tabs["mu"].to(self.device, torch.float64).contiguous()
            sd = tabs["sd"].to(self.device, torch.float64).contiguous()
            if mu.numel() == 0:
                mu = torch.zeros(1, 1, dtype=torch.float64, device=self.device)
                sd = torch.ones(1, 1, dtype=torch.float64, device=self.device)
            t = (mk(kind), mk(start), mk(width), mk(cont), mk(code_off), codes_t, mu, sd)
            self._dec[key] = t
        return t

    def _decode_ecol(self, tabs, dim: int):
        """[dim] int32: output column whose Gumbel argmax each logit enters (-1: none, e.g. the
        tanh unit of a continuous column) -- the one-wave-per-row decode kernel's element map."""
        key = (id(tabs), int(dim))
        e = self._dec.get(key)
        if e is None:
            ec = np.full(int(dim), -1, dtype=np.int32)
            for j, (kk, s, w, _, _) in enumerate(tabs["cols"]):
                o = s + 1 if kk == 0 else s
                ec[o:o + w] = j
            e = torch.from_numpy(ec).to(self.device)
            self._dec[key] = e
        return e

    def _decode_quads(self, tabs, dim: int):
        """[n, 2] int32: every run of up to 4 logits of one column that share a Philox word
        ({column | count << 24, offset-in-span << 16 | position}), the quad decode kernel's work list."""
        key = ("quads", id(tabs), int(dim))
        q = self._dec.get(key)
        if q is None:
            ent = []
            for j, (kk, s, w, _, _) in enumerate(tabs["cols"]):
                off = s + 1 if kk == 0 else s
                for i0 in range(0, w, 4):
                    cnt = min(4, w - i0)
                    if off + i0 + cnt > dim or j >= (1 << 24):
                        raise ValueError("decode tables do not fit the logits")
                    ent.append((j | (cnt << 24), (i0 << 16) | (off + i0)))
            q = torch.tensor(ent if ent else [(0, 0)], dtype=torch.int32, device=self.device).view(-1, 2)
            if not ent:
                q = q[:0]
            self._dec[key] = q
        return q

    def sample_decode(self, logits, out, tabs, stream_id=0, ctr=None):
        ctr = self.ctr if ctr is None else ctr
        kind, start, width, cont, code_off, codes, mu, sd = self._decode_tables(tabs)
        self.L.sample_decode(logits, out, kind, start, width, cont, code_off, codes, mu, sd, self.seed, ctr,
                             int(stream_id) * 16, self._decode_ecol(tabs, logits.shape[1]),
                             self._decode_quads(tabs, logits.shape[1]))
        self.L.rng_bump(ctr)
        return out
