"""CTGANEngine — the production WGAN-GP training/generation path on flat buffers.

Where the reference runs ``nn.Module`` forward passes plus autograd's double backward
with ~3.8k ATen dispatches per step and host-side NumPy samplers
(`Client/.../dtds/distributed.py:179-269`, `Server/dtds/synthesizers/ctgan.py:231-258`),
this engine:

* keeps every trainable tensor of G and D plus the BN running statistics in ONE flat fp32
  buffer (``self.flat``: ``[theta_G | theta_D | BN buffers]``) so federated aggregation is a
  single pre-scaled all-reduce and Adam is one fused multi-tensor kernel per network;
* lays out activations concat-free: the generator's residual stack writes every layer's
  ``ReLU(BN(.))`` into a column slice of one ``[B, E+n_opt+sum(gen_dims)]`` buffer, so
  ``cat([out, input])`` (`ctgan.py:44`) is free; the discriminator's fake / real /
  interpolated batches share one ``[3B, data_dim+n_opt]`` buffer whose packed view is the
  PacGAN input (`ctgan.py:28-30`);
* runs an **explicit** backward, including the hand-derived gradient-penalty double
  backward (see ``_d_step``), as a short chain of GEMMs with fused epilogues;
* draws conditional vectors, real rows, noise, Gumbel noise, dropout masks and slerp
  weights on the device, so a whole step is a static sequence of kernel launches that is
  captured once into a hipGraph and replayed.

Step semantics follow the reference client exactly (`Client/.../distributed.py:185-265`):
D step on ``loss_d = mean D(fake) - mean D(real) + GP`` then G step on
``-mean D(fake) + cond_loss``; G's BN layers run in training mode in both phases; the
gradients that the reference computes and then discards (G grads from the D phase, D
grads from the G phase) are not computed.

Gradient-penalty backward (D with hidden layers l = 0..L-1, weights V_l, dropout-masked
LeakyReLU slopes MS_l = lrelu'(u_l) * mask_l, head vector v):
    q_{L-1} = v * MS_{L-1};  q_{l-1} = (q_l V_l) * MS_{l-1};  g = q_0 V_0   (= dD/dx)
    pen = lam * mean_p (|g_p| - 1)^2;   R_{-1} = dpen/dg
    R_l = (R_{l-1} V_l^T) * MS_l;   dpen/dV_l = q_l^T R_{l-1};   dpen/dv = sum_p R_{L-1,p}
Bias gradients of the penalty are exactly zero.  The same A-chain serves the WGAN terms
of the fake/real rows (seed coefficient +-1/n_packs), so every weight gradient of the D
step is ONE GEMM over the stacked [fake; real; interp] rows.
"""
from __future__ import annotations

import contextlib
import dataclasses
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..features.transformer import SpanLayout
from .arena import TorchAlloc
from .ctgan import Discriminator, Generator
from .samplers import CondTables, RowIndex

EPI_NONE, EPI_LRELU_DROPOUT, EPI_MASK, EPI_RELU = 0, 1, 2, 3


def _ceil4(n: int) -> int:
    return (int(n) + 3) // 4 * 4


def _padded_rows(rows: int, cols: int, mem) -> torch.Tensor:
    """[rows, cols] view of a zeroed [rows, ceil4(cols)] buffer (16-B aligned row starts); ``mem`` is an
    allocator (models/arena.py) or a device."""
    if not hasattr(mem, "zeros"):
        mem = TorchAlloc(mem)
    return mem.zeros(rows, _ceil4(cols), dtype=torch.float32)[:, :cols]


def _ext(t: torch.Tensor, cols: int) -> torch.Tensor:
    """Widen a row-strided 2-D view to ``cols`` columns, into its storage's zero padding."""
    if t.shape[1] == cols:
        return t
    return t.as_strided((t.shape[0], cols), t.stride(), t.storage_offset())


@dataclasses.dataclass
class EngineConfig:
    embedding_dim: int = 128
    gen_dims: Tuple[int, ...] = (256, 256)
    dis_dims: Tuple[int, ...] = (256, 256)
    batch_size: int = 500
    pack: int = 10
    lr: float = 2e-4
    betas: Tuple[float, float] = (0.5, 0.9)
    adam_eps: float = 1e-8
    l2scale: float = 1e-6
    tau: float = 0.2
    gp_lambda: float = 10.0
    lrelu_slope: float = 0.2
    dropout_p: float = 0.5
    bn_momentum: float = 0.1
    bn_eps: float = 1e-5
    gen_chunk: int = 40960       # rows per generation pass (40k in one pass: 128x128-tile GEMMs, 455 vs 716 us)
    gen_graph: bool = True      # GPU: replay the generation pass (per sample count) as one hipGraph
    precision: str = "bf16"     # GEMM operands on the HIP path: bf16 (fp32 accumulate) or exact fp32
    graph_unroll: int = 8       # GPU: training steps captured per hipGraph (fewer graph launches)
    # GPU, one client: blocks of graph_unroll steps captured in ONE hipGraph (each block with its own multi-step
    # sampler launch on the same buffer sets, so nothing but the graph boundary changes); 0 = as many as an epoch
    # holds.  A/B knob, default 1: the device idles ~8.5 us between consecutive replays (step_breakdown_r6.txt),
    # but one 80-step graph per epoch measured slower -- bench 15.98-16.41 vs 15.83-16.24 ms, the train phase
    # 15.27-15.82 vs 15.20-15.24 ms (profiles/graph_blocks_r6.txt), as 40-step graphs did (multi_draw_ab_r6.txt)
    graph_blocks: int = 1
    streams: bool = False       # GPU: overlap independent launches of a step on side HIP streams
    paired: bool = True         # draw + generate the D- and G-phase batches of a step in one pass
    # generator GEMMs multiply only the dense part of their input [... | z | c]; the one-hot
    # conditional block c (exactly one 1 per row) is a gathered weight column in the epilogue
    onehot: bool = True
    onehot_trans: bool = False   # training: gather from per-step [C, N] copies (A/B knob; generation always does)
    dw0_tile: int = 0            # HIP: output tile of D0's weight-gradient GEMM (0 = planner's choice)
    # HIP, bf16 precision: generation keeps its activations and weight copies in bf16 (the values the
    # fp32 path rounds to bf16 when staging its GEMM operands, so the output is bit-identical) --
    # half the GEMM operand bytes and no one-hot block written into the activation buffer
    gen_bf16: bool = True
    # generator weights stored input-major (W^T, [in, out] rows) in the flat buffer: the one-hot block's
    # weights for a condition are then one contiguous row, so the epilogue gathers of G0 / G1 / G-out
    # read whole cache lines (with [out, in] rows a gather touches one line per output column).  The
    # views self.p / self.g stay the logical [out, in] (transposed views); state dicts are unchanged.
    g_wt: bool = True
    # HIP: the generator's first-layer weight gradient (the step's last GEMM) runs in the same launch
    # as the generator's Adam, its tiles applying Adam to their own outputs (gemm_adam_kernel)
    fuse_g_adam: bool = True
    # HIP, two hidden D layers: R1 = (R0 W1^T) * MS1 is computed in R0's split-K reduction launch, so
    # D1's weight gradient is the last D GEMM and shares its launch with the D Adam (as fuse_g_adam)
    fuse_d_adam: bool = True
    # the two fusions above only up to this many optimizer elements per launch (parameters x batched clients;
    # 0 = no limit): a fused launch gets the GEMM tile's LDS for every workgroup, so its Adam workgroups run at
    # 2 per CU -- fine for a few M parameters, HBM-starved for the wide table's 35-55 M (A/B knob)
    fuse_adam_max: int = 0
    # HIP, two hidden D layers: the second layer's forward is computed row by row in the first layer's
    # split-K reduction launch (chain_epilogue_kernel)
    chain_d1: bool = True
    # HIP, with chain_d1 on one client: the backward link A0 = (A1 W1) . MS0 is formed in the same chain launch
    # (each workgroup's 64-column slab of A1 times the W1 rows it just used, slabs summed by the row group's last
    # workgroup) instead of an A-chain GEMM launch after it.  A/B knob, default off: measured 191.0-192.1 us/step
    # with it vs 188.6-192.4 without (two fewer launches, but every chain workgroup re-reads its 64 W1 rows and
    # the row group's last one sums the slabs serially; profiles/achain_r6.txt)
    fuse_achain: bool = False
    # HIP, where fuse_d_adam does not apply (the batched multi-client step): D0's weight gradient -- the
    # largest gradient, 256 x 10 Din -- is held for the D Adam launch instead of sharing a launch with R0, so
    # it is never written and re-read through HBM (gemm_adam_kernel's tiles update it in place).  A/B knob,
    # default off: measured slower (8 clients 675 -> 773 us per step, 4 clients 412 -> 437 us: the 64-tile
    # Adam epilogue's per-element p / m / v traffic and R0 losing its pair partner cost more than the
    # 51 MB gradient round trip saves; profiles/batched_r3.md)
    fuse_d0_adam: bool = False
    # HIP, one client: D0's weight gradient, when it is a short-K product the persistent strip kernel takes
    # (ops.shortk_ok: <= 256 x wide N over <= 160 rows -- the wide table's 256 x 137,800 over 150), applies Adam in
    # that kernel's epilogue right before the optimizer launch, which skips its range: the 141 MB gradient is
    # neither written nor re-read.  A/B knob, default off: bitwise the same training, but measured slower (wide
    # 0.2334-0.241 s/epoch against 0.2275-0.2286 on one box): the kernel's parameter / moment traffic comes as
    # 256 rows x 128 B per strip (rows 551 KB apart) instead of the float4 Adam's contiguous stream, and runs at
    # ~3.7 TB/s where the Adam launch runs at ~6 (profiles/wide_r6.md)
    fuse_d0_shortk: bool = False
    # every launch stores the step's parameter gradients in the flat gradient buffers (gradient tests, grad-flow
    # diagnostics -- FedRuntime sets CTGANEngine.keep_grads for those); off, a fused optimizer epilogue may skip a
    # gradient nothing reads (fuse_d0_shortk)
    keep_grads: bool = False
    # HIP, bf16: each generator layer's Linear -> BatchNorm(train) -> ReLU as ONE launch, a workgroup
    # owning 16 output columns of one batch (kernels/bn_fused.hip) instead of a tile GEMM + BN launch
    bn_colown: bool = False
    # initial weights drawn from a generator of the engine's own, seeded by the engine seed ("engine": reproducible
    # whatever other threads do), or from torch's process-wide generator ("global", the reference modules' init)
    init_rng: str = "engine"
    # HIP, one-hot conditions: a generator weight gradient whose condition block (C rows of the input-major
    # weight x out) has at least this many elements is not a dense GEMM over the one-hot columns: its block rows
    # are the sums of the batch rows' upstream gradients per condition index (ops.onehot_wgrad; the block stays
    # zero between steps).  The wide table's G.out gradient: 7,018 x 7,402 dense (228 us) -> 7,018 x 640 + 500
    # scattered rows.  0 = always dense.
    onehot_wgrad_min: int = 1 << 20
    # (BatchNorm(train) + ReLU folded into the generator GEMMs around it -- round 5's bn_fold / bn_fold_publish --
    # measured slower in every variant, +11.5 / +20 us per step (profiles/bn_fold_r5.txt), and was removed.)
    # HIP step graphs (paired step, one client): ONE sampler launch at the head of each graph replay draws the
    # batches of all graph_unroll steps (step k keyed on RNG step ctr + k, into batch-buffer set k) instead of a
    # sampler launch heading every step -- bitwise the same draws; the launch is off the per-step serial path
    multi_draw: bool = True
    # HIP, paired step: each generator layer's BatchNorm + ReLU backward shares its launch with the weight gradient
    # of the layer above (independent of it; csrc gemm_bnbwd_kernel) instead of the weight gradient sharing a launch
    # with that layer's dH product -- the BN backward's 32-64 narrow workgroups then no longer run alone on the chip.
    # Off: measured no gain (189.6-191.0 us/step in every layout vs 189.0-190.2 without; profiles/bn_pair_r6.txt) --
    # the dH products lose the launch they shared with the weight gradients as much as the BN backward gains
    bn_pair: bool = False


def get_ops(backend: str, device: torch.device, seed: int = 0, precision: str = "bf16", mem=None):
    if backend == "auto":
        backend = "hip" if device.type == "cuda" else "torch"
    if backend == "torch":
        from ..ops.ref import TorchOps
        return TorchOps()
    if backend == "hip":
        if device.type != "cuda":
            raise ValueError("the hip backend needs a GPU device")
        from ..ops.hip import HipOps
        return HipOps(device, seed, precision, mem=mem)
    raise ValueError(backend)


class CTGANEngine:
    def __init__(self, layout: SpanLayout, cfg: EngineConfig | None = None, device="cpu", backend: str = "auto",
                 seed: int | None = None, mem=None):
        self.cfg = cfg = cfg or EngineConfig()
        self.layout = layout
        self.device = torch.device(device)
        # every buffer a training step touches comes from ``mem`` (models/arena.py): plain torch memory, or a
        # client slab of the batched multi-client engine (models/batched.py)
        self.mem = mem or TorchAlloc(self.device)
        self.seed = int(seed if seed is not None else torch.initial_seed() % (2 ** 31))
        self.ops = get_ops(backend, self.device, self.seed, cfg.precision, mem=self.mem)
        if hasattr(self.ops, "bn_colown"):
            self.ops.bn_colown = bool(cfg.bn_colown)
        B, P = cfg.batch_size, cfg.pack
        if B % P:
            raise ValueError("batch_size must be a multiple of pack")
        self.B, self.P, self.nP = B, P, B // P
        self.E = cfg.embedding_dim
        self.C = layout.n_opt
        self.Dd = layout.data_dim
        self.Din = self.Dd + self.C
        self.K1 = P * self.Din
        self.gdims = list(cfg.gen_dims)
        self.ddims = list(cfg.dis_dims)
        self.d0 = self.E + self.C
        self.Hw = self.d0 + sum(self.gdims)
        # column offsets in H: layer l (0-based) reads H[:, off[l]:], writes H[:, off[l+1]:off[l]]
        off = [sum(self.gdims)]
        for g in self.gdims:
            off.append(off[-1] - g)
        self.off = off            # off[0] = start of z, off[L] = 0
        self.z_cols = (off[0], off[0] + self.E)
        self.c_cols = (off[0] + self.E, self.Hw)
        self.spans = [(int(s), int(w), int(k)) for s, w, k in zip(layout.start, layout.width, layout.kind)]
        self.cond_spans = [(int(s), int(w)) for s, w in zip(layout.cond_start, layout.cond_width)]
        self.use_onehot = bool(cfg.onehot) and self.C > 0
        self._oh_pending = None   # one-hot block gradient rows written this step (cleared after the G Adam)
        self._cond_off = self.mem.tensor(np.asarray(layout.cond_offset, dtype=np.int32))
        self._build_params()
        self._build_buffers()
        # side streams ("lanes") for independent work inside a step; the captured graph keeps the
        # fork/join edges, so its branches run concurrently on the device
        self.lanes = None
        if self.device.type == "cuda" and cfg.streams:
            self.lanes = [None] + [torch.cuda.Stream(self.device) for _ in range(3)]
        self.tables: Dict[str, torch.Tensor] = {}
        self.gen_tables = None
        self._gen_bufs = None
        self._gen_graphs: Dict[int, tuple] = {}   # n -> (hipGraph, H, logits, out) of generate_decoded
        self._gen_split: Dict[int, tuple] = {}    # n -> (prep graph, body graph, H, logits, out, col, opt)
        self._gen_done = None                     # event: the last pipelined generation body has finished
        self.graphs: Dict[int, object] = {}    # steps per graph -> captured hipGraph
        self.capture_mode = "global"   # "thread_local" when several engines capture from threads
        self.bn_batches = 0       # num_batches_tracked of every BN layer
        self.batch = None         # models/batched.py BatchedClients when this engine issues K clients' steps
        self.pad_rows = None      # batched clients: row tables sized for the largest client (set_training_data)

    # ================================================================= parameters
    def _build_params(self):
        E, C, Dd = self.E, self.C, self.Dd
        spec: List[Tuple[str, Tuple[int, ...], str]] = []
        dim = E + C
        for i, g in enumerate(self.gdims):
            spec += [(f"G.{i}.W", (g, dim), "G"), (f"G.{i}.b", (g,), "G"),
                     (f"G.{i}.gamma", (g,), "G"), (f"G.{i}.beta", (g,), "G")]
            dim += g
        spec += [("G.out.W", (Dd, dim), "G"), ("G.out.b", (Dd,), "G")]
        dim = self.K1
        for i, h in enumerate(self.ddims):
            spec += [(f"D.{i}.W", (h, dim), "D"), (f"D.{i}.b", (h,), "D")]
            dim = h
        spec += [("D.out.W", (1, dim), "D"), ("D.out.b", (1,), "D")]
        for i, g in enumerate(self.gdims):
            spec += [(f"G.{i}.rm", (g,), "S"), (f"G.{i}.rv", (g,), "S")]
        order = {"G": 0, "D": 1, "S": 2}
        spec.sort(key=lambda t: order[t[2]])
        self.param_spec = spec
        self.wt_names, store, sizes, offsets, total = self._layout(bool(self.cfg.g_wt))
        self.flat = self.mem.zeros(total)
        self.p: Dict[str, torch.Tensor] = {}
        self.group_range = {}
        align = 16
        view = self._view

        for (name, shape, grp), n, o, st in zip(spec, sizes, offsets, store):
            self.p[name] = view(self.flat, o, n, shape, st, name, self.wt_names)
            a, _ = self.group_range.get(grp, (o, o))
            self.group_range[grp] = (a, (o + n + align - 1) // align * align)
        gA, gB = self.group_range["G"]
        dA, dB = self.group_range["D"]
        self.nG, self.nD = gB - gA, dB - dA
        self.flatG = self.flat[gA:gB]
        self.flatD = self.flat[dA:dB]
        self.gradG = self.mem.zeros(self.nG)
        self.gradD = self.mem.zeros(self.nD)
        self.g: Dict[str, torch.Tensor] = {}
        for (name, shape, grp), n, o, st in zip(spec, sizes, offsets, store):
            if grp == "S":
                continue
            base = o - (gA if grp == "G" else dA)
            self.g[name] = view(self.gradG if grp == "G" else self.gradD, base, n, shape, st, name, self.wt_names)
        self.mG = self.mem.zeros(self.nG)
        self.vG = self.mem.zeros(self.nG)
        self.mD = self.mem.zeros(self.nD)
        self.vD = self.mem.zeros(self.nD)
        # multi-step draws (EngineConfig.multi_draw): per-step optimizer counters [D | G] x U; the last entry of each
        # row is the canonical counter every other path reads and bumps
        self._U = max(1, int(self.cfg.graph_unroll))
        self._multi = bool(self.cfg.multi_draw) and self.device.type == "cuda" and getattr(self.ops, "name", "") == "hip" \
            and bool(self.cfg.paired) and not self.cfg.streams and self._U > 1 and isinstance(self.mem, TorchAlloc)
        if self._multi:
            self._step_sets = self.mem.zeros(2, self._U)
            self.stepD = self._step_sets[0, self._U - 1:]
            self.stepG = self._step_sets[1, self._U - 1:]
        else:
            self.stepG = self.mem.zeros(1)
            self.stepD = self.mem.zeros(1)
        self.reset_parameters()

    def _layout(self, g_wt: bool):
        """Flat-buffer layout of ``self.param_spec``: (input-major names, storage shapes, sizes, offsets, total).

        2-D weights are stored with their rows padded to a multiple of 4 floats (zero columns that stay
        zero under Adam, L2 decay and aggregation) and every tensor starts 16-B aligned, so the GEMMs read
        them with 16-B loads; self.p / self.g expose the logical [rows, cols] views, _ext() widens them to
        the padded width.  Input-major generator weights (g_wt): stored [ceil4(in), ceil4(out)] -- the
        zero rows past `in` let _kpad widen K to a multiple of 4 exactly as the padded columns of
        [out, ceil4(in)] do."""
        spec = self.param_spec
        wt_names = {n for n, s, grp in spec if grp == "G" and len(s) == 2} if g_wt else set()
        store = [((_ceil4(s[1]), _ceil4(s[0])) if nm in wt_names else (s[0], _ceil4(s[1]))) if len(s) == 2
                 else s for nm, s, _ in spec]
        sizes = [int(np.prod(s)) for s in store]
        # every group starts 64-byte aligned (vectorised optimizer / aggregation kernels)
        align = 16
        offsets, pos, prev = [], 0, None
        for (_, _, grp), n in zip(spec, sizes):
            if grp != prev:
                pos = (pos + align - 1) // align * align
                prev = grp
            pos = _ceil4(pos)
            offsets.append(pos)
            pos += n
        total = (pos + align - 1) // align * align
        return wt_names, store, sizes, offsets, total

    @staticmethod
    def _view(buf, o, n, shape, st, name, wt_names):
        v = buf[o:o + n].view(st)
        if name in wt_names:
            return v[:shape[1], :shape[0]].t()
        return v[:, :shape[1]] if len(shape) == 2 else v

    def convert_layout(self, bufs: Dict[str, torch.Tensor], g_wt: bool) -> Dict[str, torch.Tensor]:
        """State buffers (``flat`` and the group-relative ``mG`` ``vG`` ``mD`` ``vD``) saved with the
        generator-weight layout ``g_wt`` -> this engine's layout (a transpose of the G weight blocks and
        their Adam moments; everything else is copied).  Used to resume a checkpoint written with the
        other ``EngineConfig.g_wt``."""
        spec = self.param_spec
        wt_s, st_s, n_s, off_s, _ = self._layout(bool(g_wt))
        wt_d, st_d, n_d, off_d, _ = self._layout(bool(self.cfg.g_wt))

        def base(offs, grp):
            return min(o for (_, _, g), o in zip(spec, offs) if g == grp)
        out = {}
        for key, src in bufs.items():
            grp = None if key == "flat" else key[-1]
            if grp not in (None, "G", "D"):
                raise ValueError(f"convert_layout: unknown buffer {key!r}")
            src = src.detach().cpu()
            n = self.flat.numel() if grp is None else (self.nG if grp == "G" else self.nD)
            dst = torch.zeros(n, dtype=torch.float32)
            for i, (name, shape, g) in enumerate(spec):
                if grp is not None and g != grp:
                    continue
                bs, bd = (0, 0) if grp is None else (base(off_s, grp), base(off_d, grp))
                sv = self._view(src, off_s[i] - bs, n_s[i], shape, st_s[i], name, wt_s)
                dv = self._view(dst, off_d[i] - bd, n_d[i], shape, st_d[i], name, wt_d)
                dv.copy_(sv)
            out[key] = dst
        return out

    def _view_in(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        """Logical view of parameter ``name`` inside a group-relative buffer shaped like gradG / gradD
        (e.g. the Adam moments mG / vD)."""
        g = self.g[name]
        return buf.as_strided(g.shape, g.stride(), g.storage_offset())

    def reset_parameters(self):
        """PyTorch's default init of the reference modules (`Server/dtds/synthesizers/ctgan.py:15-64`:
        nn.Linear's kaiming-uniform weights and U(+-1/sqrt(fan_in)) biases, BN 1/0), drawn from a generator
        of this engine's own (seeded by the engine seed) instead of torch's process-wide one: client threads
        that build their engines concurrently (fed/local.py) would otherwise race on the global generator and
        an emulated federation would not reproduce run to run.  The draws go straight into the flat buffer in
        module order (weight then bias of each Linear, G then D) with nn.Linear's bounds: kaiming-uniform with
        a=sqrt(5) is U(+-1/sqrt(fan_in)).  No torch modules are built (a meta-device build imports
        torch._meta_registrations, 0.4 s of cold start)."""
        import math
        if self.cfg.init_rng == "global":      # torch's process-wide generator (the reference modules' own init)
            self.load_modules(Generator(self.E + self.C, self.gdims, self.Dd), Discriminator(self.Din, self.ddims, self.P))
            self.mG.zero_(); self.vG.zero_(); self.mD.zero_(); self.vD.zero_()
            self.stepG.zero_(); self.stepD.zero_()
            return
        gen = torch.Generator().manual_seed(self.seed)
        with torch.no_grad():
            for key, name in self.g_key_map() + self.d_key_map():
                p = self.p[name]
                if key.endswith("running_mean") or key.endswith("bn.bias"):
                    p.zero_()
                elif key.endswith("running_var") or key.endswith("bn.weight"):
                    p.fill_(1.0)
                elif key.endswith("weight"):
                    fan_in = p.shape[1]
                    bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
                    p.copy_(torch.empty(tuple(p.shape)).uniform_(-bound, bound, generator=gen))
                    wb = bound
                else:                                  # the Linear's bias, right after its weight
                    p.copy_(torch.empty(tuple(p.shape)).uniform_(-wb, wb, generator=gen))
        self.bn_batches = 0
        self.mG.zero_(); self.vG.zero_(); self.mD.zero_(); self.vD.zero_()
        self.stepG.zero_(); self.stepD.zero_()

    # --- reference-compatible state dicts ------------------------------------
    def g_key_map(self) -> List[Tuple[str, str]]:
        m = []
        for i in range(len(self.gdims)):
            m += [(f"seq.{i}.fc.weight", f"G.{i}.W"), (f"seq.{i}.fc.bias", f"G.{i}.b"),
                  (f"seq.{i}.bn.weight", f"G.{i}.gamma"), (f"seq.{i}.bn.bias", f"G.{i}.beta"),
                  (f"seq.{i}.bn.running_mean", f"G.{i}.rm"), (f"seq.{i}.bn.running_var", f"G.{i}.rv")]
        L = len(self.gdims)
        m += [(f"seq.{L}.weight", "G.out.W"), (f"seq.{L}.bias", "G.out.b")]
        return m

    def d_key_map(self) -> List[Tuple[str, str]]:
        m = []
        for i in range(len(self.ddims)):
            m += [(f"seq.{3 * i}.weight", f"D.{i}.W"), (f"seq.{3 * i}.bias", f"D.{i}.b")]
        L = len(self.ddims)
        m += [(f"seq.{3 * L}.weight", "D.out.W"), (f"seq.{3 * L}.bias", "D.out.b")]
        return m

    def g_state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {k: self.p[n].detach().contiguous().cpu().clone() for k, n in self.g_key_map()}
        for i in range(len(self.gdims)):
            sd[f"seq.{i}.bn.num_batches_tracked"] = torch.tensor(self.bn_batches, dtype=torch.int64)
        return sd

    def d_state_dict(self) -> Dict[str, torch.Tensor]:
        return {k: self.p[n].detach().contiguous().cpu().clone() for k, n in self.d_key_map()}

    def load_g_state_dict(self, sd):
        with torch.no_grad():
            for k, n in self.g_key_map():
                self.p[n].copy_(sd[k].reshape(self.p[n].shape))
        key = "seq.0.bn.num_batches_tracked"
        if key in sd:
            self.bn_batches = int(sd[key])

    def load_d_state_dict(self, sd):
        with torch.no_grad():
            for k, n in self.d_key_map():
                self.p[n].copy_(sd[k].reshape(self.p[n].shape))

    def load_modules(self, G: Generator, D: Discriminator):
        self.load_g_state_dict(G.state_dict())
        self.load_d_state_dict(D.state_dict())

    def to_modules(self) -> Tuple[Generator, Discriminator]:
        G = Generator(self.E + self.C, self.gdims, self.Dd)
        D = Discriminator(self.Din, self.ddims, self.P)
        G.load_state_dict(self.g_state_dict())
        D.load_state_dict(self.d_state_dict())
        return G, D

    # ================================================================= buffers
    def _build_buffers(self):
        dev, f32 = self.mem, torch.float32
        B, nP = self.B, self.nP
        z = lambda *s: self.mem.zeros(*s, dtype=f32)  # noqa: E731
        # generator forward buffers hold two batches: rows [0, B) the D phase, [B, 2B) the G phase.
        # The paired prepare runs both through ONE M = 2B GEMM chain (BN statistics per batch);
        # the per-phase paths use the G-phase rows, which are also what the G backward reads.
        if self._multi:
            # one set of the sampler's outputs per step of a graph replay: H2 (z | c behind the activations), the D
            # input block and the draws' col / opt; set 0 is also what the per-step path uses
            self._h2_sets = _padded_rows(self._U * 2 * B, self.Hw, dev)
            self.H2 = self._h2_sets[:2 * B]
        else:
            self.H2 = _padded_rows(2 * B, self.Hw, dev)
        self.abuf2 = [z(2 * B, g) for g in self.gdims]
        self.nhat2 = [z(2 * B, g) for g in self.gdims]
        self.bn_mean2 = [z(2, g) for g in self.gdims]
        self.bn_invstd2 = [z(2, g) for g in self.gdims]
        self.logits2 = _padded_rows(2 * B, self.Dd, dev)
        self.H = self.H2[B:]
        self.abuf = [t[B:] for t in self.abuf2]
        self.nhat = [t[B:] for t in self.nhat2]
        self.bn_mean = [t[1] for t in self.bn_mean2]
        self.bn_invstd = [t[1] for t in self.bn_invstd2]
        self.logits = self.logits2[B:]
        self.da = [z(B, g) for g in self.gdims]
        self.dlogits = _padded_rows(B, self.Dd, dev)
        self.dH = _padded_rows(B, self.Hw, dev)
        # discriminator inputs, one buffer: [interp | real | fake (D phase) | fake (G phase)].
        # D's stacked batch is the first 3B rows; both phases' fake rows are contiguous, so one
        # activation launch writes them; the G phase's rows are separate so its prepare can overlap
        # the D update (lanes)
        if self._multi:
            self._xall_sets = z(self._U * 4 * B, self.Din)
            self.Xall = self._xall_sets[:4 * B]
        else:
            self.Xall = z(4 * B, self.Din)
        self._x_views()
        self.dact = None
        self.dl = [z(3 * nP, h) for h in self.ddims]
        self.ms = [z(3 * nP, h) for h in self.ddims]
        self.A = [z(3 * nP, h) for h in self.ddims]
        # fused A-chain scratch (EngineConfig.fuse_achain), one set per call site (the D phase, stream base 4, and the
        # G phase, 14): slab partials [ceil(d1 / 64), rows, d0] and one arrival counter per head row (kept zero by
        # the kernel)
        self._ach = {}
        if len(self.ddims) == 2 and self.cfg.fuse_achain and getattr(self.ops, "achain_capable", False):
            for sb in (4, 14):
                self._ach[sb] = (z(-(-self.ddims[1] // 64) * 3 * nP * self.ddims[0]),
                                 self.mem.zeros(3 * nP, dtype=torch.int32))
        self.y = z(3 * nP)
        self.gbuf = z(nP, self.K1)
        inv = 1.0 / nP
        # packed-row slices of the stacked D batch: interpolates, then real, then fake
        self.rows_i, self.rows_fr = slice(0, nP), slice(nP, 3 * nP)
        self.coef3 = self.mem.tensor(torch.cat([torch.ones(nP), torch.full((nP,), -inv), torch.full((nP,), inv)]).float())
        self.wloss3 = self.mem.tensor(torch.cat([torch.zeros(nP), torch.full((nP,), -inv), torch.full((nP,), inv)]).float())
        self.coefg = self.mem.tensor(torch.full((nP,), -inv, dtype=f32))
        if self._multi:
            self._col_sets = self.mem.zeros(self._U * 2 * B, dtype=torch.int32)
            self._opt_sets = self.mem.zeros(self._U * 2 * B, dtype=torch.int32)
            self._metrics_sets = z(self._U, 4)
            self.col2, self.opt2 = self._col_sets[:2 * B], self._opt_sets[:2 * B]
            self.metrics = self._metrics_sets[self._U - 1]
        else:
            self.col2 = self.mem.zeros(2 * B, dtype=torch.int32)
            self.opt2 = self.mem.zeros(2 * B, dtype=torch.int32)
            self.metrics = z(4)     # [wgan_d, pen, wgan_g, cond_ce]
        self.col = self.col2[B:]
        self.opt = self.opt2[B:]
        # per-pack penalty / per-row cond-CE terms, summed into metrics by the column-sum launch that
        # follows (no same-address atomics in the producing kernels)
        self.pen_rows = z(nP)
        self.ce_rows = z(B)

    def _x_views(self):
        """The D input block's views: [interp | real | fake (D phase) | fake (G phase)] rows of self.Xall."""
        B, nP = self.B, self.nP
        self.X_interp = self.Xall[0:B]
        self.X_real = self.Xall[B:2 * B]
        self.X_fake = self.Xall[2 * B:3 * B]
        self.Xd = self.Xall[0:3 * B]
        self.X = self.Xd.view(3 * nP, self.K1)
        self.Xg = self.Xall[3 * B:4 * B]
        self.XgP = self.Xg.view(nP, self.K1)

    def _bind_set(self, k: int = 0, step: Optional[int] = None):
        """Multi-step draws: issue the following launches on batch-buffer set k with step ``step``'s optimizer
        counters and metrics (None: the canonical ones, the last entries)."""
        B = self.B
        self.H2 = self._h2_sets[k * 2 * B:(k + 1) * 2 * B]
        self.H = self.H2[B:]
        self.Xall = self._xall_sets[k * 4 * B:(k + 1) * 4 * B]
        self._x_views()
        self.col2 = self._col_sets[k * 2 * B:(k + 1) * 2 * B]
        self.opt2 = self._opt_sets[k * 2 * B:(k + 1) * 2 * B]
        self.col, self.opt = self.col2[B:], self.opt2[B:]
        j = self._U - 1 if step is None else int(step)
        self.stepD = self._step_sets[0, j:j + 1]
        self.stepG = self._step_sets[1, j:j + 1]
        self.metrics = self._metrics_sets[j]

    def _draw_all(self):
        """The batches of the graph's U steps in one sampler launch (bound to set 0 / the counter arrays)."""
        B, U = self.B, self._U
        self.ops.sample_train(self.tables, self.H2, self.z_cols, self.c_cols, self.Xall[2 * B:4 * B], self.X_real,
                              self.Dd, self.col2, self.opt2, step_counter=(self._step_sets[0], self._step_sets[1]),
                              metrics=self._metrics_sets, zero_metrics=True, stream_id=1, draws=U,
                              strides=(2 * B * self.H2.stride(0), 4 * B * self.Xall.stride(0), 2 * B))

    # ================================================================= data
    def set_training_data(self, encoded, rows: RowIndex | None = None, cond: CondTables | None = None):
        """encoded: the host matrix [N, data_dim], or a ``DeviceEncoded`` from the HIP encoder
        (matrix, row lists and counts already on the device)."""
        lay = self.layout
        dev_enc = hasattr(encoded, "opt") and hasattr(encoded, "rows")
        mk = self.mem.tensor
        n = len(encoded)
        # the batched engine's clients may hold different row counts (models/batched.py): every slab then
        # reserves the largest client's row tables (identical layouts), filled up to this client's rows
        pad = max(int(self.pad_rows or 0), n)

        def rows_of(data, per_row: int = 1, dtype=None):
            src = torch.as_tensor(data, dtype=dtype)
            if src.shape[0] == pad * per_row:
                return mk(src)
            out = self.mem.zeros(pad * per_row, *src.shape[1:], dtype=src.dtype)
            out[:src.shape[0]].copy_(src)
            return out
        if dev_enc:
            cond = cond or CondTables(lay, encoded.counts)
            rt = encoded.rows
            t = {"data": rows_of(encoded.data), "row_offset": mk(rt["row_offset"]), "row_count": mk(rt["row_count"]),
                 "rows": rows_of(rt["rows"], lay.n_col)}
        else:
            rows = rows or RowIndex(encoded, lay)
            cond = cond or CondTables.from_encoded(encoded, lay)
            t = {"data": rows_of(np.ascontiguousarray(encoded, dtype=np.float32)),
                 "row_offset": mk(np.asarray(rows.offset), dtype=torch.int64),
                 "row_count": mk(np.asarray(rows.count), dtype=torch.int64),
                 "rows": rows_of(np.asarray(rows.rows), lay.n_col, dtype=torch.int64)}
        t.update({
            "cdf_log": mk(np.asarray(cond.cdf_log), dtype=torch.float32),
            "cdf_emp": mk(np.asarray(cond.cdf_emp), dtype=torch.float32),
            "cond_offset": mk(np.asarray(lay.cond_offset), dtype=torch.int32),
            "cond_width": mk(np.asarray(lay.cond_width), dtype=torch.int32),
            "cond_start": mk(np.asarray(lay.cond_start), dtype=torch.int32),
        })
        self.n_rows = len(encoded)
        self.tables = t
        self.steps_per_epoch = len(encoded) // self.B
        self.graphs = {}

    def set_generation_tables(self, cond: CondTables, transformer):
        """Tables for sample_zero + fused decode (transformer: a fitted VGMTransformer)."""
        dev = self.device
        self.gen_cond = {
            "cdf_emp": torch.as_tensor(cond.cdf_emp, dtype=torch.float32, device=dev),
            "cond_offset": torch.as_tensor(self.layout.cond_offset, dtype=torch.int32, device=dev),
            "cond_width": torch.as_tensor(self.layout.cond_width, dtype=torch.int32, device=dev),
        }
        mu, sd = transformer.decode_tables()
        cols = []
        pos = 0
        c = 0
        for j, m in enumerate(transformer.meta):
            if m["type"] == "continuous":
                nv = int(transformer.components[c].sum())
                cols.append((0, pos, nv, c, None))
                pos += 1 + nv
                c += 1
            else:
                w = int(m["size"])
                codes = torch.as_tensor(np.asarray(m["i2s"], dtype=np.float64), device=dev)
                cols.append((1, pos, w, -1, codes))
                pos += w
        self.gen_tables = {"cols": cols, "mu": torch.as_tensor(mu, dtype=torch.float64, device=dev),
                           "sd": torch.as_tensor(sd, dtype=torch.float64, device=dev)}
        self._gen_bufs = None
        self._gen_graphs = {}
        self._gen_split = {}

    # ================================================================= forward pieces
    def _kpad(self, H, a: int, W: torch.Tensor):
        """(H[:, a:], W) widened over their zero padding to a K divisible by 4 when H's row
        stride allows it (16-B GEMM loads along K); otherwise the logical views."""
        x = H[:, a:]
        kp = _ceil4(x.shape[1])
        # room along K: the row stride of [out, in] storage; input-major storage has ceil4(in) rows
        room = W.stride(0) if W.stride(1) == 1 else _ceil4(W.shape[1])
        if kp != x.shape[1] and H.stride(0) >= a + kp and room >= kp:
            return _ext(x, kp), _ext(W, kp)
        return x, W

    def _g_in(self, H, a: int, W: torch.Tensor, cond):
        """GEMM operands of a generator layer reading H[:, a:]: (x, W, onehot).  With the row
        conditions ``cond`` = (col, opt[, transposed]), x / W are only the DENSE columns (up to the
        conditional block) and the one-hot block becomes the gather ``onehot`` (ops.gemm); else the
        full K.  transposed: gather from a [C, N] copy of the block made here (generation: 40k rows,
        where strided gathers from the [N, C] weight cost more than the K they save)."""
        if cond is None or not self.use_onehot:
            x, Wk = self._kpad(H, a, W)
            return x, Wk, None
        c0 = self.c_cols[0]
        kd = c0 - a
        if W.stride(0) == 1 and W.stride(1) != 1:
            # input-major storage: the block is already [C, N] rows (ops normalise transposed views)
            return H[:, a:c0], W[:, :kd], (W[:, kd:], cond[0], cond[1], self._cond_off)
        if len(cond) > 2 and cond[2]:
            return H[:, a:c0], W[:, :kd], (W[:, kd:].t().contiguous(), cond[0], cond[1], self._cond_off, True)
        return H[:, a:c0], W[:, :kd], (W[:, kd:], cond[0], cond[1], self._cond_off)

    def _g_forward(self, H, logits, training: bool, nhat=True, act_out=None, stream_id=0, slerp=None, paired=False,
                   cond=None):
        """Residual stack + output layer; with ``act_out`` the activation is fused onto the
        output GEMM (tanh / Gumbel-softmax into act_out, Philox stream ``stream_id``).
        paired: H / logits hold both batches of a step (2B rows, BN statistics per batch).
        cond: the rows' (col, opt) int32 condition indices -- the conditional block of H is then
        applied as a one-hot gather instead of a dense K range (``EngineConfig.onehot``)."""
        o = self.ops
        for i, g in enumerate(self.gdims):
            a, b_ = self.off[i], self.off[i + 1]
            x, W, oh = self._g_in(H, a, self.p[f"G.{i}.W"], cond)
            abuf, nh = (self.abuf2[i], self.nhat2[i]) if paired else (self.abuf[i], self.nhat[i])
            mean, istd = (self.bn_mean2[i], self.bn_invstd2[i]) if paired else (self.bn_mean[i], self.bn_invstd[i])
            o.linear_bn_relu(x, W, self.p[f"G.{i}.b"], self.p[f"G.{i}.gamma"],
                             self.p[f"G.{i}.beta"], H[:, b_:a],
                             abuf if nhat else None, nh if nhat else None,
                             mean, istd, self.p[f"G.{i}.rm"], self.p[f"G.{i}.rv"],
                             training, self.cfg.bn_momentum, self.cfg.bn_eps, groups=2 if paired else 1, onehot=oh)
        x, W, oh = self._g_in(H, 0, self.p["G.out.W"], cond)
        if act_out is None:
            o.gemm(x, W, logits, tb=True, bias=self.p["G.out.b"], onehot=oh)
        else:
            o.linear_activate(x, W, self.p["G.out.b"], logits, act_out, self.spans, self.cfg.tau, stream_id=stream_id,
                              slerp=slerp, onehot=oh)

    def _d_forward(self, rows: slice, stream_base: int, X=None, coef=None) -> bool:
        """D's hidden layers on the packed rows.  With ``coef`` the last layer's epilogue also
        writes the head's backward seed A_{L-1} = coef * v * MS_{L-1} (no separate head launch;
        the head's WGAN value is folded into a later column-sum launch, see _wgan_job).
        Returns True when the A chain (A_0) was formed too (EngineConfig.fuse_achain)."""
        o = self.ops
        Xs = self.X if X is None else X
        inp = Xs[rows]
        L = len(self.ddims)
        # two hidden layers: D1 (150 or 50 x 256 x 256) computed row by row in D0's split-K reduction launch
        # (not in a batched multi-client step: the row-by-row chain re-reads D1's weights per row, which pays for
        # a few dozen rows on an idle chip but not for K clients' rows -- profiles/batched_r3.md)
        chain = L == 2 and self.cfg.chain_d1 and hasattr(o, "gemm_is_split") and self.ddims[0] % 16 == 0 and \
            self.ddims[0] <= 1024 and o.gemm_is_split(inp.shape[0], self.ddims[0], inp.shape[1]) and \
            getattr(o, "batch_k", 1) == 1
        fused = False
        for i in range(L):
            head = None
            if coef is not None and i == L - 1:
                head = (coef, self.p["D.out.W"].view(-1), self.A[L - 1][rows])
            kw = {"chain": True} if (chain and i == 0) else {}
            if chain and i == 0:
                h1 = (coef, self.p["D.out.W"].view(-1), self.A[1][rows]) if coef is not None else None
                ach = self._ach.get(stream_base) if coef is not None else None
                if ach is not None:
                    o.gemm_achain_next(self.A[0][rows], *ach)
                    fused = True
                o.gemm(self.dl[0][rows], self.p["D.1.W"], self.dl[1][rows], tb=True, bias=self.p["D.1.b"],
                       epi=EPI_LRELU_DROPOUT, ms=self.ms[1][rows], slope=self.cfg.lrelu_slope,
                       p_drop=self.cfg.dropout_p, stream_id=stream_base + 1, head=h1, group=4)
            o.gemm(inp, self.p[f"D.{i}.W"], self.dl[i][rows], tb=True, bias=self.p[f"D.{i}.b"], epi=EPI_LRELU_DROPOUT,
                   ms=self.ms[i][rows], slope=self.cfg.lrelu_slope, p_drop=self.cfg.dropout_p,
                   stream_id=stream_base + i, head=head, **kw)
            if chain:
                break
            inp = self.dl[i][rows]
        return fused

    def _g_loss_metric(self):
        """The G-phase WGAN value alone (split roles: the client has no generator backward)."""
        src, out, w, dot = self._wgan_job(slice(0, self.nP), self.coefg, self.metrics[2:3])
        self.ops.colsum_many([src, self.ce_rows.view(-1, 1)], [out, self.metrics[3:4]], weights=[w, None],
                             dots=[dot, None])

    def _wgan_job(self, rows: slice, wloss, loss_out):
        """colsum job computing loss_out += sum_r wloss[r] (D(x_r) - ...) = sum_r wloss[r](d_r . v + e)."""
        L = len(self.ddims)
        return self.dl[L - 1][rows], None, wloss, (self.p["D.out.W"].view(-1), self.p["D.out.b"], loss_out)

    def _a_chain(self, rows: slice):
        o = self.ops
        for i in range(len(self.ddims) - 1, 0, -1):
            o.gemm(self.A[i][rows], self.p[f"D.{i}.W"], self.A[i - 1][rows], epi=EPI_MASK, ms=self.ms[i - 1][rows])

    # ================================================================= lanes
    @contextlib.contextmanager
    def _lane(self, k: int):
        """Issue the enclosed launches on side stream ``k`` (forked from the current stream)."""
        if self.lanes is None:
            yield
            return
        s = self.lanes[k]
        s.wait_stream(torch.cuda.current_stream(self.device))
        prev = getattr(self.ops, "lane", 0)
        self.ops.lane = k
        try:
            with torch.cuda.stream(s):
                yield
        finally:
            self.ops.lane = prev

    def _join(self, *ks: int):
        if self.lanes is None:
            return
        cur = torch.cuda.current_stream(self.device)
        for k in ks:
            cur.wait_stream(self.lanes[k])

    # ================================================================= steps
    def _d_step(self):
        self._d_prepare()
        self._d_update()

    def _d_prepare(self):
        """Draw the batch and build the D input: [slerp(real, fake) | real | fake] rows."""
        o = self.ops
        o.sample_train(self.tables, self.H, self.z_cols, self.c_cols, self.X_fake, self.X_real, self.Dd,
                       self.col, self.opt, step_counter=self.stepD, metrics=self.metrics, zero_metrics=True,
                       stream_id=1)
        # activation of the fake rows + slerp(real, fake) for the gradient penalty in one launch
        self._g_forward(self.H, self.logits, training=True, act_out=self.X_fake[:, :self.Dd], stream_id=2,
                        slerp=(self.X_real, self.X_fake, self.X_interp, 3),
                        cond=(self.col, self.opt, self.cfg.onehot_trans))

    def _prepare_paired(self, draw: bool = True):
        """Both phases' batches in one pass: one sampler launch draws the D-phase batch (with real
        rows) and the G-phase batch, and the generator runs once on the 2B stacked rows.

        Exact w.r.t. the reference's two separate forwards (`Client/.../distributed.py:185-265`):
        the D step never changes G, BN uses per-batch statistics, and the running statistics are
        updated D batch first, then G batch.  Halves the generator-side launches of a step and
        doubles their workgroups (M = 1000 fills the chip better than M = 500)."""
        o, B = self.ops, self.B
        h, cc = self.H2, self.c_cols
        if draw:                # (else drawn ahead by the graph's multi-step sampler launch, _draw_all)
            o.sample_train(self.tables, h, self.z_cols, cc, self.Xall[2 * B:4 * B], self.X_real, self.Dd,
                           self.col2, self.opt2, step_counter=(self.stepD, self.stepG), metrics=self.metrics,
                           zero_metrics=True, stream_id=1)
        self._g_forward(self.H2, self.logits2, training=True, act_out=self.Xall[2 * B:4 * B, :self.Dd], stream_id=2,
                        slerp=(self.X_real, self.X_fake, self.X_interp, 3), paired=True,
                        cond=(self.col2, self.opt2, self.cfg.onehot_trans))

    def _d_update(self):
        """D forward on the stacked rows, WGAN + GP backward, D Adam step."""
        o, B, nP = self.ops, self.B, self.nP
        L = len(self.ddims)
        allr = slice(0, 3 * nP)
        I = self.rows_i
        if not self._d_forward(allr, stream_base=4, coef=self.coef3):
            self._a_chain(allr)
        # gradient penalty: g = q_0 V_0 ; Gs written over the interpolates' input rows
        o.gemm(self.A[0][I], self.p["D.0.W"], self.gbuf)
        o.gp_scale(self.gbuf, self.X[I], self.cfg.gp_lambda, self.pen_rows)
        # R-chain on the main lane; each layer's weight-gradient GEMM (one GEMM over the stacked
        # rows) starts on a side lane as soon as its right operand is complete
        inp = self.X[I]
        prev = self.X
        pair = self.lanes is None     # weight gradient + R product of a layer: one launch
        # two hidden layers: R1 rides on R0's split-K reduction launch, and dW1 (then the last D GEMM)
        # is held for the D Adam launch (gemm_adam_kernel)
        fuse_d = pair and L == 2 and self.cfg.fuse_d_adam and getattr(o, "gemm_adam", False) and \
            self._adam_fusable(self.nD) and \
            self.ddims[0] % 16 == 0 and self.ddims[0] <= 1024 and o.gemm_is_split(self.nP, self.ddims[0], self.K1) and \
            getattr(o, "batch_k", 1) == 1
        # otherwise D0's weight gradient may be the GEMM held for the Adam launch (its operands, A0 and X, are
        # final here: the R chain below writes only dl[*][I])
        d0_fused = pair and not fuse_d and self.cfg.fuse_d0_adam and getattr(o, "gemm_adam", False)
        # a short-K D0 weight gradient (the wide table's 256 x 137,800 over 150 rows) applies Adam itself, launched
        # just before the optimizer launch (gemm(..., group=6)): R0 -- which reads W0 -- is then no pair partner
        d0_pre = pair and not d0_fused and self.cfg.fuse_d0_shortk and \
            getattr(o, "shortk_ok", lambda *a: False)(self.ddims[0], self.K1, 3 * nP)
        for i in range(L):
            last_fused = fuse_d and i == L - 1
            with self._lane(1 + i % 2):
                kw = {"tile": self.cfg.dw0_tile} if (i == 0 and self.cfg.dw0_tile and self.ops.name == "hip") else {}
                if i == 0 and d0_fused:
                    kw = {"tile": 64 if self.cfg.dw0_tile not in (32, 64) else self.cfg.dw0_tile}   # gemm_adam tiles
                    grp = 3
                elif i == 0 and d0_pre:
                    kw = {"splitk": 1}
                    grp = 7 if (self.cfg.keep_grads or getattr(self, "keep_grads", False)) else 6
                else:
                    grp = 3 if last_fused else (1 if pair else 0)
                o.gemm(self.A[i], prev, self.g[f"D.{i}.W"], ta=True, group=grp, **kw)
            if last_fused:
                break              # R_{L-1} was computed with R_{L-2}
            rk = {}
            if fuse_d and i == L - 2:      # R_{i+1} = (R_i W_{i+1}^T) . MS_{i+1}, row by row in R_i's reduction
                o.gemm(self.dl[i][I], self.p[f"D.{i + 1}.W"], self.dl[i + 1][I], tb=True, epi=EPI_MASK,
                       ms=self.ms[i + 1][I], group=4)
                rk = {"chain": True}
            o.gemm(inp, self.p[f"D.{i}.W"], self.dl[i][I], tb=True, epi=EPI_MASK, ms=self.ms[i][I],
                   group=2 if (pair and not (i == 0 and (d0_fused or d0_pre))) else 0, **rk)
            inp = self.dl[i][I]
            prev = self.dl[i]
        # (the column sums are folded into the Adam launch: those workgroups update the bias / head
        # entries themselves)
        jobs = self._d_colsum_jobs()
        self._join(1, 2)
        # d(loss)/d(e_out) = sum of the +-1/n_packs seeds = 0 (stays zero from allocation)
        b1, b2 = self.cfg.betas
        o.adam(self.flatD, self.gradD, self.mD, self.vD, self.stepD, self.cfg.lr, b1, b2, self.cfg.adam_eps, 0.0,
               jobs=jobs)

    def _d_colsum_jobs(self):
        """Bias grads + the head's weight grad (sum_r coef[r] d_r) + the WGAN and penalty values.
        (dl[L-1][I] holds R_{L-1} by then: coef = 1 there gives dpen/dv; wloss = 0 there.)
        The head's gradient and the WGAN value are one job (row weights coef / wloss over the
        same rows): in the folded Adam launch the WGAN dot then reads each head weight in the
        lane that updates it, before the update."""
        L, fr = len(self.ddims), self.rows_fr
        src, _, w, dot = self._wgan_job(slice(0, 3 * self.nP), self.wloss3, self.metrics[0:1])
        return ([self.A[i][fr] for i in range(L)] + [src, self.pen_rows.view(-1, 1)],
                [self.g[f"D.{i}.b"] for i in range(L)] + [self.g["D.out.W"].view(-1), self.metrics[1:2]],
                [None] * L + [self.coef3, None], [None] * L + [(*dot, w), None])

    def _g_colsum_jobs(self):
        """G.out bias grad + the G-phase WGAN value (-mean D(fake)) + the cond CE sum."""
        src, out, w, dot = self._wgan_job(slice(0, self.nP), self.coefg, self.metrics[2:3])
        return ([self.dlogits, src, self.ce_rows.view(-1, 1)], [self.g["G.out.b"], out, self.metrics[3:4]],
                [None, w, None], [None, dot, None])

    def _g_step(self):
        self._g_prepare()
        self._g_update()

    def _g_prepare(self):
        o, B = self.ops, self.B
        o.sample_train(self.tables, self.H, self.z_cols, self.c_cols, self.Xg, None, self.Dd,
                       self.col, self.opt, step_counter=self.stepG, stream_id=11)
        self._g_forward(self.H, self.logits, training=True, act_out=self.Xg[:, :self.Dd], stream_id=12,
                        cond=(self.col, self.opt, self.cfg.onehot_trans))

    def _g_update(self):
        """D forward on the fake rows, backward through D, activation, cond loss and G; G Adam step."""
        self._g_dlogits()
        self._g_adam(self._g_backward(fold_colsum=True, onehot_w=True))

    def _g_dlogits(self):
        """G loss (-mean D(fake) + cond CE) back to the generator's logits: self.dlogits."""
        o, B, nP = self.ops, self.B, self.nP
        L = len(self.ddims)
        fk = slice(0, nP)
        if not self._d_forward(fk, stream_base=14, X=self.XgP, coef=self.coefg):
            self._a_chain(fk)
        o.gemm(self.A[0][fk], self.p["D.0.W"], self.gbuf)            # d(-mean D)/dX, packed
        dx = self.gbuf.view(B, self.Din)
        o.act_bwd_ce(dx[:, :self.Dd], self.Xg[:, :self.Dd], self.logits, self.spans, self.cond_spans, self.col,
                     self.opt, self.dlogits, self.ce_rows, self.cfg.tau)

    def _onehot_w_ok(self, W: torch.Tensor) -> bool:
        """Is the condition block of G weight gradient W (logical [out, in]) a scattered one (onehot_wgrad_min)?"""
        lim = int(self.cfg.onehot_wgrad_min)
        return lim > 0 and self.use_onehot and bool(self.cfg.g_wt) and hasattr(self.ops, "onehot_wgrad") and \
            self.lanes is None and self.C * W.shape[0] >= lim

    def _wgrad_operands(self, a: int, W: torch.Tensor, oh: Optional[list]):
        """(x, dW) of a generator weight-gradient GEMM over H[:, a:]; with ``oh`` (a list) a large one-hot
        condition block is left out of the GEMM and queued as an (upstream-gradient slot, block rows) job."""
        if oh is not None and self._onehot_w_ok(W):
            kd = self.c_cols[0] - a
            oh.append(W[:, kd:].t())               # [C, out]: the input-major storage's condition rows
            return self.H[:, a:self.c_cols[0]], W[:, :kd]
        return self._kpad(self.H, a, W)

    def _g_backward(self, fold_colsum: bool = False, onehot_w: bool = False):
        """self.dlogits -> G parameter gradients (self.gradG), through the saved forward buffers.
        fold_colsum: return the G.out bias / metrics column-sum jobs for the Adam launch instead of
        launching them (the gradient is then complete only after _g_adam(jobs)).
        onehot_w: large one-hot condition blocks of the weight gradients by ops.onehot_wgrad (see
        EngineConfig.onehot_wgrad_min; _g_adam clears their rows again)."""
        o = self.ops
        # generator backward: the dH chain on the main lane, weight gradients on side lanes
        Lg = len(self.gdims)
        pair = self.lanes is None and Lg > 0   # weight gradient + dX product of a layer: one launch
        top = self.off[0]
        oh_w, oh_dy = ([], []) if onehot_w else (None, None)

        def wgrad(dy, a, W):
            n0 = len(oh_w) if oh_w is not None else 0
            x, dW = self._wgrad_operands(a, W, oh_w)
            if oh_w is not None and len(oh_w) > n0:
                oh_dy.append(dy)
            return x, dW
        # bn_pair: [dH_out] -> [BN_{L-1} bwd | dW_out] -> [dH_{L-1}] -> [BN_{L-2} bwd | dW_{L-1}] ... -> [dW_0 + Adam]
        bn_pair = pair and bool(self.cfg.bn_pair) and getattr(o, "bn_pair_capable", False)
        if bn_pair:
            jobs = self._g_colsum_jobs()
            if not fold_colsum:
                o.colsum_many(*jobs)
            o.gemm(self.dlogits, self.p["G.out.W"][:, :top], self.dH[:, :top])
            x, dW = wgrad(self.dlogits, 0, self.g["G.out.W"])
            o.gemm(self.dlogits, x, dW, ta=True, group=1)        # launched with the next BN backward
            for i in range(Lg - 1, -1, -1):
                a, b_ = self.off[i], self.off[i + 1]
                o.bn_relu_bwd(self.dH[:, b_:a], self.H[:, b_:a], self.nhat[i], self.p[f"G.{i}.gamma"],
                              self.bn_invstd[i], self.da[i], self.g[f"G.{i}.gamma"], self.g[f"G.{i}.beta"],
                              self.g[f"G.{i}.b"], paired=True)
                x, dW = wgrad(self.da[i], a, self.g[f"G.{i}.W"])
                if i > 0:
                    o.gemm(self.da[i], self.p[f"G.{i}.W"][:, :top - a], self.dH[:, a:top], beta=1.0)
                    o.gemm(self.da[i], x, dW, ta=True, group=1)   # launched with the next BN backward
                else:
                    fuse = fold_colsum and self.cfg.fuse_g_adam and self._adam_fusable(self.nG) and \
                        getattr(o, "gemm_adam", False)
                    o.gemm(self.da[i], x, dW, ta=True, group=3 if fuse else 0)
            if oh_w:
                o.onehot_wgrad(oh_dy, oh_w, self.col, self.opt, self._cond_off)
                self._oh_pending = (oh_dy, oh_w)
            return jobs if fold_colsum else None
        with self._lane(1):
            x, dW = wgrad(self.dlogits, 0, self.g["G.out.W"])
            o.gemm(self.dlogits, x, dW, ta=True, group=1 if pair else 0)
            if pair:
                o.gemm(self.dlogits, self.p["G.out.W"][:, :top], self.dH[:, :top], group=2)
            jobs = self._g_colsum_jobs()
            if not fold_colsum:
                o.colsum_many(*jobs)
        if Lg and not pair:
            o.gemm(self.dlogits, self.p["G.out.W"][:, :top], self.dH[:, :top])
        for i in range(Lg - 1, -1, -1):
            a, b_ = self.off[i], self.off[i + 1]
            o.bn_relu_bwd(self.dH[:, b_:a], self.H[:, b_:a], self.nhat[i], self.p[f"G.{i}.gamma"],
                          self.bn_invstd[i], self.da[i], self.g[f"G.{i}.gamma"], self.g[f"G.{i}.beta"],
                          self.g[f"G.{i}.b"])
            if i > 0:
                pair = self.lanes is None
                with self._lane(2 + i % 2):
                    x, dW = wgrad(self.da[i], a, self.g[f"G.{i}.W"])
                    o.gemm(self.da[i], x, dW, ta=True, group=1 if pair else 0)
                o.gemm(self.da[i], self.p[f"G.{i}.W"][:, :top - a], self.dH[:, a:top], beta=1.0,
                       group=2 if pair else 0)
            else:
                x, dW = wgrad(self.da[i], a, self.g[f"G.{i}.W"])
                # held for the Adam launch that follows (fold_colsum: _g_adam(jobs) is next on this stream)
                fuse = fold_colsum and self.lanes is None and self.cfg.fuse_g_adam and self._adam_fusable(self.nG) and \
                    getattr(o, "gemm_adam", False)
                o.gemm(self.da[i], x, dW, ta=True, group=3 if fuse else 0)
        if oh_w:
            # (issued before a GEMM held for the Adam launch: that launch reads these rows)
            o.onehot_wgrad(oh_dy, oh_w, self.col, self.opt, self._cond_off)
            self._oh_pending = (oh_dy, oh_w)
        self._join(1, 2, 3)
        return jobs if fold_colsum else None

    def _adam_fusable(self, n: int) -> bool:
        """May an optimizer of n parameters share its launch with a weight-gradient GEMM (fuse_adam_max)?"""
        lim = int(self.cfg.fuse_adam_max)
        return lim <= 0 or n * getattr(self.ops, "batch_k", 1) <= lim

    def _g_adam(self, jobs=None):
        b1, b2 = self.cfg.betas
        self.ops.adam(self.flatG, self.gradG, self.mG, self.vG, self.stepG, self.cfg.lr, b1, b2, self.cfg.adam_eps,
                      self.cfg.l2scale, last_in_step=True, jobs=jobs)
        if self._oh_pending is not None:   # the one-hot block rows back to zero for the next step
            dys, ws = self._oh_pending
            self.ops.onehot_wgrad(dys, ws, self.col, self.opt, self._cond_off, zero=True)
            self._oh_pending = None

    # ================================================================= split roles (MD-GAN)
    G_BUFFERS = ("H", "abuf", "nhat", "bn_mean", "bn_invstd", "da", "logits", "dlogits", "dH")

    def new_g_buffers(self) -> Dict[str, object]:
        """A private set of the generator's forward/backward buffers (one per remote client batch
        on an MD-GAN server, so K batches can be in flight between forward and backward)."""
        dev, B = self.device, self.B
        z = lambda *s: torch.zeros(*s, dtype=torch.float32, device=dev)  # noqa: E731
        return {"H": _padded_rows(B, self.Hw, dev), "abuf": [z(B, g) for g in self.gdims],
                "nhat": [z(B, g) for g in self.gdims], "bn_mean": [z(g) for g in self.gdims],
                "bn_invstd": [z(g) for g in self.gdims], "da": [z(B, g) for g in self.gdims],
                "logits": _padded_rows(B, self.Dd, dev), "dlogits": _padded_rows(B, self.Dd, dev),
                "dH": _padded_rows(B, self.Hw, dev)}

    @contextlib.contextmanager
    def use_g_buffers(self, bufs: Dict[str, object]):
        saved = {k: getattr(self, k) for k in self.G_BUFFERS}
        for k in self.G_BUFFERS:
            setattr(self, k, bufs[k])
        try:
            yield
        finally:
            for k, v in saved.items():
                setattr(self, k, v)

    def g_input_view(self, H=None) -> torch.Tensor:
        """The generator input block [z | c] of an H buffer (written by the sampler)."""
        return (self.H if H is None else H)[:, self.off[0]:]

    def _one_step(self, draw: bool = True):
        if hasattr(self.ops, "begin_step"):
            self.ops.begin_step(self)
        try:
            self._issue_step(draw)
        except BaseException:
            # a raise between a held GEMM (ops.gemm group 1/3/4) and its consumer must not leave the hold
            # behind for the next step on this thread
            if hasattr(self.ops, "reset_held"):
                self.ops.reset_held()
            raise

    def _issue_step(self, draw: bool = True):
        if self.lanes is None and self.cfg.paired:
            # both batches drawn and generated up front (G is unchanged by the D update)
            self._prepare_paired(draw)
            self._d_update()
            self._g_update()
        elif self.lanes is None:      # the reference order: D step, then G step
            self._d_step()
            self._g_step()
        else:
            # the G phase's sampling + generator forward only depends on G (unchanged by the D
            # step), so it runs on lane 3 while the D update runs on the main lane
            self._d_prepare()
            with self._lane(3):
                self._g_prepare()
            self._d_update()
            self._join(3)
            self._g_update()
        if hasattr(self.ops, "end_step"):
            self.ops.end_step(self)

    def train_steps(self, n: int, use_graph: bool | None = None, lead: int = 0):
        """n optimisation steps.  ``lead`` > 0 (graph path): ``lead_event`` is recorded on the stream before the
        last ``lead`` U-step blocks, so a host that waits on it wakes while those blocks still run (None when the
        epoch has fewer blocks or runs eagerly -- the caller then waits on the stream)."""
        if not self.tables:
            raise RuntimeError("set_training_data() first")
        self.lead_event = None
        if use_graph is None:
            use_graph = self._graphs_by_default()
        if use_graph:
            # U steps per graph launch (the per-launch gap between graphs is paid n/U times), or a graph of B
            # blocks of U steps (_graph_blocks) for the bulk of an epoch
            U = max(1, int(self.cfg.graph_unroll))
            left = n
            big = U * self._graph_blocks()
            if big > U and left >= big:
                gb = self.graphs.get(self._graph_key(big)) or self._capture(big)
                for _ in range(left // big):
                    gb.replay()
                left %= big
            if left >= U:
                g = self.graphs.get(self._graph_key(U)) or self._capture(U)
                nb = left // U
                for i in range(nb):
                    if lead and i == nb - lead:
                        self._mark_lead()
                    g.replay()
                left %= U
            if left:
                g1 = self.graphs.get(self._graph_key(1)) or self._capture(1)
                for _ in range(left):
                    g1.replay()
        else:
            for _ in range(n):
                self._one_step()
        self.bn_batches += 2 * n
        if hasattr(self.ops, "check"):
            self.ops.check()

    def train_epoch(self, use_graph: bool | None = None, lead: int = 0):
        self.train_steps(self.steps_per_epoch, use_graph, lead)

    def _mark_lead(self):
        if getattr(self, "_lead_ev", None) is None:
            self._lead_ev = torch.cuda.Event()
        self._lead_ev.record(torch.cuda.current_stream(self.device))
        self.lead_event = self._lead_ev

    def _graph_blocks(self) -> int:
        """U-step blocks per big step graph (EngineConfig.graph_blocks; 0: those of one epoch).  One client only:
        a batched engine keeps one block per graph."""
        if self.batch is not None or getattr(self.ops, "batch_k", 1) != 1:
            return 1
        U = max(1, int(self.cfg.graph_unroll))
        b = int(self.cfg.graph_blocks)
        return max(1, b if b > 0 else self.steps_per_epoch // U)

    def _graphs_by_default(self) -> bool:
        """Step graphs unless asked otherwise: on a GPU with the HIP backend.  The eager torch oracle
        (ops/ref.py) runs eagerly: on wide tables its step is tens of thousands of small ATen launches
        (Python loops over ~770 spans), and capturing 8 of them into one graph crashed HIP's graph
        instantiation (segfault in capture_end, 100k x 512 table, round 5)."""
        return self.device.type == "cuda" and self.ops.name == "hip"

    def prepare_graphs(self, steps: int | None = None, gen_rows: Sequence[int] = (), gen_split: bool = False) -> None:
        """Capture, ahead of the first round, every hipGraph that ``train_steps(steps)`` and
        ``generate_decoded(n)`` for ``n`` in ``gen_rows`` will replay: the capture (one eager warm-up step
        or pass plus the capture itself, ~40 ms for the Intrusion step graph) then happens at
        initialisation instead of inside round 0's timed window.  Capturing never changes the training
        state (``_capture_locked`` restores it).  No-op off the GPU / without graphs."""
        if self.device.type != "cuda":
            return
        steps = self.steps_per_epoch if steps is None else int(steps)
        if self.tables and steps > 0 and self._graphs_by_default():
            U = max(1, int(self.cfg.graph_unroll))
            big = U * self._graph_blocks()
            rest = steps
            if big > U and steps >= big:
                if self._graph_key(big) not in self.graphs:
                    self._capture(big)
                rest = steps % big
            if rest >= U and self._graph_key(U) not in self.graphs:
                self._capture(U)
            if rest % U and self._graph_key(1) not in self.graphs:
                self._capture(1)
        if self.gen_tables is not None and self.cfg.gen_graph and self.ops.name == "hip":
            for n in gen_rows:
                if n > 0 and gen_split and self.can_split_generation():
                    if n not in self._gen_split:
                        self._capture_gen_split(int(n))
                elif n > 0 and n not in self._gen_graphs:
                    self._capture_gen(int(n))

    def _graph_key(self, steps: int):
        """Captured step graphs are per (steps, clients): a batched engine whose clients hold different row
        counts runs the tail of an epoch with fewer clients per launch (models/batched.py)."""
        k = getattr(self.ops, "batch_k", 1)
        return steps if k == 1 else (steps, k)

    def _capture(self, steps: int = 1):
        from ..utils.devsync import CAPTURE_LOCK
        with CAPTURE_LOCK:      # no device-wide sync from another client thread meanwhile
            return self._capture_locked(steps)

    def _capture_locked(self, steps: int = 1):
        # warm up on a side stream (allocator / lazy init), then capture one step.  The state snapshot is
        # enqueued BEFORE the side stream forks from the current one, so the warm-up step cannot overtake
        # the copies (it could, racing them, when the fork came first).  (A batched engine's warm-up step
        # trains every client: all of their states are restored.)
        # (the device Philox counter too: a capture must not shift the clients' random streams, whatever step of
        # an epoch -- or which epoch segment of a batched engine with ragged clients -- it happens at)
        state = self.batch.state_tensors() if self.batch is not None else \
            [self.flat, self.mG, self.vG, self.mD, self.vD] + \
            ([self._step_sets] if self._multi else [self.stepG, self.stepD]) + \
            ([self.ops.ctr] if hasattr(self.ops, "ctr") else [])
        snap = [t.clone() for t in state]
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        try:
            with torch.cuda.stream(s):
                self._one_step()
        finally:
            # restore the state so the warm-up step does not count -- also when it raised part-way (e.g. a
            # batched arena slab overflow): the caller may fall back to other engines that copy this state
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            for dst, src in zip(state, snap):
                dst.copy_(src)
        g = torch.cuda.CUDAGraph()
        multi = self._multi and steps % self._U == 0 and self.batch is None
        try:
            with torch.cuda.graph(g, capture_error_mode=self.capture_mode):
                if multi:
                    # one launch draws every step's batch of a block into its own buffer set; step k then runs on
                    # set k with its own optimizer counters / metrics (written by that launch); blocks repeat
                    for _ in range(steps // self._U):
                        self._bind_set(0, 0)
                        self._draw_all()
                        for k in range(self._U):
                            self._bind_set(k, k)
                            self._one_step(draw=False)
                else:
                    for _ in range(steps):      # every step re-reads the device RNG/step counters
                        self._one_step()
        finally:
            if multi:
                self._bind_set(0)
        self.graphs[self._graph_key(steps)] = g
        return g

    def release(self) -> None:
        """Drop every captured hipGraph (step, generation, split generation) once the device is idle.  Called by
        FedRuntime.close() before the process exits, so the graphs are destroyed while the HIP runtime (and any
        tool attached to it, e.g. rocprofv3) is intact rather than by the interpreter's teardown in arbitrary
        order."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.graphs.clear()
        self._gen_graphs.clear()
        self._gen_split.clear()
        self._gen_done = None

    @property
    def graph(self):
        """The one-step graph, if captured (inspection / tests)."""
        return self.graphs.get(1)

    def losses(self) -> Tuple[float, float]:
        m = self.metrics.detach().cpu().numpy()
        return float(m[0] + m[1]), float(m[2] + m[3])

    # ================================================================= generation
    @torch.no_grad()
    def generate_encoded(self, n: int) -> torch.Tensor:
        """Activated generator output for n rows (eval BN): [n, data_dim]."""
        out = torch.empty(n, self.Dd, device=self.device)
        for a in range(0, n, self.cfg.gen_chunk):
            b = min(n, a + self.cfg.gen_chunk)
            H, logits, col, opt = self._gen_buffers(b - a, bf16=False)
            self.ops.sample_gen(self.gen_cond, H, self.c_cols, self.z_cols, col_out=col, opt_out=opt, stream_id=21)
            self._g_forward(H, logits, training=False, nhat=False, cond=(col, opt, True))
            self.ops.activate(logits, out[a:b], self.spans, self.cfg.tau, stream_id=22)
        return out

    @torch.no_grad()
    def generate_decoded(self, n: int, use_graph: bool | None = None) -> torch.Tensor:
        """Fused sample -> G(eval) -> Gumbel-argmax/tanh decode: [n, n_cols] float64 on device.

        On a GPU the whole pass for a given n (every chunk's sampler, eval-BN GEMMs and decode
        launches) is captured once into a hipGraph and replayed each round; the result is a fresh
        tensor (a device copy of the graph's static output)."""
        if self.gen_tables is None:
            raise RuntimeError("set_generation_tables() first")
        if use_graph is None:
            use_graph = self.device.type == "cuda" and self.cfg.gen_graph and self.ops.name == "hip"
        if self._gen_done is not None:    # a pipelined body may still read the shared weight copies
            torch.cuda.current_stream(self.device).wait_event(self._gen_done)
        if use_graph:
            ent = self._gen_graphs.get(n) or self._capture_gen(n)
            ent[0].replay()
            out = ent[3].clone()
        else:
            out = torch.empty(n, len(self.gen_tables["cols"]), dtype=torch.float64, device=self.device)
            self._gen_pass(n, out, self._gen_buffers)
        if hasattr(self.ops, "check"):
            self.ops.check()
        return out

    # ------------------------------------------------------------------ pipelined generation
    def can_split_generation(self) -> bool:
        """generate_decoded_split applies: HIP bf16 generation with graphs."""
        return (self.device.type == "cuda" and self.gen16 and self.cfg.gen_graph and self.ops.name == "hip" and
                self.gen_tables is not None and getattr(self.ops, "batch_k", 1) == 1)

    def generate_decoded_split(self, n: int, gen_stream: "torch.cuda.Stream") -> torch.Tensor:
        """generate_decoded(n) in two parts, so the table of round r is generated while round r + 1 trains.

        The prep graph (on the current stream, ~10 us) copies everything the generation reads from the live model
        -- the bf16 / transposed weight copies of gen_weight_prep, each layer's bias, BatchNorm affine and running
        statistics, the output bias -- and snapshots the RNG step counter, advancing the live one by the body's
        bumps; the body graph (sampler, eval generator, decode) then runs on ``gen_stream`` reading only those
        copies.  The table is bit-identical to generate_decoded(n), and training's random numbers are unchanged
        (the live counter moves exactly as the unsplit pass would move it).  Returns a fresh tensor whose
        producer is ``gen_stream``."""
        self.generation_prep(n)
        return self.generation_body(n, gen_stream)

    def generation_prep(self, n: int) -> None:
        """The prep half of generate_decoded_split(n), on the current stream (see there)."""
        ent = self._gen_split.get(n) or self._capture_gen_split(n)
        cur = torch.cuda.current_stream(self.device)
        if self._gen_done is not None:          # the previous body still reads the snapshot
            cur.wait_event(self._gen_done)
        ent[0].replay()
        self._gen_prepped = torch.cuda.Event()
        self._gen_prepped.record(cur)

    def generation_body(self, n: int, gen_stream: "torch.cuda.Stream") -> torch.Tensor:
        """The body half, on ``gen_stream``: it waits for the prep (an event), not for whatever the current stream
        queued since -- the body of round r may be issued after round r + 1's training."""
        ent = self._gen_split[n]
        gen_stream.wait_event(self._gen_prepped)
        with torch.cuda.stream(gen_stream):
            ent[1].replay()
            out = ent[4].clone()
            done = torch.cuda.Event()
            done.record(gen_stream)
        self._gen_done = done
        if hasattr(self.ops, "check"):
            self.ops.check()
        return out

    def _gen_snapshot(self):
        if getattr(self, "_gsnap", None) is None:
            names = [f"G.{i}.{k}" for i in range(len(self.gdims)) for k in ("b", "gamma", "beta", "rm", "rv")]
            names.append("G.out.b")
            self._gsnap = {nm: torch.empty_like(self.p[nm]) for nm in names}
            self._gsnap_pairs = ([self._gsnap[nm] for nm in names], [self.p[nm] for nm in names])
            self._gsnap_ctr = torch.zeros_like(self.ops.ctr)
        return self._gsnap

    def _gen_prep(self, n: int):
        self._gen_weights16()
        self._gen_snapshot()
        torch._foreach_copy_(*self._gsnap_pairs)
        self._gsnap_ctr.copy_(self.ops.ctr)
        for _ in range(-(-n // self.cfg.gen_chunk)):     # the body's decode bumps, once per chunk
            self.ops.L.rng_bump(self.ops.ctr)

    def _gen_body(self, n: int, out: torch.Tensor, bufs):
        w16 = (self._gw16, self._gwt)
        for a in range(0, n, self.cfg.gen_chunk):
            b = min(n, a + self.cfg.gen_chunk)
            H, logits, col, opt = bufs(b - a)
            self.ops.sample_gen(self.gen_cond, H, self.c_cols, self.z_cols, col_out=col, opt_out=opt, stream_id=21,
                                ctr=self._gsnap_ctr)
            self._g_forward16(H, logits, w16, (col, opt), params=self._gsnap)
            self.ops.sample_decode(logits, out[a:b], self.gen_tables, stream_id=23, ctr=self._gsnap_ctr)

    def _capture_gen_split(self, n: int):
        from ..utils.devsync import CAPTURE_LOCK
        m = min(n, self.cfg.gen_chunk)
        H = self._gen_h16(m)
        lg = _padded_rows(m, self.Dd, self.device)
        col, opt = (torch.zeros(m, dtype=torch.int32, device=self.device) for _ in range(2))
        out = torch.empty(n, len(self.gen_tables["cols"]), dtype=torch.float64, device=self.device)
        bufs = lambda k: (H[:k], lg[:k], col[:k], opt[:k])  # noqa: E731
        lane = self.ops.lane
        with CAPTURE_LOCK:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            # the body runs beside training: its own split-K / scratch slots (ops lane 7), never the step's
            self.ops.lane = 7
            try:
                with torch.cuda.stream(s):      # warm-up (decode tables, lazy init); advances the RNG once
                    self._gen_prep(n)
                    self._gen_body(n, out, bufs)
                torch.cuda.current_stream(self.device).wait_stream(s)
                torch.cuda.synchronize(self.device)
                gp, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(gp, capture_error_mode=self.capture_mode):
                    self._gen_prep(n)
                with torch.cuda.graph(gb, capture_error_mode=self.capture_mode):
                    self._gen_body(n, out, bufs)
            finally:
                self.ops.lane = lane
        self._gen_split[n] = (gp, gb, H, lg, out, col, opt)
        return self._gen_split[n]

    def _gen_pass(self, n: int, out: torch.Tensor, bufs):
        w16 = self._gen_weights16() if self.gen16 else None
        for a in range(0, n, self.cfg.gen_chunk):
            b = min(n, a + self.cfg.gen_chunk)
            H, logits, col, opt = bufs(b - a)
            self.ops.sample_gen(self.gen_cond, H, self.c_cols, self.z_cols, col_out=col, opt_out=opt, stream_id=21)
            if w16 is None:
                self._g_forward(H, logits, training=False, nhat=False, cond=(col, opt, True))
            else:
                self._g_forward16(H, logits, w16, (col, opt))
            self.ops.sample_decode(logits, out[a:b], self.gen_tables, stream_id=23)

    @property
    def gen16(self) -> bool:
        """Generation in bf16 storage (EngineConfig.gen_bf16): HIP bf16 backend, one-hot generator
        GEMMs, and 8-aligned column offsets (16-B bf16 operand rows)."""
        return (self.cfg.gen_bf16 and self.ops.name == "hip" and not getattr(self.ops, "f32", True) and
                self.use_onehot and all(o % 8 == 0 for o in self.off))

    def _gen_h16(self, rows: int) -> torch.Tensor:
        """bf16 generator activations [rows, ceil8(c0)]: [out_{L-1} | ... | out_0 | z] (no one-hot block)."""
        return torch.zeros(rows, -(-self.c_cols[0] // 8) * 8, dtype=torch.bfloat16, device=self.device)

    def _gen_weights16(self):
        """Generation views of the generator weights, refreshed from the current fp32 weights inside
        the generation graph (every replay sees the aggregated model), in ONE launch: per layer the
        bf16 copy of the dense columns and the one-hot block transposed to [C, N] fp32.
        Returns (bf16 copies, transposed blocks), one per layer (G-out last)."""
        c0 = self.c_cols[0]
        names = [f"G.{i}.W" for i in range(len(self.gdims))] + ["G.out.W"]
        starts = list(self.off[:len(self.gdims)]) + [0]
        if getattr(self, "_gw16", None) is None:
            self._gw16 = [torch.zeros(self.p[nm].shape[0], -(-(c0 - a) // 8) * 8, dtype=torch.bfloat16,
                                      device=self.device) for nm, a in zip(names, starts)]
            self._gwt = [torch.zeros(self.p[nm].shape[1] - (c0 - a), self.p[nm].shape[0], device=self.device)
                         for nm, a in zip(names, starts)]
        self.ops.L.gen_weight_prep([self.p[nm] for nm in names], [c0 - a for a in starts], self._gw16, self._gwt)
        return self._gw16, self._gwt

    def _g_forward16(self, H16, logits, w16, cond, params=None):
        """Eval-mode generator on the bf16 buffer: each layer's GEMM reads bf16 rows and weights,
        gathers the one-hot block from col / opt, and writes bf16 (BN-eval + ReLU epilogue); the output
        layer writes fp32 logits.  w16 = _gen_weights16(); params: biases / BN tensors by name (default the
        live ones; the pipelined generation passes its snapshot)."""
        o, p = self.ops, (self.p if params is None else params)
        c0 = self.c_cols[0]
        col, opt = cond
        wd, wt = w16
        for i, g in enumerate(self.gdims):
            a, b_ = self.off[i], self.off[i + 1]
            oh = (wt[i], col, opt, self._cond_off, True)
            o.linear_bn_relu(H16[:, a:c0], wd[i], p[f"G.{i}.b"], p[f"G.{i}.gamma"], p[f"G.{i}.beta"], H16[:, b_:a],
                             None, None, None, None, p[f"G.{i}.rm"], p[f"G.{i}.rv"], False, self.cfg.bn_momentum,
                             self.cfg.bn_eps, onehot=oh)
        oh = (wt[-1], col, opt, self._cond_off, True)
        o.gemm(H16[:, :c0], wd[-1], logits, tb=True, bias=p["G.out.b"], onehot=oh)

    def _capture_gen(self, n: int):
        """Capture generate_decoded(n) with its own static buffers (graphs hold no tensor refs)."""
        from ..utils.devsync import CAPTURE_LOCK
        m = min(n, self.cfg.gen_chunk)
        H = self._gen_h16(m) if self.gen16 else _padded_rows(m, self.Hw, self.device)
        lg = _padded_rows(m, self.Dd, self.device)
        col, opt = (torch.zeros(m, dtype=torch.int32, device=self.device) for _ in range(2))
        out = torch.empty(n, len(self.gen_tables["cols"]), dtype=torch.float64, device=self.device)
        bufs = lambda k: (H[:k], lg[:k], col[:k], opt[:k])  # noqa: E731
        with CAPTURE_LOCK:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):      # warm-up (decode tables, lazy init); advances the RNG once
                self._gen_pass(n, out, bufs)
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=self.capture_mode):
                self._gen_pass(n, out, bufs)
        self._gen_graphs[n] = (g, H, lg, out, col, opt)
        return self._gen_graphs[n]

    def _gen_buffers(self, n: int, bf16: bool | None = None):
        bf16 = self.gen16 if bf16 is None else bf16
        if self._gen_bufs is None or self._gen_bufs[0].shape[0] < n or \
                (self._gen_bufs[0].dtype == torch.bfloat16) != bf16:
            m = max(n, min(self.cfg.gen_chunk, n))
            H = self._gen_h16(m) if bf16 else _padded_rows(m, self.Hw, self.device)
            self._gen_bufs = (H, _padded_rows(m, self.Dd, self.device),
                              torch.zeros(m, dtype=torch.int32, device=self.device),
                              torch.zeros(m, dtype=torch.int32, device=self.device))
        H, lg, col, opt = self._gen_bufs
        return H[:n], lg[:n], col[:n], opt[:n]
