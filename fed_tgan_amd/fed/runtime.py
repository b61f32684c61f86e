"""The federated runtime: initialisation protocol, training rounds, aggregation, sampling.

Roles (one process per rank):

* **client** — owns a local table shard and a :class:`CTGANEngine` on its GPU
  (``cuda:LOCAL_RANK``) or the CPU; trains one local epoch per round
  (`Client/.../dtds/distributed.py:179-269`).
* **federator** — rank 0.  In *dedicated* mode (the reference topology, ``world_size = K+1``,
  `R/README.md:7-25`) it holds no data, like ``MDGANServer`` (`Server/dtds/distributed.py:543-835`).
  In *co-located* mode (one process per GPU, every rank a client — the MI355X layout) rank 0
  is a client *and* the federator.

Initialisation (`Server/dtds/distributed.py:865-873`), now as collectives:
    A. meta all-gather -> vocabulary merge + JSD client distances (federator) -> broadcast
    B. local VGM fits -> all-gather of GMM parameters -> pooled resampling, W1 distances and
       global VGM fit (federator) -> broadcast
    C. every rank refits its transformer with the global GMMs and encodes its rows
    D. aggregation weights (federator) -> broadcast
    E. global span counts (all-reduce) -> the generation-time conditional sampler.  The
       reference reads the raw training table at the server for this (`:565-580`); here no
       raw row ever leaves a client.
    F. initial weights broadcast from the first client.

Each round (`Server/dtds/distributed.py:794-825`): local epoch on every client; ONE
weighted all-reduce of the flat parameter buffer (every client now holds the aggregate,
so there is no push-back); sampling of ``n_sample`` rows (sharded over the client GPUs in
co-located mode) with eval-mode BN; decode; CSV dump; per-round wall time.  After the
last round ``timestamp_experiment.csv`` is written (`:827-829`).
"""
from __future__ import annotations

import contextlib
import dataclasses
import json
import os
import threading
import time
from typing import Dict, List, Optional

import numpy as np
import pandas as pd
import torch

from ..data.constants import CATEGORICAL
from ..data.decode import csv_layout, decode_frame
from ..data.schema import DatasetSpec
from ..data.synthetic import generate, shard
from ..data.table import TablePreprocessor, dump_meta_json, read_csv_table
from ..data.vocab import CategoryVocab
from ..features.gmm import VGMBank, fit_vgm, sample_pool
from ..features.transformer import VGMTransformer
from ..models.engine import CTGANEngine, EngineConfig
from ..models.samplers import CondTables
from ..parallel.comm import Comm
from ..utils.metrics import MetricsLog, PhaseTimer, cgroup_cpu_stat
from ..utils.devsync import PendingHost, stream_sync
from .stats import (aggregation_weights, continuous_client_distances, continuous_client_distances_device,
                    merge_categorical_metas, uniform_weights)


@dataclasses.dataclass
class FedConfig:
    spec: DatasetSpec
    epochs: int = 10
    datapath: Optional[str] = None          # CSV per client ('{client}' / '{rank}' are substituted)
    synthetic_rows: int = 40000             # rows per client when no CSV is given
    shard_mode: str = "independent"         # independent | iid | dirichlet | skew
    dirichlet_alpha: float = 0.5
    out_dir: str = "."
    n_sample: Optional[int] = None          # rows per epoch CSV (default spec.n_sample)
    aggregation: str = "weighted"           # weighted | uniform
    gmm_backend: str = "torch"              # torch | sklearn
    gmm_pool_cap: int = 0                   # cap on pooled GMM re-fit sample size (0 = reference: N)
    backend: str = "auto"                   # engine ops: auto | hip | torch
    write_csv: bool = True
    csv_writer: str = "auto"                # auto | native | pandas
    table_reader: str = "auto"              # client CSVs: auto | pandas | arrow (data/table.py read_csv_table)
    async_csv: bool = True                  # write each epoch CSV in the background (overlaps next round)
    # formatter threads of a CSV write (0: min(cores, 16)).  Measured: 4 background threads fall
    # behind a 21 ms round (the last flush then waits for a backlog): 20.9 -> 23.4 ms/epoch
    csv_threads: int = 0
    client_streams: bool = True             # in-process emulation: one HIP stream per client thread
    seed: int = 0
    engine: EngineConfig = dataclasses.field(default_factory=EngineConfig)
    ckpt_every: int = 0
    resume: bool = False
    use_graph: Optional[bool] = None
    verbose: bool = True
    metrics_log: Optional[str] = None
    drop_client_prob: float = 0.0           # fault injection: a client misses a round with this probability
    mode: str = "fedavg"                    # fedavg | mdgan
    device_encode: bool = True              # GPU: VGM-encode with the HIP kernel (csrc/kernels/vgm.hip)
    grad_flow: bool = False                 # record per-layer mean |grad| each round (utils/gradflow.py)
    e_interval: int = 1                     # fedavg: local epochs per aggregation; mdgan: D-swap period
    heartbeat_s: float = 0.0                # >0: per-round monitored barrier naming dead ranks
    profile_dir: Optional[str] = None       # export a torch.profiler trace of round `profile_epoch`
    profile_epoch: int = 1
    dump_real: bool = False                 # write the synthetic client shards (for the evaluators)
    # initial G/D weights: "independent" = every client its own random init, as the reference's
    # clients build their own modules (`Client/.../dtds/distributed.py:156-165`); the federator's copy
    # comes from the first client (`Server/dtds/distributed.py:789`).  "broadcast" = every rank
    # starts from the first client's weights.
    init: str = "independent"
    # sample + write the epoch CSV every N rounds (and after the last); 1 = every round (reference)
    csv_every: int = 1
    csv_epochs: Optional[List[int]] = None  # if set: sample + write only these epochs (and the last)
    # per-collective sub-phase timers (allreduce / share / generate / gather / d2h): HIP event pairs on a
    # GPU (no host sync), wall time on the CPU.  None = on when real process groups exist (multi-rank
    # runs, --force-dist), off otherwise
    phase_detail: Optional[bool] = None
    # phase timers on a GPU: "events" (HIP event pairs, no host sync) or "sync" (stream-synchronised wall
    # time at every phase boundary, the round-2 behaviour)
    phase_timer: str = "events"
    # wait on the host for the local epoch's kernels before issuing the aggregation / sampling work.
    # Measured (bench.py, 1 GPU, 20 rounds): 18.5 ms/round with the wait, 20.4-20.6 ms without it -- issuing
    # the generation graph, the pinned D2H copy and the CSV hand-off while the 80-step epoch still runs
    # stretches the epoch's kernels by ~2 ms (profiles/bench_train_sync_r3.txt)
    train_sync: bool = True
    # train_sync's wait, early: the host waits for the epoch's kernels up to (not including) the last N U-step
    # graph blocks, so the aggregation / sampling issue and the next round's launches are queued while those
    # blocks run instead of the device idling behind the host's round boundary (0 = wait for the whole epoch;
    # used with round_sync=False -- its wait would put the idle back)
    sync_lead_blocks: int = 0
    # wait on the host for the round's device work (aggregation, generation) before returning: the round time
    # then is device time; without it the next round's launches queue behind the generation and the host
    # returns at once (the epoch CSV's own hand-off waits for the table copy either way)
    round_sync: bool = True
    # generate round r's epoch table while round r + 1 trains (CTGANEngine.generate_decoded_split: a ~10 us prep
    # on the training stream snapshots what generation reads, the sampler / generator / decode run on a side
    # stream).  None = on where it applies (one process per GPU, HIP bf16 generation with graphs, FedAvg)
    pipeline_sample: Optional[bool] = None
    # pipelined sampling: issue the table's body / gather / copy / writer hand-off after the next round's training
    # is queued (their host time then overlaps it).  None = on without real process groups.  Default off: on the
    # round-6 tree one box measured 15.76-15.81 vs 15.88-15.98 ms per round, a second box no gain (15.87-15.93 vs
    # 15.79-15.86 on its settled pairs; profiles/round_sync_r6.txt), round 5 no gain either; over an RCCL
    # communicator that work queued beside the epoch stretched its kernels by ~2 ms as train_sync=0 does
    # (profiles/sync_r5.txt)
    defer_handoff: Optional[bool] = False
    # HIP stream priority of the pipelined generation stream (torch convention: lower = higher priority; 0 normal).
    # HIP maps streams onto hardware queues round-robin in creation order, so a normal-priority side stream can
    # share the training stream's in-order queue (seen in a kernel trace: both on queue 1)
    gen_stream_priority: int = 0
    # sample_round: gather the epoch table's shares even when one rank samples it all (a one-rank RCCL run then
    # exercises the multi-rank data path -- the side-stream gather over the communicator -- on one GPU; tests)
    force_gather: bool = False
    # after the last round the federator writes models/{name}_generator.pt (python -m dtds.sample)
    save_generator: bool = True
    # several clients on one GPU (in-process emulation): "on" runs their training steps as ONE batched launch
    # sequence (models/batched.py) when they allow it (HIP backend, no fault injection); "off" keeps one engine,
    # stream and step graph per client thread; "auto" batches up to batched_max_auto clients.  Round 4 made the
    # thread path's aggregation event-ordered (no device sync), so client threads start the next epoch while the
    # federator samples and writes: 12-epoch runs, 40k-row Intrusion clients, sum of rounds 1-11
    # (profiles/multiclient_r4.txt): 2 clients 337 ms batched vs 311 ms threads, 4 clients 416 vs 325, 8 clients
    # 609 vs 525 -- the threads are faster at every K (with 3-4x the round-to-round variance), so "auto" keeps
    # them (batched_max_auto = 1); the batched engine stays available ("on": one arena, lower variance).
    batched_clients: str = "auto"
    batched_max_auto: int = 1
    batched_arena_mb: float = 0.0           # per-client arena slab of the batched engine (0: estimated)
    # write models/label_encoders_{name}.pickle during initialisation (a helper process, as the reference writes it
    # there) instead of after the last round
    label_encoders_early: bool = True


def _log(cfg: FedConfig, rank: int, *msg):
    if cfg.verbose and rank == 0:
        print(*msg, flush=True)


def _warm_device(device):
    """HIP context creation and the first load of this library's code objects (one tiny launch of ours) while
    stage A's pandas work runs.  The initialisation path launches no ATen compute kernel any more (pooled GMM
    sample, row index, code checks and centring are this library's kernels or host numpy), so none of torch's
    code objects -- tens to hundreds of ms each on a box's first GPU process -- is loaded before round 0."""
    from ..ops import native
    ctr = torch.zeros(1, dtype=torch.int64, device=device)
    native.require().rng_bump(ctr)
    torch.cuda.synchronize(device)


def federate_gmm(banks: List[VGMBank], rows: List[int], cfg: FedConfig, device) -> tuple:
    """Federator side of ``uniform_continuous_gmm`` (`Server/dtds/distributed.py:689-765`).

    Draw ``int(N * n_i / N)`` samples from every client's VGM per continuous column, measure each
    client's Wasserstein-1 distance to the pooled sample, and fit one global VGM on the pool.
    Returns (global bank as dict, valid-component masks, normalised W1 distances [K, n_cont]).
    """
    rng = np.random.default_rng(cfg.seed + 12345)
    n_total = int(np.sum(rows))
    if cfg.gmm_pool_cap and n_total > cfg.gmm_pool_cap:
        n_total = cfg.gmm_pool_cap
    share = [float(r) / float(np.sum(rows)) for r in rows]
    n_cont = banks[0].n
    if cfg.gmm_backend == "torch" and n_cont:
        # the pool stays on the device: sampled there, W1 distances and the global fit read it in place
        pool, off = sample_pool(banks, [int(n_total * sh) for sh in share], rng, device, cfg.seed + 4242)
        e_hat = continuous_client_distances_device(pool, off)
        gb = fit_vgm(pool, backend="torch", seed=cfg.seed, device=device)
        return gb.to_dict(), gb.components().tolist(), e_hat
    pooled, per_client = [], [[] for _ in banks]
    for j in range(n_cont):
        parts = [b.sample_column(j, int(n_total * share[i]), rng) for i, b in enumerate(banks)]
        for i, p in enumerate(parts):
            per_client[i].append(p)
        pooled.append(np.concatenate(parts))
    e_hat = continuous_client_distances(pooled, per_client) if n_cont else np.zeros((len(banks), 0))
    gb = fit_vgm(pooled, backend=cfg.gmm_backend, seed=cfg.seed, device=device)
    comps = gb.components()
    return gb.to_dict(), comps.tolist(), e_hat


def round_alive_mask(cfg: FedConfig, epoch: int, k: int) -> np.ndarray:
    """Fault injection: which clients take part in round ``epoch`` (deterministic in the seed).

    At least one client always survives.  With ``drop_client_prob == 0`` every client is alive.
    """
    if cfg.drop_client_prob <= 0:
        return np.ones(k, dtype=bool)
    rng = np.random.default_rng([cfg.seed, 7, epoch])
    alive = rng.random(k) >= cfg.drop_client_prob
    if not alive.any():
        alive[rng.integers(0, k)] = True
    return alive


def effective_weights(weights: np.ndarray, alive: np.ndarray) -> np.ndarray:
    w = np.where(alive, weights, 0.0)
    return w / w.sum()


class FedRuntime:
    def __init__(self, cfg: FedConfig, comm: Comm, device: torch.device, federator: int = 0):
        self.cfg = cfg
        self.comm = comm
        self.device = device
        self.federator = federator
        self.rank = comm.rank
        self.is_fed = self.rank == federator
        self.is_client = comm.is_client
        self.name = cfg.spec.name
        self.n_sample = cfg.n_sample or cfg.spec.n_sample
        self._writer = None
        self._losses = None
        self.gradflow = None
        if cfg.grad_flow and comm.is_client and comm.client_index == 0:
            from ..utils.gradflow import GradFlow
            self.gradflow = GradFlow()
        # phase boundaries as HIP events on a GPU (no host sync inside a round; read after the fact)
        self.timer = PhaseTimer(events=device.type == "cuda" and cfg.phase_timer == "events",
                                sync=cfg.phase_timer == "sync")
        self.round_times: List[float] = []
        self.start_epoch = 0
        self.metrics = MetricsLog(cfg.metrics_log) if (cfg.metrics_log and self.is_fed) else None
        self.dump_csv = None
        self._round_start: Dict[int, float] = {}    # epoch -> wall time its round began
        self._csv_done: Dict[int, float] = {}       # epoch -> wall time its CSV was on disk
        self._csv_times: Dict[int, tuple] = {}      # epoch -> (copy wait, format + write) seconds, writer side

    # ================================================================= data
    def _local_frame(self) -> pd.DataFrame:
        cfg, c = self.cfg, self.comm
        k, idx = c.n_clients, c.client_index
        if cfg.datapath:
            path = cfg.datapath.format(client=idx, rank=self.rank)
            if os.path.exists(path):
                return read_csv_table(path, cfg.table_reader)
            print(f"[data] rank {self.rank}: {path} not found; using the synthetic {cfg.spec.name}-schema "
                  f"generator ({cfg.synthetic_rows} rows, shard mode {cfg.shard_mode})", flush=True)
        if cfg.shard_mode == "independent":
            df = generate(cfg.spec, cfg.synthetic_rows, seed=cfg.seed * 1000 + idx, as_category=True)
        else:
            full = generate(cfg.spec, cfg.synthetic_rows * k, seed=cfg.seed, as_category=True)
            df = shard(full, k, cfg.shard_mode, seed=cfg.seed, target=cfg.spec.target_column,
                       alpha=cfg.dirichlet_alpha)[idx]
        if cfg.dump_real:
            d = os.path.join(cfg.out_dir, "data", "raw")
            os.makedirs(d, exist_ok=True)
            df.to_csv(os.path.join(d, f"{self.name}_train_client{idx}.csv"), index=False)
        return df

    def merge_real_shards(self):
        """Federator: concatenate the clients' synthetic shards into data/raw/{name}_train.csv (for the
        evaluators, which compare against the full real table like `Server/similarity_analysis.py:96`)."""
        d = os.path.join(self.cfg.out_dir, "data", "raw")
        parts = [os.path.join(d, f"{self.name}_train_client{i}.csv") for i in range(self.comm.n_clients)]
        if all(os.path.exists(p) for p in parts):
            pd.concat([pd.read_csv(p) for p in parts]).to_csv(os.path.join(d, f"{self.name}_train.csv"), index=False)

    # ================================================================= init protocol
    def initialize(self):
        cfg, c = self.cfg, self.comm
        spec = cfg.spec
        t0 = time.time()
        warm = None
        if self.device.type == "cuda":
            # HIP context creation and the first load of this library's code objects overlap the pandas work
            # of stage A on a side thread
            warm = threading.Thread(target=_warm_device, args=(self.device,), daemon=True)
            warm.start()
        # ---- A. categorical meta
        self.table = None
        if self.is_client:
            df = self._local_frame()
            if list(df.columns) != list(spec.selected_variables):
                df = df[spec.selected_variables]
            self.table = TablePreprocessor(df, f"{self.name}_train", spec.problem_type,
                                           "" if spec.target_column == "none" else spec.target_column,
                                           spec.categorical_list, spec.nonnegative_list, spec.date_dic)
        metas = c.all_gather_object(self.table.local_meta() if self.is_client else None)
        client_metas = [metas[r] for r in c.client_ranks]
        payload = None
        if self.is_fed:
            merged, vocabs, d_hat = merge_categorical_metas(client_metas)
            payload = (merged, [(v.column_name, v.tolist()) for v in vocabs], d_hat)
        merged, vocab_lists, d_hat = c.broadcast_object(payload, src=self.federator)
        self.global_meta = merged
        self.vocabs = [CategoryVocab(lst, name) for name, lst in vocab_lists]
        self.d_hat = np.asarray(d_hat)
        cat_idx = [j for j, col in enumerate(merged["columns"]) if col["type"] == CATEGORICAL]
        self.cat_idx = cat_idx
        if self.is_fed:
            self._write_meta_artifacts()
            if cfg.label_encoders_early:
                self.start_label_encoders()
        if warm is not None:
            warm.join()
        self.init_times = {"meta": time.time() - t0}
        _log(cfg, self.rank, f"[init] categorical merge done ({time.time() - t0:.2f}s)")
        # ---- B. local VGMs -> global VGM
        info = None
        self.encoded = None
        if self.is_client:
            self.encoded = self.table.encode(self.vocabs)
            local = VGMTransformer().fit(self.encoded, cat_idx, (), backend=cfg.gmm_backend,
                                         seed=cfg.seed + 7 * c.client_index, device=self.device)
            info = (local.bank.to_dict(), len(self.encoded))
        infos = c.all_gather_object(info)
        client_infos = [infos[r] for r in c.client_ranks]
        self.rows = [n for _, n in client_infos]
        payload = None
        if self.is_fed:
            payload = self._global_gmm([VGMBank.from_dict(b) for b, _ in client_infos], self.rows)
        gbank, comps, e_hat = c.broadcast_object(payload, src=self.federator)
        self.bank = VGMBank.from_dict(gbank)
        self.components = np.asarray(comps, dtype=bool)
        self.e_hat = np.asarray(e_hat)
        self.init_times["vgm"] = time.time() - t0
        _log(cfg, self.rank, f"[init] global VGM fitted ({time.time() - t0:.2f}s)")
        # ---- C. refit + encode
        self.transformer = VGMTransformer().refit(self.encoded, merged, self.vocabs, cat_idx, (), self.bank,
                                                  self.components)
        lay = self.transformer.layout
        if self.is_client:
            self.train_matrix = self._encode_training_table()
        self.init_times["encode"] = time.time() - t0
        # ---- D. weights
        if cfg.aggregation == "uniform":
            self.weights = uniform_weights(c.n_clients)
        else:
            self.weights = aggregation_weights(self.d_hat, self.e_hat, self.rows)
        _log(cfg, self.rank, f"final aggregation weights {self.weights}")
        # ---- E. global span counts for generation
        maxw = int(lay.cond_width.max()) if lay.n_col else 0
        cnt = torch.zeros(lay.n_col, maxw, dtype=torch.float64)
        if self.is_client:
            cnt += torch.as_tensor(self.train_matrix.counts if hasattr(self.train_matrix, "counts")
                                   else CondTables.span_counts(self.train_matrix, lay))
        c.all_reduce_cpu(cnt)
        self.gen_cond = CondTables(lay, cnt.numpy())
        # ---- engine + F. initial weights
        # this process' generators only: torch.manual_seed seeds every visible GPU, and counting them
        # initialises the SMI library (0.1 s)
        torch.random.default_generator.manual_seed(cfg.seed + self.rank)
        if self.device.type == "cuda":
            with torch.cuda.device(self.device):
                torch.cuda.manual_seed(cfg.seed + self.rank)
        self.steps = [n // cfg.engine.batch_size for n in self.rows]
        self.engine = None
        batch = self._batch_group(lay)
        if batch is not None:
            # (a slab too small for a client's tables raises here: in "auto" mode every thread of the process
            # then falls back to an engine of its own, see _batch_ready)
            failed = None
            try:
                self.engine = batch.engine_for(self.batch_slab, lay, cfg.engine, self.batch_seed, backend=cfg.backend)
                self.engine.set_training_data(self.train_matrix)
            except MemoryError as e:
                failed = e
            if not self._batch_ready(failed):
                self.engine = None
        if self.engine is None:
            self.engine = CTGANEngine(lay, cfg.engine, self.device, backend=cfg.backend,
                                      seed=cfg.seed * 7919 + self.rank)
            if self.is_client:
                self.engine.set_training_data(self.train_matrix)
        if getattr(self, "thread_local_capture", False):
            self.engine.capture_mode = "thread_local"
        if self.gradflow is not None:     # the diagnostics read every parameter gradient after the epoch
            self.engine.keep_grads = True
        self.engine.set_generation_tables(self.gen_cond, self.transformer)
        self._initial_weights()
        if cfg.resume:
            self.load_checkpoint()
        if self.batched:
            # freeze the arena and capture the epoch's step graphs now (collective over the process' client
            # threads): a failure falls back to per-thread engines instead of aborting round 0
            self._prepare_batched()
        self.csv_cols = csv_layout(merged, self.vocabs)     # None: a date format only the pandas path handles
        if getattr(self, "thread_local_capture", False):
            # client threads of one process: none captures its graphs while another still uploads its tables (a
            # pageable host-to-device copy fails while any stream of the process captures -- with independent
            # initial weights nothing else orders the threads here)
            self.comm.barrier()
        self._prepare_round_zero()
        self.init_times["engine"] = time.time() - t0
        # RCCL's lazy communicator / P2P setup happens here, not in round 0
        c.warmup(dst=self.federator, gather=self.federator in c.client_ranks)
        self.init_times["total"] = time.time() - t0     # cumulative seconds at the end of each stage
        _log(cfg, self.rank, f"[init] done in {time.time() - t0:.2f}s: data_dim={lay.data_dim} n_opt={lay.n_opt} "
                             f"steps/epoch={self.steps}")

    def _prepare_round_zero(self):
        """Everything round 0 would otherwise do for the first time, done at initialisation: capture the
        local epoch's step graphs and the generation graph of this rank's share of the epoch table, create
        the table's copy stream and background writer, and page in one pinned host buffer of the table's
        size (torch's caching host allocator hands it back in round 0).  Round 0 then costs what every
        later round costs (`Server/dtds/distributed.py:790-829` times every round the same way)."""
        cfg, c = self.cfg, self.comm
        if self.device.type != "cuda" or cfg.mode != "fedavg" or cfg.use_graph is False:
            return
        gen = []
        samplers = c.client_ranks if (self.federator in c.client_ranks and not getattr(self, "batched", False)) \
            else [self.federator]
        if self.rank in samplers:
            i = samplers.index(self.rank)
            gen.append(self.n_sample // len(samplers) + (1 if i < self.n_sample % len(samplers) else 0))
        if self.is_fed and int(cfg.e_interval) > 1 and len(samplers) > 1:
            gen.append(self.n_sample)           # rounds without aggregation: the federator's table alone
        # (a batched engine's step graphs were captured by _prepare_batched)
        train = 0 if getattr(self, "batched", False) or not self.is_client or not self.engine.tables \
            else self.engine.steps_per_epoch
        self._pipe = self._pipeline_sample()
        if self._pipe:
            self._gen_stream = torch.cuda.Stream(self.device, priority=int(self.cfg.gen_stream_priority))
        self.engine.prepare_graphs(train, gen, gen_split=self._pipe)
        if self.is_fed and cfg.write_csv and cfg.async_csv:
            self._copy_stream = torch.cuda.Stream(self.device)
            # the table of round r is held by the writer while round r + 1 copies its own: two (three if the
            # writer lags) pinned buffers are live at once.  A second first-time pinned allocation in round 1
            # (hipHostMalloc of the 40k-row table, ~80 ms) was the "round-1 stall" of round 4
            n_cols = len(self.global_meta["columns"])
            bufs = [torch.empty((self.n_sample, n_cols), dtype=torch.float64, pin_memory=True) for _ in range(3)]
            del bufs                                # back to torch's caching host allocator
            from ..utils.csvio import AsyncTableWriter
            if self._writer is None:
                self._writer = AsyncTableWriter()
            self._writer.submit(self._warm_csv, n_cols)     # the writer thread (and the formatter's) start now
            self._writer.flush()

    def _pipeline_sample(self) -> bool:
        """FedConfig.pipeline_sample resolved: the table of round r is generated on a side stream while round
        r + 1 trains.  Off in the in-process client emulations (their threads order the gather with events of
        their own streams) and for a batched engine."""
        cfg = self.cfg
        if cfg.pipeline_sample is False or self.device.type != "cuda" or cfg.mode != "fedavg":
            return False
        if getattr(self, "batched", False) or type(self.comm).__name__ != "Comm":
            return False
        return bool(self.engine.can_split_generation())

    def _warm_csv(self, n_cols: int):
        """One table of the real size and shape through the native formatter to the null device, on the writer
        thread.  The first table a process formats costs ~18x a steady one (83 vs 4.6 ms on the box: the
        formatter threads' fresh malloc arenas fault in every page of the formatted text), and while it ran the
        main thread stalled as long (round 1: 78 ms waiting to enter the train phase, profiles/stall_r5.txt).
        Formatting plausible values (long float reprs, every vocabulary index) pays that at initialisation."""
        from ..data.decode import KIND_FLOAT, KIND_NONNEG, KIND_VOCAB
        from ..utils import csvio
        lay = self.csv_cols
        if lay is None or self.cfg.csv_writer not in ("auto", "native") or not csvio.available():
            return
        t0 = time.perf_counter()
        rows = max(int(self.n_sample), 1)
        vals = np.zeros((rows, n_cols))
        rng = np.random.default_rng(0)
        for j, k in enumerate(lay.kinds):
            s = lay.src[j]
            if k == KIND_VOCAB:
                vals[:, s] = np.arange(rows) % max(len(lay.vocabs[j]), 1)
            elif k == KIND_FLOAT:
                vals[:, s] = rng.standard_normal(rows) * 1e3
            elif k == KIND_NONNEG:
                vals[:, s] = rng.standard_normal(rows)
        try:
            csvio.write_layout(os.devnull, vals, lay, threads=self.cfg.csv_threads)
        except (RuntimeError, ValueError) as e:     # a warm-up only: the real tables report their own errors
            _log(self.cfg, self.rank, f"csv warm-up skipped: {e}")
        self.csv_warm_s = time.perf_counter() - t0

    def _batch_group(self, lay):
        """The batched multi-client engine's arena when this process' clients run as one (threads of an
        in-process emulation on a GPU; see FedConfig.batched_clients), else None."""
        cfg, c = self.cfg, self.comm
        g = getattr(c, "g", None)
        self.batched = False
        kind = type(c).__name__
        if cfg.batched_clients == "off" or g is None or kind not in ("ThreadComm", "HierComm") or not self.is_client:
            return None
        # this process' clients are the threads of g: client (rank - t) + i is thread i
        t = c.t if kind == "HierComm" else c.rank
        first = self.rank - t
        local_rows = self.rows[first:first + g.k]
        ok = (self.device.type == "cuda" and cfg.backend in ("auto", "hip") and cfg.drop_client_prob <= 0 and
              c.client_ranks == list(range(c.world_size)) and g.k > 1 and cfg.mode == "fedavg")
        if ok and cfg.batched_clients == "auto" and g.k > cfg.batched_max_auto:
            return None
        if not ok:
            if cfg.batched_clients == "on":
                raise RuntimeError("batched_clients='on' needs a GPU, the HIP backend, several clients per process, "
                                   "every rank a client and no fault injection")
            return None
        from ..models.arena import Arena
        from ..models.batched import BatchedClients, slab_order
        # slabs in non-increasing order of steps per epoch (clients with fewer rows finish their epoch first and
        # leave the batched launches; models/batched.py); engine seeds consecutive in slab order
        order = slab_order([n // cfg.engine.batch_size for n in local_rows])
        self.batch_slab = order.index(t)
        self.batch_seed = cfg.seed * 7919 + first + self.batch_slab
        self._local_t = t
        with g.lock:
            if g.batch is None:
                slab = int(cfg.batched_arena_mb * (1 << 20)) or \
                    Arena.estimate_slab_bytes(lay, cfg.engine, max(local_rows))
                g.batch = BatchedClients.empty(g.k, self.device, slab, n_rows=max(local_rows))
                g.batch.client_of_slab = order
        self.batched = True
        self.batch_clients = g.batch       # (strong reference: the engine only holds a weak one)
        return g.batch

    def _batch_ready(self, err: Optional[BaseException]) -> bool:
        """Collective over the process' client threads: did every thread build its slab engine?  If not,
        "auto" mode falls back to one engine per thread (False), "on" mode raises."""
        g = self.comm.g
        if g.local_all(self._local_t, err is None):
            return True
        if self.cfg.batched_clients == "on":
            raise RuntimeError(f"batched clients: a client's engine does not fit its arena slab ({err}); "
                               "raise FedConfig.batched_arena_mb") from err
        _log(self.cfg, self.rank, f"[init] batched clients do not fit the arena ({err}): one engine per client")
        self._drop_batch()
        return False

    def _drop_batch(self):
        g = self.comm.g
        g.wait()
        if self._local_t == 0:
            g.batch = None
        self.batched = False
        self.batch_clients = None
        g.wait()

    def _prepare_batched(self):
        """Collective over the process' client threads: thread 0 freezes the arena (one device sync: every
        thread's initial state is on the device) and captures the epoch's step graphs.  On a failure
        ("auto" mode) every thread continues with an engine of its own, holding its client's state."""
        g, t = self.comm.g, self._local_t
        g.wait()                    # every thread's initial weights / checkpoint are enqueued
        err = None
        if t == 0:
            try:
                self.batch_clients.prepare(self.cfg.use_graph)
                # the FedAvg matrix-vector product's library kernels load on first use (~60 ms in round 0)
                b = self.batch_clients
                torch.mv(torch.zeros(b.k, 64, device=self.device).t(), torch.zeros(b.k, device=self.device))
            except (MemoryError, RuntimeError) as e:
                err = e
                if hasattr(self.engine.ops, "reset_held"):
                    self.engine.ops.reset_held()
        if g.local_all(t, err is None):
            return
        if self.cfg.batched_clients == "on":
            raise RuntimeError(f"batched clients: preparing the batched step failed ({err})") from err
        _log(self.cfg, self.rank, f"[init] batched step unavailable ({err}): one engine per client")
        if t == 0:
            from ..utils.devsync import device_sync
            device_sync(self.device)
        g.wait()
        old = self.engine
        e = CTGANEngine(old.layout, self.cfg.engine, self.device, backend=self.cfg.backend,
                        seed=self.cfg.seed * 7919 + self.rank)
        e.capture_mode = old.capture_mode
        e.set_training_data(self.train_matrix)
        e.set_generation_tables(self.gen_cond, self.transformer)
        for name in ("flat", "mG", "vG", "mD", "vD", "stepG", "stepD"):
            getattr(e, name).copy_(getattr(old, name))
        if hasattr(e.ops, "ctr"):
            e.ops.ctr.copy_(old.ops.ctr)
        e.bn_batches = old.bn_batches
        self.engine = e
        self._drop_batch()

    def _initial_weights(self):
        """Step F: the clients keep their own random init (reference) or adopt the first client's;
        a dataless federator always takes the first client's copy (`Server/dtds/distributed.py:789`)."""
        c, src = self.comm, self.comm.client_ranks[0]
        if self.cfg.init == "broadcast":
            c.broadcast_tensor(self.engine.flat, src=src)
        elif self.cfg.init == "independent":
            if not all(r in c.client_ranks for r in range(c.world_size)):
                buf = self.engine.flat.detach().clone()
                c.broadcast_tensor(buf, src=src)
                if not self.is_client:
                    self.engine.flat.copy_(buf)
        else:
            raise ValueError(f"init must be independent or broadcast, got {self.cfg.init!r}")

    def _encode_training_table(self):
        """VGM-encode the local table: on the GPU with the HIP kernel (matrix and row lists stay
        resident), else with the numpy reference path."""
        cfg = self.cfg
        if self.device.type == "cuda" and cfg.backend in ("auto", "hip") and cfg.device_encode:
            from ..features.encode_gpu import encode_on_device
            try:
                return encode_on_device(self.transformer, self.encoded, self.device, seed=cfg.seed * 131 + self.rank)
            except ValueError:
                pass   # e.g. non-integer category codes: host path below
        return self.transformer.transform(self.encoded, np.random.default_rng(cfg.seed + self.rank))

    def _global_gmm(self, banks: List[VGMBank], rows: List[int]):
        return federate_gmm(banks, rows, self.cfg, self.device)

    def _write_meta_artifacts(self):
        mdir = os.path.join(self.cfg.out_dir, "models")
        os.makedirs(mdir, exist_ok=True)
        dump_meta_json(self.global_meta, os.path.join(mdir, f"{self.name}.json"))

    def _label_encoder_path(self) -> str:
        mdir = os.path.join(self.cfg.out_dir, "models")
        os.makedirs(mdir, exist_ok=True)
        return os.path.join(mdir, f"label_encoders_{self.name}.pickle")

    def start_label_encoders(self):
        """Start writing ``models/label_encoders_{name}.pickle`` during initialisation, as the reference
        does (`Server/dtds/distributed.py:679-684`), so a crashed or killed run still leaves it next to
        the meta JSON.  Building sklearn ``LabelEncoder`` objects imports scikit-learn (0.5-0.9 s of
        Python), so a helper process does it (data/vocab.py ``__main__``): neither this process' GIL nor
        its critical path sees the import.  ``write_label_encoders`` waits for it."""
        import subprocess
        import sys
        self._le_proc = None
        req = json.dumps({"path": os.path.abspath(self._label_encoder_path()),
                          "vocabs": [[v.column_name, v.tolist()] for v in self.vocabs]})
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
        # the request goes through a file and the helper's stderr into another: no pipe that this process
        # must write (the wide table's vocabularies are large) or drain (a chatty helper would block on a
        # full pipe) while it initialises
        import tempfile
        try:
            with tempfile.TemporaryFile() as f:
                f.write(req.encode())
                f.flush()
                f.seek(0)
                self._le_err = tempfile.TemporaryFile()
                p = subprocess.Popen([sys.executable, "-m", "fed_tgan_amd.data.vocab"], stdin=f,
                                     stdout=subprocess.DEVNULL, stderr=self._le_err, env=env)
            self._le_proc = p
        except OSError:
            self._le_proc = None

    def write_label_encoders(self):
        """Make sure ``models/label_encoders_{name}.pickle`` exists: wait for the helper process of
        ``start_label_encoders``, or write the file here if there was none or it failed."""
        p = getattr(self, "_le_proc", None)
        self._le_proc = None
        if p is not None:
            try:
                p.wait(timeout=120)
                if p.returncode == 0 and os.path.exists(self._label_encoder_path()):
                    return self._label_encoder_path()
                self._le_err.seek(0)
                err = self._le_err.read().decode(errors="replace")
                print(f"[init] label-encoder helper failed ({p.returncode}): {err[-300:]}", flush=True)
            except Exception:            # noqa: BLE001 - fall back to an in-process write
                p.kill()
            finally:
                self._le_err.close()
        from ..data.vocab import write_label_encoders
        return write_label_encoders(self._label_encoder_path(), self.vocabs)

    # ================================================================= rounds
    def _sub(self, name: str):
        """Sub-phase timer (see FedConfig.phase_detail), or nothing."""
        on = self.cfg.phase_detail
        if on is None:
            on = bool(getattr(self.comm, "dist_active", False))
        return self.timer.phase(name, self.device) if on else contextlib.nullcontext()

    def aggregate(self, alive: np.ndarray | None = None):
        """Weighted FedAvg of every G/D parameter and BN statistic (`Server/dtds/distributed.py:86-106`)
        as one all-reduce of the pre-scaled flat buffer; clients that missed the round get weight 0."""
        c = self.comm
        wts = self.weights if alive is None else effective_weights(self.weights, alive)
        w = float(wts[c.client_index]) if self.is_client else 0.0
        if getattr(self, "_pipe", False) and getattr(c, "_native", None) is not None:
            # the previous round's pipelined gather runs on torch's RCCL communicator on the generation stream,
            # this all-reduce on the native one: two communicators with collectives in flight at once and no
            # cross-rank order between them can deadlock, so every rank orders the all-reduce after its gather
            torch.cuda.current_stream(self.device).wait_stream(self._gen_stream)
        with self._sub("allreduce"):
            c.weighted_all_reduce(self.engine.flat, w)
        with self._sub("share"):
            # a dedicated federator (RCCL among the clients) gets the clients' mean last-step losses with the
            # aggregate: one device all-reduce and the same message, no host round trip per client
            m = None
            if self.federator not in c.client_ranks and c.data_backend == "nccl" and c.dist_active:
                m = self._loss_buf
                if self.is_client:
                    m.copy_(self.engine.metrics.detach().view(-1))
                    c.client_mean(m)
            shared = c.share_with_federator(self.engine.flat, self.federator, extra=m)
            self._losses_shared = shared and m is not None
            if self._losses_shared and self.is_fed:
                self._losses = m.cpu()   # (the federator's stream was synchronised by the receive)
        # num_batches_tracked: weighted average of every client's counter, truncated (reference cast)
        ep = self.engine
        counts = np.asarray([2 * s for s in self.steps], dtype=np.float64) * (self._epoch_done)
        ep.bn_batches = int(np.sum(wts * counts))

    def sample_round(self, epoch: int, aggregated: bool = True):
        """Generate n_sample rows, decode, and (federator) write the epoch CSV.

        After an aggregation every client holds the global model, so the rows are generated sharded
        over the client GPUs; on a round without aggregation (-E_interval > 1) the clients' models
        differ and the whole table comes from the federator's model alone."""
        c = self.comm
        colocated = self.federator in c.client_ranks
        # (batched clients: the federator's engine generates the whole table -- the other clients' threads
        # issue no GPU work at all)
        samplers = c.client_ranks if (colocated and aggregated and not getattr(self, "batched", False)) \
            else [self.federator]
        share = None
        per = [self.n_sample // len(samplers) + (1 if i < self.n_sample % len(samplers) else 0)
               for i in range(len(samplers))]
        # on a GPU with the background writer, the table's device-to-host copy runs on a side
        # stream and the writer waits for it: round r's copy + CSV overlap round r + 1's training
        # (bench.py's timed region still ends with every table on disk)
        async_copy = self.cfg.async_csv and self.device.type == "cuda"
        # (pipelined: the rows come from the generation side stream, and the gather / copy are ordered on it, so
        # the round ends without waiting for them -- the next round's training overlaps them)
        pipe = bool(getattr(self, "_pipe", False)) and self.rank in samplers
        defer = self.cfg.defer_handoff
        if defer is None:
            defer = not bool(getattr(c, "dist_active", False))
        if pipe and async_copy and defer:
            # only the prep (snapshot of the model) is issued now; the body, the gather, the copy and the writer
            # hand-off are issued by _complete_handoff once the next round's training is queued, so their host
            # time overlaps that training instead of the GPU idling behind it
            k = per[samplers.index(self.rank)]
            with self._sub("generate"):
                self.engine.generation_prep(k)
            self._handoff = (k, per, samplers, epoch)
            return None
        gen = (lambda k: self.engine.generate_decoded_split(k, self._gen_stream)) if pipe \
            else self.engine.generate_decoded
        on_gen = (lambda: torch.cuda.stream(self._gen_stream)) if pipe else contextlib.nullcontext
        if len(samplers) == 1 and not self._force_gather(samplers):
            if self.rank in samplers:
                with self._sub("generate"):
                    vals = gen(per[0])
                with self._sub("d2h"), on_gen():
                    share = self._host(vals) if async_copy else vals.cpu().numpy()
        else:
            # every client decodes its share on its GPU; one gather to the federator (RCCL over
            # xGMI when the data plane is RCCL), one device-to-host copy there
            with self._sub("generate"):
                vals = gen(per[samplers.index(self.rank)])
            with self._sub("gather"), on_gen():
                rows = c.gather_rows(vals, per, samplers, dst=self.federator, to_host=not async_copy)
            with self._sub("d2h"), on_gen():
                if self.is_fed:
                    if rows.device.type == "cuda":
                        share = self._host(rows)
                    else:
                        share = rows.numpy()
        if self.is_fed and self.cfg.write_csv:
            self.write_epoch_csv(share, epoch)
        return share if self.is_fed else None

    def close(self) -> None:
        """Orderly teardown (idempotent): every epoch CSV on disk, the writer and label-encoder helper joined,
        the device drained, the captured graphs and side streams released, then the communicators destroyed --
        all before interpreter exit, whose destructor order is arbitrary (a run under rocprofv3 segfaulted in
        exit() after the tool's finalisation, profiles/exit_r6.txt)."""
        if getattr(self, "_closed", False):
            return
        self._closed = True
        try:
            self.flush_writes()
        finally:
            w, self._writer = getattr(self, "_writer", None), None
            if w is not None:
                w.close()
            if getattr(self, "_le_proc", None) is not None:
                self.write_label_encoders()
            eng = getattr(self, "engine", None)
            if eng is not None:
                eng.release()
            self._gen_stream = self._copy_stream = None
            if getattr(self, "comm", None) is not None:
                self.comm.destroy()

    def _force_gather(self, samplers) -> bool:
        """FedConfig.force_gather applies: a real process group whose every client samples (co-located federator)."""
        c = self.comm
        return bool(self.cfg.force_gather) and c.dist_active and list(samplers) == list(c.client_ranks) and \
            self.federator in c.client_ranks

    def _complete_handoff(self):
        """Issue the deferred part of the last pipelined sample_round: the generation body on the side stream,
        the gather to the federator, the pinned copy and the CSV writer hand-off."""
        h = getattr(self, "_handoff", None)
        if h is None:
            return
        self._handoff = None
        k, per, samplers, epoch = h
        share = None
        with torch.cuda.stream(self._gen_stream):
            vals = self.engine.generation_body(k, self._gen_stream)
            if len(samplers) == 1 and not self._force_gather(samplers):
                share = self._host(vals)
            else:
                rows = self.comm.gather_rows(vals, per, samplers, dst=self.federator, to_host=False)
                if self.is_fed:
                    share = self._host(rows) if rows.device.type == "cuda" else rows.numpy()
        if self.is_fed and self.cfg.write_csv:
            self.write_epoch_csv(share, epoch)

    def _host(self, t: torch.Tensor) -> PendingHost:
        if getattr(self, "_copy_stream", None) is None:
            self._copy_stream = torch.cuda.Stream(t.device)
        return PendingHost(t, self._copy_stream)

    def result_dir(self) -> str:
        d = os.path.join(self.cfg.out_dir, f"{self.name}_result")
        os.makedirs(d, exist_ok=True)
        return d

    def write_epoch_csv(self, values: np.ndarray, epoch: int):
        if self.cfg.async_csv:
            if self._writer is None:
                from ..utils.csvio import AsyncTableWriter
                self._writer = AsyncTableWriter()
            self._writer.submit(self._write_epoch_csv, values, epoch)
            return os.path.join(self.result_dir(), f"{self.name}_synthesis_epoch_{epoch}.csv")
        return self._write_epoch_csv(values, epoch)

    def flush_writes(self):
        """Block until every submitted epoch CSV is on disk (a deferred pipelined hand-off is issued first)."""
        self._complete_handoff()
        if self._writer is not None:
            self._writer.flush()

    def _write_epoch_csv(self, values, epoch: int):
        t0 = time.perf_counter()
        if isinstance(values, PendingHost):
            values = values.get()
        t1 = time.perf_counter()
        path = self._write_epoch_csv_body(values, epoch)
        self._csv_done[epoch] = time.time()
        # writer-side seconds of this table: waiting for its device-to-host copy, formatting + writing
        self._csv_times[epoch] = (t1 - t0, time.perf_counter() - t1)
        return path

    def _write_epoch_csv_body(self, values, epoch: int):
        if isinstance(values, PendingHost):
            values = values.get()
        path = os.path.join(self.result_dir(), f"{self.name}_synthesis_epoch_{epoch}.csv")
        use_native = self.cfg.csv_writer in ("auto", "native") and self.csv_cols is not None
        if use_native:
            from ..utils import csvio
            if csvio.available() or self.cfg.csv_writer == "native":
                csvio.write_layout(path, values, self.csv_cols, threads=self.cfg.csv_threads)
                return path
        decode_frame(values, self.global_meta, self.vocabs).to_csv(path, index=False)
        return path

    def run_round(self, epoch: int) -> float:
        c = self.comm
        t0 = time.time()
        self._round_start[epoch] = t0
        alive = round_alive_mask(self.cfg, epoch, c.n_clients)
        h0 = time.perf_counter()
        cpu0 = time.process_time()
        thr0 = cgroup_cpu_stat() if self.metrics is not None else {}
        hw = hi = 0.0
        with self.timer.phase("train", self.device):
            if getattr(self, "batched", False):
                # every client's epoch in one batched launch sequence, issued by the process' thread 0 (host
                # barriers over the process' threads only; the device work is on thread 0's stream)
                c.g.wait()
                hw = time.perf_counter()
                if self._local_t == 0:
                    self.batch_clients.train_epoch(self.cfg.use_graph)
                    if self.gradflow is not None:
                        self.gradflow.update(self.engine)
                hi = time.perf_counter()
                c.g.wait()
            elif self.is_client and alive[c.client_index]:
                hw = time.perf_counter()
                self.engine.train_epoch(self.cfg.use_graph, lead=max(int(self.cfg.sync_lead_blocks), 0))
                hi = time.perf_counter()
                if self.gradflow is not None:
                    self.gradflow.update(self.engine)
            # the previous round's deferred table work, now that this round's training is queued
            self._complete_handoff()
            if self.cfg.train_sync and self.device.type == "cuda":
                ev = getattr(self.engine, "lead_event", None) if self.cfg.sync_lead_blocks > 0 else None
                if ev is not None:
                    ev.synchronize()
                else:
                    stream_sync(self.device)
        # host-side seconds of the train phase: waiting at the entry barrier, issuing the epoch, until its end
        self._host_train = {"h_wait": (hw - h0) if hw else 0.0, "h_issue": (hi - hw) if hi else 0.0,
                            "h_total": time.perf_counter() - h0}
        self._epoch_done = epoch + 1
        h1 = time.perf_counter()
        with self.timer.phase("aggregate", self.device):
            # -E_interval (accepted but unused by the reference, `Server/dtds/distributed.py:904`):
            # local epochs between aggregations (1 = aggregate every round, the reference behaviour)
            aggregated = (epoch + 1) % max(int(self.cfg.e_interval), 1) == 0
            if aggregated:
                self.aggregate(alive if self.cfg.drop_client_prob > 0 else None)
        every = max(int(self.cfg.csv_every), 1)
        if self.cfg.csv_epochs is not None:
            dump = epoch in self.cfg.csv_epochs or epoch + 1 == self.cfg.epochs
        else:
            dump = (epoch + 1) % every == 0 or epoch + 1 == self.cfg.epochs
        h2 = time.perf_counter()
        if dump:
            with self.timer.phase("sample_dump", self.device):
                self.sample_round(epoch, aggregated)
        h3 = time.perf_counter()
        if self.device.type == "cuda" and self.cfg.round_sync:
            stream_sync(self.device)
        dt = time.time() - t0
        # host seconds of the round's phases after the train phase: aggregation, sampling + CSV hand-off, final wait
        self._host_train.update({"h_agg": h2 - h1, "h_sample": h3 - h2, "h_end": time.perf_counter() - h3})
        if self.metrics is not None:
            # process CPU seconds of the round (all threads) and the cgroup's CFS throttling during it
            self._host_train["cpu_s"] = time.process_time() - cpu0
            thr1 = cgroup_cpu_stat()
            for k in ("throttled_usec", "nr_throttled", "usage_usec"):
                if k in thr0 and k in thr1:
                    self._host_train[k] = thr1[k] - thr0[k]
        self._sync_losses()
        return dt

    @property
    def _loss_buf(self) -> torch.Tensor:
        """Device buffer of the four last-step loss terms (loss_d, pen, loss_g, cond CE), float32."""
        if getattr(self, "_lbuf", None) is None:
            self._lbuf = torch.zeros(4, dtype=torch.float32, device=self.engine.flat.device)
        return self._lbuf

    def _sync_losses(self):
        """Collective when the federator holds no data: the clients' last-step losses, averaged.  With an
        RCCL data plane they already travelled with the aggregate (``aggregate``); on gloo they take one
        host all-reduce over the control plane."""
        c = self.comm
        if c.world_size == 1 or self.federator in c.client_ranks:
            self._losses = None
            return
        if getattr(self, "_losses_shared", False):
            self._losses_shared = False
            return
        m = self.engine.metrics.detach().cpu().double() if self.is_client else torch.zeros(4, dtype=torch.float64)
        c.all_reduce_cpu(m)
        self._losses = m / max(c.n_clients, 1)

    def _profiled_round(self, epoch: int) -> float:
        """One round under torch.profiler (host ops + HIP kernels), exported as a Chrome trace."""
        from torch.profiler import ProfilerActivity, profile
        acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.device.type == "cuda" else [])
        os.makedirs(self.cfg.profile_dir, exist_ok=True)
        with profile(activities=acts, record_shapes=False) as prof:
            dt = self.run_round(epoch)
        prof.export_chrome_trace(os.path.join(self.cfg.profile_dir, f"trace_rank{self.rank}_epoch{epoch}.json"))
        return dt

    def round_losses(self):
        """(loss_d, loss_g) of the last step, as the federator reports them."""
        m = getattr(self, "_losses", None)
        if m is not None:
            return float(m[0] + m[1]), float(m[2] + m[3])
        return self.engine.losses() if self.is_client else (float("nan"), float("nan"))

    def fit(self):
        cfg = self.cfg
        for ep in range(self.start_epoch, cfg.epochs):
            # (one profiler per process: in a threaded emulation only the federator's thread profiles)
            if cfg.profile_dir and ep == cfg.profile_epoch and (self.is_fed or getattr(self.comm, "g", None) is None):
                dt = self._profiled_round(ep)
            else:
                dt = self.run_round(ep)
            fault = os.environ.get("FEDTGAN_FAULT_EXIT")   # "rank:epoch" -- test hook: that rank dies
            if fault and fault == f"{self.rank}:{ep}":
                os._exit(3)
            if cfg.heartbeat_s > 0:
                self.comm.heartbeat(cfg.heartbeat_s)
            self.round_times.append(dt)
            if self.is_fed:
                ld, lg = self.round_losses()
                _log(cfg, self.rank, f"EPOCH {ep}: loss_d:{ld:>6.2f}   loss_g:{lg:>6.2f}   round time: {dt:.3f} sec")
                if self.metrics is not None:
                    csv_t = self._csv_times.get(ep - 1)      # the previous table, written during this round
                    self.metrics.write({"epoch": ep, "round_s": dt, "loss_d": ld, "loss_g": lg,
                                        **self.timer.last(), **getattr(self, "_host_train", {}),
                                        **({"csv_wait_prev": csv_t[0], "csv_write_prev": csv_t[1]} if csv_t else {}),
                                        **({"csv_warm_s": self.csv_warm_s}
                                           if ep == self.start_epoch and hasattr(self, "csv_warm_s") else {})})
            if cfg.ckpt_every and (ep + 1) % cfg.ckpt_every == 0:
                self.flush_writes()      # the checkpoint's per-round stamps include every CSV so far
                self.save_checkpoint(ep + 1)
        self.flush_writes()
        if self.gradflow is not None:
            d = os.path.join(cfg.out_dir, "reports")
            os.makedirs(d, exist_ok=True)
            self.gradflow.save_csv(os.path.join(d, "grad_flow.csv"))
            self.gradflow.plot(d)
        if self.is_fed:
            self.write_label_encoders()
            self.write_timestamps()
            if cfg.dump_real:
                self.merge_real_shards()
            if cfg.save_generator:
                self.save_generator()

    def epoch_stamps(self) -> List[float]:
        """Per-round entries of ``timestamp_experiment.csv``, each INCLUDING that round's CSV dump.

        The reference times the round with the dump inside it (`Server/dtds/distributed.py:795-825`),
        so the cumulative sum (``time_stamp`` in `Server/similarity_analysis.py:111-115`) is the wall
        time at which each epoch's CSV exists.  With the background writer the dump of round r
        overlaps round r + 1, so entry r is the time from the previous epoch's CSV completion (or
        the first round's start) to this epoch's CSV completion: the cumulative sum again equals the
        wall time at which epoch r's table is on disk.  Rounds without a recorded CSV keep their
        round time."""
        fitted = sorted(self._round_start)
        if not fitted or any(e not in self._csv_done for e in fitted):
            return list(self.round_times)
        prior = list(self.round_times[:max(0, len(self.round_times) - len(fitted))])   # resumed: checkpointed rounds
        out, prev = [], self._round_start[fitted[0]]
        for e in fitted:
            done = self._csv_done[e]
            out.append(done - prev)
            prev = done
        return prior + out

    def save_generator(self, path: Optional[str] = None) -> str:
        """The aggregated generator + transformer + sampler tables + decode metadata in one
        weights-only file (`fed_tgan_amd.models.generator_io`); the reference's unused
        ``save_model`` (`Server/dtds/distributed.py:560-563`) made usable."""
        from ..models.generator_io import export_generator
        if path is None:
            d = os.path.join(self.cfg.out_dir, "models")
            os.makedirs(d, exist_ok=True)
            path = os.path.join(d, f"{self.name}_generator.pt")
        return export_generator(path, self.engine, self.transformer, self.gen_cond, self.global_meta, self.vocabs,
                                self.name)

    def write_timestamps(self):
        """One per-round wall time per line, no header (`Server/dtds/distributed.py:827-829`)."""
        import csv
        path = os.path.join(self.cfg.out_dir, "timestamp_experiment.csv")
        with open(path, "w", newline="") as f:
            csv.writer(f, dialect="excel").writerows([[t] for t in self.epoch_stamps()])
        return path

    # ================================================================= checkpoint / resume
    def _ckpt_path(self) -> str:
        d = os.path.join(self.cfg.out_dir, "ckpt")
        os.makedirs(d, exist_ok=True)
        return os.path.join(d, f"rank{self.rank}.pt")

    def save_checkpoint(self, epoch: int):
        e = self.engine
        if getattr(self, "batched", False):
            from ..utils.devsync import device_sync
            device_sync(self.device)      # the state was written by client 0's stream
        state = {"epoch": epoch, "flat": e.flat.cpu(), "mG": e.mG.cpu(), "vG": e.vG.cpu(), "mD": e.mD.cpu(),
                 "vD": e.vD.cpu(), "stepG": e.stepG.cpu(), "stepD": e.stepD.cpu(), "bn_batches": e.bn_batches,
                 "round_times": self.epoch_stamps(), "cpu_rng": torch.get_rng_state(),
                 "g_wt": bool(e.cfg.g_wt)}       # flat-buffer layout of the generator weights
        if hasattr(e.ops, "ctr"):          # HIP backend: the device Philox step counter
            state["rng_ctr"] = e.ops.ctr.cpu()
        torch.save(state, self._ckpt_path())

    def load_checkpoint(self):
        p = self._ckpt_path()
        if not os.path.exists(p):
            return
        st = torch.load(p, weights_only=True)
        e = self.engine
        keys = ("flat", "mG", "vG", "mD", "vD")
        # a checkpoint without the key predates input-major generator weights: [out, in] storage
        saved_wt = bool(st.get("g_wt", False))
        if saved_wt != bool(e.cfg.g_wt):
            st.update(e.convert_layout({k: st[k] for k in keys}, saved_wt))
        for k in keys + ("stepG", "stepD"):
            getattr(e, k).copy_(st[k])
        e.bn_batches = int(st["bn_batches"])
        if "cpu_rng" in st:
            torch.set_rng_state(st["cpu_rng"])
        if "rng_ctr" in st and hasattr(e.ops, "ctr"):
            e.ops.ctr.copy_(st["rng_ctr"])
        self.start_epoch = int(st["epoch"])
        self.round_times = list(st["round_times"])
        self._epoch_done = self.start_epoch
