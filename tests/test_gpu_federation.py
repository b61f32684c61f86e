"""Federation on the GPU: the HIP engine inside FedRuntime (single client, and the in-process
multi-client emulation with one HIP stream per client), several clients per process over several
processes (HierComm), and the asynchronous table path (pinned side-stream copy awaited by the
background CSV writer)."""
import os

import numpy as np
import pandas as pd
import pytest
import torch

from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.fed.local import run_local_emulation
from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
from fed_tgan_amd.models.engine import EngineConfig
from fed_tgan_amd.parallel.comm import Comm
from fed_tgan_amd.utils.devsync import PendingHost

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _cfg(tmp, **kw):
    base = dict(spec=intrusion_spec(), epochs=2, synthetic_rows=4000, n_sample=3000, out_dir=str(tmp),
                backend="hip", gmm_backend="torch", engine=EngineConfig(batch_size=500), verbose=False)
    base.update(kw)
    return FedConfig(**base)


def _check_outputs(tmp, epochs, n_sample):
    res = os.path.join(tmp, "Intrusion_result")
    for ep in range(epochs):
        df = pd.read_csv(os.path.join(res, f"Intrusion_synthesis_epoch_{ep}.csv"))
        assert df.shape == (n_sample, 42) and list(df.columns) == intrusion_spec().selected_variables
    ts = pd.read_csv(os.path.join(tmp, "timestamp_experiment.csv"), header=None)
    assert ts.shape == (epochs, 1) and bool((ts.iloc[:, 0] > 0).all())


def test_gpu_single_client_runtime(tmp_path):
    from fed_tgan_amd.ops import native
    native.require()
    rt = FedRuntime(_cfg(tmp_path), Comm(0, 1, [0], "gloo", device=DEV), DEV)
    rt.initialize()
    assert rt.engine.ops.name == "hip"
    rt.fit()
    rt.flush_writes()
    _check_outputs(tmp_path, 2, 3000)
    assert np.isfinite(rt.engine.losses()).all()


def test_gpu_emulated_clients_on_streams(tmp_path):
    """Two clients, one HIP stream each, weighted aggregation through the thread communicator."""
    from fed_tgan_amd.ops import native
    native.require()
    rt = run_local_emulation(_cfg(tmp_path, shard_mode="iid"), 2, backend="hip", device=DEV)
    _check_outputs(tmp_path, 2, 3000)
    assert np.isclose(rt.weights.sum(), 1.0) and len(rt.weights) == 2
    assert bool(torch.isfinite(rt.engine.flat).all())


def test_pending_host_copy_matches_sync_copy():
    """The side-stream pinned copy waits for the producing kernels and survives the source being
    released (record_stream)."""
    s = torch.cuda.Stream(DEV)
    vals = torch.randn(40000, 42, dtype=torch.float64, device=DEV) * 3
    ref = vals.cpu().numpy().copy()
    ph = PendingHost(vals * 1.0, s)           # a temporary: its memory is released right away
    junk = torch.empty_like(vals).fill_(7.0)  # may be placed in that memory on the compute stream
    got = ph.get()
    torch.cuda.synchronize()
    assert ph.shape == (40000, 42) and np.array_equal(got, ref)
    assert float(junk[0, 0]) == 7.0


def test_gpu_two_process_federation_gloo_data_plane(tmp_path):
    """Two client processes driving HIP engines on the one GPU of the box (RCCL needs a GPU per rank,
    so the data plane is gloo here): weighted all-reduce of device buffers, sharded generation
    gathered to rank 0, uneven shares."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    cmd = [sys.executable, "-m", "dtds.distributed", "-world_size", "2", "-colocated", "-data_backend", "gloo",
           "-backend", "hip", "-epochs", "2", "-synthetic_rows", "4000", "-n_sample", "3001", "-out_dir", str(tmp_path),
           "-quiet"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    _check_outputs(tmp_path, 2, 3001)


def _run(cmd, env=None, timeout=180):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable] + cmd, cwd=root, env=env or dict(os.environ), capture_output=True,
                          text=True, timeout=timeout)


def test_rccl_branches_one_rank():
    """The nccl branches of Comm (weighted all-reduce, gather_rows, batched P2P exchange) on a one-rank
    RCCL communicator; the RCCL debug log must show the AllReduce being enqueued."""
    import json
    env = dict(os.environ, NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="COLL")
    r = _run(["tools/rccl_selftest.py"], env=env, timeout=150)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["ok"] and res["data_backend"] == "nccl" and res["data_ranks"] == 1, res
    assert res["hier_allreduce_ok"] and res["hier_gather_ok"], res      # HierComm (K=2 threads) over RCCL
    assert "AllReduce" in (r.stdout + r.stderr)


def test_bench_one_gpu_rccl_data_plane():
    """bench.py on one GPU with a real one-rank RCCL data plane (--force-dist): the round's
    aggregation is an RCCL all-reduce; every rank (one) agrees on the aggregate, full CSV written."""
    import json
    r = _run(["bench.py", "--steps", "1", "--warmup", "1", "--rows", "4000", "--n-sample", "3000", "--quiet",
              "--no-eval", "--check", "--force-dist"], timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["config"]["data_plane"] == "nccl" and rec["n_gpus"] == 1
    assert rec["consistency"]["flat_identical"] and rec["consistency"]["csv_rows"] == 3000
    assert "allreduce" in rec["phase_s"]
    # the self-verification record of the driver's multi-GPU line
    assert rec["comm"]["data_world_size"] == 1 and rec["comm"]["data_backend"] == "nccl"
    assert rec["comm"]["rccl_version"] and rec["comm"]["transport"]["files"] >= 1


def test_saved_generator_on_gpu(tmp_path):
    """models/{name}_generator.pt from a HIP run reloads into a fresh HIP engine (weights-only load)
    holding exactly the run's final weights, and generates / writes a full-width table."""
    from fed_tgan_amd.models.generator_io import load_generator
    from fed_tgan_amd.ops import native
    native.require()
    rt = FedRuntime(_cfg(tmp_path, epochs=1), Comm(0, 1, [0], "gloo", device=DEV), DEV)
    rt.initialize()
    rt.fit()
    gen = load_generator(str(tmp_path / "models" / "Intrusion_generator.pt"), DEV, backend="hip", seed=5)
    assert gen.engine.ops.name == "hip" and torch.equal(gen.engine.flat, rt.engine.flat)
    a = gen.sample(3000)
    assert a.shape == (3000, 42) and np.isfinite(a).all()
    gen.write_csv(str(tmp_path / "g.csv"), 2500)
    assert pd.read_csv(tmp_path / "g.csv").shape == (2500, 42)


def test_hier_one_rank_rccl_two_clients(tmp_path):
    """Two clients as threads over a one-rank RCCL process group (HierComm): the thread-level sum
    on the GPU, then the process-level RCCL all-reduce and gather."""
    from fed_tgan_amd.cli import free_port
    from fed_tgan_amd.ops import native
    native.require()
    comm = Comm(0, 1, [0], "nccl", port=free_port(), device=DEV, force_dist=True)
    try:
        rt = run_local_emulation(_cfg(tmp_path, shard_mode="iid"), 2, backend="hip", device=DEV, outer=comm)
        rt.flush_writes()
        assert comm.data_world_size() == 1 and rt.comm.data_world_size() == 2
    finally:
        comm.destroy()
    _check_outputs(tmp_path, 2, 3000)
    assert len(rt.weights) == 2 and bool(torch.isfinite(rt.engine.flat).all())


def test_hier_two_processes_two_clients_each(tmp_path):
    """-world_size 2 -local_clients 2: four HIP clients, two per process, on the box's one GPU (gloo
    data plane between the processes, as RCCL needs a GPU per rank)."""
    r = _run(["-m", "dtds.distributed", "-world_size", "2", "-local_clients", "2", "-data_backend", "gloo", "-backend",
              "hip", "-epochs", "2", "-synthetic_rows", "4000", "-n_sample", "3001", "-out_dir", str(tmp_path),
              "-dump_real", "-quiet"], timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    _check_outputs(tmp_path, 2, 3001)
    assert len(list((tmp_path / "data" / "raw").glob("Intrusion_train_client*.csv"))) == 4


def test_gpu_emulated_clients_batched(tmp_path):
    """Three emulated clients with equal row counts run as ONE batched engine (models/batched.py): client 0's
    thread issues every client's steps, the FedAvg reduces over the arena, every client ends each round
    holding the same aggregate, and the federator writes every epoch table."""
    from fed_tgan_amd.ops import native
    native.require()
    rt = run_local_emulation(_cfg(tmp_path, epochs=3, batched_clients="on"), 3, backend="hip", device=DEV)
    assert rt.batched and rt.engine.batch is not None
    b = rt.batch_clients
    torch.cuda.synchronize()
    flats = [e.flat for e in b.engines]
    assert all(torch.equal(f, flats[0]) for f in flats[1:])
    assert bool(torch.isfinite(flats[0]).all())
    assert all(e.bn_batches == b.engines[0].bn_batches for e in b.engines)
    _check_outputs(tmp_path, 3, 3000)


def test_gpu_emulated_clients_batched_off_and_unequal_rows(tmp_path):
    """batched_clients='off' keeps the per-thread engines; clients with different row counts (Dirichlet
    shards) batch, each training its own steps per epoch (slabs in non-increasing order of steps)."""
    from fed_tgan_amd.ops import native
    native.require()
    rt = run_local_emulation(_cfg(tmp_path, epochs=1, batched_clients="off"), 2, backend="hip", device=DEV)
    assert not rt.batched and rt.engine.batch is None
    rt = run_local_emulation(_cfg(tmp_path / "u", epochs=2, shard_mode="dirichlet", batched_clients="on"), 3,
                             backend="hip", device=DEV)
    assert len(set(rt.rows)) > 1 and rt.batched
    b = rt.batch_clients
    steps = [n // 500 for n in rt.rows]
    assert b.steps() == sorted(steps, reverse=True) and [steps[c] for c in b.client_of_slab] == b.steps()
    torch.cuda.synchronize()
    for s, e in enumerate(b.engines):
        assert float(e.stepD) == 2 * b.steps()[s]       # each client trained its own epoch length, twice
        assert torch.equal(e.flat, b.engines[0].flat)   # and holds the aggregate
    _check_outputs(tmp_path / "u", 2, 3000)


def _final_flats(tmp, n, **kw):
    rt = run_local_emulation(_cfg(tmp, **kw), n, backend="hip", device=DEV)
    torch.cuda.synchronize()
    return rt, rt.engine.flat.detach().clone()


def test_gpu_batched_matches_threads_broadcast_init(tmp_path):
    """The same federation with batched clients and with one engine per client thread (init='broadcast':
    every client starts from client 0's weights) ends the rounds with the same aggregate, to the
    reassociation noise of the other split-K plans and epilogue fusions (the clients' streams
    are ordered before the batched steps)."""
    from fed_tgan_amd.ops import native
    native.require()
    # (IID shards: equal rows keep every client in its own slab, so both paths give it the same seed)
    kw = dict(epochs=2, synthetic_rows=2000, init="broadcast", shard_mode="iid", seed=3,
              engine=EngineConfig(batch_size=500, precision="fp32"))
    rb, fb = _final_flats(tmp_path / "b", 3, batched_clients="on", **kw)
    rt, ft = _final_flats(tmp_path / "t", 3, batched_clients="off", **kw)
    assert rb.batched and not rt.batched and rb.rows == rt.rows
    # a lost ordering race leaves garbage (rel ~ 1, seen with the unordered broadcast); reassociation noise leaves
    # each element within the +-lr per step that Adam's normalised steps allow (2 epochs x 4 steps)
    rel = ((fb - ft).norm() / ft.norm()).item()
    assert rel < 2e-2, rel
    n = rb.engine.group_range["D"][1]       # the parameters (the BN running statistics follow them)
    assert (fb[:n] - ft[:n]).abs().max().item() <= 2 * 8 * 2e-4 + 1e-5


def test_hier_one_rank_rccl_four_batched_clients(tmp_path):
    """-local_clients 4 over a one-rank RCCL process group (HierComm) batch like the in-process emulation:
    the arena's weighted sum, then the process-level RCCL all-reduce; the aggregate equals ThreadComm's."""
    from fed_tgan_amd.cli import free_port
    from fed_tgan_amd.ops import native
    native.require()
    kw = dict(epochs=2, shard_mode="dirichlet", batched_clients="on")
    comm = Comm(0, 1, [0], "nccl", port=free_port(), device=DEV, force_dist=True)
    try:
        rh = run_local_emulation(_cfg(tmp_path / "h", **kw), 4, backend="hip", device=DEV, outer=comm)
        rh.flush_writes()
        torch.cuda.synchronize()
        fh = rh.engine.flat.detach().clone()
        assert rh.batched and type(rh.comm).__name__ == "HierComm" and comm.data_backend == "nccl"
    finally:
        comm.destroy()
    rt, ft = _final_flats(tmp_path / "t", 4, **kw)
    assert rt.batched and rh.rows == rt.rows
    assert torch.equal(fh, ft)
    _check_outputs(tmp_path / "h", 2, 3000)


def test_dedicated_federator_rccl_among_clients(tmp_path):
    """The reference topology (`R/README.md:7-25`): rank 0 a dataless federator, rank 1 the client, on the
    box's one GPU.  The aggregation is RCCL among the client ranks (the federator sits outside the group)
    and the federator receives the aggregate over its pair group: both ranks end with the same weights."""
    r = _run(["tools/topology_probe.py", "--world-size", "2", "--epochs", "2", "--out", str(tmp_path)], timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    import json
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["data_backend"] == ["nccl", "nccl"] and res["data_world_size"][1] == 1
    assert res["flat_equal"] and res["epochs"] == 2
    _check_outputs(tmp_path, 2, 3000)


_ROUNDS_SCRIPT = r"""
import json, sys, torch
import pandas as pd
from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
from fed_tgan_amd.parallel.comm import Comm
out = sys.argv[1]
dev = torch.device("cuda:0")
cfg = FedConfig(spec=intrusion_spec(), epochs=4, synthetic_rows=40000, out_dir=out, backend="hip", gmm_backend="torch",
                verbose=False, metrics_log=out + "/m.jsonl")
rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=dev), dev)
rt.initialize()
rt.fit()
stamps = pd.read_csv(out + "/timestamp_experiment.csv", header=None)[0].tolist()
print(json.dumps({"rounds": rt.round_times, "stamps": stamps, "metrics": [json.loads(l) for l in open(out + "/m.jsonl")]}))
"""


def test_gpu_round_zero_costs_a_steady_round(tmp_path):
    """Nothing first-time happens inside the rounds (FedRuntime._prepare_round_zero: the step and generation
    graphs, the table writer, the pinned table buffers and the CSV formatter's first table are made at init):
    every round of a 4-round run -- round 0 and round 1 included, which used to pay 40-80 ms of captures, a
    second pinned allocation and the formatter's first table -- costs within 1.5x of the steady round
    (`Server/dtds/distributed.py:790-829` times every round alike).  In a fresh process: earlier tests of this
    session would have paid the one-time costs already."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    p = subprocess.run([sys.executable, "-c", _ROUNDS_SCRIPT, str(tmp_path)], capture_output=True, text=True,
                       timeout=110, env=env, cwd=root)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    r, stamps = res["rounds"], res["stamps"]
    steady = sorted(r[1:])[1]
    assert max(r) <= 1.5 * steady, (r, res["metrics"])
    # timestamp_experiment.csv: entry e ends when epoch e's table is on disk; the first one also holds the
    # write of table 0 that no earlier round overlaps
    assert len(stamps) == 4 and all(s > 0 for s in stamps)
    assert max(stamps[1:]) <= 1.5 * steady, (stamps, r, res["metrics"])
    # entry 0 = round 0 + table 0's write, which nothing overlaps: bounded by the steady round plus that write as the
    # writer measured it (round 1's csv_write_prev; ~5-7 ms against a ~15 ms round since the round-6 step speed-up)
    w0 = res["metrics"][1].get("csv_write_prev", 0.0)
    assert stamps[0] <= 1.5 * steady + w0, (stamps, r, res["metrics"])


def test_gpu_pipelined_sampling_matches_unpipelined(tmp_path):
    """FedConfig.pipeline_sample: round r's table generated on a side stream while round r + 1 trains
    (CTGANEngine.generate_decoded_split) writes the same epoch CSVs byte for byte, leaves the same trained model and
    the same RNG counter as the unsplit generation after the round's training -- also with the body / copy /
    writer hand-off deferred past the next round's training issue (FedConfig.defer_handoff)."""
    from fed_tgan_amd.ops import native
    native.require()
    res = []
    for pipe, defer in ((False, False), (True, False), (True, True)):
        out = tmp_path / f"p{int(pipe)}{int(defer)}"
        cfg = FedConfig(spec=intrusion_spec(), epochs=3, synthetic_rows=8000, out_dir=str(out), backend="hip",
                        gmm_backend="torch", verbose=False, pipeline_sample=pipe, defer_handoff=defer)
        rt = FedRuntime(cfg, Comm(0, 1, [0], "gloo", device=DEV), DEV)
        rt.initialize()
        assert rt._pipe == pipe
        rt.fit()
        torch.cuda.synchronize()
        csvs = [(out / f"{rt.name}_result" / f"{rt.name}_synthesis_epoch_{e}.csv").read_bytes() for e in range(3)]
        res.append((csvs, rt.engine.flat.clone(), rt.engine.ops.ctr.clone()))
    c0, f0, k0 = res[0]
    for c1, f1, k1 in res[1:]:            # pipelined, and pipelined with the hand-off deferred past the next issue
        assert all(a == b for a, b in zip(c0, c1))
        assert torch.equal(f0, f1)
        assert torch.equal(k0, k1)


_TWO_RANK_SCRIPT = r"""
import json, os, sys, torch
from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
from fed_tgan_amd.parallel.comm import Comm
rank, port, out, pipe = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4] == "1"
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
comm = Comm(rank, 2, [0, 1], "auto", port=port, device=dev)
cfg = FedConfig(spec=intrusion_spec(), epochs=3, synthetic_rows=4000, out_dir=out, backend="hip", gmm_backend="torch",
                verbose=False, pipeline_sample=pipe)
rt = FedRuntime(cfg, comm, dev)
rt.initialize()
rt.fit()
torch.cuda.synchronize()
print(json.dumps({"rank": rank, "pipe": bool(getattr(rt, "_pipe", False)), "backend": comm.data_backend,
                  "flat": float(rt.engine.flat.double().sum())}), flush=True)
comm.destroy()
"""


def test_gpu_two_ranks_pipelined_sampling_gathers_the_same_tables(tmp_path):
    """Two rank processes on the one GPU (the data-plane vote picks gloo: one device) with pipelined sampling: each
    rank generates its share on its side stream and the shares are gathered to rank 0 -- the epoch CSVs equal the
    unpipelined run's byte for byte, and the two ranks agree on the aggregate."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    res = {}
    for pipe in ("0", "1"):
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        out = tmp_path / f"p{pipe}"
        procs = [subprocess.Popen([sys.executable, "-c", _TWO_RANK_SCRIPT, str(r), str(port), str(out), pipe],
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env, cwd=root)
                 for r in (0, 1)]
        outs = [p.communicate(timeout=150) for p in procs]
        for p, (o, e) in zip(procs, outs):
            assert p.returncode == 0, e[-3000:]
        recs = [json.loads(o.strip().splitlines()[-1]) for o, _ in outs]
        assert all(r["pipe"] == (pipe == "1") for r in recs) and recs[0]["backend"] == "gloo"
        assert recs[0]["flat"] == recs[1]["flat"]
        res[pipe] = [(out / "Intrusion_result" / f"Intrusion_synthesis_epoch_{e}.csv").read_bytes() for e in range(3)]
    assert res["0"] == res["1"]


_ONE_RANK_RCCL_SCRIPT = r"""
import json, sys, torch
from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime
from fed_tgan_amd.parallel.comm import Comm
port, out, pipe, native = int(sys.argv[1]), sys.argv[2], sys.argv[3] == "1", sys.argv[4] == "1"
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
comm = Comm(0, 1, [0], "auto", port=port, device=dev, force_dist=True, native_rccl=native)
cfg = FedConfig(spec=intrusion_spec(), epochs=3, synthetic_rows=4000, out_dir=out, backend="hip", gmm_backend="torch",
                verbose=False, pipeline_sample=pipe, force_gather=True)
rt = FedRuntime(cfg, comm, dev)
rt.initialize()
rt.fit()
torch.cuda.synchronize()
print(json.dumps({"pipe": bool(getattr(rt, "_pipe", False)), "backend": comm.data_backend,
                  "native": getattr(comm, "_native", None) is not None,
                  "flat": float(rt.engine.flat.double().sum())}), flush=True)
rt.close()
"""


def test_gpu_one_rank_rccl_pipelined_gather_matches_unpipelined(tmp_path):
    """on a one-rank RCCL data plane (force_dist) with FedConfig.force_gather, every round's
    table goes through Comm.gather_rows over the RCCL communicator -- on the generation side stream when sampling is
    pipelined.  The epoch CSVs equal the unpipelined run's byte for byte, and the native RCCL plane for the weight
    all-reduce gives the same model and tables as torch's."""
    import json
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root + os.pathsep + os.environ.get("PYTHONPATH", ""))
    res = {}
    for pipe, native in (("0", "0"), ("1", "0"), ("1", "1")):
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        out = tmp_path / f"p{pipe}n{native}"
        p = subprocess.run([sys.executable, "-c", _ONE_RANK_RCCL_SCRIPT, str(port), str(out), pipe, native],
                           capture_output=True, text=True, env=env, cwd=root, timeout=150)
        assert p.returncode == 0, p.stderr[-3000:]
        rec = json.loads(p.stdout.strip().splitlines()[-1])
        assert rec["backend"] == "nccl" and rec["pipe"] == (pipe == "1") and rec["native"] == (native == "1")
        res[(pipe, native)] = (rec["flat"], [(out / "Intrusion_result" / f"Intrusion_synthesis_epoch_{e}.csv").read_bytes()
                                             for e in range(3)])
    base = res[("0", "0")]
    for key, val in res.items():
        assert val[0] == base[0], key
        assert val[1] == base[1], key
