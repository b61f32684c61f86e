"""Federation on the CPU: gloo multi-process runs, in-process emulation, aggregation math, fault
injection, checkpoint/resume, and the reference-compatible CLI + evaluator outputs."""
import os
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest
import torch

from fed_tgan_amd.data.schema import intrusion_spec
from fed_tgan_amd.fed.local import run_local_emulation
from fed_tgan_amd.fed.runtime import FedConfig, FedRuntime, effective_weights, round_alive_mask
from fed_tgan_amd.models.engine import EngineConfig
from fed_tgan_amd.parallel.comm import Comm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cfg(tmp, **kw):
    base = dict(spec=intrusion_spec(), epochs=2, synthetic_rows=1000, n_sample=600, out_dir=str(tmp), backend="torch",
                gmm_backend="torch", engine=EngineConfig(batch_size=100), verbose=False)
    base.update(kw)
    return FedConfig(**base)


def test_local_emulation_two_clients(tmp_path):
    rt = run_local_emulation(_cfg(tmp_path, dump_real=True), 2, backend="torch", device=torch.device("cpu"))
    res = tmp_path / "Intrusion_result"
    assert sorted(os.listdir(res)) == ["Intrusion_synthesis_epoch_0.csv", "Intrusion_synthesis_epoch_1.csv"]
    df = pd.read_csv(res / "Intrusion_synthesis_epoch_1.csv")
    assert df.shape == (600, 42) and list(df.columns) == intrusion_spec().selected_variables
    ts = pd.read_csv(tmp_path / "timestamp_experiment.csv", header=None)
    assert ts.shape == (2, 1)
    assert (tmp_path / "models" / "Intrusion.json").exists()
    assert (tmp_path / "models" / "label_encoders_Intrusion.pickle").exists()
    assert (tmp_path / "data" / "raw" / "Intrusion_train.csv").exists()
    assert np.isclose(rt.weights.sum(), 1.0) and len(rt.weights) == 2


def test_label_encoders_written_during_init(tmp_path):
    """The pickle exists once initialisation is over (the reference writes it there,
    `Server/dtds/distributed.py:679-684`): a run killed mid-training still leaves it."""
    import pickle
    from fed_tgan_amd.fed.local import LocalGroup, ThreadComm
    from fed_tgan_amd.fed.runtime import FedRuntime
    rt = FedRuntime(_cfg(tmp_path), ThreadComm(LocalGroup(1), 0, torch.device("cpu")), torch.device("cpu"))
    rt.initialize()
    rt._le_proc.wait(timeout=120)
    path = tmp_path / "models" / "label_encoders_Intrusion.pickle"
    with open(path, "rb") as f:       # our own file
        les = pickle.load(f)
    assert [d["column_name"] for d in les] == [v.column_name for v in rt.vocabs]
    assert all(d["label_encoder"].classes_.tolist() == v.tolist() for d, v in zip(les, rt.vocabs))
    assert rt.write_label_encoders() == str(path)


def test_weighted_aggregation_is_weighted_average(tmp_path):
    """Every client ends the round holding sum_i w_i * theta_i of ALL flat entries (incl. BN stats)."""
    from fed_tgan_amd.fed.local import LocalGroup, ThreadComm
    import threading
    k = 3
    g = LocalGroup(k)
    bufs = [torch.randn(1000) for _ in range(k)]
    orig = [b.clone() for b in bufs]
    w = [0.2, 0.5, 0.3]

    def run(r):
        ThreadComm(g, r, torch.device("cpu")).weighted_all_reduce(bufs[r], w[r])

    ts = [threading.Thread(target=run, args=(r,)) for r in range(k)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    ref = sum(wi * o for wi, o in zip(w, orig))
    for b in bufs:
        assert torch.allclose(b, ref, atol=1e-6)


def test_fault_injection_masks():
    cfg = _cfg("/tmp", drop_client_prob=0.5, seed=3)
    for ep in range(20):
        alive = round_alive_mask(cfg, ep, 4)
        assert alive.any()
        w = effective_weights(np.array([0.1, 0.2, 0.3, 0.4]), alive)
        assert np.isclose(w.sum(), 1.0) and np.all(w[~alive] == 0)
    assert round_alive_mask(_cfg("/tmp"), 0, 4).all()


def test_local_emulation_with_dropped_clients(tmp_path):
    rt = run_local_emulation(_cfg(tmp_path, drop_client_prob=0.5, epochs=3), 3, backend="torch",
                             device=torch.device("cpu"))
    assert len(rt.round_times) == 3


def test_checkpoint_resume(tmp_path):
    cfg = _cfg(tmp_path, epochs=2, ckpt_every=1)
    rt = run_local_emulation(cfg, 1, backend="torch", device=torch.device("cpu"))
    flat = rt.engine.flat.clone()
    cfg2 = _cfg(tmp_path, epochs=3, resume=True)
    comm = Comm(0, 1, [0], "gloo", device=torch.device("cpu"))
    rt2 = FedRuntime(cfg2, comm, torch.device("cpu"))
    rt2.initialize()
    assert rt2.start_epoch == 2
    assert torch.equal(rt2.engine.flat, flat)
    rt2.fit()
    assert len(rt2.round_times) == 3


@pytest.mark.parametrize("saved_wt", [False, True])
def test_checkpoint_resume_across_generator_layouts(tmp_path, saved_wt):
    """a checkpoint written with the other EngineConfig.g_wt (e.g. before input-major generator
    weights became the default: no 'g_wt' key) resumes into the same logical weights and Adam moments."""
    import dataclasses
    eng_a = EngineConfig(batch_size=100, g_wt=saved_wt)
    cfg = _cfg(tmp_path, epochs=2, ckpt_every=1, engine=eng_a)
    rt = run_local_emulation(cfg, 1, backend="torch", device=torch.device("cpu"))
    if not saved_wt:     # the pre-g_wt checkpoint format had no layout key
        path = rt._ckpt_path()
        st = torch.load(path, weights_only=True)
        st.pop("g_wt", None)
        torch.save(st, path)
    eng_b = dataclasses.replace(eng_a, g_wt=not saved_wt)
    rt2 = FedRuntime(_cfg(tmp_path, epochs=3, resume=True, engine=eng_b), Comm(0, 1, [0], "gloo",
                     device=torch.device("cpu")), torch.device("cpu"))
    rt2.initialize()
    assert rt2.start_epoch == 2
    a, b = rt.engine, rt2.engine
    for name in a.p:
        assert torch.equal(a.p[name], b.p[name]), name
    for name in a.g:        # Adam moments through the gradient-shaped views
        for buf in ("m", "v"):
            grp = "G" if name.startswith("G.") else "D"
            va = a._view_in(getattr(a, buf + grp), name)
            vb = b._view_in(getattr(b, buf + grp), name)
            assert torch.equal(va, vb), (buf, name)
    rt2.fit()
    assert len(rt2.round_times) == 3


def _run_cli(args, cwd, timeout=420):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    return subprocess.run([sys.executable, "-m", "dtds.distributed"] + args, cwd=cwd, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.slow
def test_cli_reference_topology_gloo(tmp_path):
    """world_size=3: a dataless federator + 2 clients as three gloo processes (README demo topology)."""
    r = _run_cli(["-world_size", "3", "-epochs", "2", "-backend", "torch", "-synthetic_rows", "1000", "-n_sample",
                  "500", "-batch_size", "100", "-out_dir", str(tmp_path), "-dump_real", "-quiet"], cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert (tmp_path / "Intrusion_result" / "Intrusion_synthesis_epoch_1.csv").exists()
    ts = pd.read_csv(tmp_path / "timestamp_experiment.csv", header=None)
    assert len(ts) == 2
    # evaluator CLIs on the produced outputs
    env = dict(os.environ, PYTHONPATH=ROOT)
    s = subprocess.run([sys.executable, os.path.join(ROOT, "similarity_analysis.py"), "-nepoch", "2"], cwd=tmp_path,
                       env=env, capture_output=True, text=True, timeout=300)
    assert s.returncode == 0, s.stderr[-2000:]
    sim = pd.read_csv(tmp_path / "Intrusion_statistical_similarity_analysis.csv")
    assert list(sim.columns) == ["Epoch_No.", "Avg_JSD", "Avg_WD", "time_stamp"]
    assert sim["Avg_JSD"].between(0, 1).all() and np.isfinite(sim["Avg_WD"]).all()


def test_local_epochs_between_aggregations(tmp_path):
    """-E_interval 2: clients train two local epochs between weighted aggregations."""
    rt = run_local_emulation(_cfg(tmp_path, epochs=3, e_interval=2), 2, backend="torch", device=torch.device("cpu"))
    assert len(rt.round_times) == 3


def test_cli_colocated_two_ranks(tmp_path):
    """-colocated (the MI355X layout, every rank a client): weighted all-reduce + sharded sampling
    gathered to rank 0, here over gloo with two processes; uneven shares (501 rows)."""
    r = _run_cli(["-world_size", "2", "-colocated", "-epochs", "2", "-backend", "torch", "-synthetic_rows", "1000",
                  "-n_sample", "501", "-batch_size", "100", "-out_dir", str(tmp_path), "-quiet"], cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    df = pd.read_csv(tmp_path / "Intrusion_result" / "Intrusion_synthesis_epoch_1.csv")
    assert df.shape == (501, 42)


def test_profiled_round_exports_trace(tmp_path):
    cfg = _cfg(tmp_path, epochs=2, profile_dir=str(tmp_path / "prof"))
    run_local_emulation(cfg, 1, backend="torch", device=torch.device("cpu"))
    assert (tmp_path / "prof" / "trace_rank0_epoch1.json").stat().st_size > 0


@pytest.mark.slow
def test_heartbeat_names_a_dead_rank(tmp_path):
    """Failure detection: rank 1 (its own process, reference-style explicit -rank launch) dies
    after its first round; with -heartbeat, rank 0 fails fast with a monitored-barrier error
    naming rank 1 instead of waiting out the process-group timeout."""
    import socket
    import time
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = str(so.getsockname()[1])
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", FEDTGAN_FAULT_EXIT="1:0")
    args = ["-world_size", "2", "-colocated", "-epochs", "3", "-backend", "torch", "-synthetic_rows", "1000",
            "-n_sample", "200", "-batch_size", "100", "-heartbeat", "5", "-out_dir", str(tmp_path), "-quiet",
            "-ip", "127.0.0.1", "-port", port]
    procs = [subprocess.Popen([sys.executable, "-m", "dtds.distributed", "-rank", str(r)] + args, cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (0, 1)]
    t0 = time.time()
    out0, err0 = procs[0].communicate(timeout=300)
    procs[1].communicate(timeout=60)
    assert procs[1].returncode == 3
    assert procs[0].returncode != 0
    assert "monitoredBarrier" in err0 and "1" in err0, err0[-2000:]
    assert time.time() - t0 < 240


def test_real_csv_datapath_per_client(tmp_path):
    """-datapath with '{client}' reads each client's own CSV (the reference's real-data path), with
    blanks in a categorical column; the clients' row counts drive steps and weights."""
    from fed_tgan_amd.data.synthetic import generate
    spec = intrusion_spec()
    for i, n in enumerate((1200, 700)):
        df = generate(spec, n, seed=40 + i)
        df.loc[df.index[:5], "protocol_type"] = np.nan          # blanks -> "empty" category
        df.to_csv(tmp_path / f"intr_client{i}.csv", index=False)
    cfg = _cfg(tmp_path, datapath=str(tmp_path / "intr_client{client}.csv"), synthetic_rows=999999)
    rt = run_local_emulation(cfg, 2, backend="torch", device=torch.device("cpu"))
    assert rt.rows == [1200, 700] and rt.steps == [12, 7]
    out = pd.read_csv(tmp_path / "Intrusion_result" / "Intrusion_synthesis_epoch_1.csv")
    assert out.shape == (600, 42)


def _init_two_clients(tmp, init):
    """Initialise a 2-client in-process federation (threads) and return both runtimes."""
    import threading
    from fed_tgan_amd.fed.local import LocalGroup, ThreadComm
    g = LocalGroup(2)
    rts = [None, None]

    def run(r):
        rt = FedRuntime(_cfg(tmp, init=init, shard_mode="iid"), ThreadComm(g, r, torch.device("cpu")),
                        torch.device("cpu"))
        rt.initialize()
        rts[r] = rt

    ts = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    return rts


def test_initial_weights_independent_by_default(tmp_path):
    """Reference: every client builds its own randomly initialised G/D (`Client/.../distributed.py:156-165`);
    -init broadcast gives every client the first client's weights."""
    a, b = _init_two_clients(tmp_path / "ind", "independent")
    assert not torch.equal(a.engine.flat, b.engine.flat)
    a, b = _init_two_clients(tmp_path / "bc", "broadcast")
    assert torch.equal(a.engine.flat, b.engine.flat)


def test_timestamps_include_the_background_csv(tmp_path, monkeypatch):
    """timestamp_experiment.csv: with the background writer each entry still ends when its epoch's CSV
    is on disk, so the cumulative sum is the wall time at which each table exists (the reference's
    `time_stamp`, `Server/similarity_analysis.py:111-115`)."""
    import time as _t
    slow = FedRuntime._write_epoch_csv_body

    def delayed(self, values, epoch):
        _t.sleep(0.4)
        return slow(self, values, epoch)

    monkeypatch.setattr(FedRuntime, "_write_epoch_csv_body", delayed)
    rt = FedRuntime(_cfg(tmp_path, epochs=3, async_csv=True), Comm(0, 1, [0], "gloo", device=torch.device("cpu")),
                    torch.device("cpu"))
    rt.initialize()
    t0 = _t.time()
    rt.fit()
    ts = pd.read_csv(tmp_path / "timestamp_experiment.csv", header=None).iloc[:, 0].to_numpy()
    assert len(ts) == 3
    # the three writes are serial: the stamps cover at least 3 x 0.4 s of CSV writing
    assert ts.sum() >= 1.2 and (ts >= 0).all()
    assert abs(ts.sum() - (rt._csv_done[2] - rt._round_start[0])) < 1e-6
    assert ts.sum() <= _t.time() - t0 + 1e-3
    for e in range(3):
        assert abs(np.cumsum(ts)[e] - (rt._csv_done[e] - rt._round_start[0])) < 1e-6


def test_saved_generator_samples_standalone(tmp_path):
    """The federator's models/{name}_generator.pt reloads with weights_only=True into a fresh engine
    that reproduces the run's generator and writes a reference-format CSV (python -m dtds.sample)."""
    from fed_tgan_amd.models.generator_io import load_generator
    rt = run_local_emulation(_cfg(tmp_path, epochs=1), 2, backend="torch", device=torch.device("cpu"))
    path = tmp_path / "models" / "Intrusion_generator.pt"
    assert path.exists()
    gen = load_generator(str(path), torch.device("cpu"), backend="torch")
    assert torch.equal(gen.engine.flat, rt.engine.flat)
    r = subprocess.run([sys.executable, "-m", "dtds.sample", "-model", str(path), "-n", "700", "-out",
                        str(tmp_path / "s.csv"), "-backend", "torch"], cwd=ROOT,
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2"), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    df = pd.read_csv(tmp_path / "s.csv")
    ref = pd.read_csv(tmp_path / "Intrusion_result" / "Intrusion_synthesis_epoch_0.csv")
    assert df.shape == (700, 42) and list(df.columns) == list(ref.columns)
    vocab = {v.column_name: set(v.tolist()) for v in rt.vocabs}
    for c in intrusion_spec().categorical_list:          # decoded categories come from the same vocab
        assert set(df[c].astype(str)) <= vocab[c] | {" "}, c


def test_cli_round5_flags_reach_the_config():
    """-pipeline_sample / -table_reader land in FedConfig; -native_rccl is accepted (it only changes the RCCL plane)."""
    from fed_tgan_amd.cli import build_parser, fed_config_from_args
    a = build_parser().parse_args(["-pipeline_sample", "off", "-table_reader", "arrow", "-native_rccl"])
    cfg = fed_config_from_args(a)
    assert cfg.pipeline_sample is False and cfg.table_reader == "arrow" and a.native_rccl
    cfg = fed_config_from_args(build_parser().parse_args([]))
    assert cfg.pipeline_sample is None and cfg.table_reader == "auto"
