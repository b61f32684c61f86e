"""The bench.py driver contract: one JSON line from rank 0, single process and under
``torch.distributed.run`` with two gloo ranks (the launch the driver uses for N > 1)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{") and '"metric"' in l]


def _env():
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    env.pop("RANK", None); env.pop("WORLD_SIZE", None); env.pop("LOCAL_RANK", None)
    return env


def test_bench_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1",
                        "--rows", "1000", "--n-sample", "1500", "--quiet"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    rec = lines[0]
    assert KEYS <= set(rec)
    assert rec["metric"] == "sec_per_epoch" and rec["n_gpus"] == 1 and rec["higher_is_better"] is False
    assert rec["value"] > 0 and abs(rec["ms_per_step"] - 1000 * rec["value"]) < 1e-2


def test_bench_torchrun_two_ranks():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "1", "--rows", "1000", "--n-sample", "1500", "--quiet"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout          # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "fed2" and rec["scaling"] == "weak"
    assert rec["avg_jsd"] is not None and rec["avg_wd"] is not None


def test_bench_self_launch_four_ranks():
    """`bench.py --gpus 4` with no launcher: the script starts the 4 ranks itself (GPUs hidden -> gloo)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1", "--warmup",
                        "1", "--rows", "1000", "--n-sample", "1500", "--quiet", "--no-eval"],
                       capture_output=True, text=True, timeout=400, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    rec = lines[0]
    assert rec["n_gpus"] == 4 and rec["config"]["parallelism"] == "fed4"
    for k in ("train", "allreduce", "gather", "d2h", "generate"):
        assert k in rec["phase_s"], rec["phase_s"]


def test_bench_eight_ranks_identical_aggregate():
    """8 self-launched ranks: every rank holds a bit-identical aggregate after the last round and the
    epoch CSV (sharded generation, gathered on rank 0) has all 40,000 rows -- checked by DEFAULT for
    N > 1 (the driver's 8-GPU line must verify itself), with the data-plane record."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "1", "--warmup",
                        "1", "--rows", "1000", "--n-sample", "40000", "--quiet", "--no-eval"],
                       capture_output=True, text=True, timeout=600, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["n_gpus"] == 8
    assert rec["consistency"] == {"flat_identical": True, "ranks": 8, "csv_rows": 40000}
    assert rec["comm"]["data_world_size"] == 8 and rec["comm"]["data_backend"] == "gloo"
    assert "transport" in rec["comm"]


def test_bench_world_size_mismatch_fails():
    env = dict(_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--rows", "1000", "--quiet"], capture_output=True, text=True, timeout=120, env=env,
                       cwd="/tmp")
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_bench_engine_override_and_force_dist():
    """--engine KEY=VALUE reaches EngineConfig (reported back); --force-dist builds real process groups
    for one rank (gloo here; RCCL on a GPU box)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--rows",
                        "1000", "--n-sample", "600", "--quiet", "--no-eval", "--engine", "onehot=0", "--force-dist",
                        "--check"], capture_output=True, text=True, timeout=300, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_lines(r.stdout)[0]
    assert rec["engine_overrides"] == ["onehot=0"] and rec["config"]["data_plane"] == "gloo"
    assert rec["consistency"]["csv_rows"] == 600
