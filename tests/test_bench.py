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
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
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
