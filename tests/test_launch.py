"""Launcher helpers that must not touch HIP: GPU counting from the KFD topology, the device map of
the reference topology, and the shared-GPU queue cap."""
import os

import pytest

from fed_tgan_amd import cli
from fed_tgan_amd.utils import gpus


def _fake_kfd(tmp_path, simds):
    for i, s in enumerate(simds):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count {s}\nmem_banks_count 1\n")
    return str(tmp_path)


def test_visible_gpu_count_from_kfd_and_env(tmp_path, monkeypatch):
    root = _fake_kfd(tmp_path, [0, 1024, 1024, 1024])      # one CPU node, three GPUs
    for v in gpus._VIS_VARS:
        monkeypatch.delenv(v, raising=False)
    assert gpus.visible_gpu_count(root) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert gpus.visible_gpu_count(root) == 2
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    assert gpus.visible_gpu_count(root) == 0


def test_device_map_of_the_reference_topology():
    # dedicated federator (rank 0) on GPU 0 with client 1; co-located: one rank per GPU
    assert [cli.device_index(r, 8, False) for r in range(9)] == [0, 0, 1, 2, 3, 4, 5, 6, 7]
    assert [cli.device_index(r, 8, True) for r in range(8)] == list(range(8))
    assert [cli.device_index(r, 1, False) for r in range(3)] == [0, 0, 0]


@pytest.mark.parametrize("world,colocated,ngpu,shared", [(3, False, 1, True), (9, False, 8, True),
                                                         (8, True, 8, False), (2, True, 1, True),
                                                         (3, False, 0, False)])
def test_gpus_shared(monkeypatch, world, colocated, ngpu, shared):
    monkeypatch.setattr(gpus, "visible_gpu_count", lambda *a, **k: ngpu)
    assert cli.gpus_shared(world, colocated) is shared


def test_cap_shared_queues(monkeypatch):
    monkeypatch.delenv("FEDTGAN_SHARED_HW_QUEUES", raising=False)
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")          # the box default is lowered
    cli.cap_shared_queues()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "2"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "1")          # a lower choice is kept
    cli.cap_shared_queues()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "1"
    monkeypatch.delenv("GPU_MAX_HW_QUEUES")
    monkeypatch.setenv("FEDTGAN_SHARED_HW_QUEUES", "3")
    cli.cap_shared_queues()
    assert os.environ["GPU_MAX_HW_QUEUES"] == "3"
