"""Count the node's GPUs WITHOUT loading the HIP runtime.

Launchers (``python -m dtds.distributed`` without ``-rank``, ``bench.py --gpus N``) must decide how
many ranks share a GPU, and set per-process HIP variables such as ``GPU_MAX_HW_QUEUES`` for their
children, before any process touches HIP.  A parent that loads HIP itself stays resident on GPU 0
with its own queues for the whole run, so the count comes from the kernel driver's topology
(``/sys/class/kfd/kfd/topology/nodes/*/properties``: nodes with SIMDs are GPUs), restricted by
``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` when set.
"""
from __future__ import annotations

import glob
import os

_VIS_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _kfd_gpu_nodes(root: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    n = 0
    for p in glob.glob(os.path.join(root, "*", "properties")):
        try:
            with open(p) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count":
                        n += int(v) > 0
                        break
        except OSError:
            continue
    return n


def visible_gpu_count(root: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process would see, without initialising HIP: the driver's GPU nodes, capped by the
    length of every *_VISIBLE_DEVICES list that is set (an empty list hides every GPU)."""
    total = _kfd_gpu_nodes(root)
    for var in _VIS_VARS:
        v = os.environ.get(var)
        if v is None:
            continue
        total = min(total, len([x for x in v.split(",") if x.strip()]))
    return total
