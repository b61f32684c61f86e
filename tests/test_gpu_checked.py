"""The device bounds-checked build (``csrc/build.py --checked`` -> ``_C_checked.so``,
``FEDTGAN_CHECKED=1``): a clean training + generation run raises nothing; a corrupted CSR row-count
table makes the sampler's pick leave the row lists, which the check reports (the access itself is
clamped, so the kernel never faults).  Each case runs in its own process (one native library per
process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, torch
sys.path[:0] = [{root!r}, {tests!r}]
from fed_tgan_amd.ops import native
from fed_tgan_amd.models.engine import CTGANEngine, EngineConfig
from fed_tgan_amd.models.samplers import CondTables
from helpers import small_table
L = native.require()
assert native.CHECKED and L.is_checked(), "checked library not loaded"
_, _, _, _, _, _, tr, X = small_table()
eng = CTGANEngine(tr.layout, EngineConfig(batch_size=500), torch.device("cuda:0"), backend="hip", seed=3)
eng.set_training_data(X)
eng.set_generation_tables(CondTables.from_encoded(X, tr.layout), tr)
eng.train_steps(3, use_graph=True)
eng.generate_decoded(2000)
if {corrupt}:
    eng.tables["row_count"].mul_(1000)
    try:
        eng.train_steps(1, use_graph=False)
    except RuntimeError as e:
        print("CHECK:", e)
        sys.exit(0)
    sys.exit(3)
print("CLEAN")
"""


def _run(corrupt: bool):
    env = dict(os.environ, FEDTGAN_CHECKED="1")
    code = SCRIPT.format(root=ROOT, tests=os.path.join(ROOT, "tests"), corrupt=corrupt)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=150, cwd=ROOT)


def test_checked_build_clean_run():
    r = _run(False)
    assert r.returncode == 0 and "CLEAN" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_checked_build_flags_bad_csr_table():
    r = _run(True)
    assert r.returncode == 0 and "sampler CSR pick outside the row lists" in r.stdout, (r.stdout[-2000:],
                                                                                       r.stderr[-3000:])
