"""Host C++ under sanitizers (the GPU sanitizers are not available on this pool): the native CSV
writer built with AddressSanitizer + UndefinedBehaviorSanitizer, and with ThreadSanitizer for
its worker pool, formats a table of every column kind identically to its single-threaded path."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "csrc", "host")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_csv_writer_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "csvchk")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-pthread", "-I" + HOST,
           os.path.join(HOST, "tests", "csv_writer_check.cpp"), os.path.join(HOST, "csv_writer.cpp"), "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(tmp_path / "out.csv")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    assert r.stdout.startswith("ok")
