"""Build ``fed_tgan_amd/_C.so``: HIP kernels (hipcc, gfx950) + host C++ + torch bindings.

No torch cpp_extension / hipify step: sources are written for CDNA4 directly and compiled
with explicit hipcc lines.  Objects are cached under ``build/`` and only rebuilt when a
source or header is newer than its object.  The library links against the HIP runtime that
ships inside the torch wheel (same soname as /opt/rocm's), so one HIP runtime is loaded per
process.

    python csrc/build.py [--force] [-j N] [--debug] [--checked]

``--checked`` builds ``fed_tgan_amd/_C_checked.so`` (objects under ``build/native_checked``):
the same kernels with -DFEDTGAN_CHECKED=1, which verify every table-derived index on the device
(see ``kernels/common.h`` FT_CHECK).  ``FEDTGAN_CHECKED=1`` at run time loads it instead of _C.so.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
BUILD = os.path.join(ROOT, "build", "native")
OUT = os.path.join(ROOT, "fed_tgan_amd", "_C.so")
ARCH = os.environ.get("FEDTGAN_ARCH", "gfx950")


def rocm() -> str:
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc() -> str:
    p = os.path.join(rocm(), "bin", "hipcc")
    return p if os.path.exists(p) else shutil.which("hipcc") or "hipcc"


def torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(tdir, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def newer(src_list, obj) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(s) > t for s in src_list)


def run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise SystemExit(f"build failed: {cmd[-1] if cmd else ''}")
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--save-temps", action="store_true")
    ap.add_argument("--checked", action="store_true", help="device bounds-checked build -> _C_checked.so")
    args = ap.parse_args()
    build_dir = BUILD + ("_checked" if args.checked else "")
    out = OUT.replace("_C.so", "_C_checked.so") if args.checked else OUT
    os.makedirs(build_dir, exist_ok=True)
    inc, tlib, abi = torch_paths()
    headers = glob.glob(os.path.join(HERE, "**", "*.h"), recursive=True)
    opt = ["-O0", "-g"] if args.debug else ["-O3"]
    common = ["-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I" + HERE] + opt
    if args.checked:
        common.append("-DFEDTGAN_CHECKED=1")
    jobs = []
    for src in sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip"))):
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        cmd = [hipcc(), "-c", src, "-o", obj, f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + common
        if args.save_temps:
            cmd += ["-save-temps=obj"]
        jobs.append((src, obj, cmd))
    for src in sorted(glob.glob(os.path.join(HERE, "host", "*.cpp"))):
        obj = os.path.join(build_dir, os.path.basename(src) + ".o")
        jobs.append((src, obj, ["g++", "-c", src, "-o", obj, "-pthread"] + common))
    for src in sorted(glob.glob(os.path.join(HERE, "comm", "*.cpp"))):   # native RCCL plane (host code, HIP headers)
        obj = os.path.join(build_dir, "comm_" + os.path.basename(src) + ".o")
        jobs.append((src, obj, [hipcc(), "-c", src, "-o", obj, "-x", "c++", "-D__HIP_PLATFORM_AMD__=1",
                                "-I" + os.path.join(rocm(), "include")] + common))
    bsrc = os.path.join(HERE, "bindings.cpp")
    bobj = os.path.join(build_dir, "bindings.cpp.o")
    jobs.append((bsrc, bobj, [hipcc(), "-c", bsrc, "-o", bobj, "-x", "c++", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                              "-I" + os.path.join(rocm(), "include")] + ["-I" + p for p in inc] + common))
    todo = [(s, o, c) for s, o, c in jobs if args.force or newer([s] + headers, o)]
    with cf.ThreadPoolExecutor(max_workers=max(1, args.j)) as ex:
        list(ex.map(lambda j: run(j[2]), todo))
    objs = [o for _, o, _ in jobs]
    if args.force or todo or newer(objs, out):
        # linked beside the library and renamed over it: a reader (an import, a gpurun snapshot) never sees a
        # half-written file
        tmp = out + ".tmp"
        run([hipcc(), "-shared", "-o", tmp] + objs + [f"--offload-arch={ARCH}", "-L" + tlib, "-lc10", "-lc10_hip",
                                                       "-ltorch", "-ltorch_cpu", "-l:libamdhip64.so", "-ldl", "-pthread",
                                                       "-Wl,-rpath," + tlib])
        os.replace(tmp, out)
    print(f"built {out} ({len(todo)} objects recompiled)")


if __name__ == "__main__":
    main()
