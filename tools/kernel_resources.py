"""Per-kernel register, scratch and LDS usage of a built HIP object (gfx950 code object metadata).

    python tools/kernel_resources.py [build/native/gemm.hip.o] [--match REGEX]

Unbundles the object's ``.hip_fatbin`` (clang-offload-bundler), reads the AMDGPU metadata notes (llvm-readelf
--notes) and prints, per kernel, VGPRs / AGPRs / SGPRs / scratch bytes per lane / static LDS bytes.  A kernel
whose scratch is non-zero spills or indexes a register array at run time (round 5: the BN-on-load GEMMs had 80 B of
scratch from runtime-indexed range arrays, the fix took their step cost from +39 to +11 us).
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def notes_of(obj: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin.bin"), os.path.join(d, "k.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                        f"--input={fat}", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                              text=True).stdout


def kernels(notes: str):
    """(demangled name, {field: int}) per kernel.  The metadata lists each kernel's fields alphabetically, from
    .agpr_count to .wavefront_size."""
    blocks = re.findall(r"(\.agpr_count:.*?\.wavefront_size:\s+\d+)", notes, re.S)
    names = [re.search(r"\.name:\s+(\S+)", b).group(1) for b in blocks]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    for b, n in zip(blocks, dem):
        f = {}
        for k in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size"):
            m = re.search(r"\.%s:\s+(\d+)" % k, b)
            f[k] = int(m.group(1)) if m else -1
        yield n, f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("obj", nargs="?", default=os.path.join(os.path.dirname(__file__), "..", "build", "native",
                                                          "gemm.hip.o"))
    ap.add_argument("--match", default=".")
    args = ap.parse_args()
    rows = [(n, f) for n, f in kernels(notes_of(args.obj)) if re.search(args.match, n)]
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'scratch':>8} {'lds':>7}  kernel")
    for n, f in rows:
        print(f"{f['vgpr_count']:5d} {f['agpr_count']:5d} {f['sgpr_count']:5d} {f['private_segment_fixed_size']:8d} "
              f"{f['group_segment_fixed_size']:7d}  {n[:160]}")
    return 0 if rows else 1


if __name__ == "__main__":
    sys.exit(main())
