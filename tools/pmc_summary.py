"""Per-kernel hardware-counter summary of rocprofv3 --pmc runs (one directory per pass).

Reads every *counter_collection.csv under the given directories and reports, per kernel (name +
grid), the dispatch count and the MEAN counter value per dispatch. Then derived ratios:
  * MFMA busy   = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES
  * wave stall  = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (parked on s_waitcnt / barriers)
  * issue stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  * LDS conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  * HBM-side bytes per dispatch = FETCH_SIZE / WRITE_SIZE (KB)

    python tools/pmc_summary.py gpurun_out/pmc_a gpurun_out/pmc_b gpurun_out/pmc_c [--out=F] [--top=N]
"""
import collections
import csv
import glob
import os
import sys


def load(dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> values
    disp = collections.defaultdict(set)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    name = row.get("Kernel_Name", "?").split("(")[0].replace("void ", "").replace("fedtgan::", "")
                    key = f"{name[:60]} grid={row.get('Grid_Size', '?')}"
                    per[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    disp[key].add((path, row.get("Dispatch_Id", row.get("Correlation_Id"))))
    return per, disp


def main(argv):
    dirs = [a for a in argv if not a.startswith("--")]
    out = next((a.split("=", 1)[1] for a in argv if a.startswith("--out=")), None)
    top = int(next((a.split("=", 1)[1] for a in argv if a.startswith("--top=")), "40"))
    per, disp = load(dirs)

    def mean(k, c):
        v = per[k].get(c)
        return sum(v) / len(v) if v else None

    rows = []
    for k in per:
        n = len(disp[k])
        busy, mfma = mean(k, "SQ_BUSY_CYCLES"), mean(k, "SQ_VALU_MFMA_BUSY_CYCLES")
        wc, wa, wi = mean(k, "SQ_WAVE_CYCLES"), mean(k, "SQ_WAIT_ANY"), mean(k, "SQ_WAIT_INST_ANY")
        lc, la = mean(k, "SQ_LDS_BANK_CONFLICT"), mean(k, "SQ_LDS_IDX_ACTIVE")
        fs, ws = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
        pct = lambda a, b: f"{100 * a / b:5.1f}%" if (a is not None and b) else "   -  "  # noqa: E731
        kb = lambda x: f"{x:9.1f}" if x is not None else "      -  "  # noqa: E731
        rows.append((n, k, pct(mfma, busy), pct(wa, wc), pct(wi, wc), pct(lc, la), kb(fs), kb(ws)))
    rows.sort(key=lambda r: -r[0])
    lines = [f"{'disp':>5}  {'MFMA busy':>9} {'wait':>6} {'issue':>6} {'LDS cf':>6} {'fetch KB':>9} {'write KB':>9}  kernel"]
    for n, k, a, b, c, d, e, f in rows[:top]:
        lines.append(f"{n:5d}  {a:>9} {b:>6} {c:>6} {d:>6} {e} {f}  {k}")
    # then every counter's mean per dispatch, kernel by kernel
    lines.append("")
    for k in sorted(per, key=lambda k: -len(disp[k]))[:top]:
        lines.append(k)
        for c, v in sorted(per[k].items()):
            lines.append(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
