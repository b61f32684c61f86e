"""Per-kernel critical-path time of the captured training step from a rocprofv3 kernel trace.

rocprofv3's kernel start stamps include the wait for the previous kernel of the graph, so the
honest per-kernel cost is the increment it adds to the completion timeline:
inc_k = end_k - max(end_{k-1}, start_k).  Usage: step_breakdown.py run_results.db [--out=F]"""
import collections

import numpy as np
import sqlite3
import sys


def main(db, out=None):
    rows = sqlite3.connect(db).execute(
        "select start, end, name, grid_x, grid_y, grid_z, workgroup_x from kernels order by start").fetchall()
    n = len(rows)
    rows = rows[int(n * 0.35):int(n * 0.75)]      # steady-state graph replays
    inc = collections.defaultdict(list)
    prev = rows[0][1]
    for s, e, name, gx, gy, gz, wx in rows[1:]:
        key = name.split("(")[0].replace("void ", "").replace("fedtgan::", "")[:44] + f" grid=({gx // wx},{gy},{gz})"
        inc[key].append((e - max(prev, s)) / 1000.0)
        prev = max(prev, e)
    tot = sum(sum(v) for v in inc.values())
    lines = [f"critical-path total {tot:.1f} us over {sum(len(v) for v in inc.values())} kernels"]
    for k, v in sorted(inc.items(), key=lambda kv: -sum(kv[1])):
        lines.append(f"{100 * sum(v) / tot:5.1f}%  n={len(v):4d}  avg {sum(v) / len(v):6.2f} us  {k}")
    # one steady-state step in issue order (the last full window of kernels-per-step launches): where the
    # launches sit relative to each other, with each one's start gap after the previous end and its duration
    n_samp = sum(len(v) for k, v in inc.items() if k.startswith("sample_kernel") or k.startswith("sample_multi"))
    per = max(1, round(len(rows) / max(1, n_samp)))
    if "--order" in sys.argv and len(rows) > 2 * per:
        lines.append(f"one step in order (~{per} kernels): gap_us dur_us inc_us kernel")
        seq = rows[len(rows) // 2: len(rows) // 2 + per + 1]
        for (ps, pe, *_), (s, e, name, gx, gy, gz, wx) in zip(seq, seq[1:]):
            key = name.split("(")[0].replace("void ", "").replace("fedtgan::", "")[:44] + f" grid=({gx // wx},{gy},{gz})"
            lines.append(f"  {(s - pe) / 1000.0:6.2f} {(e - s) / 1000.0:6.2f} {(e - max(pe, s)) / 1000.0:6.2f}  {key}")
    if "--gaps" in sys.argv:
        # idle time between consecutive kernels (start_k - end_{k-1} > 0): where the device waits for the host /
        # the graph's packet submission; the critical-path totals above exclude it
        gaps = []
        pe = rows[0][1]
        for i, (s, e, name, *_rest) in enumerate(rows[1:], 1):
            if s > pe:
                gaps.append(((s - pe) / 1000.0, i, rows[i - 1][2].split("(")[0][-40:], name.split("(")[0][-40:]))
            pe = max(pe, e)
        big = [g for g in gaps if g[0] > 3.0]
        span = (rows[-1][1] - rows[0][0]) / 1000.0
        lines.append(f"gaps: {len(gaps)} idle intervals, {sum(g[0] for g in gaps):.1f} us idle of {span:.1f} us "
                     f"({len(big)} longer than 3 us, {sum(g[0] for g in big):.1f} us)")
        for g in big[:12]:
            lines.append(f"  gap {g[0]:7.2f} us before kernel #{g[1]}: {g[2]} -> {g[3]}")
        if len(big) > 1:
            idx = [g[1] for g in big]
            d = np.diff(idx)
            lines.append(f"  kernels between long gaps: min {d.min()} median {int(np.median(d))} max {d.max()}")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], out=next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--out=")), None))
