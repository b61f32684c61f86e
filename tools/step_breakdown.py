"""Per-kernel critical-path time of the captured training step from a rocprofv3 kernel trace.

rocprofv3's kernel start stamps include the wait for the previous kernel of the graph, so the
honest per-kernel cost is the increment it adds to the completion timeline:
inc_k = end_k - max(end_{k-1}, start_k).  Usage: step_breakdown.py run_results.db [--out=F]"""
import collections
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
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main(sys.argv[1], out=next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--out=")), None))
