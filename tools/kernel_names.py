"""Distinct kernel names (full template arguments) and grids of a rocprofv3 kernel trace, with counts and mean
duration -- for telling apart instantiations that step_breakdown.py's short names merge.

    python tools/kernel_names.py run_results.db [substring]
"""
import sqlite3
import sys


def main(db, sub=""):
    rows = sqlite3.connect(db).execute("select name, grid_x, grid_y, grid_z, workgroup_x, end - start from kernels").fetchall()
    agg = {}
    for n, gx, gy, gz, wx, d in rows:
        if sub and sub not in n:
            continue
        k = (n.split("(")[0], f"({gx // wx},{gy},{gz})")
        c, t = agg.get(k, (0, 0.0))
        agg[k] = (c + 1, t + d)
    for (n, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"n={c:5d} avg {t / c / 1e3:8.2f} us grid={g} {n}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
