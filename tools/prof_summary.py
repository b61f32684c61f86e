"""Summarise a rocprofv3 rocpd database: per-kernel (and per-shape) time table."""
import sqlite3
import sys


def main(db, top=30, by_shape=False, out=None):
    con = sqlite3.connect(db)
    cur = con.cursor()
    if by_shape:
        q = ("select name, grid_x/workgroup_x, grid_y, grid_z, count(*), sum(end-start)/1000.0, avg(end-start)/1000.0, "
             "vgpr_count, lds_size from kernels group by name, grid_x, grid_y, grid_z order by sum(end-start) desc")
    else:
        q = ("select name, count(*), sum(end-start)/1000.0, avg(end-start)/1000.0 from kernels group by name "
             "order by sum(end-start) desc")
    rows = cur.execute(q).fetchall()
    total = sum(r[5] if by_shape else r[2] for r in rows)
    lines = [f"total kernel time {total:.1f} us over {sum(r[4] if by_shape else r[1] for r in rows)} dispatches"]
    for r in rows[:top]:
        if by_shape:
            lines.append(f"{r[4]:6d} {r[5]:10.1f}us avg {r[6]:7.2f}us wg=({r[1]},{r[2]},{r[3]}) vgpr={r[7]} lds={r[8]} "
                         f"{r[0][:70]}")
        else:
            lines.append(f"{r[1]:6d} {r[2]:10.1f}us avg {r[3]:7.2f}us {100 * r[2] / total:5.1f}%  {r[0][:90]}")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


def timeline(db, period=None, out=None):
    """Busy vs idle time of the device in the steady-state part of the trace: consecutive
    kernels are merged into busy intervals; reports the kernel-time sum, the wall span and the
    average idle gap between dependent launches (the graph's per-kernel dispatch cost)."""
    con = sqlite3.connect(db)
    rows = con.execute("select start, end, name from kernels order by start").fetchall()
    if not rows:
        return
    # steady state: the last 60 % of the trace (warm-up and capture excluded)
    rows = rows[int(len(rows) * 0.4):]
    busy = sum(e - s for s, e, _ in rows) / 1000.0
    span = (rows[-1][1] - rows[0][0]) / 1000.0
    gaps = [(b[0] - a[1]) / 1000.0 for a, b in zip(rows, rows[1:])]
    pos = [g for g in gaps if g > 0]
    lines = [f"kernels {len(rows)}  kernel time {busy:.1f} us  wall span {span:.1f} us  "
             f"device busy {100 * busy / span:.1f} %",
             f"gaps between consecutive kernels: mean {sum(gaps) / len(gaps):.2f} us  "
             f"median {sorted(gaps)[len(gaps) // 2]:.2f} us  overlapping pairs {len(gaps) - len(pos)}"]
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "a") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    if "--timeline" in sys.argv:
        timeline(sys.argv[1], out=next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--out=")), None))
        sys.exit(0)
    main(sys.argv[1], by_shape="--shape" in sys.argv, out=next((a.split("=", 1)[1] for a in sys.argv
                                                                   if a.startswith("--out=")), None))
