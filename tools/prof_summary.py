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


if __name__ == "__main__":
    main(sys.argv[1], by_shape="--shape" in sys.argv, out=next((a.split("=", 1)[1] for a in sys.argv
                                                                   if a.startswith("--out=")), None))
