"""Summarise a rocprofv3 --kernel-trace --stats database into a text table
(committed under profiles/)."""
import sqlite3
import sys


def main(db, out=None):
    con = sqlite3.connect(db)
    cur = con.cursor()
    rows = list(cur.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    res = {}
    for r in cur.execute("select name, vgpr_count, sgpr_count, lds_size, scratch_size, grid_x, workgroup_x from kernels"):
        res.setdefault(r[0], r[1:])
    lines = ["%-58s %6s %12s %11s %6s  %s" % ("kernel", "calls", "total_us", "avg_us", "pct", "vgpr sgpr lds scratch grid wg")]
    for name, calls, tot, avg, pct in rows:
        k = res.get(name, ())
        lines.append("%-58s %6d %12.1f %11.3f %6.2f  %s" % (name[:58], calls, tot / 1e3 if tot > 1e6 else tot, avg, pct,
                                                         " ".join(str(x) for x in k)))
    txt = "\n".join(lines)
    print(txt)
    if out:
        open(out, "w").write("# rocprofv3 --kernel-trace --stats (durations in microseconds)\n# source: %s\n" % db + txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
