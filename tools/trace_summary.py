"""Per-kernel totals and the dispatch sequence of one frame from a rocprofv3
--kernel-trace CSV (kernel_trace.csv): python trace_summary.py <csv> [n_last]."""
import csv
import collections
import sys


def main(path, n_last=60):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tot = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = r["Kernel_Name"].split("(")[0][:70]
        tot[k][0] += 1
        tot[k][1] += d
    print("%-70s %6s %10s %9s" % ("kernel", "calls", "total_us", "avg_us"))
    for k, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1]):
        print("%-70s %6d %10.1f %9.2f" % (k, c, t, t / c))
    print("\nlast %d dispatches (us: duration, gap to previous end):" % int(n_last))
    prev = None
    for r in rows[-int(n_last):]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%-70s %9.1f %8.1f  grid %s" % (r["Kernel_Name"].split("(")[0][:70], (e - s) / 1e3,
                                             0 if prev is None else (s - prev) / 1e3, r.get("Grid_Size_X", r.get("Grid_Size", ""))))
        prev = e


if __name__ == "__main__":
    main(*sys.argv[1:])
