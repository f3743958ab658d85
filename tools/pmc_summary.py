"""Summarise tools/pmc.sh output per config: kernel-trace stats and the HBM
bytes per launch of each bench pass, for bench.py's roofline.

    hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB; on gfx950
FETCH_SIZE counts 128-B read requests at 64 B, i.e. half the bytes
(MI355X_MICROARCH.md, HBM section), hence the factor 2.  Both count L2 ->
fabric requests, so Infinity-Cache hits are included: an upper bound on DRAM
bytes.  Only the timed (uninstrumented, COUNT = false) kernel instantiations
are used.  Pass mapping: primary = primary_kernel; shade = shade1_kernel, or
shade_kernel (gen + resolve, or fused chains) + shadow_kernel, or
adaptive_kernel (one fused launch)."""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

PASS = {"primary_kernel": "primary", "frame1_kernel": "primary", "shade1_kernel": "shade", "shade_kernel": "shade", "shadow_kernel": "shade",
        "adaptive_kernel": "shade", "chain_trace_kernel": "shade", "chain0_kernel": "shade",
        "chain_shade_kernel": "shade", "chain_compact_kernel": "shade", "chain_finish_kernel": "shade"}
# kernels without a COUNT template argument: the instrumented frame runs the same
# instantiation, so their dispatches are averaged over every frame
NO_COUNT_ARG = {"chain0_kernel", "chain_shade_kernel", "chain_compact_kernel", "chain_finish_kernel"}


def parse_name(name):
    """'void mrt::shade_kernel<false, true, ...>(mrt::RenderParams)' -> ('shade_kernel', 'false, true, ...')"""
    m = re.search(r"mrt::(\w+)<([^>]*)>", name)
    if not m:
        m2 = re.search(r"mrt::(\w+)", name)
        return (m2.group(1) if m2 else name.strip()), ""
    return m.group(1), m.group(2)


def counters(root):
    per = defaultdict(lambda: defaultdict(list))      # full kernel -> counter -> values per dispatch
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                per[row.get("Kernel_Name", "?")][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def stats(root):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
        with open(f, newline="") as fh:
            rows += list(csv.DictReader(fh))
    return rows


def summarise(cfg, root):
    lines = [f"## {cfg}"]
    tr = stats(os.path.join(root, "trace"))
    if tr:
        lines.append("kernel-trace --stats (rocprofv3):")
        for r in sorted(tr, key=lambda r: -float(r.get("TotalDurationNs", 0))):
            base, targs = parse_name(r["Name"])
            lines.append("    %-34s calls %5s  avg %12.1f ns  total %14.1f ns  [%s]" % (
                base, r.get("Calls"), float(r.get("AverageNs", 0)), float(r.get("TotalDurationNs", 0)), targs))
    per = counters(root)
    passes = defaultdict(float)
    # frames in each PMC pass: one primary_kernel (or adaptive_kernel) dispatch per frame
    def frames(counter, timed_only):
        n = 0
        for k, cs in per.items():
            base, targs = parse_name(k)
            if base in ("primary_kernel", "adaptive_kernel", "frame1_kernel") and cs.get(counter):
                if not timed_only or targs.split(",")[0].strip() == "false":
                    n += len(cs[counter])
        return max(1, n)
    lines.append("PMC (mean per dispatch; per-frame pass totals below):")
    for k in sorted(per):
        base, targs = parse_name(k)
        cs = per[k]
        f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) if cs.get("FETCH_SIZE") else None
        w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) if cs.get("WRITE_SIZE") else None
        lines.append("    %-34s FETCH_SIZE %s KiB  WRITE_SIZE %s KiB  dispatches %s  [%s]" % (
            base, "-" if f is None else "%.1f" % f, "-" if w is None else "%.1f" % w,
            len(cs.get("FETCH_SIZE") or cs.get("WRITE_SIZE") or []), targs))
        if base not in PASS or f is None or w is None:
            continue
        every = base in NO_COUNT_ARG
        if not every and targs.split(",")[0].strip() != "false":
            continue   # the instrumented (COUNT = true) launch
        # bytes per frame: all of this kernel's dispatches over the frames they ran in
        fb = sum(cs["FETCH_SIZE"]) / frames("FETCH_SIZE", not every)
        wb = sum(cs["WRITE_SIZE"]) / frames("WRITE_SIZE", not every)
        passes[PASS[base]] += 2 * fb * 1024 + wb * 1024
    for p, b in sorted(passes.items()):
        lines.append("    pass %-8s hbm_bytes_per_launch %16.0f   (2*FETCH_SIZE + WRITE_SIZE)" % (p, b))
    return lines, {p: int(b) for p, b in passes.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--round", default="r02")
    ap.add_argument("--json", default="profiles/r02_pmc_traffic.json")
    a = ap.parse_args()
    out = json.load(open(a.json)) if os.path.exists(a.json) else {}
    out.setdefault("configs", {})
    out.setdefault("source", {})
    out["formula"] = ("2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per frame, summed over the pass's dispatches "
                      "(gfx950 FETCH_SIZE half-count correction)")
    for d in sorted(glob.glob(os.path.join(a.root, "*"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d)
        lines, passes = summarise(cfg, d)
        txt = "\n".join(lines) + "\n"
        print(txt)
        path = f"profiles/{a.round}_{cfg.lower()}_rocprof.txt"
        open(path, "w").write(f"# rocprofv3 summaries: python3 bench.py --config {cfg} --steps 5 --warmup 1 "
                              f"--no-cpu-baseline (tools/pmc.sh)\n" + txt)
        if passes:
            out["configs"][cfg] = {"per_launch_hbm_bytes": passes}
            out["source"][cfg] = path
    json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
