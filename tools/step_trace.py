"""Kernel-busy time of bench.py's timed region, from a rocprofv3 kernel trace of the
driver's own command (tools/gpu_steptrace.sh: `rocprofv3 --kernel-trace --stats --
python3 bench.py --config CFG --steps 20 --warmup 5`, frames in flight as the bench runs).

bench.py prints the timed region's host clocks (`timed_region`: CLOCK_MONOTONIC and
CLOCK_BOOTTIME, ns); the clock whose window holds the trace's dispatches is used.  Per
config this reports, over the dispatches of the timed region (clipped to it):

  busy_union_ms_per_step   union of the kernel-busy intervals / steps (GPU busy time)
  ms_per_step_traced_run   the traced run's own host ms_per_step (the window / steps)
  union_over_step          busy union / window: 1.0 = the GPU never idles between frames
  kernel_sum_over_union    sum of dispatch durations / union: the overlap of frames in flight
  frac_l2_per_step         algorithmic bytes per step / busy union per step / L2 peak
  frac_hbm_per_step        the same against the HBM peak
  kernels                  per kernel: dispatches in the region, average duration (us)

    python3 tools/step_trace.py <trace dir> <bench log> <CFG> [profiles/r04_steptrace.json]
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

HBM_PEAK_GBS, L2_PEAK_GBS = 8000.0, 34500.0


def bench_line(path):
    for line in reversed(open(path).read().splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"{path}: no bench JSON line")


def dispatches(root):
    out = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    if not out:
        raise SystemExit(f"{root}: no kernel_trace.csv")
    return sorted(out)


def short(name):
    m = re.search(r"mrt::(\w+)(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name.split("(")[0].strip()[:60]


def analyse(root, log, cfg):
    b = bench_line(log)
    reg = b.get("timed_region")
    if not reg:
        raise SystemExit(f"{log}: bench line has no timed_region (bench.py older than round 4)")
    ds = dispatches(root)
    best = None
    for key, (t0, t1) in reg.items():
        sel = [d for d in ds if t0 <= d[0] <= t1]
        if best is None or len(sel) > len(best[2]):
            best = (key, (t0, t1), sel)
    key, (t0, t1), sel = best
    if not sel:
        raise SystemExit("no dispatch inside the timed region on any host clock")
    steps = b["steps"]
    iv = sorted((max(s, t0), min(e, t1)) for s, e, _ in sel)
    union, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    ksum = sum(e - s for s, e in iv)
    per = defaultdict(list)
    for s, e, n in sel:
        per[short(n)].append((e - s) / 1e3)
    window = t1 - t0
    ps = b["roofline"].get("per_step") or {}
    step_b = ps.get("algorithmic_bytes_per_step")
    u_step = union / steps / 1e6   # ms
    rec = {
        "config": cfg, "command": b.get("_command", "bench.py --config %s --steps %d --warmup %d" % (cfg, steps, b["warmup"])),
        "clock": key, "steps": steps, "dispatches": len(sel), "dispatches_per_step": round(len(sel) / steps, 2),
        "busy_union_ms_per_step": round(u_step, 4), "ms_per_step_traced_run": round(window / steps / 1e6, 4),
        "bench_ms_per_step": b["ms_per_step"], "union_over_step": round(union / window, 4),
        "kernel_sum_over_union": round(ksum / union, 3),
        "kernels": {k: {"dispatches": len(v), "avg_us": round(sum(v) / len(v), 2)} for k, v in
                    sorted(per.items(), key=lambda kv: -sum(kv[1]))},
    }
    if step_b:
        gbs = step_b / (u_step * 1e-3) / 1e9
        rec.update({"algorithmic_bytes_per_step": step_b, "achieved_gbs_per_step": round(gbs, 1),
                    "frac_l2_per_step": round(gbs / L2_PEAK_GBS, 4), "frac_hbm_per_step": round(gbs / HBM_PEAK_GBS, 4),
                    "bench_frac_l2_per_step": ps.get("frac_l2")})
    return rec


def main():
    root, log, cfg = sys.argv[1:4]
    out = sys.argv[4] if len(sys.argv) > 4 else None
    rec = analyse(root, log, cfg)
    rec["source"] = os.path.relpath(root)
    print(json.dumps(rec, indent=1))
    if out:
        data = json.load(open(out)) if os.path.exists(out) else {"configs": {}}
        data["configs"][cfg] = rec
        json.dump(data, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
