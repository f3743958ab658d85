"""Summarise tools/pmc.sh output (rocprofv3 --pmc CSV passes) per kernel.

Writes a text table (mean counter value per dispatch) and, with --json, the
per-launch HBM traffic that bench.py reports as roofline.traffic:

    hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB.  On gfx950
FETCH_SIZE counts 128-B read requests at 64 B, i.e. half the bytes
(MI355X_MICROARCH.md, HBM section), hence the factor 2; WRITE_SIZE is exact
for 16-B-per-lane stores.  Both count L2 -> fabric traffic, so Infinity-Cache
hits are included: an upper bound on HBM bytes.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*\)$", "", name.strip())
    name = name.replace("void ", "").replace("mrt::", "")
    return name


def load(root):
    per = defaultdict(lambda: defaultdict(list))      # kernel -> counter -> [values per dispatch]
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", "?"))
                per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--out", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--config", default="C3")
    a = ap.parse_args()
    per = load(a.root)
    lines = ["# rocprofv3 --pmc (one counter set per pass), mean value per dispatch",
             "# workload: python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline (config %s)" % a.config]
    traffic = {}
    for k in sorted(per):
        cs = per[k]
        lines.append(k)
        for c in sorted(cs):
            v = cs[c]
            lines.append("    %-32s %16.1f   (n=%d)" % (c, sum(v) / len(v), len(v)))
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            hbm = 2 * fetch * 1024 + write * 1024
            lines.append("    %-32s %16.0f   (2*FETCH_SIZE + WRITE_SIZE, bytes)" % ("hbm_bytes_per_launch", hbm))
            if "<false" in k:      # uninstrumented (timed) instantiation
                base = k.split("<")[0]
                traffic[base] = int(hbm)
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            h = sum(cs["TCC_HIT_sum"]); m = sum(cs["TCC_MISS_sum"])
            lines.append("    %-32s %16.4f" % ("L2 hit rate", h / max(1.0, h + m)))
        if "SQ_WAVE_CYCLES" in cs:
            wc = sum(cs["SQ_WAVE_CYCLES"])
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in cs:
                    lines.append("    %-32s %16.4f" % (c + " / WAVE_CYCLES", sum(cs[c]) / max(1.0, wc)))
    txt = "\n".join(lines) + "\n"
    print(txt)
    if a.out:
        open(a.out, "w").write(txt)
    if a.json:
        json.dump({"config": a.config, "per_launch_hbm_bytes": traffic,
                   "formula": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)",
                   "source": a.out}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
