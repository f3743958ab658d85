"""DESIGN.md results table from the tracked bench lines (profiles/<round>_<cfg>_bench.json)
and the rocprofv3 record (profiles/<round>_profile.json): per config Mray/s, ms per
frame (frames in flight), single-frame latency, the dominant pass's L2-priced fraction
(live and recomputed from the tracked rocprof average), its PMC HBM fraction, and the
CPU oracle baseline when the line carries one."""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = ["C3", "C2", "C3L", "C4", "D1", "C5", "A3", "R3", "P4", "G3", "FS"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", default="r06")
    ap.add_argument("--prev", default="r04", help="round whose tracked lines give the last column")
    a = ap.parse_args()
    print("| config | Mray/s | ms / frame | frame latency | frac (L2, live) | frac (tracked rocprof avg) | "
          "HBM frac (PMC) | CPU oracle (ref.-equiv.) | previous round |")
    print("|---|---|---|---|---|---|---|---|---|")
    for c in CONFIGS:
        p = os.path.join(ROOT, "profiles", f"{a.round}_{c.lower()}_bench.json")
        if not os.path.exists(p):
            continue
        d = json.loads(open(p).read().strip().splitlines()[-1])
        r = d["roofline"]
        tr = (r.get("tracked_profile") or {}).get("frac")
        hbm = (r.get("hbm") or {}).get("frac")
        cpu = d.get("cpu_baseline") or {}
        cpu_s = f"{cpu['value']} ({cpu.get('reference_equivalent')})" if cpu.get("value") else "—"
        pp = os.path.join(ROOT, "profiles", f"{a.prev}_{c.lower()}_bench.json")
        prev = "—"
        if os.path.exists(pp):
            q = json.loads(open(pp).read().strip().splitlines()[-1])
            prev = f"{q['value']:.0f} ({q['ms_per_step']:.3f} ms)"
        print(f"| {c} {d['config']['workload'][:60]} | {d['value']:.0f} | {d['ms_per_step']:.3f} | "
              f"{d.get('frame_latency_ms', 0):.3f} ms | {r['frac']:.3f} | {tr if tr is not None else '—'} | "
              f"{hbm if hbm is not None else '—'} | {cpu_s} | {prev} |")


if __name__ == "__main__":
    main()
