"""Summarise tools/prof_all.sh output per config into profiles/<round>_<cfg>_rocprof.txt
and one JSON (profiles/<round>_profile.json) that bench.py reads.

Per config directory (gpurun_out/prof3/<CFG>/):
  trace/  rocprofv3 --kernel-trace --stats of `bench.py --config CFG --inflight 1`
          (one frame in flight: every dispatch's duration is its own launch time)
          + trace.log, whose last line is that run's bench JSON
  fetch/  --pmc FETCH_SIZE          write/  --pmc WRITE_SIZE
  sq/     --pmc SQ_* wave-state counters + TCP (L1) / GRBM counters (one pass)

Reported per kernel instantiation: calls, average / min / max duration (us),
VGPR, AGPR, SGPR, LDS bytes, scratch bytes per lane (kernel_trace.csv columns),
then the PMC means per dispatch.  HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE
(KiB; gfx950 FETCH_SIZE half-count, MI355X_MICROARCH.md HBM section).

Latency evidence (SQ counters count quad-cycles; WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~= WAVE_CYCLES, MI355X_MICROARCH.md PMC section):
  wave_active / wave_wait_mem / wave_issue_stall = the three shares of WAVE_CYCLES
  valu_share = ACTIVE_INST_VALU / WAVE_CYCLES (a wave's cycles issuing VALU)
  simd_valu_busy = 2 * INSTS_VALU / (SIMDs * clock * duration): the share of the SIMDs'
      VALU throughput used -- a wave64 f32 VALU instruction occupies a SIMD for 2 cycles
      (SIMD-32; MI355X_MICROARCH.md cycle constants); clock from GRBM_GUI_ACTIVE / 8 XCDs / duration
  wave_issue_share = 4 * ACTIVE_INST_VALU / (SIMDs * clock * duration): the same instructions at
      one wave's own issue cost (4 cycles each); above 1 only because waves of a SIMD overlap
  l2_req_per_vmem_load = TCP_TCC_READ_REQ_sum / SQ_INSTS_VMEM_RD
  l1_hit = 1 - TCP_TCC_READ_REQ_sum / TCP_TOTAL_CACHE_ACCESSES_sum
Only the timed (COUNT = false) instantiations enter the pass totals."""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
import statistics
from collections import defaultdict

SIMDS = 256 * 4
# bench pass of each kernel (bench.py roofline: "primary" = the primary-ray launch or
# the fused frame1_kernel; "shade" = everything after it)
PASS = {"primary_kernel": "primary", "frame1_kernel": "primary", "shade1_kernel": "shade", "shade_kernel": "shade",
        "shadow_kernel": "shade", "adaptive_kernel": "shade", "chain_trace_kernel": "shade",
        "chain0_kernel": "shade", "chain_shade_kernel": "shade", "chain_compact_kernel": "shade",
        "chain_finish_kernel": "shade", "chain_path_kernel": "shade", "tile_order_kernel": "shade",
        "chain_fold_kernel": "shade", "unit_eye_kernel": "shade", "adapt_combine_kernel": "shade"}
NO_COUNT_ARG = {"chain0_kernel", "chain_shade_kernel", "chain_compact_kernel", "chain_finish_kernel",
                "chain_path_kernel", "tile_order_kernel", "chain_fold_kernel", "adapt_combine_kernel"}
FRAME_KERNELS = ("primary_kernel", "frame1_kernel", "adaptive_kernel")
# frames of one tools/prof_all.sh run (bench.py --inflight 1 --steps 6 --warmup 1): one
# setup frame, the instrumented (count-mode) frame, 1 warmup, 6 timed, 5 latency frames
FRAMES_TIMED, FRAMES_COUNT = 13, 1


def parse_name(name):
    m = re.search(r"mrt::(\w+)<([^>]*)>", name)
    if not m:
        m2 = re.search(r"mrt::(\w+)", name)
        return (m2.group(1) if m2 else name.strip().split("(")[0]), ""
    return m.group(1), m.group(2)


def timed(base, targs):
    return base in NO_COUNT_ARG or targs.split(",")[0].strip() == "false"


def rows(root, pattern):
    out = []
    for f in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        with open(f, newline="") as fh:
            out += list(csv.DictReader(fh))
    return out


def trace_table(root):
    per = defaultdict(list)
    res = {}
    for r in rows(root, "*kernel_trace.csv"):
        k = r["Kernel_Name"]
        per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        res.setdefault(k, {key: r.get(col) for key, col in (
            ("vgpr", "VGPR_Count"), ("agpr", "Accum_VGPR_Count"), ("sgpr", "SGPR_Count"), ("lds", "LDS_Block_Size"),
            ("scratch", "Scratch_Size"), ("wg", "Workgroup_Size_X"), ("grid", "Grid_Size_X"))})
    return per, res


def counters(root):
    per = defaultdict(lambda: defaultdict(list))
    for r in rows(root, "*counter_collection.csv"):
        per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def code_objects(objs):
    """Code-object resources of the built kernels (tools/kmeta.py), keyed by the
    demangled name as rocprofv3 prints it: vgpr / sgpr / scratch bytes per lane /
    VGPR spills.  (rocprofv3's VGPR_Count column is in allocation granules.)"""
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import kmeta
    out = {}
    for o in objs:
        for r in kmeta.kernels(o):
            name = subprocess.run(["c++filt", r.get("name", "")], capture_output=True, text=True).stdout.strip()
            out[name] = {"vgpr": r.get("vgpr_count"), "sgpr": r.get("sgpr_count"),
                         "scratch": r.get("private_segment_fixed_size"), "vgpr_spill": r.get("vgpr_spill_count")}
    return out


CODE = {}


def mean(v):
    return sum(v) / len(v) if v else None


def summarise(cfg, d):
    lines = [f"## {cfg}"]
    durs, res = trace_table(os.path.join(d, "trace"))
    bench = None
    log = os.path.join(d, "trace.log")
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                bench = json.loads(line)
    lines.append("kernel-trace (rocprofv3, one frame in flight; durations in us; resources per lane):")
    lines.append("    %-46s %5s %10s %9s %9s %11s  rocprof: vgpr agpr sgpr   lds scratch | code object: vgpr sgpr "
                 "scratch spills" % ("kernel", "calls", "avg", "min", "max", "total"))
    for k in sorted(durs, key=lambda k: -sum(durs[k])):
        base, targs = parse_name(k)
        v = durs[k]
        r = res[k]
        co = CODE.get(k.strip(), {})
        lines.append("    %-46s %5d %10.2f %9.2f %9.2f %11.1f           %4s %4s %4s %5s %7s |              %4s %4s %7s "
                     "%6s" % ((base + "<" + targs + ">")[:46], len(v), mean(v), min(v), max(v), sum(v), r["vgpr"],
                              r["agpr"], r["sgpr"], r["lds"], r["scratch"], co.get("vgpr", "-"), co.get("sgpr", "-"),
                              co.get("scratch", "-"), co.get("vgpr_spill", "-")))
    cnt = {}
    for sub in ("fetch", "write", "sq"):
        for k, cs in counters(os.path.join(d, sub)).items():
            for c, vals in cs.items():
                cnt.setdefault(k, {})[c] = vals
    # frames per PMC pass: one frame kernel dispatch per frame (timed instantiations)
    out = {"kernels": {}, "passes": {}}
    if cnt:
        lines.append("PMC (mean per dispatch):")
    for k in sorted(cnt):
        base, targs = parse_name(k)
        cs = cnt[k]
        m = {c: mean(v) for c, v in cs.items()}
        ent = {"counters": {c: round(x, 3) for c, x in m.items()}, "dispatches": max(len(v) for v in cs.values())}
        if k.strip() in CODE:
            ent["code_object"] = CODE[k.strip()]
        dur = mean(durs.get(k, []))
        if dur:
            ent["avg_us"] = round(dur, 3)
        if m.get("FETCH_SIZE") is not None and m.get("WRITE_SIZE") is not None:
            ent["hbm_bytes"] = int(2 * m["FETCH_SIZE"] * 1024 + m["WRITE_SIZE"] * 1024)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            lat = {}
            for name, c in (("wave_active", "SQ_ACTIVE_INST_ANY"), ("wave_wait_mem", "SQ_WAIT_ANY"),
                            ("wave_issue_stall", "SQ_WAIT_INST_ANY"), ("valu_share", "SQ_ACTIVE_INST_VALU")):
                if m.get(c) is not None:
                    lat[name] = round(m[c] / wc, 4)
            if m.get("GRBM_GUI_ACTIVE") and dur and m.get("SQ_ACTIVE_INST_VALU") is not None:
                clk = m["GRBM_GUI_ACTIVE"] / 8 / (dur * 1e-6)
                lat["clock_ghz"] = round(clk / 1e9, 3)
                if m.get("SQ_INSTS_VALU") is not None:
                    lat["simd_valu_busy"] = round(2 * m["SQ_INSTS_VALU"] / (SIMDS * clk * dur * 1e-6), 4)
                lat["wave_issue_share"] = round(4 * m["SQ_ACTIVE_INST_VALU"] / (SIMDS * clk * dur * 1e-6), 4)
            if m.get("TCP_TCC_READ_REQ_sum") is not None and m.get("SQ_INSTS_VMEM_RD"):
                lat["l2_req_per_vmem_load"] = round(m["TCP_TCC_READ_REQ_sum"] / m["SQ_INSTS_VMEM_RD"], 4)
            if m.get("TCP_TCC_READ_REQ_sum") is not None and m.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
                lat["l1_hit"] = round(1 - m["TCP_TCC_READ_REQ_sum"] / m["TCP_TOTAL_CACHE_ACCESSES_sum"], 4)
            if m.get("SQ_WAVES"):
                lat["waves"] = int(m["SQ_WAVES"])
            if m.get("SQ_INSTS_VALU") and m.get("SQ_WAVES"):
                lat["valu_insts_per_wave"] = round(m["SQ_INSTS_VALU"] / m["SQ_WAVES"], 1)
            ent["latency"] = lat
        out["kernels"][base + "<" + targs + ">"] = ent
        lines.append("    %-46s %s" % ((base + "<" + targs + ">")[:46], "  ".join(
            "%s %.4g" % (c, x) for c, x in sorted(m.items()))))
        if "latency" in ent:
            lines.append("    %-46s latency %s" % ("", json.dumps(ent["latency"])))
    # pass totals of the timed kernels: summed per frame
    frames = defaultdict(int)
    for k, cs in cnt.items():
        base, targs = parse_name(k)
        if base in FRAME_KERNELS and timed(base, targs):
            for c, v in cs.items():
                frames[c] = max(frames[c], len(v))
    n_trace = sum(len(v) for k, v in durs.items() if parse_name(k)[0] in FRAME_KERNELS and timed(*parse_name(k)))
    if not n_trace:   # no frame kernel (adaptive passes over the chain engine): the run's own frame count
        n_trace = FRAMES_TIMED
    # kernels without a count-mode variant also ran in the instrumented frame(s)
    def per_frame(base, n):
        return n + FRAMES_COUNT if base in NO_COUNT_ARG else n
    passes = defaultdict(lambda: {"hbm_bytes": 0.0, "avg_us": 0.0, "kernels": []})
    for k in set(list(cnt) + list(durs)):
        base, targs = parse_name(k)
        if base not in PASS or not timed(base, targs):
            continue
        p = passes[PASS[base]]
        p["kernels"].append(base + "<" + targs + ">")
        if k in durs and n_trace:
            p["avg_us"] += sum(durs[k]) / per_frame(base, n_trace)   # per frame, all of this kernel's launches
        cs = cnt.get(k, {})
        if cs.get("FETCH_SIZE") and cs.get("WRITE_SIZE"):
            ff = frames["FETCH_SIZE"] or FRAMES_TIMED
            fw = frames["WRITE_SIZE"] or FRAMES_TIMED
            p["hbm_bytes"] += (2 * sum(cs["FETCH_SIZE"]) * 1024 / per_frame(base, ff)
                               + sum(cs["WRITE_SIZE"]) * 1024 / per_frame(base, fw))
    for name, p in sorted(passes.items()):
        p["hbm_bytes"] = int(p["hbm_bytes"])
        p["avg_us"] = round(p["avg_us"], 3)
        lines.append("    pass %-8s per frame: %10.2f us (rocprof)  hbm_bytes %14d (2*FETCH_SIZE + WRITE_SIZE)  %s" % (
            name, p["avg_us"], p["hbm_bytes"], ", ".join(sorted(p["kernels"]))))
        out["passes"][name] = p
    if bench:
        r = bench.get("roofline", {})
        lines.append("bench line of the traced run: value %s Mray/s, launch_ms %s, roofline kernel %s, achieved %s GB/s"
                     % (bench.get("value"), bench.get("launch_ms"), r.get("kernel"), r.get("achieved")))
        out["bench_launch_ms"] = bench.get("launch_ms")
    return lines, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out/prof3")
    ap.add_argument("--round", default="r06")
    ap.add_argument("--objs", nargs="*", default=sorted(glob.glob(os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "rendering-algorithms-raytracer_amd", "lib", "build",
        "mrt_*.o"))))
    a = ap.parse_args()
    CODE.update(code_objects(a.objs))
    js = f"profiles/{a.round}_profile.json"
    allout = json.load(open(js)) if os.path.exists(js) else {"configs": {}}
    allout["note"] = ("rocprofv3 at --inflight 1 (tools/prof_all.sh); hbm_bytes = 2*FETCH_SIZE*1024 + "
                      "WRITE_SIZE*1024 per launch (gfx950 FETCH_SIZE half-count); latency from SQ/TCP/GRBM counters "
                      "(tools/prof3.py docstring)")
    for d in sorted(glob.glob(os.path.join(a.root, "*"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d)
        lines, out = summarise(cfg, d)
        txt = "\n".join(lines) + "\n"
        print(txt)
        path = f"profiles/{a.round}_{cfg.lower()}_rocprof.txt"
        open(path, "w").write(f"# tools/prof_all.sh: rocprofv3 --kernel-trace --stats and --pmc passes of "
                              f"python3 bench.py --config {cfg} --inflight 1 --no-cpu-baseline\n" + txt)
        out["source"] = path
        allout["configs"][cfg] = out
    json.dump(allout, open(js, "w"), indent=1)


if __name__ == "__main__":
    main()
