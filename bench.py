#!/usr/bin/env python3
"""Headline benchmark: Mray/s (primary + shadow) on the Sponza config C3
(1920x1080, 1 spp, Blinn + PointLight; synthetic ~68k-triangle stand-in for the
missing sponza.obj) -- BASELINE.json `metric` / configs[2].

One "step" = one full frame: primary rays + shadow rays + shading + Image::Map.
N = 1: the frame renders straight into HBM buffers.  N > 1 (torch.distributed,
one process per GPU, backend nccl = RCCL): 32x32 buckets are dealt b mod N
(reference bucket grid, src/Scene.cpp:90-95), every rank renders its buckets
into a packed tile buffer, one RCCL gather brings them to rank 0, which
scatters them into the frame.  value = rays of the whole frame / max-over-ranks
wall time.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
NODE_B, LEAF_B = 128, 160      # QNode / DLeaf bytes (csrc/mrt_types.h)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-thread-seconds for the oracle sample")
    return ap.parse_args()


def kernel_bytes(st, px, hits):
    """Algorithmic bytes per launch: node/leaf visits x
    their sizes + per-pixel ray I/O + per-hit shading gathers."""
    pn, pl = st["primary_node_visits"], st["primary_leaf_visits"]
    sn, sl = st["node_visits"] - pn, st["leaf_visits"] - pl
    primary = pn * NODE_B + pl * LEAF_B + px * 16                 # write the 16-B hit record
    # read the hit record, write float RGB + RGB8; per hit: PrimShade + 3 vertices + 3 normals
    shade = sn * NODE_B + sl * LEAF_B + px * (16 + 12 + 3) + hits * (32 + 3 * 16 + 3 * 16)
    return primary, shade


def cpu_baseline(cfg_key, seconds):
    """The CPU oracle (C restatement, OpenMP) on this host's cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from miro import scenes
    cfg = scenes.CONFIGS[cfg_key]
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    s = O.OracleScene()
    m = s.add_material(cfg["material"]["kind"], kd=cfg["material"]["kd"])
    if cfg["mesh"] == "sponza":
        s.add_obj(scenes.sponza_obj(), m)
    elif cfg["mesh"] == "bunny":
        s.add_obj(scenes.bunny_obj(), m)
        s.add_mesh([(-100, 0, -100), (0, 0, 100), (100, 0, -100)], [(0, 1, 0)] * 3, [(0, 1, 2)], [(0, 1, 2)], m)
    else:
        import numpy as np
        f = np.load(os.path.join(ROOT, "tests", "golden", "cornell_box_mesh.npz"))
        s.add_mesh(f["verts"], f["normals"], f["vidx"], f["nidx"], m)
    for l in cfg["lights"]:
        s.add_point_light(l["pos"], l["power"])
    s.set_bg(cfg["bg"])
    s.build()
    W, H = cfg["W"], cfg["H"]
    rays, t_total, frames = 0, 0.0, 0
    band = 64
    y = 0
    while t_total * threads < seconds and t_total < 60.0:
        y0 = y % H
        t0 = time.perf_counter()
        r = s.render(cfg["camera"], W, H, rect=(0, y0, W, min(H, y0 + band)), threads=threads, want_hits=False)
        t_total += time.perf_counter() - t0
        rays += r["primary_rays"] + r["shadow_rays"]
        y += band
        frames += 1
    return {"value": round(rays / t_total / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{cfg_key} {W}x{H}: {frames} bands of {band} rows ({rays} rays, {t_total:.1f} s wall, "
                      f"{threads} OpenMP threads, oracle/mrt_oracle.c -O2)"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import miro
    from miro import _lib, scenes

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    scene, cam, cfg = scenes.build_config(args.config, device=dev)
    W, H = cfg["W"], cfg["H"]
    L = miro.lib()
    stream = torch.cuda.current_stream()
    sh = stream.cuda_stream
    camc = cam._c()
    bx, by = (W + 31) // 32, (H + 31) // 32
    nb = bx * by
    frame = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
    frame8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    if world > 1:
        mine = list(range(rank, nb, world))
        per = (nb + world - 1) // world
        ids = torch.tensor(mine + [mine[-1]] * (per - len(mine)), dtype=torch.int32, device="cuda")
        tiles = torch.empty(per * 1024 * 3, dtype=torch.float32, device="cuda")
        all_ids = [torch.tensor(list(range(r, nb, world)) + [list(range(r, nb, world))[-1]] * (per - len(range(r, nb, world))),
                                dtype=torch.int32, device="cuda") for r in range(world)]
        gathered = [torch.empty_like(tiles) for _ in range(world)] if rank == 0 else None
    opts_count = _lib.mrt_render_opts(W, H, dev, 1, 1, 0, 0)
    opts = _lib.mrt_render_opts(W, H, dev, 0, 1, 0, 0)

    def step(o):
        if world == 1:
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), frame.data_ptr(),
                                                frame8.data_ptr(), sh), "render")
        else:
            _lib.check(L.mrt_render_buckets_async(scene.handle, C.byref(camc), C.byref(o), ids.data_ptr(), len(ids),
                                                  tiles.data_ptr(), sh), "render buckets")
            dist.gather(tiles, gathered, dst=0)
            if rank == 0:
                for r in range(world):
                    _lib.check(L.mrt_unpack_buckets_async(all_ids[r].data_ptr(), len(all_ids[r]), gathered[r].data_ptr(),
                                                          W, H, frame.data_ptr(), frame8.data_ptr(), scene.handle, sh),
                               "unpack")

    # instrumented frame: node/leaf visits + per-launch times (not timed below)
    step(opts_count)
    torch.cuda.synchronize()
    st = scene.stats()
    shadow_mine = st["shadow_rays"]
    if world > 1:
        t = torch.tensor([shadow_mine], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        shadow_total = int(t.item())
    else:
        shadow_total = shadow_mine
    rays_per_frame = W * H + shadow_total
    hits_px = st["primary_hits"]

    for _ in range(args.warmup):
        step(opts)
    # per-launch durations of the uninstrumented kernels (HIP events on this stream)
    prim_ms, shade_ms = [], []
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(opts)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st_last = scene.stats()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # separate short loop for per-launch event timing
    for _ in range(5):
        step(opts)
        torch.cuda.synchronize()
        s2 = scene.stats()
        prim_ms.append(s2["primary_ms"])
        shade_ms.append(s2["shade_ms"])
    if rank != 0:
        dist.destroy_process_group()
        return
    value = rays_per_frame * args.steps / elapsed / 1e6
    px_mine = W * H if world == 1 else len(range(0, nb, world)) * 1024
    hits_mine = hits_px
    b_prim, b_shade = kernel_bytes(st, px_mine, hits_mine)
    pm, sm = float(np.median(prim_ms)), float(np.median(shade_ms))
    one_light = len(cfg["lights"]) == 1 and cfg.get("num_paths", 1) == 1
    shade_name = "shade1_kernel" if one_light else "shade_kernel"
    if sm >= pm:
        dom, dom_ms, dom_b = shade_name + " (shade + any-hit shadow rays)", sm, b_shade
    else:
        dom, dom_ms, dom_b = "primary_kernel (camera rays, closest hit)", pm, b_prim
    achieved = dom_b / (dom_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            prof = json.load(open(pmc))
            if prof.get("config") == args.config:
                traffic = prof.get("per_launch_hbm_bytes", {}).get(dom.split()[0])
        except Exception:
            traffic = None
    out = {
        "metric": "Mray/s (primary+shadow) on Sponza 1920x1080",
        "value": round(value, 2), "unit": "Mray/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (deterministic Sponza stand-in, %d tris; sponza.obj is not in the reference snapshot)"
                % scene.bvh_info["prims"],
        "config": {"workload": cfg["name"], "config": args.config, "width": W, "height": H, "spp": 1,
                   "rays_per_frame": rays_per_frame, "shadow_rays": shadow_total,
                   "qbvh_nodes": scene.bvh_info["nodes"], "qbvh_leaves": scene.bvh_info["leaves"],
                   "parallelism": "replica" if world == 1 else f"bucket-tiles b mod {world} + RCCL gather"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "launch_ms": round(dom_ms, 4), "algorithmic_bytes_per_launch": int(dom_b),
                     "visits_per_ray": round((st["node_visits"]) / max(1, rays_per_frame if world == 1 else
                                              px_mine + shadow_mine), 3)},
        "launch_ms": {"primary": round(pm, 4), "shade": round(sm, 4)},
    }
    if not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
