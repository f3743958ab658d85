#!/usr/bin/env python3
"""Headline benchmark: Mray/s (primary + shadow) on the Sponza config C3
(1920x1080, 1 spp, Blinn + PointLight; synthetic ~68k-triangle stand-in for the
missing sponza.obj) -- BASELINE.json `metric` / configs[2].

One "step" = one pass of the hot path over one batch: primary rays + shadow
rays + shading + Image::Map.
N = 1: one frame per step, rendered straight into HBM buffers (whole-frame
launch pair); consecutive steps alternate over --inflight (4) HIP streams, each
with its own scratch in libmrt, so the tail of one frame's persistent launches
overlaps the start of the next frame (4 streams = the HIP hardware queues per process).  N > 1 (torch.distributed, one process per GPU, backend nccl =
RCCL): weak scaling -- a step renders a camera path of N frames (frame 0 is the
config camera, then 2.5-degree pans), the 32x32 buckets of all N frames are
dealt id mod N (reference bucket grid, src/Scene.cpp:90-95), every rank renders
its share in one launch pair into packed 8-bit tiles, one RCCL gather per step
brings them to rank 0, which scatters them into the N frames; the gather of
step k overlaps the render of step k + 1 (miro/tiles.py BatchPipeline).
value = rays of all frames of all steps / max-over-ranks wall time.  Rank 0
prints one JSON line.
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
    ap.add_argument("--frames", type=int, default=0, help="frames per step (default: 1 at N=1, N at N>1)")
    ap.add_argument("--inflight", type=int, default=4,
                    help="N = 1 frame path: frames in flight (consecutive steps alternate over this many HIP "
                         "streams, so one frame's launch tail overlaps the next frame's start)")
    ap.add_argument("--path", choices=["auto", "batch"], default="auto",
                    help="batch: use the bucket-batch path even for one frame on one GPU (A/B)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-thread-seconds for the oracle sample")
    return ap.parse_args()


def _camera(c):
    import miro
    cam = miro.Camera()
    cam.setEye(c["eye"]); cam.setLookAt(c["lookAt"]); cam.setUp(c["up"]); cam.setFOV(c["fov"])
    return cam


def _pixels_in_frame(ids, bpf, bx, W, H):
    n = 0
    for i in ids:
        b = i % bpf
        n += min(32, W - (b % bx) * 32) * min(32, H - (b // bx) * 32)
    return n


def kernel_bytes(st, px, hits, float_out=True, wavefront=False):
    """Algorithmic bytes per launch: node/leaf visits x
    their sizes + per-pixel ray I/O + per-hit shading gathers.  With the
    wavefront shadow pass each shadow ray is also written (32 B), read back
    (32 B) and answered (1 B write + 1 B read), the hit record and the shading
    gathers are read twice (kernels 2a and 2c) and each pixel's ray count once."""
    pn, pl = st["primary_node_visits"], st["primary_leaf_visits"]
    sn, sl = st["node_visits"] - pn, st["leaf_visits"] - pl
    primary = pn * NODE_B + pl * LEAF_B + px * 16                 # write the 16-B hit record
    # read the hit record, write float RGB + RGB8; per hit: PrimShade + 3 vertices + 3 normals
    gathers = 2 if wavefront else 1
    shade = (sn * NODE_B + sl * LEAF_B + px * (16 * gathers + (12 if float_out else 0) + 3)
             + hits * (32 + 3 * 16 + 3 * 16) * gathers)
    if wavefront:
        shade += st["shadow_rays"] * (32 + 32 + 1 + 1) + px * 2
    return primary, shade


def cpu_baseline(cfg_key, seconds):
    """The CPU oracle (C restatement, OpenMP) on this host's cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from miro import scenes
    cfg = scenes.CONFIGS[cfg_key]
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    s = O.OracleScene()
    mat = cfg["material"]
    m = s.add_material(mat["kind"], kd=mat["kd"], specExp=mat.get("specExp", 1.0), specAmt=mat.get("specAmt", 0.0),
                       reflectAmt=mat.get("reflectAmt", 0.0), refractAmt=mat.get("refractAmt", 0.0),
                       ior=mat.get("ior", 1.5))
    if cfg["mesh"] == "sponza":
        s.add_obj(scenes.sponza_obj(), m)
    elif cfg["mesh"] in ("bunny", "instances"):
        if cfg["mesh"] == "bunny":
            s.add_obj(scenes.bunny_obj(), m)
        else:   # two ProxyObject BVHs, instances alternating (as scenes.build_config)
            blas = [s.make_blas([s.add_obj(p, m)]) for p in (scenes.dragon_obj(), scenes.buddha_obj())]
            for i, M in enumerate(scenes.instance_transforms(**cfg["instances"])):
                s.add_instance(blas[i % 2], M)
        s.add_mesh([(-100, 0, -100), (0, 0, 100), (100, 0, -100)], [(0, 1, 0)] * 3, [(0, 1, 2)], [(0, 1, 2)], m)
    else:
        import numpy as np
        f = np.load(os.path.join(ROOT, "tests", "golden", "cornell_box_mesh.npz"))
        s.add_mesh(f["verts"], f["normals"], f["vidx"], f["nidx"], m)
    skies = {}

    def sky(size):
        if size not in skies:
            skies[size] = s.add_texture(scenes.sky_rgb(*size))
        return skies[size]

    for l in cfg["lights"]:
        if l["type"] == "point":
            s.add_point_light(l["pos"], l["power"])
        elif l["type"] == "dome":
            s.add_dome_light(sky(tuple(l["sky"])), l["power"], l.get("samples", 1), l.get("noise", 0.001))
        else:
            s.add_rect_light(l["v1"], l["v2"], l["v3"], l["power"], l.get("samples", 1), l.get("noise", 0.001))
    s.set_bg(cfg["bg"])
    if cfg.get("env"):
        s.set_env_map(sky(tuple(cfg["env"]["sky"])), cfg["env"]["exposure"])
    s.set_num_paths(cfg.get("num_paths", 1))
    if cfg.get("subdivs"):
        s.set_subdivs(*cfg["subdivs"])
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
        rays += r["primary_rays"] + r["shadow_rays"] + r["secondary_rays"]
        y += band
        frames += 1
    return {"value": round(rays / t_total / 1e6, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{cfg_key} {W}x{H}: {frames} bands of {band} rows ({rays} rays, {t_total:.1f} s wall, "
                      f"{threads} OpenMP threads, oracle/mrt_oracle.c -O2)"}


def _scene_setup(scene):
    """One-time host BVH::build (src/BVH.cpp:457-575), outside the timed region."""
    ms = getattr(scene, "bvh_build_ms", None)
    prims = scene.bvh_info["prims"]
    return {"bvh_build_ms": None if ms is None else round(ms, 2), "prims": prims, "threads": 1,
            "build_mprims_per_s": None if not ms else round(prims / ms / 1e3, 3),
            # instanced scenes: the BLAS builds (mrt_scene_make_blas) happen before the world QBVH
            "blas_build_ms": round(getattr(scene, "blas_build_ms", 0.0), 2)}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import miro
    from miro import _lib, scenes
    from miro import tiles as tiles_mod

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
    # frames per step: 1 at N = 1; N > 1 renders a camera path of N frames per
    # step (weak scaling: one frame of work per GPU per step), every frame's
    # buckets dealt over all ranks, 8-bit tiles gathered once per step
    n_frames = args.frames or (1 if world == 1 else min(world, 16))
    cams = [cam] if n_frames == 1 else [_camera(c) for c in scenes.camera_path(cfg["camera"], n_frames)]
    bx, by = (W + 31) // 32, (H + 31) // 32
    bpf = bx * by
    use_frame_path = world == 1 and n_frames == 1 and args.path == "auto"
    inflight = max(1, args.inflight) if use_frame_path else 1
    streams = [stream] + [torch.cuda.Stream() for _ in range(inflight - 1)]
    frame = [torch.empty(H * W * 3, dtype=torch.float32, device="cuda") for _ in range(inflight)] \
        if use_frame_path else None
    frame8 = [torch.empty(H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(inflight)]
    frames8 = [frame8[0]] if use_frame_path else \
        [torch.empty(n_frames * H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(2)]
    camc = (_lib.mrt_camera * n_frames)(*[c._c() for c in cams])
    opts_count = _lib.mrt_render_opts(W, H, dev, 1, 1, 0, 0)
    opts = _lib.mrt_render_opts(W, H, dev, 0, 1, 0, 0)
    if not use_frame_path:
        mine = tiles_mod.batch_items(bpf, n_frames, world, rank)
        items = torch.tensor(mine, dtype=torch.int32, device="cuda")
        all_items = torch.tensor([i for r in range(world) for i in tiles_mod.batch_items(bpf, n_frames, world, r)],
                                 dtype=torch.int32, device="cuda")
        per = len(mine)

        def render(ids, out, o=opts):
            _lib.check(L.mrt_render_batch_async(scene.handle, camc, n_frames, C.byref(o), ids.data_ptr(), len(ids),
                                                None, out.data_ptr(), torch.cuda.current_stream().cuda_stream),
                       "render batch")

        def unpack(ids, gathered, b):
            _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), len(ids), None, gathered.data_ptr(), W, H, n_frames,
                                                None, frames8[b].data_ptr(), scene.handle,
                                                torch.cuda.current_stream().cuda_stream), "unpack")

        # two streams: consecutive steps' launch pairs overlap (libmrt keeps scratch per stream)
        pipe = tiles_mod.BatchPipeline(world, rank, dist, items, all_items,
                                       lambda k: torch.empty(k * per * 1024 * 3, dtype=torch.uint8, device="cuda"),
                                       render, unpack, streams=[torch.cuda.Stream(), torch.cuda.Stream()])

    nstep = [0]

    def step(o, serial=False):
        if use_frame_path:
            i = 0 if serial else nstep[0] % inflight
            nstep[0] += 1
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc[0]), C.byref(o), frame[i].data_ptr(),
                                                frame8[i].data_ptr(), streams[i].cuda_stream), "render")
        elif o is opts_count:
            render(items, pipe.tiles[0], opts_count)     # instrumented launch only (no gather)
        else:
            pipe.step()

    # instrumented frame: node/leaf visits + per-launch times (not timed below)
    step(opts_count, serial=True)
    torch.cuda.synchronize()
    st = scene.stats()
    shadow_mine = st["shadow_rays"]
    # adaptive supersampling (subdivs > 1): eye rays per pixel vary, counted by the kernel
    adaptive = bool(cfg.get("subdivs")) and max(cfg["subdivs"][:2]) > 1
    eye_mine = st["primary_rays"] if adaptive else 0
    second_mine = st["secondary_rays"]   # Blinn reflection / refraction rays
    if world > 1:
        t = torch.tensor([shadow_mine, eye_mine, second_mine], dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        shadow_total, eye_total, second_total = int(t[0].item()), int(t[1].item()), int(t[2].item())
    else:
        shadow_total, eye_total, second_total = shadow_mine, eye_mine, second_mine
    primary_total = eye_total if adaptive else n_frames * W * H
    rays_per_step = primary_total + shadow_total + second_total      # all frames of the batch, all ranks
    hits_px = st["primary_hits"]

    for _ in range(args.warmup):
        step(opts)
    if not use_frame_path:
        pipe.flush()
    # per-launch durations of the uninstrumented kernels (HIP events on this stream)
    prim_ms, shade_ms = [], []
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(opts)
    if not use_frame_path:
        pipe.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st_last = scene.stats()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    # separate short loop for per-launch event timing (render launches only)
    for _ in range(5):
        if use_frame_path:
            step(opts, serial=True)
        else:
            render(items, pipe.tiles[0])
        torch.cuda.synchronize()
        s2 = scene.stats()
        prim_ms.append(s2["primary_ms"])
        shade_ms.append(s2["shade_ms"])
    if rank != 0:
        dist.destroy_process_group()
        return
    value = rays_per_step * args.steps / elapsed / 1e6
    px_mine = W * H if use_frame_path else _pixels_in_frame(sorted(set(mine)), bpf, bx, W, H)
    hits_mine = hits_px
    # the specialised kernel runs for one point light, one path and no environment map
    mat = cfg["material"]
    recursive = mat["kind"] == "blinn" and (mat.get("reflectAmt", 0) > 0 or mat.get("refractAmt", 0) > 0)
    one_light = (len(cfg["lights"]) == 1 and cfg["lights"][0]["type"] == "point" and cfg.get("num_paths", 1) == 1
                 and not cfg.get("env") and not recursive)
    b_prim, b_shade = kernel_bytes(st, px_mine, hits_mine, float_out=use_frame_path,
                                   wavefront=not one_light and not recursive)
    if recursive:   # each secondary hit gathers its PrimShade + 3 vertices + 3 normals
        b_shade += second_mine * (16 + 32 + 3 * 16 + 3 * 16)
    pm, sm = float(np.median(prim_ms)), float(np.median(shade_ms))
    shade_name = ("shade1_kernel (shade + any-hit shadow rays)" if one_light else
                  "shade_kernel (fused: shade + reflection/refraction rays + any-hit shadow rays)" if recursive else
                  "shade pass (shade_kernel<gen> + shadow_kernel any-hit + shade_kernel<resolve>)")
    if adaptive:   # one fused launch: eye rays, shading, inline shadow rays (its time is shade_ms)
        dom, dom_ms = "adaptive_kernel (eye rays + shading + any-hit shadow rays)", sm
        dom_b = (st["node_visits"] * NODE_B + st["leaf_visits"] * LEAF_B
                 + px_mine * (16 + (12 if use_frame_path else 0) + 3) + hits_px * (32 + 3 * 16 + 3 * 16))
    elif sm >= pm:
        dom, dom_ms, dom_b = shade_name, sm, b_shade
    else:
        dom, dom_ms, dom_b = "primary_kernel (camera rays, closest hit)", pm, b_prim
    achieved = dom_b / (dom_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if use_frame_path and os.path.exists(pmc):   # PMC pass was taken on the N = 1 frame path
        try:
            prof = json.load(open(pmc))
            if prof.get("config") == args.config:
                traffic = prof.get("per_launch_hbm_bytes", {}).get(dom.split()[0])
        except Exception:
            traffic = None
    out = {
        "metric": ("Mray/s (primary+shadow) on Sponza 1920x1080" if args.config == "C3" else
                   f"Mray/s (primary+shadow{'+secondary' if second_total else ''}) [{args.config}: {cfg['name']}]"),
        "value": round(value, 2), "unit": "Mray/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic (deterministic %s stand-in, %d tris; %s.obj is not in the reference snapshot%s)"
                 % ({"sponza": "Sponza", "bunny": "bunny", "instances": "dragon_2 / buddha_smooth"}.get(
                     cfg["mesh"], cfg["mesh"]), scene.bvh_info["prims"],
                    {"instances": "dragon_2.obj / buddha_smooth"}.get(cfg["mesh"], cfg["mesh"]),
                    "; procedural lat-long sky for the dome / environment map" if cfg.get("env") else "")),
        "config": {"workload": cfg["name"], "config": args.config, "width": W, "height": H, "spp": 1 if not adaptive else f"adaptive {cfg['subdivs'][0]}..{cfg['subdivs'][1]} subdivs, "
                   f"{primary_total / (n_frames * W * H):.2f} eye rays/px",
                   "frames_per_step": n_frames, "rays_per_step": rays_per_step, "shadow_rays": shadow_total,
                   "secondary_rays": second_total,
                   "qbvh_nodes": scene.bvh_info["nodes"], "qbvh_leaves": scene.bvh_info["leaves"],
                   "frames_in_flight": inflight,
                   "parallelism": "single GPU, whole frame" if use_frame_path else
                   f"{n_frames}-frame camera path per step, 32x32 buckets dealt id mod {world}, "
                   f"one RCCL gather of 8-bit tiles per step (double-buffered)"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "launch_ms": round(dom_ms, 4), "algorithmic_bytes_per_launch": int(dom_b),
                     "visits_per_ray": round(st["node_visits"] / max(1, (eye_mine if adaptive else px_mine) + shadow_mine + second_mine), 3)},
        "launch_ms": {"primary": round(pm, 4), "shade": round(sm, 4)},
        # one-time host side (outside the timed region): BVH::build over the scene's triangles
        "scene_setup": _scene_setup(scene),
        # instrumented (count-mode) launch: wall-clock spread of the persistent waves
        "wave_timing_us": {k: round(st[k], 1) for k in ("primary_span_us", "primary_ramp_us", "primary_tail_us",
                                                       "shade_span_us", "shade_ramp_us", "shade_tail_us")},
        "lane_util": round(st["primary_node_visits"] / max(1, 64 * st["primary_wave_steps"]), 4),
    }
    if not args.no_cpu_baseline and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
