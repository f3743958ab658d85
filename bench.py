#!/usr/bin/env python3
"""Headline benchmark: Mray/s (primary + shadow) on the Sponza config C3
(1920x1080, 1 spp, Blinn + PointLight; synthetic ~68k-triangle stand-in for the
missing sponza.obj) -- BASELINE.json `metric` / configs[2].  --config picks the
other presets of miro/scenes.py (C2, C4, C5, D1, A3, R3, P4).

One "step" = one pass of the hot path over one batch: primary rays + shadow
rays (+ secondary / GI rays) + shading + Image::Map, inputs resident in HBM.

N = 1: one frame per step, rendered straight into HBM buffers (whole-frame
launch pair); consecutive steps alternate over --inflight (4) HIP streams, each
with its own scratch in libmrt, so the tail of one frame's persistent launches
overlaps the start of the next frame.

N > 1: one process per GPU (torch.distributed, backend nccl = RCCL).  `python
bench.py --gpus N` spawns the N ranks itself when WORLD_SIZE is not set (the
parent never touches torch or HIP); under torch.distributed.run WORLD_SIZE must
equal --gpus.  The headline `value` is the north-star split (strong scaling):
ONE frame per step, its 32x32 buckets dealt id mod N (reference bucket grid,
src/Scene.cpp:90-95), every rank renders its share in one launch into packed
float tiles, one RCCL gather of the framebuffer brings them to rank 0, which
scatters them into the frame; the gather of step k overlaps the render of
step k + 1 (miro/tiles.py BatchPipeline).  `split_times` gives each rank's
render and the gather alone; `weak` times a camera path of N frames per step
(buckets of all N frames dealt id mod N, 8-bit tiles), i.e. weak scaling.

value = rays of all frames of all steps / max-over-ranks wall time.  Rank 0
prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
L2_PEAK_GBS = 34500.0          # MI355X_MICROARCH.md: L2 ~34.5 TB/s aggregate
NODE_B, LEAF_B = 128, 160      # QNode / DLeaf bytes (csrc/mrt_types.h)
# rocprofv3 evidence of this round (tools/prof_all.sh + tools/prof3.py): per config and
# bench pass, HBM bytes per launch (PMC) and the rocprof average duration at one
# frame in flight; per kernel, the SQ / TCP latency counters
PROFILE_FILE = os.path.join(ROOT, "profiles", "r06_profile.json")
CPU_CAL_FILE = os.path.join(ROOT, "profiles", "r02_cpu_calibration.json")
# kernel traces of the driver-settings runs (tools/step_trace.py): busy union per timed step
STEP_TRACE_FILE = os.path.join(ROOT, "profiles", "r06_steptrace.json")
# N > 1 split: frames of the camera path per step when --frames-per-launch is not given
DEFAULT_FPL = 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--frames", type=int, default=0, help="frames per step (default: 1 at N=1, N at N>1)")
    ap.add_argument("--settle-s", type=float, default=0.3,
                    help="untimed rendering before the warmup steps until this many seconds have passed (clock settle)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="N = 1 frame path: frames in flight (consecutive steps alternate over this many HIP "
                         "streams and hardware queues, so one frame's launch tail overlaps the next frame's "
                         "start); 0 = the config's `inflight` (4, or 8 where a few heavy tiles set the frame's "
                         "latency: C2, C4)")
    ap.add_argument("--path", choices=["auto", "batch"], default="auto",
                    help="batch: use the bucket-batch path even for one frame on one GPU (A/B)")
    ap.add_argument("--split", choices=["frame", "batch"], default="frame",
                    help="N > 1: frame = one frame per step split over the GPUs (headline); batch = N frames per step "
                         "(weak scaling; also reported as the `weak` key of a frame-split line)")
    ap.add_argument("--strong-steps", type=int, default=0, help="N > 1: steps of the secondary (weak) measurement")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-thread-seconds for the oracle sample")
    ap.add_argument("--share", default="",
                    help="N = 1 only: comma list of split widths (e.g. 2,4,8); renders rank 0's bucket share of each "
                         "N-way split alone (no gather) with --inflight streams, times the full-frame unpack, and "
                         "prints a modeled N-GPU curve (gather modeled from --xgmi-gbs; unmeasured on hardware)")
    ap.add_argument("--xgmi-gbs", type=float, default=50.0,
                    help="--share model: assumed effective RCCL point-to-point rate per xGMI link and direction (GB/s)")
    ap.add_argument("--xgmi-lat-us", type=float, default=15.0, help="--share model: assumed per-gather latency (us)")
    ap.add_argument("--size", default="", help="WxH override of the config's frame size (exploration runs only)")
    ap.add_argument("--assemble", choices=["ipc", "gather"], default="ipc",
                    help="N > 1 split (and --share): ipc = every rank writes its buckets straight into rank 0's frames "
                         "through an IPC mapping (mrt_ipc_open) and one barrier per step marks the frame whole, no gather "
                         "or unpack (falls back to gather when a rank cannot map them); gather = packed float tiles, one "
                         "RCCL gather to rank 0 and its unpack")
    ap.add_argument("--split-float", action="store_true",
                    help="N > 1 split with --assemble ipc: rank 0's frames also hold the float RGB before Image::Map "
                         "(12 more bytes per pixel across xGMI); by default the split assembles the reference's "
                         "framebuffer, the 8-bit Image (src/Image.cpp:19-35)")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="strong split (N > 1, and --share): frames per step, the first K frames of the config's "
                         "camera path (distinct cameras; frame 0 = the headline camera), each rank's buckets of all of "
                         "them rendered in ONE launch; K > 1 is reported as batched (1..16; 0 = DEFAULT_FPL)")
    ap.add_argument("--latency-frames", type=int, default=5,
                    help="single frames (nothing else in flight) timed after the run for launch_ms / frame latency")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="libmrt tuning switch (mrt_set_tuning) for A/B and profiling runs; reported in the line")
    return ap.parse_args()


# ------------------------------------------------------------------ launcher
def spawn(args):
    """--gpus N without WORLD_SIZE: start N fresh rank processes (one per GPU)
    before anything in this process touches torch / HIP; return rank 0's code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    # poll every rank: when one exits non-zero the others would block in a
    # collective (or in init_process_group) forever, so they are terminated
    # and that rank's code is returned
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


# ------------------------------------------------------------------ helpers
def progress(msg):
    """A progress line on stderr (long configs: a GPU run that prints nothing for
    minutes is taken to be hung)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _camera(c):
    import miro
    cam = miro.Camera()
    cam.setEye(c["eye"]); cam.setLookAt(c["lookAt"]); cam.setUp(c["up"]); cam.setFOV(c["fov"])
    return cam


def _pixels_in_frame(ids, bpf, bx, W, H):
    n = 0
    for i in ids:
        if i < 0:
            continue
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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads():
    """The host cores this process may use: the affinity mask, capped by
    OMP_NUM_THREADS when the environment sets it (the GPU box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(cfg_key, seconds):
    """The CPU oracle (C restatement, OpenMP) on this host's cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from miro import scenes
    cfg = scenes.CONFIGS[cfg_key]
    threads = cpu_threads()
    if cfg["mesh"] == "final":   # the reference's final scene (oracle/final_scene.py)
        from miro import final_scene
        import final_scene as oracle_final
        s, _ = oracle_final.build(final_scene.spec())
        return _cpu_sample(s, cfg_key, cfg, threads, seconds)
    s = O.OracleScene()

    def material(mat):
        return s.add_material(mat["kind"], kd=mat["kd"], specExp=mat.get("specExp", 1.0),
                              specAmt=mat.get("specAmt", 0.0), reflectAmt=mat.get("reflectAmt", 0.0),
                              refractAmt=mat.get("refractAmt", 0.0), ior=mat.get("ior", 1.5),
                              specGloss=mat.get("specGloss", 1.0), translucency=mat.get("translucency", 0.0),
                              le=mat.get("le", (0, 0, 0)), emitted=mat.get("emitted", 0.0),
                              sampleEnv=mat.get("sampleEnv", True), disperse=mat.get("disperse", False),
                              ior3=mat.get("ior3"))

    m = material(cfg["material"])
    if cfg["mesh"] in ("sponza", "sponza_large"):
        s.add_obj(scenes.mesh_obj(cfg), m)
    elif cfg["mesh"] in ("bunny", "instances"):
        if cfg["mesh"] == "bunny":
            s.add_obj(scenes.bunny_obj(), m)
        else:   # two ProxyObject BVHs, instances alternating (as scenes.build_config)
            blas = [s.make_blas([s.add_obj(p, m)]) for p in scenes.proto_objs(cfg)]
            for i, M in enumerate(scenes.instance_transforms(**cfg["instances"])):
                s.add_instance(blas[i % 2], M)
    else:
        import numpy as np
        f = np.load(os.path.join(ROOT, "tests", "golden", "cornell_box_mesh.npz"))
        s.add_mesh(f["verts"], f["normals"], f["vidx"], f["nidx"], m)
    for name, emat in cfg.get("extra", ()):
        s.add_obj(scenes.EXTRA_OBJS[name], material(emat))
    if cfg["mesh"] in ("bunny", "instances"):
        s.add_mesh([(-100, 0, -100), (0, 0, 100), (100, 0, -100)], [(0, 1, 0)] * 3, [(0, 1, 2)], [(0, 1, 2)], m)
    skies = {}

    def sky(spec):
        k = scenes.sky_key(spec)
        if k not in skies:
            skies[k] = s.add_texture(scenes.env_image(spec, hdr_loader=O.hdr_load))
        return skies[k]

    for l in cfg["lights"]:
        if l["type"] == "point":
            s.add_point_light(l["pos"], l["power"])
        elif l["type"] == "dome":
            s.add_dome_light(sky(l["sky"]), l["power"], l.get("samples", 1), l.get("noise", 0.001))
        else:
            s.add_rect_light(l["v1"], l["v2"], l["v3"], l["power"], l.get("samples", 1), l.get("noise", 0.001))
    s.set_bg(cfg["bg"])
    if cfg.get("env"):
        s.set_env_map(sky(cfg["env"]["sky"]), cfg["env"]["exposure"])
    s.set_num_paths(cfg.get("num_paths", 1))
    if cfg.get("path_trace"):
        s.set_path_trace(True, *cfg["path_trace"])
    if cfg.get("subdivs"):
        s.set_subdivs(*cfg["subdivs"])
    s.build()
    return _cpu_sample(s, cfg_key, cfg, threads, seconds)


def _cpu_sample(s, cfg_key, cfg, threads, seconds):
    """Time the oracle scene `s` over row bands of the config's frame for about
    `seconds` CPU-thread-seconds (at most 60 s wall)."""
    W, H = cfg["W"], cfg["H"]
    rays, t_total, frames = 0, 0.0, 0
    band = 64 if not (cfg.get("path_trace") or cfg["mesh"] == "final") else 8
    y = 0
    while t_total * threads < seconds and t_total < 60.0:
        y0 = y % H
        t0 = time.perf_counter()
        r = s.render(cfg["camera"], W, H, rect=(0, y0, W, min(H, y0 + band)), threads=threads, want_hits=False)
        t_total += time.perf_counter() - t0
        rays += r["primary_rays"] + r["shadow_rays"] + r["secondary_rays"]
        y += band
        frames += 1
    value = rays / t_total / 1e6
    omp = os.environ.get("OMP_NUM_THREADS")
    out = {"value": round(value, 3), "unit": "Mray/s", "cores": threads, "kind": "port",
           "cpu": cpu_model(), "affinity_cpus": len(os.sched_getaffinity(0)),
           "cores_reason": (f"OMP_NUM_THREADS={omp}: the CPU share the GPU pool grants one GPU's job (the affinity "
                            f"mask lists the whole host, whose other cores belong to other GPUs' jobs)")
           if omp and omp.isdigit() and int(omp) < len(os.sched_getaffinity(0)) else "every core in the affinity mask",
           "sample": f"{cfg_key} {W}x{H}: {frames} bands of {band} rows ({rays} rays, {t_total:.1f} s wall, "
                     f"{threads} OpenMP threads, oracle/mrt_oracle.c -O2)"}
    if os.path.exists(CPU_CAL_FILE):   # oracle vs the reference's own 1-thread rate, same Xeon
        cal = json.load(open(CPU_CAL_FILE))
        out["reference_equivalent"] = round(value * cal["ratio_reference_over_oracle"], 3)
        out["calibration"] = (f"x{cal['ratio_reference_over_oracle']}: the reference renders explosion01 1920x1080 "
                              f"at {cal['reference_mray_s'][0]}-{cal['reference_mray_s'][1]} Mray/s on 1 thread, the "
                              f"oracle at {cal['oracle_mray_s']} on the same {cal['cpu']} "
                              f"(profiles/r02_cpu_calibration.json); ASSUMED to carry over to this host's CPU: the "
                              f"reference (SSE, MSVC-shaped) cannot be built or run on the GPU box, so the ratio is "
                              f"measured on the build container's Intel CPU only")
    return out


def _scene_setup(scene):
    """One-time host BVH::build (src/BVH.cpp:457-575), outside the timed region."""
    ms = getattr(scene, "bvh_build_ms", None)
    prims = scene.bvh_info["prims"]
    return {"bvh_build_ms": None if ms is None else round(ms, 2), "prims": prims,
            "build_mprims_per_s": None if not ms else round(prims / ms / 1e3, 3),
            # instanced scenes: the BLAS builds (mrt_scene_make_blas) happen before the world QBVH
            "blas_build_ms": round(getattr(scene, "blas_build_ms", 0.0), 2),
            "blas_prims": getattr(scene, "blas_prims", 0)}


def step_trace_evidence(config):
    """This config's tracked kernel trace of a driver-settings run (profiles/r06_steptrace.json,
    tools/step_trace.py): kernel-busy union per timed step, overlap, per-step fraction."""
    if not os.path.exists(STEP_TRACE_FILE):
        return None
    rec = json.load(open(STEP_TRACE_FILE)).get("configs", {}).get(config)
    if not rec:
        return None
    keep = ("busy_union_ms_per_step", "ms_per_step_traced_run", "union_over_step", "kernel_sum_over_union",
            "frac_l2_per_step", "frac_hbm_per_step", "dispatches_per_step", "command", "source")
    return {k: rec[k] for k in keep if k in rec}


def profile_evidence(config):
    """This config's tracked rocprofv3 record (profiles/r06_profile.json): per pass
    {hbm_bytes, avg_us, kernels}, per kernel {latency, code_object, ...}, source."""
    if not os.path.exists(PROFILE_FILE):
        return None
    return json.load(open(PROFILE_FILE)).get("configs", {}).get(config)


# ------------------------------------------------------------------ worker
def main():
    args = parse()
    sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
    from miro import scenes as _scenes   # (imports no torch / HIP)
    if not args.inflight:   # the config's frames in flight
        args.inflight = int(_scenes.CONFIGS[args.config].get("inflight", 4))
    # hardware queues of this process's HIP runtime (read when HIP initialises, so before
    # torch is imported): one per frame in flight.  With HIP's default 4 the N = 1 pipeline
    # holds at most 4 frames, so a frame whose latency is set by a few heavy tiles caps
    # the step at latency / 4 (C2: 0.2011 -> 0.1644 ms per step with 8)
    # (the GPU box's environment sets GPU_MAX_HW_QUEUES=4, HIP's default, so a larger need replaces it)
    want_q = min(32, max(4, args.inflight))
    try:
        have_q = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        have_q = 0
    if have_q < want_q:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn(args))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}")
    import numpy as np
    import torch
    import torch.distributed as dist
    import miro
    from miro import _lib, scenes
    from miro import tiles as tiles_mod

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MRT_BENCH_REHEARSE=gloo: the N > 1 path rehearsed on ONE GPU -- every rank on cuda:0, the
    # collectives over gloo through host copies (_HostDist); its numbers mean nothing, its job
    # is to run the multi-rank code (split pipeline, timing, the JSON line) where only one GPU is
    rehearse = world > 1 and os.environ.get("MRT_BENCH_REHEARSE") == "gloo"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import datetime
        if rehearse:
            torch.cuda.set_device(0)
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=300))
            dist = _HostDist(dist, torch)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=datetime.timedelta(seconds=300))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    # the config's own switches (miro/scenes.py "tune": a measured per-scene choice, e.g. C3's
    # nested camera-ray walk), then --tune on top; both reported in the line
    tuning = dict(_scenes.CONFIGS[args.config].get("tune", {}))
    for kv in args.tune:
        k, v = kv.split("=")
        tuning[k] = int(v)
    for k, v in tuning.items():
        _lib.check(miro.lib().mrt_set_tuning(k.encode(), int(v)), f"tuning {k}")
    progress(f"building {args.config}")
    scene, cam, cfg = scenes.build_config(args.config, device=dev)
    progress(f"built: {scene.bvh_info['prims']} world objects")
    if args.size:   # exploration only: the line's config reports the size used
        w_, h_ = (int(x) for x in args.size.lower().split("x"))
        cfg = dict(cfg, W=w_, H=h_, name=cfg["name"] + f" (at {w_}x{h_})")
    W, H = cfg["W"], cfg["H"]
    L = miro.lib()
    stream = torch.cuda.current_stream()
    # N = 1: one frame per step through the whole-frame path.  N > 1 (default
    # --split frame): the north-star split, ONE frame per step, its 32x32 buckets
    # dealt id mod N, float tiles, one RCCL gather of the framebuffer to rank 0,
    # consecutive frames double-buffered (BatchPipeline); --split batch: weak
    # scaling, a camera path of N frames per step (8-bit tiles), measured as the
    # secondary key of the split line.
    # (--path batch at N = 1 runs the split path on one GPU: same pipeline, N = 1)
    split = (world > 1 and args.split == "frame") or (world == 1 and args.path == "batch")
    fpl = max(1, min(16, args.frames_per_launch or DEFAULT_FPL))
    n_frames = (fpl if split else 1) if (world == 1 or split) else (args.frames or min(world, 16))
    bx, by = (W + 31) // 32, (H + 31) // 32
    bpf = bx * by
    use_frame_path = world == 1 and n_frames == 1 and args.path == "auto"
    inflight = max(1, args.inflight) if use_frame_path else 1
    streams = [stream] + [torch.cuda.Stream() for _ in range(inflight - 1)]
    frame = [torch.empty(H * W * 3, dtype=torch.float32, device="cuda") for _ in range(inflight)]
    frame8 = [torch.empty(H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(inflight)]
    opts_count = _lib.mrt_render_opts(W, H, dev, 1, 1, 0, 0)
    opts = _lib.mrt_render_opts(W, H, dev, 0, 1, 0, 0)
    camc = (_lib.mrt_camera * 1)(cam._c())

    depth = max(1, args.inflight)

    def make_pipe(nf, float_tiles, nsplit=None, srank=None, pipe_streams=None, share_unpack="own"):
        """This rank's share of an nf-frame step (items id mod N), its render /
        unpack closures and the gather pipeline over `depth` buffers and streams
        (--inflight).  nsplit / srank: the share of rank srank of an nsplit-way
        split rendered without the gather (bench.py --share); share_unpack "none":
        no unpack (a rank > 0 of the split only renders and sends), "full": rank 0's
        unpack of all nsplit shares' tiles each step (its buffers hold nsplit shares).
        The nf frames are the first nf frames of the config's camera path (frame 0 is
        the headline camera)."""
        nsplit = world if nsplit is None else nsplit
        srank = rank if srank is None else srank
        cc = path_cameras(nf)
        mine, all_ids, per = tiles_mod.split_items(bpf * nf, nsplit, srank)
        shares = 1
        if nsplit != world and share_unpack != "full":   # one share on its own: its unpadded items are the whole "gathered" buffer
            all_ids = mine
        elif nsplit != world:   # rank 0 of the split: every share's (padded) tiles unpacked each step
            shares = nsplit
        items = torch.tensor(mine, dtype=torch.int32, device="cuda")
        all_items = torch.tensor(all_ids, dtype=torch.int32, device="cuda")
        out_f = [torch.empty(nf * H * W * 3, dtype=torch.float32, device="cuda") for _ in range(depth)] \
            if float_tiles else None
        out_8 = [torch.empty(nf * H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(depth)]
        dt = torch.float32 if float_tiles else torch.uint8

        def render(ids, out, o=opts):
            tf, t8 = (out.data_ptr(), None) if float_tiles else (None, out.data_ptr())
            _lib.check(L.mrt_render_batch_async(scene.handle, cc, nf, C.byref(o), ids.data_ptr(), len(mine), tf, t8,
                                                torch.cuda.current_stream().cuda_stream), "render batch")

        def unpack(ids, gathered, b):
            if share_unpack == "none":
                return
            gf, g8 = (gathered.data_ptr(), None) if float_tiles else (None, gathered.data_ptr())
            _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), len(ids), gf, g8, W, H, nf,
                                                out_f[b].data_ptr() if float_tiles else None, out_8[b].data_ptr(),
                                                scene.handle, torch.cuda.current_stream().cuda_stream), "unpack")

        # `depth` streams: consecutive steps' launches overlap (libmrt keeps scratch per stream)
        pipe = tiles_mod.BatchPipeline(world, rank, dist, items, all_items,
                                       lambda k: torch.empty(k * shares * per * 1024 * 3, dtype=dt, device="cuda"),
                                       render, unpack,
                                       streams=pipe_streams or [torch.cuda.Stream() for _ in range(depth)])
        for b in range(depth):   # per-stream scratch allocated before any timing
            with torch.cuda.stream(pipe.streams[b]):
                render(items, pipe.tiles[b])
        torch.cuda.synchronize()
        pipe.out_f, pipe.out_8 = out_f, out_8   # rank 0's assembled frames, one per buffer
        return pipe, render, items, mine, out_f

    def path_cameras(nf):
        """mrt_camera[nf]: the first nf frames of the config's camera path (frame 0 = the headline camera)."""
        cams_ = [cam] if nf == 1 else [_camera(c) for c in scenes.camera_path(cfg["camera"], nf)]
        return (_lib.mrt_camera * nf)(*[c._c() for c in cams_])

    def hip_rt():
        """The HIP runtime torch and libmrt share (one per process)."""
        lib_ = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
        h_ = C.CDLL(lib_ if os.path.exists(lib_) else "libamdhip64.so")
        h_.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        return h_

    def make_ipc_pipe(nf, nsplit=None, srank=None, pipe_streams=None):
        """The split with direct writes (--assemble ipc): rank 0 owns `depth` frame buffers
        (nf frames each: the 8-bit framebuffer, Image::m_pixels, and with --split-float the
        float frame before Image::Map), exports them (mrt_ipc_export), every rank maps
        them (mrt_ipc_open) and renders its buckets of each step straight into buffer
        k % depth (mrt_render_batch_frames_async); one stream-ordered all-reduce of one
        int per step is the frame-end barrier (tiles.FramePipeline).  nsplit / srank: one
        rank's share rendered alone on this GPU into local frames (--share: no barrier).
        Returns (pipe, render(b, opts), mine, frames) or raises when a rank cannot map."""
        nsplit = world if nsplit is None else nsplit
        srank = rank if srank is None else srank
        nb = len(pipe_streams) if pipe_streams else max(2, depth)   # frame buffers (FramePipeline needs 2)
        cc = path_cameras(nf)
        mine = tiles_mod.rank_buckets(bpf * nf, nsplit, srank)
        items = torch.tensor(mine, dtype=torch.int32, device="cuda")
        alone = nsplit != world
        owner = alone or rank == 0
        # per buffer: (float frames or None, 8-bit frames)
        own = [(torch.empty(nf * H * W * 3, dtype=torch.float32, device="cuda") if args.split_float else None,
                torch.empty(nf * H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(nb)] if owner else None
        ptrs, opened, err = [], [], ""

        def ptr(t):
            return None if t is None else t.data_ptr()
        if alone or world == 1:
            ptrs = [(ptr(f), ptr(f8)) for f, f8 in own]
        else:
            obj = [None]
            if rank == 0:
                try:
                    hs = []
                    for pair in own:
                        for t in pair:
                            if t is None:
                                hs.append(None)
                                continue
                            h = _lib.mrt_ipc_handle()
                            _lib.check(L.mrt_ipc_export(C.c_void_p(t.data_ptr()), C.byref(h)), "ipc export")
                            hs.append(bytes(h))
                    obj = [hs]
                except Exception as e:   # reported through the agreement below
                    err = repr(e)
            dist.broadcast_object_list(obj, src=0)
            try:
                if rank == 0:
                    ptrs = [(ptr(f), ptr(f8)) for f, f8 in own]
                elif obj[0] is None:
                    err = "rank 0 could not export its frames"
                else:
                    for i in range(nb):
                        pair = []
                        for j in range(2):
                            hb = obj[0][2 * i + j]
                            if hb is None:
                                pair.append(None)
                                continue
                            h = _lib.mrt_ipc_handle.from_buffer_copy(hb)
                            p = C.c_void_p()
                            _lib.check(L.mrt_ipc_open(C.byref(h), dev, C.byref(p)), "ipc open")
                            opened.append(p.value)
                            # the mapping must be usable before a kernel stores through it: a 4-byte
                            # copy from it through the HIP runtime (an error here falls back to the
                            # gather; a bad mapping met by a kernel would fault instead)
                            probe = (C.c_uint8 * 4)()
                            if hip_rt().hipMemcpy(probe, C.c_void_p(p.value), C.c_size_t(4), 2) != 0:   # DtoH
                                raise RuntimeError("rank 0's frame mapped but not readable from this device")
                            pair.append(p.value)
                        ptrs.append(tuple(pair))
            except Exception as e:
                err = repr(e)
            # every rank takes the same decision: all mapped, or all fall back
            ok = torch.tensor([0.0 if err else 1.0], dtype=torch.float64, device="cuda")
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if ok.item() < 1.0:
                for p in opened:
                    L.mrt_ipc_close(C.c_void_p(p))
                raise RuntimeError(err or "another rank could not map rank 0's frames")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")

        def render(b, o=opts):
            _lib.check(L.mrt_render_batch_frames_async(scene.handle, cc, nf, C.byref(o), items.data_ptr(), len(mine),
                                                       ptrs[b][0], ptrs[b][1],
                                                       torch.cuda.current_stream().cuda_stream), "render frames")

        def barrier():
            if alone or world == 1:
                return None
            return dist.all_reduce(flag, async_op=True)

        pipe = tiles_mod.FramePipeline(world if not alone else 1, rank if not alone else 0, render, barrier, None,
                                       streams=pipe_streams or [torch.cuda.Stream() for _ in range(nb)])
        for b in range(nb):   # per-stream scratch allocated before any timing
            with torch.cuda.stream(pipe.streams[b]):
                render(b)
        torch.cuda.synchronize()
        if not alone and world > 1:
            dist.barrier()
        pipe.own, pipe.opened, pipe.items_n = own, opened, len(mine)
        return pipe, render, mine, own

    def count_rays(render_count):
        """Rays of one step over all ranks from an instrumented launch (+ this rank's stats)."""
        render_count()
        torch.cuda.synchronize()
        st_ = scene.stats()
        adaptive_ = bool(cfg.get("subdivs")) and max(cfg["subdivs"][:2]) > 1
        v = [st_["shadow_rays"], st_["primary_rays"] if adaptive_ else 0, st_["secondary_rays"]]
        if world > 1:
            t_ = torch.tensor(v, dtype=torch.float64, device="cuda")
            dist.all_reduce(t_)
            v = [int(x) for x in t_.tolist()]
        return st_, v

    region = {}

    def clocks():
        return {"monotonic_ns": time.clock_gettime_ns(time.CLOCK_MONOTONIC),
                "boottime_ns": time.clock_gettime_ns(time.CLOCK_BOOTTIME)}

    settle = {}

    def timed(step_fn, flush, k):
        # clock settle before the warmup: the GPU renders groups of `inflight` steps until
        # --settle-s of wall time have passed, so clocks and caches are at their sustained
        # state when the W warmup steps start (C3, one box: 20 steps after 5 warmups 0.444 ms
        # per step, after 20 warmups 0.424, 100 steps 0.414)
        # (N > 1: every rank takes the same decision from the slowest rank's clock, so all
        # ranks run the same steps and their gathers pair up)
        t_s, n_s = time.perf_counter(), 0
        while True:
            e_s = time.perf_counter() - t_s
            if world > 1:
                t_ = torch.tensor([e_s], dtype=torch.float64, device="cuda")
                dist.all_reduce(t_, op=dist.ReduceOp.MAX)
                e_s = t_.item()
            if e_s >= args.settle_s:
                break
            for _ in range(max(1, inflight, depth if not use_frame_path else 1)):
                step_fn()
            n_s += max(1, inflight, depth if not use_frame_path else 1)
            flush()
            torch.cuda.synchronize()
        if not settle:
            settle.update({"seconds": round(time.perf_counter() - t_s, 3), "steps": n_s})
        for _ in range(args.warmup):
            step_fn()
        flush()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        c0 = clocks()
        t0_ = time.perf_counter()
        for _ in range(k):
            step_fn()
        flush()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        e = time.perf_counter() - t0_
        c1 = clocks()
        # the timed region on the host clocks a kernel trace may use (tools/step_trace.py
        # selects the dispatches inside it); the first timed region is the headline's
        if not region:
            region.update({key: [c0[key], c1[key]] for key in c0})
        if world > 1:
            t_ = torch.tensor([e], dtype=torch.float64, device="cuda")
            dist.all_reduce(t_, op=dist.ReduceOp.MAX)
            e = t_.item()
        return e

    nstep = [0]

    def frame_step(o=opts, serial=False):
        i = 0 if serial else nstep[0] % inflight
        nstep[0] += 1
        _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc[0]), C.byref(o), frame[i].data_ptr(),
                                            frame8[i].data_ptr(), streams[i].cuda_stream), "render")

    def check_timed_frame(t_f, t_8):
        """The last timed frame (rank 0's assembled frame at N > 1) against the same
        camera rendered once on its own through mrt_render_frame_async, the path the
        full-size parity tests compare with the oracle (tests/test_full_size.py):
        sha256 of the float and 8-bit frames, after the timed region."""
        import hashlib
        torch.cuda.synchronize()
        ref_f = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
        ref_8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
        _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc[0]), C.byref(opts), ref_f.data_ptr(),
                                            ref_8.data_ptr(), stream.cuda_stream), "render (frame check)")
        torch.cuda.synchronize()

        def digest(a, b):
            h = hashlib.sha256()
            if a is not None:
                h.update(a.reshape(-1)[:H * W * 3].cpu().numpy().tobytes())
            h.update(b.reshape(-1)[:H * W * 3].cpu().numpy().tobytes())
            return h.hexdigest()[:16]
        got, ref = digest(t_f, t_8), digest(ref_f if t_f is not None else None, ref_8)
        return {"timed_frame_sha256": got, "single_frame_sha256": ref, "equal": got == ref,
                "compared": ("float + 8-bit" if t_f is not None else "8-bit") + " RGB of the last timed step's frame"}

    adaptive = bool(cfg.get("subdivs")) and max(cfg["subdivs"][:2]) > 1
    assemble = None
    if args.share:
        share_mode(args, dict(scene=scene, cfg=cfg, W=W, H=H, bpf=bpf, L=L, _lib=_lib, tiles_mod=tiles_mod, torch=torch, np=np, make_pipe=make_pipe, make_ipc_pipe=make_ipc_pipe, count_rays=count_rays, timed=timed, frame_step=frame_step, streams=streams, frame=frame, frame8=frame8, opts=opts, opts_count=opts_count, camc=camc, adaptive=adaptive, inflight=inflight), [int(x) for x in args.share.split(",") if x.strip()])
        return
    if use_frame_path:
        # setup: every in-flight stream renders once, so libmrt's per-stream scratch
        # (hit records, stacks, counters) is allocated before the warmup / timed steps
        for i in range(inflight):
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc[0]), C.byref(opts), frame[i].data_ptr(),
                                                frame8[i].data_ptr(), streams[i].cuda_stream), "render")
        torch.cuda.synchronize()
        progress("setup frames done; instrumented frame")
        st, (shadow_total, eye_total, second_total) = count_rays(lambda: frame_step(opts_count, serial=True))
        mine, items = None, None
        progress("timed region")
        elapsed = timed(frame_step, lambda: None, args.steps)
        last = (nstep[0] - 1) % inflight
        frame_check = check_timed_frame(frame[last], frame8[last])
    else:
        assemble = "gather"
        if split and args.assemble == "ipc":
            try:
                pipe, render_b, mine, own = make_ipc_pipe(n_frames)
                assemble = "ipc"
            except Exception as e:   # every rank took the same decision (make_ipc_pipe)
                assemble = f"gather (ipc unavailable: {e})"
                progress(f"IPC frame mapping failed ({e}); the split gathers tiles instead")
        if assemble == "ipc":
            def render_one(o=opts):
                render_b(0, o)
            items = None
            st, (shadow_total, eye_total, second_total) = count_rays(lambda: render_one(opts_count))
            elapsed = timed(pipe.step, pipe.flush, args.steps)
            last = (pipe.k - 1) % pipe.depth
            frame_check = check_timed_frame(own[last][0], own[last][1]) if rank == 0 else None
            out_bytes_px = 3 + (12 if args.split_float else 0)
        else:
            pipe, render, items, mine, _ = make_pipe(n_frames, float_tiles=split)

            def render_one(o=opts):
                render(items, pipe.tiles[0], o)
            st, (shadow_total, eye_total, second_total) = count_rays(lambda: render_one(opts_count))
            elapsed = timed(pipe.step, pipe.flush, args.steps)
            last = (pipe.k - 1) % pipe.depth
            frame_check = check_timed_frame(pipe.out_f[last] if split else None, pipe.out_8[last]) \
                if rank == 0 and (n_frames == 1 or split) else None
    shadow_mine, eye_mine, second_mine = st["shadow_rays"], (st["primary_rays"] if adaptive else 0), st["secondary_rays"]
    primary_total = eye_total if adaptive else n_frames * W * H
    rays_per_step = primary_total + shadow_total + second_total      # all frames of the batch, all ranks
    hits_px = st["primary_hits"]

    # N > 1: per-rank render and assembly times of the split (median of 5, each
    # alone: render = HIP events of one launch on this rank's stream; ipc: one frame-end
    # barrier (all-reduce of one int) between barriers, gather: one RCCL gather of the
    # tile buffer), and the weak-scaling batch of N frames per step as the secondary key
    split_times, weak = None, None
    if world > 1 and split:
        r_ms, g_ms = [], []
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            dist.barrier()
            e0.record()
            render_one()
            e1.record()
            torch.cuda.synchronize()
            r_ms.append(e0.elapsed_time(e1))
            dist.barrier()
            tg = time.perf_counter()
            if assemble == "ipc":
                dist.all_reduce(flag)
            else:
                dist.gather(pipe.tiles[0], list(pipe.recv[0].chunk(world)) if rank == 0 else None, dst=0)
            torch.cuda.synchronize()
            g_ms.append((time.perf_counter() - tg) * 1e3)
        t_ = torch.tensor([float(np.median(r_ms)), float(np.median(g_ms))], dtype=torch.float64, device="cuda")
        dist.all_reduce(t_, op=dist.ReduceOp.MAX)
        if assemble == "ipc":
            split_times = {"render_ms_max_rank": round(t_[0].item(), 4), "barrier_ms": round(t_[1].item(), 4),
                           "assemble": "ipc: every rank's kernel stores its buckets' pixels into rank 0's frames "
                                       "(mrt_ipc_open mapping, xGMI); no gather, no unpack",
                           "framebuffer": "RGB8 (Image::m_pixels)" + (" + float RGB" if args.split_float else ""),
                           "remote_bytes_per_rank_max": int(max(0, len(mine)) * 1024 * out_bytes_px)}
        else:
            split_times = {"render_ms_max_rank": round(t_[0].item(), 4), "gather_ms": round(t_[1].item(), 4),
                           "assemble": assemble, "gather_bytes_per_rank": int(pipe.tiles[0].numel() * 4)}
        # the same split at ONE frame per step (frames_per_step 1: strong scaling of a single frame,
        # whose 1/N share cannot fill the GPU)
        single = None
        if n_frames > 1:
            try:
                if assemble == "ipc":
                    spipe, srender_b, smine, _ = make_ipc_pipe(1)

                    def srender_one(o=opts):
                        srender_b(0, o)
                else:
                    spipe, srender, sitems, smine, _ = make_pipe(1, float_tiles=True)

                    def srender_one(o=opts):
                        srender(sitems, spipe.tiles[0], o)
                _, (ssh, seye, ssec) = count_rays(lambda: srender_one(opts_count))
                s_rays = (seye if adaptive else W * H) + ssh + ssec
                se = timed(spipe.step, spipe.flush, args.steps)
                single = {"value": round(s_rays * args.steps / se / 1e6, 2), "unit": "Mray/s", "scaling": "strong",
                          "frames_per_step": 1, "steps": args.steps, "ms_per_step": round(se / args.steps * 1e3, 4),
                          "split": "one frame (the headline camera) per step, the same split and assembly"}
                if assemble == "ipc":
                    torch.cuda.synchronize()
                    dist.barrier()
                    for p_ in spipe.opened:
                        L.mrt_ipc_close(C.c_void_p(p_))
            except Exception as e:   # reported, never fatal
                single = {"error": repr(e)}
        nf_w = args.frames or min(world, 16)
        wpipe, wrender, witems, _, _ = make_pipe(nf_w, float_tiles=False)
        _, (wsh, weye, wsec) = count_rays(lambda: wrender(witems, wpipe.tiles[0], opts_count))
        w_rays = (weye if adaptive else nf_w * W * H) + wsh + wsec
        k_w = args.strong_steps or args.steps
        we = timed(wpipe.step, wpipe.flush, k_w)
        weak = {"value": round(w_rays * k_w / we / 1e6, 2), "unit": "Mray/s", "scaling": "weak",
                "frames_per_step": nf_w, "steps": k_w, "ms_per_step": round(we / k_w * 1e3, 4),
                "split": f"{nf_w}-frame camera path per step, 32x32 buckets of all frames dealt id mod {world}, one "
                         f"RCCL gather of 8-bit tiles per step (double-buffered)"}

    # per-launch durations of the uninstrumented kernels (HIP events on the
    # launch's stream), and the latency of one frame with nothing else in flight
    prim_ms, shade_ms, lat_ms = [], [], []
    progress("latency frames")
    for _ in range(max(1, args.latency_frames)):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if use_frame_path:
            frame_step(opts, serial=True)
        else:
            render_one()
        torch.cuda.synchronize()
        lat_ms.append((time.perf_counter() - t1) * 1e3)
        s2 = scene.stats()
        prim_ms.append(s2["primary_ms"])
        shade_ms.append(s2["shade_ms"])
    if split and world > 1 and assemble == "ipc":   # unmap rank 0's frames once every rank is done with them
        torch.cuda.synchronize()
        dist.barrier()
        for p_ in pipe.opened:
            L.mrt_ipc_close(C.c_void_p(p_))
    if rank != 0:
        dist.destroy_process_group()
        return
    value = rays_per_step * args.steps / elapsed / 1e6
    px_mine = W * H if use_frame_path else _pixels_in_frame(sorted(set(mine)), bpf, bx, W, H)
    hits_mine = hits_px
    # the specialised kernel runs for one point light, one path and no environment map
    chain = scenes.chain_level(cfg)
    one_light = (len(cfg["lights"]) == 1 and cfg["lights"][0]["type"] == "point" and cfg.get("num_paths", 1) == 1
                 and not cfg.get("env") and chain == 0 and not cfg.get("extra"))
    # float RGB is written by the frame path and the split's tiles; the IPC split writes the 8-bit framebuffer only
    float_out = use_frame_path or (split and (assemble != "ipc" or args.split_float))
    b_prim, b_shade = kernel_bytes(st, px_mine, hits_mine, float_out=float_out,
                                   wavefront=not one_light and chain == 0)
    if chain:   # each secondary / GI hit gathers its PrimShade + 3 vertices + 3 normals (+ its level record)
        b_shade += second_mine * (16 + 32 + 3 * 16 + 3 * 16 + 12)
    pm, sm = float(np.median(prim_ms)), float(np.median(shade_ms))
    shade_name = ("shade1_kernel (shade + any-hit shadow rays)" if one_light else
                  "chain engine (per level: chain gen + compact + chain_trace [closest hits + any-hit shadow rays]; "
                  "resolve + combine)" if chain else
                  "shade pass (shade_kernel<gen> + shadow_kernel any-hit + shade_kernel<resolve>)")
    if st.get("fused"):   # frame1_kernel: the whole frame in one launch (its time is primary_ms)
        dom, dom_key, dom_ms = ("frame1_kernel (camera rays + closest hit + shading + any-hit shadow rays, "
                                "one launch)"), "primary", pm
        dom_b = (st["node_visits"] * NODE_B + st["leaf_visits"] * LEAF_B
                 + px_mine * ((12 if float_out else 0) + 3) + hits_px * (32 + 3 * 16 + 3 * 16))
    elif adaptive and st.get("chain"):   # adaptive passes, each a chain-engine tree walk (G3)
        dom, dom_key, dom_ms, dom_b = ("chain engine, adaptive passes (per pass: unit_eye + per level chain gen + compact "
                                       "+ chain_trace + resolve, per-level folds, adapt_combine)"), "shade", sm, b_shade
    elif adaptive:   # one fused launch: eye rays, shading, inline shadow rays (its time is shade_ms)
        dom, dom_key, dom_ms = "adaptive_kernel (eye rays + shading + any-hit shadow rays)", "shade", sm
        dom_b = (st["node_visits"] * NODE_B + st["leaf_visits"] * LEAF_B
                 + px_mine * (16 + (12 if use_frame_path else 0) + 3) + hits_px * (32 + 3 * 16 + 3 * 16))
    elif sm >= pm:
        dom, dom_key, dom_ms, dom_b = shade_name, "shade", sm, b_shade
    else:
        dom, dom_key, dom_ms, dom_b = "primary_kernel (camera rays, closest hit)", "primary", pm, b_prim
    achieved = dom_b / (dom_ms * 1e-3) / 1e9
    # the whole step: algorithmic bytes of every pass of one step (all frames of the
    # step on this rank) over the timed ms_per_step -- what the timed region achieved,
    # frames in flight included (the per-launch `frac` above is one launch alone)
    ms_step = elapsed / args.steps * 1e3
    step_b = (dom_b if st.get("fused") or adaptive else b_prim + b_shade) * (n_frames if not split else 1)
    step_gbs = step_b / (ms_step * 1e-3) / 1e9
    prof = profile_evidence(args.config) if use_frame_path else None
    ppass = ((prof or {}).get("passes") or {}).get(dom_key) or {}
    dom_traffic = ppass.get("hbm_bytes") or None
    hbm = None
    if dom_traffic:
        hbm_gbs = dom_traffic / (dom_ms * 1e-3) / 1e9
        hbm = {"achieved": round(hbm_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(hbm_gbs / HBM_PEAK_GBS, 4), "bytes_per_launch": int(dom_traffic),
               "source": prof.get("source")}
    # the tracked rocprofv3 average of the same pass (one frame in flight): the
    # fraction recomputed from it must agree with `frac` (HIP events, live)
    tracked = None
    if ppass.get("avg_us"):
        f_t = dom_b / (ppass["avg_us"] * 1e-6) / 1e9 / L2_PEAK_GBS
        tracked = {"avg_us": ppass["avg_us"], "frac": round(f_t, 4), "kernels": ppass.get("kernels"),
                   "source": prof.get("source")}
    per_step = {"algorithmic_bytes_per_step": int(step_b), "ms_per_step": round(ms_step, 4),
                "achieved": round(step_gbs, 1), "unit": "GB/s",
                "frac_l2": round(step_gbs / L2_PEAK_GBS, 4), "frac_hbm": round(step_gbs / HBM_PEAK_GBS, 4)}
    frame_hbm = sum((p_ or {}).get("hbm_bytes") or 0 for p_ in ((prof or {}).get("passes") or {}).values())
    if frame_hbm:   # PMC DRAM-side bytes of one frame (tracked profile) over the timed step
        per_step["hbm_traffic_per_step"] = int(frame_hbm)
        per_step["hbm_frac_counters"] = round(frame_hbm / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    st_rec = step_trace_evidence(args.config)
    if st_rec:      # the kernel trace of this config's driver-settings run: busy union per step
        per_step["tracked_trace"] = st_rec
    # latency evidence of the pass's longest kernel (SQ wave-state shares, VALU busy,
    # L2 requests per vector load): why neither bandwidth roofline binds
    latency = None
    # (the pass's most-dispatched kernel: the timed instantiation, not the walk-exit probe's few launches)
    for kname, ent in sorted(((prof or {}).get("kernels") or {}).items(),
                             key=lambda kv: (-kv[1].get("dispatches", 0), -kv[1].get("avg_us", 0))):
        if kname in (ppass.get("kernels") or []) and ent.get("latency"):
            latency = dict(ent["latency"], kernel=kname)
            if ent.get("code_object"):
                latency["code_object"] = ent["code_object"]
            break
    # SURVEY.md 8(d)'s own pricing of the same bytes: algorithmic bytes against HBM.  Above 1
    # it is non-physical -- those node / leaf bytes are served by L1 (98% hits) and L2, and the
    # PMC-measured DRAM-side bytes (`hbm`, per_step.hbm_frac_counters) are a few % of HBM
    hbm_alg = {"frac_per_launch": round(achieved / HBM_PEAK_GBS, 4), "frac_per_step": round(step_gbs / HBM_PEAK_GBS, 4),
               "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "note": "SURVEY.md 8(d) pricing (algorithmic bytes / 8 TB/s); non-physical above 1: the bytes are "
                       "served by L1 / L2, not HBM (see hbm / per_step.hbm_frac_counters for the DRAM-side bytes)"}
    # latency model of the one-launch frame kernel.  Every wave walks its tiles' rays one
    # dependent node step at a time (a step = node fetch -> box test -> stack op, plus the
    # step's leaf triangles, for the whole wave); count mode counts those wave steps.  The
    # launch's SIMD-cycles divided by them give the SIMD time one wave step costs; the
    # tracked profile's VALU instruction count (SQ_INSTS_VALU, 2 cycles per wave64 op on a
    # SIMD-32, MI355X_MICROARCH.md) gives the part of it spent issuing VALU, and the rest is
    # latency the other resident waves did not cover.
    lat_model = None
    wsteps = st.get("primary_wave_steps", 0) + st.get("shadow_wave_steps", 0)
    if st.get("fused") and wsteps:
        simds = 4 * int(torch.cuda.get_device_properties(dev).multi_processor_count)
        waves = int(tuning.get("frame1_waves", 7))
        clk = float((latency or {}).get("clock_ghz") or 2.4)
        simd_cyc = dom_ms * 1e-3 * clk * 1e9 * simds / wsteps
        lat_model = {
            "wave_steps_per_frame": int(wsteps), "resident_waves": simds * waves, "waves_per_simd": waves,
            "steps_per_wave": round(wsteps / (simds * waves), 1), "clock_ghz": clk,
            "simd_cycles_per_wave_step": round(simd_cyc, 1),
            "wave_cycles_per_step": round(simd_cyc * waves, 0),
            "lane_use": round((st["primary_node_visits"] + st.get("shadow_node_visits", 0)) / (64.0 * wsteps), 4)}
        # the timed steps keep several frames in flight, so the launch tails overlap: the same
        # wave steps over ms_per_step (per frame) give the steady-state SIMD time per step
        pipe_cyc = elapsed / args.steps / max(1, n_frames) * clk * 1e9 * simds / wsteps
        lat_model["pipelined_simd_cycles_per_wave_step"] = round(pipe_cyc, 1)
        vpw = (latency or {}).get("valu_insts_per_wave")
        if vpw and (latency or {}).get("waves"):
            valu_step = vpw * latency["waves"] / wsteps
            lat_model.update({
                "valu_insts_per_wave_step": round(valu_step, 1),
                "valu_issue_cycles_per_step": round(2 * valu_step, 1),
                "valu_issue_share": round(2 * valu_step / simd_cyc, 3),
                "pipelined_valu_issue_share": round(2 * valu_step / pipe_cyc, 3),
                "uncovered_latency_cycles_per_step": round(simd_cyc - 2 * valu_step, 1),
                "source": "valu counts from the tracked profile (%s)" % (prof or {}).get("source")})
            lat_model["reading"] = (
                "one launch alone: a SIMD spends %.0f cycles per wave step, %.0f%% of them issuing its %.0f VALU "
                "instructions (2 cycles each) and the rest with all %d resident waves waiting on dependent node / "
                "triangle fetches (L1 / L2 hits, 180-225+ cycles each, MI355X_MICROARCH.md) or in the launch's "
                "ramp and tail. In the timed steps (frames in flight, tails overlapped) a step costs %.0f SIMD "
                "cycles, %.0f%% of them VALU issue: the frame is bound by VALU issue first and dependent-fetch "
                "latency second. Bandwidth is not the bound: L2 frac %.2f, counter HBM frac %s."
                % (simd_cyc, 100 * 2 * valu_step / simd_cyc, valu_step, waves, pipe_cyc, 100 * 2 * valu_step / pipe_cyc,
                   achieved / L2_PEAK_GBS, "n/a" if hbm is None else "%.3f" % hbm["frac"]))
        else:
            lat_model["reading"] = ("a SIMD spends %.0f cycles per wave step (%d waves resident); no tracked VALU "
                                    "counts for this config, so the issue / latency split is not given"
                                    % (simd_cyc, waves))
    # primary-kernel lanes doing node work per issued wave step (adaptive: no primary launch)
    lane_util = round(st["primary_node_visits"] / (64 * st["primary_wave_steps"]), 4) if st["primary_wave_steps"] else None
    out = {
        "metric": ("Mray/s (primary+shadow) on Sponza 1920x1080" if args.config == "C3" else
                   f"Mray/s (primary+shadow{'+secondary' if second_total else ''}) [{args.config}: {cfg['name']}]"),
        "value": round(value, 2), "unit": "Mray/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        # N = 1 and the split: one frame per step whatever N is (total work fixed);
        # --split batch: N frames per step (work per GPU fixed)
        "scaling": "strong" if (world == 1 or split) else "weak", "vs_baseline": None, "dtype": "f32",
        "data": ("the reference's own final-scene data (Models/Final, Textures, Images/sky.hdr; assets/final) with "
                 "seeded stand-ins for the 7 meshes and the environment .tga missing from the snapshot; %d world objects, "
                 "%d BLAS triangles" % (scene.bvh_info["prims"], getattr(scene, "blas_prims", 0))
                 if cfg["mesh"] == "final" else
                 "synthetic (deterministic %s stand-in, %d tris; %s.obj is not in the reference snapshot%s)"
                 % ({"sponza": "Sponza", "sponza_large": "Sponza (262k variant)", "bunny": "bunny",
                     "instances": "dragon_2 / buddha_smooth"}.get(cfg["mesh"], cfg["mesh"]), scene.bvh_info["prims"],
                    {"instances": "dragon_2.obj / buddha_smooth", "sponza_large": "sponza"}.get(cfg["mesh"], cfg["mesh"]),
                    "; Images/Arches_E_PineTree.hdr dome / environment map" if cfg.get("env") else "")),
        "config": {"workload": cfg["name"], "config": args.config, "width": W, "height": H,
                   "spp": 1 if not adaptive else f"adaptive {cfg['subdivs'][0]}..{cfg['subdivs'][1]} subdivs, "
                   f"{primary_total / (n_frames * W * H):.2f} eye rays/px",
                   "frames_per_step": n_frames, "rays_per_step": rays_per_step, "shadow_rays": shadow_total,
                   "secondary_rays": second_total,
                   "qbvh_nodes": scene.bvh_info["nodes"], "qbvh_leaves": scene.bvh_info["leaves"],
                   "frames_in_flight": inflight, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                   "parallelism": "single GPU, whole frame" if use_frame_path else
                   ((f"one {W}x{H} frame per step" if n_frames == 1 else
                     f"batched: {n_frames} {W}x{H} frames of the camera path per step (distinct cameras), rendered "
                     f"by each rank in ONE launch (--frames-per-launch)") +
                    f" split over {world} GPUs: its 32x32 buckets dealt id mod {world} (src/Scene.cpp:90-174), " +
                    ("each rank's kernel stores its pixels straight into rank 0's frames through an IPC mapping, one "
                     "frame-end barrier (all-reduce of one int) per step, no gather or unpack"
                     if assemble == "ipc" else
                     "float32 tiles, one RCCL gather of the framebuffer(s) to rank 0 per step" +
                     ("" if assemble == "gather" else f" [{assemble}]")) +
                    f", consecutive steps pipelined over {depth} buffers" if split else
                    f"{n_frames}-frame camera path per step, 32x32 buckets dealt id mod {world}, "
                    f"one RCCL gather of 8-bit tiles per step (double-buffered)")},
        # The traversal is bound by latency along each wave's dependent chain
        # (~35% VALU busy, 41% memory wait); its algorithmic bytes
        # are served by L1/L2, so the ceiling they are priced against is the L2
        # bandwidth; `hbm` prices the counter-measured DRAM-side bytes.
        "roofline": {"bound": "l2", "kernel": dom, "achieved": round(achieved, 1), "peak": L2_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / L2_PEAK_GBS, 4),
                     "traffic": None if dom_traffic is None else int(dom_traffic),
                     "hbm": hbm, "hbm_algorithmic": hbm_alg, "latency_model": lat_model,
                     "tracked_profile": tracked, "latency": latency, "lane_util": lane_util,
                     "launch_ms": round(dom_ms, 4), "algorithmic_bytes_per_launch": int(dom_b),
                     "per_step": per_step,
                     # count-mode chunks of the chain engine re-rendered by the fused fallback: their node /
                     # leaf visits are not in the counts above, so visits_per_ray is a floor then
                     "chain_fallbacks_in_count_frame": int(st.get("chain_fallbacks", 0)),
                     "visits_per_ray": round(st["node_visits"] / max(1, (eye_mine if adaptive else px_mine)
                                                                    + shadow_mine + second_mine), 3)},
        "launch_ms": {"primary": round(pm, 4), "shade": round(sm, 4)},
        "frame_latency_ms": round(float(np.median(lat_ms)), 4),
        # one-time host side (outside the timed region): BVH::build over the scene's triangles
        "scene_setup": _scene_setup(scene),
        # instrumented (count-mode) launch: wall-clock spread of the persistent waves
        # (null where a pass records no wave clocks: the chain engine's many launches)
        "wave_timing_us": {k: (round(st[k], 1) if 0 <= st[k] < 1e9 else None)
                           for k in ("primary_span_us", "primary_ramp_us", "primary_tail_us",
                                     "shade_span_us", "shade_ramp_us", "shade_tail_us")},
    }
    if cfg["mesh"] == "final":   # the reference's only published absolute number is this scene's
        out["reference_published"] = {
            "render": "20 minutes on an i7 quadcore desktop (webpage/aguzman_jschwarzhaupt.html:147), 1904x1042",
            "this_frame_s": round(elapsed / args.steps, 4),
            "note": "not the same measurement: the reference frame is its CPU path on its own full assets (seven of "
                    "them, and the environment image, are stand-ins here) and a different RNG stream"}
    if region:
        out["timed_region"] = region
    if settle:   # untimed clock-settle steps before the warmup (see timed())
        out["settle"] = settle
    try:   # the library's embedded source hash against the sources beside it (tools/source_hash.py)
        out["build"] = _lib.build_info(L)
    except Exception as e:   # reported, never fatal
        out["build"] = {"error": str(e)}
    if tuning:
        out["tuning"] = tuning
    if rehearse:
        out["rehearsal"] = (f"MRT_BENCH_REHEARSE=gloo: {world} ranks sharing ONE GPU, collectives over gloo through "
                            f"host copies -- a run of the multi-rank code, not a measurement")
    if frame_check is not None:
        out["frame_check"] = frame_check
    if st.get("fused"):   # the frame kernel's walk (LDS top nodes only with tuning lds_nodes 1)
        out["walk"] = scene.walk_info()
        # the camera-ray walk's loop end (mrt_device.hip: one latch unless tuned off, or the
        # two-exit / LDS top-node walks, which are nested)
        one = tuning.get("walk_latch", 1) != 0 and out["walk"]["walk_exits"] == 1 and out["walk"]["lds_nodes"] != 1
        out["walk"]["latch"] = "one" if one else "nested"
    if split_times is not None:
        out["split_times"] = split_times
    if weak is not None:
        out["weak"] = weak
    if world > 1 and split and n_frames > 1:
        out["single_frame"] = single
    if not args.no_cpu_baseline and world == 1:
        try:
            out["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        except Exception as e:  # report, never hide
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


class _HostDist:
    """torch.distributed over gloo through host copies (bench rehearsal, MRT_BENCH_REHEARSE=gloo):
    barrier, all_reduce, gather and destroy_process_group as bench.py and BatchPipeline call them,
    on CUDA tensors.  A gather returns an already completed work object."""

    def __init__(self, dist, torch):
        self._d, self._t = dist, torch
        self.ReduceOp = dist.ReduceOp

    def barrier(self):
        self._d.barrier()

    def all_reduce(self, t, op=None, async_op=False):
        if t.is_cuda:   # stream order: the collective follows this rank's enqueued work
            self._t.cuda.current_stream().synchronize()
        h = t.cpu()
        self._d.all_reduce(h, op=op if op is not None else self._d.ReduceOp.SUM)
        t.copy_(h)
        return self._done() if async_op else None

    def broadcast_object_list(self, obj, src=0):
        self._d.broadcast_object_list(obj, src=src)

    @staticmethod
    def _done():
        class _Done:
            @staticmethod
            def wait():
                return True
        return _Done()

    def gather(self, t, outs=None, dst=0, async_op=False):
        if t.is_cuda:
            self._t.cuda.current_stream().synchronize()
        h = t.cpu()
        ho = [self._t.empty_like(h) for _ in outs] if outs is not None else None
        self._d.gather(h, ho, dst=dst)
        if outs is not None:
            for o, x in zip(outs, ho):
                o.copy_(x)

        class _Done:
            @staticmethod
            def wait():
                return True
        return _Done() if async_op else None

    def destroy_process_group(self):
        self._d.destroy_process_group()


def share_mode(args, E, widths):
    """--share N1,N2,...: the strong split's per-rank work measured on ONE GPU.

    The whole frame first (the N = 1 frame path with --inflight streams); then, per
    split width N, every rank r's share of buckets (id mod N == r) rendered alone
    through the split pipeline (--inflight buffers and streams).

    --assemble ipc (default): every share renders straight into frames
    (mrt_render_batch_frames_async), as a rank does into rank 0's mapped frames; no
    unpack anywhere.  The N-GPU step is modeled as
        max(slowest rank's render, one rank's frame bytes / per-link xGMI rate,
            barrier latency / (buffers - 1))
    -- the kernel stores of rank r > 0 cross one xGMI link into rank 0 (each rank its
    own link), and the per-step barrier of step k only gates the render of step
    k + buffers - 1.  --assemble gather: ranks r > 0 render into float tiles; rank 0
    renders its share and unpacks all N shares' tiles every step, as after the
    gather; step = max(rank 0's render + full unpack, slowest rank > 0, gather) with
    gather = latency + one rank's float tiles / per-link rate.  The xGMI rate and
    latency are ASSUMED (--xgmi-gbs, --xgmi-lat-us); nothing here ran on more than
    one GPU.  --frames-per-launch K: each share renders the first K frames of the
    camera path in one launch per step (per-frame times reported)."""
    torch, np, C_ = E["torch"], E["np"], C
    scene, L, _lib, tiles_mod = E["scene"], E["L"], E["_lib"], E["tiles_mod"]
    W, H, bpf = E["W"], E["H"], E["bpf"]
    ipc = args.assemble == "ipc"
    for i in range(E["inflight"]):
        _lib.check(L.mrt_render_frame_async(scene.handle, C_.byref(E["camc"][0]), C_.byref(E["opts"]),
                                            E["frame"][i].data_ptr(), E["frame8"][i].data_ptr(),
                                            E["streams"][i].cuda_stream), "render")
    torch.cuda.synchronize()
    _, (sh_full, eye_full, sec_full) = E["count_rays"](lambda: E["frame_step"](E["opts_count"], serial=True))
    rays_full = (eye_full if E["adaptive"] else W * H) + sh_full + sec_full
    e_full = E["timed"](E["frame_step"], lambda: None, args.steps)
    frame_ms = e_full / args.steps * 1e3
    out = {"metric": f"modeled strong-split curve from single-GPU share measurements [{args.config}]",
           "config": {"workload": E["cfg"]["name"], "config": args.config, "width": W, "height": H,
                      "buckets": bpf, "inflight": E["inflight"], "steps": args.steps, "warmup": args.warmup,
                      "assemble": args.assemble},
           "frame": {"ms_per_step": round(frame_ms, 4), "mray_s": round(rays_full / (frame_ms * 1e-3) / 1e6, 1)},
           "assumptions": {"xgmi_gbs_per_link": args.xgmi_gbs,
                           ("barrier_latency_us" if ipc else "gather_latency_us"): args.xgmi_lat_us,
                           "note": "xGMI rate and latency assumed, not measured: this box has one GPU; every "
                                   "other number in this line is measured on it"},
           "shares": {}}
    # one set of streams for every share pipeline (libmrt keeps scratch per stream, at most 16 per scene)
    share_streams = [torch.cuda.Stream() for _ in range(max(2, args.inflight))]
    K = max(1, min(16, args.frames_per_launch or DEFAULT_FPL))   # frames per share launch (camera path)
    out["config"]["frames_per_launch"] = K
    bxs = (W + 31) // 32
    for N in widths:
        per_rank = []
        for r in range(N):
            if ipc:
                pipe, render_b, mine, _ = E["make_ipc_pipe"](K, nsplit=N, srank=r, pipe_streams=share_streams)

                def render_one(o=E["opts"]):
                    render_b(0, o)
            else:
                pipe, render, items, mine, _ = E["make_pipe"](K, True, nsplit=N, srank=r, pipe_streams=share_streams,
                                                              share_unpack="full" if r == 0 else "none")

                def render_one(o=E["opts"]):
                    render(items, pipe.tiles[0], o)
            _, (sh, eye, sec) = E["count_rays"](lambda: render_one(E["opts_count"]))
            px = sum(min(32, W - (b % bpf % bxs) * 32) * min(32, H - (b % bpf // bxs) * 32)
                     for b in mine)   # over the K frames of a launch
            e = E["timed"](pipe.step, pipe.flush, args.steps)
            ms = e / args.steps * 1e3 / K   # per frame
            # host issue time of the same steps (the Python loop alone, before the device drains)
            torch.cuda.synchronize()
            t_i = time.perf_counter()
            for _ in range(args.steps):
                pipe.step()
            issue_ms = (time.perf_counter() - t_i) / args.steps * 1e3 / K
            pipe.flush()
            torch.cuda.synchronize()
            # one share launch alone (HIP events, nothing else in flight)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            alone = []
            for _ in range(5):
                e0.record()
                render_one()
                e1.record()
                torch.cuda.synchronize()
                alone.append(e0.elapsed_time(e1) / K)
            per_rank.append({"rank": r, "buckets": len(mine), "pixels": px, "ms_per_step": round(ms, 4),
                             "host_issue_ms_per_step": round(issue_ms, 4),
                             "launch_alone_ms": round(float(np.median(alone)), 4),
                             "rays": (eye if E["adaptive"] else px) + sh + sec})
            del pipe
        slow = max(per_rank, key=lambda x: x["ms_per_step"])
        if ipc:
            # rank r > 0's pixels cross its xGMI link as stores, per frame
            bpp = 3 + (12 if args.split_float else 0)   # RGB8 framebuffer (+ float RGB with --split-float)
            link_b = max(x["pixels"] for x in per_rank[1:]) * bpp / K if N > 1 else 0
            link_ms = link_b / (args.xgmi_gbs * 1e9) * 1e3
            bar_ms = args.xgmi_lat_us * 1e-3 / max(1, len(share_streams) - 1) / K
            step_ms = max(slow["ms_per_step"], link_ms, bar_ms)
            bound = "render" if step_ms == slow["ms_per_step"] else ("xgmi stores" if step_ms == link_ms else "barrier")
            rec = {"remote_bytes_per_link_per_frame": int(link_b), "link_ms_model": round(link_ms, 4),
                   "barrier_ms_model": round(bar_ms, 4)}
        else:
            # rank 0's unpack of the whole gathered frame (N ranks' padded float tiles)
            _, all_ids, per = tiles_mod.split_items(bpf * K, N, 0)
            ids = torch.tensor(all_ids, dtype=torch.int32, device="cuda")
            gathered = torch.zeros(len(all_ids) * 1024 * 3, dtype=torch.float32, device="cuda")
            ff = torch.empty(K * W * H * 3, dtype=torch.float32, device="cuda")
            f8 = torch.empty(K * W * H * 3, dtype=torch.uint8, device="cuda")
            un = []
            for _ in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), len(all_ids), gathered.data_ptr(), None, W, H, K,
                                                    ff.data_ptr(), f8.data_ptr(), scene.handle,
                                                    torch.cuda.current_stream().cuda_stream), "unpack")
                e1.record()
                torch.cuda.synchronize()
                un.append(e0.elapsed_time(e1))
            unpack_ms = float(np.median(un[2:])) / K   # per frame
            tile_bytes = per * 1024 * 3 * 4                      # one gather: K frames' tiles
            gather_ms = (args.xgmi_lat_us * 1e-3 + tile_bytes / (args.xgmi_gbs * 1e9) * 1e3) / K   # per frame
            step_ms = max(slow["ms_per_step"], gather_ms)   # rank 0's line includes its full unpack
            bound = "render" if slow["ms_per_step"] >= gather_ms else "gather"
            rec = {"rank0_render_plus_unpack_ms": per_rank[0]["ms_per_step"], "unpack_ms_rank0_alone": round(unpack_ms, 4),
                   "gather_bytes_per_rank": tile_bytes, "gather_ms_model": round(gather_ms, 4)}
        out["shares"][str(N)] = dict(
            {"per_rank": per_rank, "slowest_rank_ms": slow["ms_per_step"], "slowest_rank": slow["rank"],
             "mean_rank_ms": round(sum(x["ms_per_step"] for x in per_rank) / N, 4)}, **rec,
            step_ms_model=round(step_ms, 4), bound=bound,
            predicted_mray_s=round(rays_full / (step_ms * 1e-3) / 1e6, 1),
            predicted_speedup=round(frame_ms / step_ms, 3))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
