"""Interleaved A/B of tuning switches on config C3 (one process, one device).
Usage: python tools/ab_bench.py key=v1,v2 [key2=...] [--rounds R] [--inflight K]
Per variant: serial kernel times (HIP events of single frames) and the
pipelined rate with K frames in flight on K streams (bench.py's N = 1 mode)."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import miro  # noqa: E402
from miro import _lib, scenes  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if "=" in a]
    rounds = 7
    if "--rounds" in sys.argv:
        rounds = int(sys.argv[sys.argv.index("--rounds") + 1])
    cfgkey = os.environ.get("AB_CONFIG", "C3")
    inflight = int(sys.argv[sys.argv.index("--inflight") + 1]) if "--inflight" in sys.argv else 4
    variants = [{}]
    for a in args:   # key=v1,v2 (product with the other keys); k1+k2=a1+a2,b1+b2 (paired values)
        k, vs = a.split("=")
        ks = k.split("+")
        variants = [dict(v, **{kk: int(xx) for kk, xx in zip(ks, x.split("+"))}) for v in variants for x in vs.split(",")]
    scene, cam, cfg = scenes.build_config(cfgkey)
    W, H = cfg["W"], cfg["H"]
    L = miro.lib()
    frame = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
    frame8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    camc = cam._c()
    streams = [torch.cuda.Stream() for _ in range(inflight)]
    fr = [torch.empty(H * W * 3, dtype=torch.float32, device="cuda") for _ in range(inflight)]
    fr8 = [torch.empty(H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(inflight)]

    def pipelined(v, frames=40):
        for k, x in v.items():
            _lib.check(L.mrt_set_tuning(k.encode(), x), k)
        o = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
        for i in range(inflight):   # per-stream scratch + warm
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), fr[i].data_ptr(),
                                                fr8[i].data_ptr(), streams[i].cuda_stream), "render")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for f in range(frames):
            i = f % inflight
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), fr[i].data_ptr(),
                                                fr8[i].data_ptr(), streams[i].cuda_stream), "render")
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / frames * 1e3
    ref = None

    def run(v, count=False, reps=10):
        for k, x in v.items():
            _lib.check(L.mrt_set_tuning(k.encode(), x), k)
        o = _lib.mrt_render_opts(W, H, 0, int(count), 1, 0, 0)
        pm, sm = [], []
        t0 = time.perf_counter()
        for _ in range(reps):
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), frame.data_ptr(),
                                                frame8.data_ptr(), sh), "render")
            st = scene.stats()
            pm.append(st["primary_ms"]); sm.append(st["shade_ms"])
        return pm, sm, st

    res = {json.dumps(v): ([], []) for v in variants}
    pipe = {json.dumps(v): [] for v in variants}
    for v in variants:  # warm + correctness vs the first variant
        run(v, reps=2)
        out = frame.cpu().numpy().view(np.uint32).copy()
        if ref is None:
            ref = out
        assert np.array_equal(ref, out), f"variant {v} changed the frame!"
        _, _, st = run(v, count=True, reps=1)
        print("variant", v, "counts", {k: st[k] for k in ("node_visits", "leaf_visits", "primary_node_visits",
                                                          "max_stack", "shadow_rays", "primary_hits", "primary_uniform_visits")},
              "primary SIMD util %.3f" % (st["primary_node_visits"] / max(1, 64 * st["primary_wave_steps"])),
              "shadow SIMD util %.3f" % (st["shadow_node_visits"] / max(1, 64 * st["shadow_wave_steps"])), flush=True)
    for r in range(rounds):
        for v in variants:
            pm, sm, _ = run(v)
            res[json.dumps(v)][0].extend(pm)
            res[json.dumps(v)][1].extend(sm)
            pipe[json.dumps(v)].append(pipelined(v))
    rays = W * H + st["shadow_rays"]
    for k, (pm, sm) in res.items():
        p, s = np.median(pm), np.median(sm)
        q = np.median(pipe[k])
        print(f"{k:64s} primary {p:.4f} ms  shade {s:.4f} ms  "
              f"frame {p + s:.4f} ms  -> {rays / (p + s) / 1e3:.0f} Mray/s (kernel time); "
              f"{inflight} in flight {q:.4f} ms/frame -> {rays / q / 1e3:.0f} Mray/s", flush=True)


if __name__ == "__main__":
    main()
