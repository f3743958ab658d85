"""Wave timeline of one count-mode frame (diagnostics for the launch tail):
per-wave start/end/tiles/node visits of the primary and shade launches of a
config, saved to gpurun_out/wave_log_<config>.npz with a printed summary."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--tune", nargs="*", default=[], help="tuning switches key=value (mrt_set_tuning)")
    ap.add_argument("--frames", type=int, default=0, help="render a camera-path batch of N frames (bucket path)")
    ap.add_argument("--timed", action="store_true", help="log the uninstrumented kernels (wave_log=1, no counters)")
    a = ap.parse_args()
    import torch
    import miro
    from miro import _lib, scenes
    for kv in a.tune:
        k, v = kv.split("=")
        _lib.check(miro.lib().mrt_set_tuning(k.encode(), int(v)), k)
    if a.timed:
        _lib.check(miro.lib().mrt_set_tuning(b"wave_log", 1), "wave_log")
    count = 0 if a.timed else 1
    scene, cam, cfg = scenes.build_config(a.config)
    W, H = cfg["W"], cfg["H"]
    img = miro.Image()
    img.resize(W, H)
    if a.frames:
        bpf = ((W + 31) // 32) * ((H + 31) // 32)
        cams = []
        for c in scenes.camera_path(cfg["camera"], a.frames):
            m = miro.Camera(); m.setEye(c["eye"]); m.setLookAt(c["lookAt"]); m.setUp(c["up"]); m.setFOV(c["fov"])
            cams.append(m._c())
        camc = (_lib.mrt_camera * a.frames)(*cams)
        ids = torch.arange(bpf * a.frames, dtype=torch.int32, device="cuda")
        t8 = torch.empty(len(ids) * 1024 * 3, dtype=torch.uint8, device="cuda")
        o = _lib.mrt_render_opts(W, H, 0, count, 0, 0, 0)
        for _ in range(10):
            _lib.check(miro.lib().mrt_render_batch_async(scene.handle, camc, a.frames, C.byref(o), ids.data_ptr(),
                                                         len(ids), None, t8.data_ptr(), None), "batch")
            torch.cuda.synchronize()
    else:
        # back-to-back async frames like bench.py (host copies between frames
        # would idle the GPU and drop its clocks); the last one is logged
        fr = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
        fr8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
        o = _lib.mrt_render_opts(W, H, 0, count, 1, 0, 0)
        camc = cam._c()
        for _ in range(30):
            _lib.check(miro.lib().mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), fr.data_ptr(),
                                                         fr8.data_ptr(), None), "render")
        torch.cuda.synchronize()
    out = {}
    st = scene.stats()
    print("event-timed launches: primary %.3f ms, shade %.3f ms" % (st["primary_ms"], st["shade_ms"]))
    for k, name in enumerate(("primary", "shade")):
        log, khz = scene.wave_log(k)
        out[name + "_full"] = log
        log = log[:, :4]
        if len(log) == 0:   # (the one-launch frame kernel has no shade launch)
            continue
        t0 = log[:, 0].astype(np.float64)
        t1 = log[:, 1].astype(np.float64)
        base = t0.min()
        us = 1e3 / khz
        s, e = (t0 - base) * us, (t1 - base) * us
        tiles = log[:, 2].astype(np.int64)
        nodes = log[:, 3].astype(np.int64)
        out[name] = log
        q = np.percentile(e, [0, 1, 10, 50, 90, 99, 100])
        print(f"{name}: waves {len(log)} tiles/wave mean {tiles.mean():.2f} min {tiles.min()} max {tiles.max()}")
        print(f"  end us percentiles 0/1/10/50/90/99/100: " + " ".join(f"{x:.0f}" for x in q))
        print(f"  start spread {s.max():.1f} us; busy fraction (sum wave time / waves x span) "
              f"{(e - s).sum() / (len(e) * e.max()):.3f}")
        late = e > np.percentile(e, 99)
        print(f"  slowest 1% waves: tiles {tiles[late].mean():.2f} nodes/tile {(nodes[late] / np.maximum(1, tiles[late])).mean():.0f}"
              f" vs all {(nodes / np.maximum(1, tiles)).mean():.0f}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"wave_log_{a.config}{'_' + '_'.join(a.tune) if a.tune else ''}{'_f%d' % a.frames if a.frames else ''}{'_timed' if a.timed else ''}.npz"), khz=khz, **out)


if __name__ == "__main__":
    main()
