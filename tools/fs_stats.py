"""Config FS diagnostics (one process, one device): per tuning variant, the count-mode
statistics of one frame (visits per ray, lane utilisation of the chain trace launches) and
the kernel time of one uncounted frame.  Usage: python tools/fs_stats.py [WxH] [key=v,...]..."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import torch  # noqa: E402
import miro  # noqa: E402
from miro import _lib, scenes  # noqa: E402


def main():
    size = [a for a in sys.argv[1:] if "x" in a and "=" not in a]
    W, H = (int(x) for x in (size[0] if size else "476x260").split("x"))
    variants = [{}]
    for a in sys.argv[1:]:
        if "=" in a:
            variants.append({k: int(v) for k, v in (kv.split("=") for kv in a.split(","))})
    cfgkey = os.environ.get("FS_CONFIG", "FS")
    scene, cam, cfg = scenes.build_config(cfgkey)
    print("built", cfgkey, flush=True)
    L = miro.lib()
    frame = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
    frame8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    camc = cam._c()
    for v in variants:
        for k, x in v.items():
            _lib.check(L.mrt_set_tuning(k.encode(), x), k)
        o = _lib.mrt_render_opts(W, H, 0, 1, 1, 0, 0)
        _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), frame.data_ptr(), frame8.data_ptr(), sh), "render")
        torch.cuda.synchronize()
        st = scene.stats()
        rays = st["primary_rays"] + st["shadow_rays"] + st["secondary_rays"]
        o = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
        ts = []
        for _ in range(int(os.environ.get("FS_REPS", "1"))):
            t0 = time.perf_counter()
            _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), frame.data_ptr(), frame8.data_ptr(), sh), "render")
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        dt = sorted(ts)[len(ts) // 2]
        print(json.dumps({"variant": v, "ms": round(dt * 1e3, 1), "mray_s": round(rays / dt / 1e6, 2), "rays": rays,
                          "nodes_per_ray": round(st["node_visits"] / rays, 2), "leaves_per_ray": round(st["leaf_visits"] / rays, 2),
                          "trace_lane_util": round(st["shadow_node_visits"] / max(1, 64 * st["shadow_wave_steps"]), 4),
                          "primary_lane_util": round(st["primary_node_visits"] / max(1, 64 * st["primary_wave_steps"]), 4),
                          **{k: st[k] for k in ("primary_rays", "shadow_rays", "secondary_rays", "node_visits", "leaf_visits",
                                                "shadow_node_visits", "shadow_wave_steps", "primary_node_visits", "primary_wave_steps")}}),
              flush=True)


if __name__ == "__main__":
    main()
