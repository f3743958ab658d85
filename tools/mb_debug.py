"""GPU vs oracle pixel diffs for motion-blur path-tracing variants (debug aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "rendering-algorithms-raytracer_amd"), os.path.join(ROOT, "oracle"), ROOT,
          os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import miro  # noqa: E402
from miro import _lib  # noqa: E402
from helpers import bits, camera  # noqa: E402
from test_motion_blur import CAM, cornell, moved, sphere  # noqa: E402


def run(tag, P, O_, cam, W=48, H=40):
    img = miro.Image()
    img.resize(W, H)
    P.raytraceImage(camera(cam), img, want_hits=True)
    ref = O_.render(cam, W, H, threads=8)
    d = (bits(img.rgb) != bits(ref["rgb"])).any(axis=2)
    ys, xs = np.nonzero(d)
    print(f"{tag}: {d.sum()} px differ; sec gpu {P.last_stats['secondary_rays']} ref {ref['secondary_rays']};"
          f" shadow gpu {P.last_stats['shadow_rays']} ref {ref['shadow_rays']}", list(zip(ys[:5], xs[:5])), flush=True)
    for y, x in list(zip(ys, xs))[:3]:
        print("   ", img.rgb[y, x], ref["rgb"][y, x], ref["hits"]["prim"][y, x])


L = miro.lib()
ball = sphere()
gi = dict(kind="blinn", kd=(0.2, 0.7, 0.3))
for chain in (1, 0):
    L.mrt_set_tuning(b"chain", chain)
    for sh in (1.0, 0.0):
        P, O_, _ = cornell(moving=[(ball, moved(ball), gi)], num_paths=2, path_trace=(2, False))
        run(f"chain={chain} MB shutter={sh}", P, O_, dict(CAM, shutterSpeed=sh))
    P, O_, _ = cornell(extra=[(ball, gi)], num_paths=2, path_trace=(2, False))
    run(f"chain={chain} static", P, O_, CAM)
    P, O_, _ = cornell(moving=[(ball, moved(ball), gi)], num_paths=1, path_trace=(1, False))
    run(f"chain={chain} MB 1 path 1 bounce", P, O_, dict(CAM, shutterSpeed=1.0))
