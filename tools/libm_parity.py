"""CPU-only: how far a libm evaluated in double and rounded once moves each config's frame
against the reference's own calls.

The reference's source resolves its libm calls (Fresnel's sin(acosf), Blinn's pow, the
lat-long lookups' atan2 / acos, the cosine sampler's cos / sin) to the float overloads
(glibc sinf / acosf / powf / atan2f / cosf).  Round 5's device evaluated sinf / cosf / powf
in double and rounded once (oracle.LIBM_DOUBLE); since round 6 it restates all five glibc
functions bit for bit (csrc/mrt_libm.h), i.e. it equals oracle.LIBM_FLOAT.  This tool
keeps the comparison of the two conventions (profiles/r06_libm_parity.json: round 5's
device convention against the reference's, per config):

    python3 tools/libm_parity.py [--threads 8] [--out profiles/r05_libm_parity.json] [KEY[:WxH] ...]

Reports channels beyond north_star's 1e-4 relative (no floor), the bit-exact
share, primary hit ids, and the ray counts of both conventions."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "rendering-algorithms-raytracer_amd"),
          os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import oracle as O  # noqa: E402
from miro import scenes  # noqa: E402
from helpers import config_scene  # noqa: E402

DEFAULT = ["C3:1920x1080", "C4:1920x1080", "D1:1024x1024", "R3:1920x1080", "G3:960x540", "P4:256x256",
           "A3:960x540", "C5:960x540", "FS:160x88"]


def compare(key, W, H, threads):
    _, Osc, cam = config_scene(key)
    t0 = time.time()
    dev = Osc.render(cam, W, H, threads=threads, libm=O.LIBM_DOUBLE)
    ref = Osc.render(cam, W, H, threads=threads, libm=O.LIBM_FLOAT)
    g, r = dev["rgb"].astype(np.float64), ref["rgb"].astype(np.float64)
    bad = np.abs(g - r) > 1e-4 * np.abs(r)
    px_bad = bad.any(axis=2)
    exact = float((dev["rgb"].view(np.uint32) == ref["rgb"].view(np.uint32)).mean())
    worst = float(np.max(np.abs(g - r) / np.maximum(np.abs(r), 1e-30))) if bad.any() else 0.0
    return {
        "config": key, "W": W, "H": H,
        "channels_beyond_1e-4": int(bad.sum()), "pixels_beyond_1e-4": int(px_bad.sum()),
        "bit_exact_share": exact, "worst_rel": worst,
        "rgb8_diff_px": int((dev["rgb8"] != ref["rgb8"]).any(axis=2).sum()),
        "primary_hits_equal": bool(np.array_equal(dev["hits"]["prim"], ref["hits"]["prim"])),
        "shadow_rays": [dev["shadow_rays"], ref["shadow_rays"]],
        "secondary_rays": [dev["secondary_rays"], ref["secondary_rays"]],
        "seconds": round(time.time() - t0, 2),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    ap.add_argument("keys", nargs="*")
    a = ap.parse_args()
    rows = []
    for spec in a.keys or DEFAULT:
        key, _, size = spec.partition(":")
        W, H = (int(v) for v in size.split("x")) if size else (scenes.CONFIGS[key]["W"], scenes.CONFIGS[key]["H"])
        row = compare(key, W, H, a.threads)
        print(json.dumps(row), flush=True)
        rows.append(row)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"note": "oracle LIBM_DOUBLE (round 5's device convention) vs LIBM_FLOAT (the reference's "
                               "float overloads, glibc); tools/libm_parity.py", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
