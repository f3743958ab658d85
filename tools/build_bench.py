"""Host scene-build throughput: OBJ load
(TriangleMesh::loadObj restatement) and BVH::build (binned SAH + QBVH collapse)
for the Sponza stand-in and a 1.09 M-triangle buddha_smooth-sized stand-in, on
1 thread and on the host's build threads (MRT_BUILD_THREADS / affinity /
OMP_NUM_THREADS).  The parallel tree must equal the 1-thread tree bit for bit.
Prints one JSON line (profiles/r02_build_bench.json when --out is given)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import miro  # noqa: E402
from miro import _lib, scenes  # noqa: E402


def build(path, threads, reps=3):
    L = miro.lib()
    os.environ["MRT_BUILD_THREADS"] = str(threads)
    best_load = best_build = None
    arrays = None
    for _ in range(reps):
        h = L.mrt_scene_create()
        m = _lib.mrt_material(0, _lib.f3((1, 1, 1)), _lib.f3((0, 0, 0)), _lib.f3((1, 1, 1)), 1.0, 0.0,
                              _lib.f3((0, 0, 0)), 0.0)
        mat = L.mrt_scene_add_material(h, C.byref(m))
        t0 = time.perf_counter()
        _lib.check(L.mrt_scene_add_obj(h, path.encode(), None, mat), "load")
        t1 = time.perf_counter()
        _lib.check(L.mrt_scene_build_bvh(h), "build")
        t2 = time.perf_counter()
        info = _lib.mrt_bvh_info()
        _lib.check(L.mrt_scene_bvh_info(h, C.byref(info)), "info")
        if arrays is None:
            nb = np.zeros((info.nodes, 24), np.float32); nc = np.zeros((info.nodes, 4), np.int32)
            lt = np.zeros((info.leaves, 36), np.float32); lp = np.zeros((info.leaves, 4), np.int32)
            fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int32)
            _lib.check(L.mrt_scene_bvh_export(h, nb.ctypes.data_as(fp), nc.ctypes.data_as(ip), lt.ctypes.data_as(fp),
                                              lp.ctypes.data_as(ip)), "export")
            arrays = (nb.view(np.uint32), nc, lt.view(np.uint32), lp)
        L.mrt_scene_destroy(h)
        best_load = (t1 - t0) if best_load is None else min(best_load, t1 - t0)
        best_build = (t2 - t1) if best_build is None else min(best_build, t2 - t1)
    return best_load * 1e3, best_build * 1e3, info.prims, info.nodes, info.leaves, arrays


def main():
    sys.path.insert(0, ROOT)
    import bench
    threads = int(os.environ.get("MRT_BUILD_THREADS_MAX", 0)) or bench.cpu_threads()
    out = {"cpu": bench.cpu_model(), "threads": threads, "scenes": {}}
    for name, path in (("sponza", scenes.sponza_obj()), ("buddha_full", scenes.buddha_full_obj())):
        l1, b1, prims, nodes, leaves, a1 = build(path, 1)
        ln, bn, _, _, _, an = build(path, threads)
        same = all(np.array_equal(x, y) for x, y in zip(a1, an))
        out["scenes"][name] = {"prims": prims, "qbvh_nodes": nodes, "qbvh_leaves": leaves,
                               "obj_load_ms": round(min(l1, ln), 1),
                               "build_ms_1_thread": round(b1, 1), f"build_ms_{threads}_threads": round(bn, 1),
                               "build_mprims_per_s": round(prims / bn / 1e3, 2), "speedup": round(b1 / bn, 2),
                               "tree_identical": bool(same)}
        if not same:
            print(json.dumps(out))
            sys.exit("parallel build differs from the 1-thread build")
    print(json.dumps(out))
    if "--out" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
