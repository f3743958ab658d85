"""Regenerate the committed fixtures (run in the build container, where the
reference's model files are readable at /root/reference/Models).

Inputs: the reference's own test assets, loaded by the CPU oracle's restatement
of TriangleMesh::loadObj (so the arrays carry the loader's x0.99999994 scaling
and face normals).  Outputs: oracle renders of config C1 (full 256x256 frame)
and digests of small C2/C3 frames.  Data only -- no reference source is copied.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import oracle as O  # noqa: E402
from miro import scenes  # noqa: E402

MODELS = "/root/reference/Models"
MESHES = {"cornell_box": "cornell_box.obj", "teapot": "teapot.obj", "explosion01": "Final/explosion01.obj"}


def load_mesh(rel):
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_obj(os.path.join(MODELS, rel), m)
    return s.mesh_arrays(0)


def digest(*arrs):
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def oracle_scene(cfg, mesh_arrays=None, obj=None, floor=False):
    s = O.OracleScene()
    mat = cfg["material"]
    m = s.add_material(mat["kind"], kd=mat["kd"])
    if mesh_arrays is not None:
        s.add_mesh(*mesh_arrays, m)
    else:
        s.add_obj(obj, m)
    if floor:
        s.add_mesh([(-100, 0, -100), (0, 0, 100), (100, 0, -100)], [(0, 1, 0)] * 3, [(0, 1, 2)], [(0, 1, 2)], m)
    for l in cfg["lights"]:
        s.add_point_light(l["pos"], l["power"])
    s.set_bg(cfg["bg"])
    s.build()
    return s


def motion_fixture():
    """cannonBallT1/T2 (the reference's makeMBMeshObjs pair, src/main.cpp:216-221)
    and its groundPlane: time-0 arrays, time-1 vertices (same topology)."""
    v1, n1, vi1, ni1 = load_mesh("Final/cannonBallT1.obj")
    v2, _, vi2, _ = load_mesh("Final/cannonBallT2.obj")
    assert v1.shape == v2.shape and np.array_equal(vi1, vi2), "MBObject meshes need one topology"
    gv, gn, gvi, gni = load_mesh("Final/groundPlane.obj")
    np.savez_compressed(os.path.join(HERE, "cannonball_mb.npz"), verts=v1, normals=n1, vidx=vi1, nidx=ni1,
                        verts2=v2, ground_verts=gv, ground_normals=gn, ground_vidx=gvi, ground_nidx=gni)


def main():
    if sys.argv[1:] == ["motion"]:
        return motion_fixture()
    meta = {}
    for name, rel in MESHES.items():
        v, n, vi, ni = load_mesh(rel)
        np.savez_compressed(os.path.join(HERE, f"{name}_mesh.npz"), verts=v, normals=n, vidx=vi, nidx=ni)
        meta[name] = {"tris": int(len(vi)), "sha256": digest(v, n, vi, ni)}
    # C1 golden frame
    fx = np.load(os.path.join(HERE, "cornell_box_mesh.npz"))
    cfg = scenes.CONFIGS["C1"]
    s = oracle_scene(cfg, (fx["verts"], fx["normals"], fx["vidx"], fx["nidx"]))
    r = s.render(cfg["camera"], cfg["W"], cfg["H"])
    np.savez_compressed(os.path.join(HERE, "c1_cornell_256.npz"), rgb=r["rgb"], rgb8=r["rgb8"],
                        t=r["hits"]["t"], a=r["hits"]["a"], b=r["hits"]["b"], prim=r["hits"]["prim"],
                        shadow=r["shadow"])
    meta["C1"] = {"W": cfg["W"], "H": cfg["H"], "shadow_rays": r["shadow_rays"],
                  "sha256": digest(r["rgb"], r["rgb8"], r["hits"])}
    # C2 / C3 small-frame digests (synthetic stand-ins)
    for key, W, H in (("C2", 128, 128), ("C3", 192, 108)):
        cfg = scenes.CONFIGS[key]
        obj = scenes.bunny_obj() if cfg["mesh"] == "bunny" else scenes.sponza_obj()
        s = oracle_scene(cfg, obj=obj, floor=(cfg["mesh"] == "bunny"))
        r = s.render(cfg["camera"], W, H, threads=8)
        meta[key] = {"W": W, "H": H, "qbvh": s.qbvh_info(), "shadow_rays": r["shadow_rays"],
                     "sha256_rgb": digest(r["rgb"]), "sha256_hits": digest(r["hits"])}
    with open(os.path.join(HERE, "fixtures.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(json.dumps(meta, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
