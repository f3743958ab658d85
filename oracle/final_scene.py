"""TEST INFRASTRUCTURE (the checker, never the product): the reference's final
scene (makeFinalScene, src/main.cpp:132-670) in the CPU oracle, from the same
description miro/final_scene.py.spec() hands the product, with the same calls in
the same order (materials, world meshes, MBObject pairs via set_motion, BLASes
built at their first instance as miro.Scene.preCalc does, ProxyObject
instances, dome light, environment map, subdivisions), so object and hit ids
agree with libmrt's."""
from __future__ import annotations

import oracle as O


def material(s, m):
    """oracle material id of a spec material (helpers.materials_pair's mapping)."""
    ior3 = m.get("ior3")
    ior = ior3[1] if ior3 else m.get("ior", 1.5)
    return s.add_material(m["kind"], kd=m["kd"], specExp=m.get("specExp", 1.0), specAmt=m.get("specAmt", 0.0),
                          reflectAmt=m.get("reflectAmt", 0.0), refractAmt=m.get("refractAmt", 0.0), ior=ior,
                          specGloss=m.get("specGloss", 1.0), translucency=m.get("translucency", 0.0),
                          disperse=m.get("disperse", False), ior3=ior3)


def build(sp):
    """(OracleScene, camera dict) of a final-scene spec."""
    s = O.OracleScene()
    textures = {}

    def texture(path):
        if path not in textures:
            if path.endswith(".hdr"):
                textures[path] = s.add_texture(O.hdr_load(path))
            else:
                data, typ = O.image_load(path)
                textures[path] = s.add_texture_typed(data, typ)
        return textures[path]

    # libmrt registers a material at the first mesh that uses it; the oracle ids are
    # local to the oracle, so registering them up front changes nothing it computes
    mats = {}
    for name, m in sp["materials"].items():
        mats[name] = material(s, m)
        maps = {k: texture(p) for k, p in m.get("maps", {}).items()}
        if maps:
            s.set_material_maps(mats[name], **maps)
    blas = {}
    for o in sp["objects"]:
        if "blas" in o:
            b = o["blas"]
            if b not in blas:
                blas[b] = s.make_blas([s.add_obj(path, mats[mn]) for path, mn in sp["blas"][b]])
            s.add_instance(blas[b], o["m"])
            continue
        mid = s.add_obj(o["obj"], mats[o["mat"]])
        if "obj2" in o:   # makeMBMeshObjs: the time-1 mesh's vertices, loaded on the side
            tmp = O.OracleScene()
            v2 = tmp.mesh_arrays(tmp.add_obj(o["obj2"], tmp.add_material("lambert")))[0]
            s.set_motion(mid, v2)
    s.add_dome_light(texture(sp["dome"]["image"]), sp["dome"]["power"], sp["dome"]["samples"])
    s.set_env_map(texture(sp["env"]["image"]), sp["env"]["exposure"])
    s.set_bg(sp["bg"])
    s.set_num_paths(sp["num_paths"])
    s.set_subdivs(*sp["subdivs"])
    s.build()
    return s, dict(sp["camera"])
