"""Shared scene builders for tests: the same scene description fed to the
product (miro / libmrt.so) and to the CPU oracle."""
import os

import numpy as np

import miro
import oracle as O
from miro import scenes

from conftest import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fixture_mesh(name):
    f = np.load(os.path.join(GOLDEN, f"{name}_mesh.npz"))
    return f["verts"], f["normals"], f["vidx"], f["nidx"]


MAP_KINDS = ("color", "normal", "specular", "reflect", "refract", "alpha")


def material_maps(pm, O_, om, mat):
    """mat["maps"]: {kind: (data (H, W, channels), RawImage type)} -> the same
    Texture on the product material (Material::set*Map) and in the oracle."""
    maps = mat.get("maps")
    if not maps:
        return
    ids = {}
    for kind in MAP_KINDS:
        if kind not in maps:
            continue
        data, typ = maps[kind]
        tex = miro.Texture(miro.RawImage(data.shape[1], data.shape[0], data, typ))
        getattr(pm, "set%sMap" % kind.capitalize())(tex)
        ids[kind] = O_.add_texture_typed(data, typ)
    O_.set_material_maps(om, **ids)


def materials_pair(P, O_, mat):
    """One material description -> (product material, oracle material id)."""
    optics = dict(reflectAmt=mat.get("reflectAmt", 0.0), refractAmt=mat.get("refractAmt", 0.0), ior=mat.get("ior", 1.5),
                  specGloss=mat.get("specGloss", 1.0))
    if mat["kind"] == "lambert":
        pm = miro.Lambert(mat["kd"])
        return pm, O_.add_material("lambert", kd=mat["kd"])
    pm = miro.Blinn(mat["kd"], specExp=mat.get("specExp", 1.0), specAmt=mat.get("specAmt", 0.0), **optics)
    if "ior3" in mat:   # setIor(ior, i) for i = 0..2, src/Blinn.h:38
        for i, v in enumerate(mat["ior3"]):
            pm.setIor(v, i)
    pm.m_disperse = bool(mat.get("disperse", False))
    pm.setTranslucency(mat.get("translucency", 0.0))
    pm.setLightEmittedIntensity(mat.get("emitted", 0.0))
    pm.setLightEmittedColor(mat.get("le", (0, 0, 0)))
    pm.setSampleEnv(mat.get("sampleEnv", True))
    om = O_.add_material("blinn", kd=mat["kd"], specExp=mat.get("specExp", 1.0), specAmt=mat.get("specAmt", 0.0),
                         translucency=mat.get("translucency", 0.0), le=mat.get("le", (0, 0, 0)),
                         emitted=mat.get("emitted", 0.0), sampleEnv=mat.get("sampleEnv", True),
                         disperse=mat.get("disperse", False), ior3=mat.get("ior3"),
                         **dict(optics, ior=mat["ior3"][1] if "ior3" in mat else optics["ior"]))
    return pm, om


def scene_pair(cfg, meshes=None, obj=None, floor=False, lights=None, num_paths=1, instances=None, subdivs=None,
               extra=None, path_trace=None, moving=None):
    """Build (miro.Scene, OracleScene, camera dict) for a config dict.
    extra: [(mesh arrays, material dict), ...] added after the main geometry;
    moving: [(mesh arrays, time-1 vertices, material dict), ...] MBObject meshes
    (makeMBMeshObjs) added after those;
    path_trace: (max_bounces, sample_env) turns Scene::m_pathTrace on."""
    lights = cfg["lights"] if lights is None else lights
    mat = cfg["material"]
    P = miro.Scene()
    O_ = O.OracleScene()
    all_mats = []   # (product, oracle id, description): per-material environment maps come last

    def materials_pair_(P, O_, m):
        pm_, om_ = materials_pair(P, O_, m)
        all_mats.append((pm_, om_, m))
        return pm_, om_
    pm, om = materials_pair_(P, O_, mat)
    material_maps(pm, O_, om, mat)
    for arrs in (meshes or []):
        tm = miro.TriangleMesh()
        tm.setArrays(*arrs)
        miro.makeMeshObjs(P, tm, pm)
        O_.add_mesh(*arrs, om)
    if obj is not None:
        tm = miro.TriangleMesh()
        tm.load(obj)
        miro.makeMeshObjs(P, tm, pm)
        O_.add_obj(obj, om)
    if instances:  # ((obj path, ...) per BLAS, [(blas index, 4x4), ...]) -- ProxyObjects
        paths, placed = instances
        protos, oblas = [], []
        for path in paths:
            tm = miro.TriangleMesh()
            tm.load(path)
            objs, bvh = miro.Objects(), miro.BVH()
            miro.ProxyObject.setupProxy(tm, pm, objs, bvh)
            protos.append((objs, bvh))
            oblas.append(O_.make_blas([O_.add_obj(path, om)]))
        for b, M in placed:
            P.addObject(miro.ProxyObject(*protos[b], miro.Matrix4x4(M)))
            O_.add_instance(oblas[b], M)
    for arrs, emat in (extra or []):   # mesh arrays (+ uv, tidx), or an OBJ path
        xm, oxm = materials_pair_(P, O_, emat)
        tm = miro.TriangleMesh()
        if isinstance(arrs, str):
            tm.load(arrs)
            O_.add_obj(arrs, oxm)
        else:
            tm.setArrays(*arrs[:4])
            mid = O_.add_mesh(*arrs[:4], oxm)
            if len(arrs) == 6:   # texture coordinates
                tm.setTexCoords(arrs[4], arrs[5])
                O_.set_texcoords(mid, arrs[4], arrs[5])
        miro.makeMeshObjs(P, tm, xm)
        material_maps(xm, O_, oxm, emat)
    for arrs, v2, emat in (moving or []):
        xm, oxm = materials_pair_(P, O_, emat)
        tm, tm2 = miro.TriangleMesh(), miro.TriangleMesh()
        tm.setArrays(*arrs[:4])
        tm2.setArrays(v2, *arrs[1:4])
        mid = O_.add_mesh(*arrs[:4], oxm)
        O_.set_motion(mid, v2)
        miro.makeMBMeshObjs(P, tm, tm2, xm)
    if floor:
        fl = miro.TriangleMesh()
        fl.createSingleTriangle()
        fl.setV1((-100, 0, -100)); fl.setV2((0, 0, 100)); fl.setV3((100, 0, -100))
        fl.setN1((0, 1, 0)); fl.setN2((0, 1, 0)); fl.setN3((0, 1, 0))
        miro.makeMeshObjs(P, fl, pm)
        O_.add_mesh(fl.verts, fl.normals, fl.vidx, fl.nidx, om)
    textures = {}

    def texture(rgb):  # one product Texture + one oracle texture per image
        if id(rgb) not in textures:
            tex = miro.Texture(miro.RawImage(rgb.shape[1], rgb.shape[0], rgb))
            textures[id(rgb)] = (tex, O_.add_texture(rgb))
        return textures[id(rgb)]

    skies = {}

    def sky(spec):   # a config sky spec -> one image per spec (HDR files: the oracle's decoder)
        if isinstance(spec, np.ndarray):
            return spec
        key = scenes.sky_key(spec)
        if key not in skies:
            skies[key] = scenes.env_image(spec, hdr_loader=O.hdr_load)
        return skies[key]

    for l in lights:
        if l["type"] == "point":
            pl = miro.PointLight(); pl.setPosition(l["pos"]); pl.setPower(l["power"])
            fast = l.get("fast_shadows", True)
            pl.setFastShadows(fast)
            P.addLight(pl)
            # Light::setFastShadows(false): the point light's transparent-shadow walk never
            # traces (src/PointLight.cpp:49-70 loops while sampleHit.t < distance, from t =
            # distance), so the oracle's light casts no shadow ray
            O_.add_point_light(l["pos"], l["power"], cast_shadows=fast)
        elif l["type"] == "dome":
            rgb = sky(l["sky"])
            l = dict(l, sky=rgb)
            tex, otex = texture(rgb)
            dl = miro.DomeLight(); dl.setTexture(tex); dl.setPower(l["power"])
            dl.setSamples(l.get("samples", 1)); dl.setNoiseThreshold(l.get("noise", 0.001))
            dl.setFastShadows(l.get("fast_shadows", True))
            P.addLight(dl)
            O_.add_dome_light(otex, l["power"], l.get("samples", 1), l.get("noise", 0.001),
                              fast_shadows=l.get("fast_shadows", True))
        else:
            rl = miro.RectangleLight(); rl.setVertices(l["v1"], l["v2"], l["v3"]); rl.setPower(l["power"])
            rl.setSamples(l.get("samples", 1)); rl.setNoiseThreshold(l.get("noise", 0.001))
            rl.setFastShadows(l.get("fast_shadows", True))
            P.addLight(rl)
            O_.add_rect_light(l["v1"], l["v2"], l["v3"], l["power"], l.get("samples", 1), l.get("noise", 0.001),
                              fast_shadows=l.get("fast_shadows", True))
    P.setBGColor(cfg["bg"])
    O_.set_bg(cfg["bg"])
    env = cfg.get("env")
    if env:
        tex, otex = texture(sky(env["sky"]))
        P.setEnvMap(tex); P.setEnvExposure(env["exposure"])
        O_.set_env_map(otex, env["exposure"])
    for pm_, om_, m in all_mats:   # Material::setEnvMap / m_envExposure
        if m.get("env"):
            tex, otex = texture(sky(m["env"]["sky"]))
            pm_.setEnvMap(tex); pm_.setEnvExposure(m["env"]["exposure"])
            O_.set_material_env_map(om_, otex, m["env"]["exposure"])
    P.setNumPaths(num_paths)
    O_.set_num_paths(num_paths)
    if path_trace is not None:
        P.setPathTrace(True); P.setMaxBounces(path_trace[0]); P.setSampleEnv(path_trace[1])
        O_.set_path_trace(True, path_trace[0], path_trace[1])
    if subdivs is not None:  # (min, max, noise): Scene::adaptiveSampleScene
        P.setMinSubdivs(subdivs[0]); P.setMaxSubdivs(subdivs[1]); P.setNoise(subdivs[2])
        O_.set_subdivs(*subdivs)
    P.preCalc()
    O_.build()
    return P, O_, cfg["camera"]


def camera(c):
    cam = miro.Camera()
    cam.setEye(c["eye"]); cam.setLookAt(c["lookAt"]); cam.setUp(c.get("up", (0, 1, 0))); cam.setFOV(c["fov"])
    cam.setAperture(c.get("aperture", 0.0)); cam.setFocusPlane(c.get("focusPlane", 1.0))
    cam.setShutterSpeed(c.get("shutterSpeed", 0.001))
    return cam


def final_scene_pair(grid=201):
    """(miro.Scene, OracleScene, camera dict) of the reference's final scene (config FS)."""
    from miro import final_scene
    import final_scene as oracle_final
    sp = final_scene.spec(grid=grid)
    P, _ = final_scene.build_product(sp)
    O_, cam = oracle_final.build(sp)
    return P, O_, cam


def config_scene(key, **kw):
    cfg = scenes.CONFIGS[key]
    if cfg["mesh"] == "final":
        return final_scene_pair(**kw)
    kw.setdefault("num_paths", cfg.get("num_paths", 1))
    kw.setdefault("subdivs", cfg.get("subdivs"))
    kw.setdefault("path_trace", cfg.get("path_trace"))
    kw.setdefault("extra", [(scenes.EXTRA_OBJS[n], m) for n, m in cfg.get("extra", ())])
    if cfg["mesh"] == "cornell":
        return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], **kw)
    if cfg["mesh"] == "bunny":
        return scene_pair(cfg, obj=scenes.bunny_obj(), floor=True, **kw)
    if cfg["mesh"] == "instances":
        placed = [(i % 2, M) for i, M in enumerate(scenes.instance_transforms(**cfg["instances"]))]
        return scene_pair(cfg, floor=True, instances=(scenes.proto_objs(cfg), placed), **kw)
    return scene_pair(cfg, obj=scenes.mesh_obj(cfg), **kw)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)
