"""The compiled reference-side C++ bridge (shim/miro_shim.cpp): reference-layout
types (16-B Vector3 arrays, TupleI3 indices, one Object per triangle) marshalled
into libmrt by Scene::preCalc, then Scene::raytraceImage and Scene::trace
(reference src/Scene.h:31-32).  The GPU test renders config C1 through the
binary and compares with the CPU oracle: 8-bit pixels and hit records exact."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import miro
import oracle as O
from helpers import fixture_mesh
from miro import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "shim", "build", "shim_test")


def write_mesh(path):
    v, n, vi, ni = fixture_mesh("cornell_box")
    with open(path, "wb") as f:
        np.array([len(v), len(n), len(vi)], np.int32).tofile(f)
        for a, t in ((v, np.float32), (n, np.float32), (vi, np.uint32), (ni, np.uint32)):
            np.ascontiguousarray(a, t).tofile(f)


def write_rays(path, n=2000, seed=11):
    rng = np.random.default_rng(seed)
    o = np.tile(np.array([[2.75, 2.75, 5.0]], np.float32), (n, 1)) + rng.uniform(-0.5, 0.5, (n, 3)).astype(np.float32)
    d = (rng.normal(size=(n, 3)) * 0.35 + np.array([0.0, 0.0, -1.0])).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmax = np.where(rng.uniform(size=n) < 0.2, 4.0, 1e12).astype(np.float32)
    with open(path, "wb") as f:
        np.array([n], np.int32).tofile(f)
        o.tofile(f); d.tofile(f); tmax.tofile(f)
    return o, d, tmax


def oracle_c1():
    cfg = scenes.CONFIGS["C1"]
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_mesh(*fixture_mesh("cornell_box"), m)
    s.add_point_light(cfg["lights"][0]["pos"], cfg["lights"][0]["power"])
    s.set_bg(cfg["bg"])
    s.build()
    return s, cfg["camera"]


def test_shim_binary_builds_the_scene_without_a_gpu(tmp_path):
    """Scene::preCalc runs on the host (BVH build through the C-ABI); without a
    device the frame entry reports MRT_ERR_NO_DEVICE instead of crashing."""
    assert os.path.exists(BIN), "shim/build/shim_test not built (__graft_entry__.build())"
    mesh = tmp_path / "mesh.bin"
    write_mesh(mesh)
    r = subprocess.run([BIN, str(mesh), "64", "64", str(tmp_path / "out.rgb8")], capture_output=True, text=True,
                       timeout=120)
    if miro.device_count() > 0:
        assert r.returncode == 0, r.stderr
    else:
        assert r.returncode == 1 and "raytraceImage: -7" in r.stderr, (r.returncode, r.stderr)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[], [0, 0]])
def test_shim_renders_c1_like_the_oracle(tmp_path, devices):
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 256, 256
    mesh, rays, hits, out = (str(tmp_path / n) for n in ("mesh.bin", "rays.bin", "hits.bin", "out.rgb8"))
    write_mesh(mesh)
    o, d, tmax = write_rays(rays)
    r = subprocess.run([BIN, mesh, str(W), str(H), out, rays, hits] + [str(x) for x in devices], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    img = np.fromfile(out, np.uint8).reshape(H, W, 3)
    s, cam = oracle_c1()
    ref = s.render(cam, W, H, threads=8)
    assert np.array_equal(img, ref["rgb8"])
    got = np.fromfile(hits, np.dtype([("t", "<f4"), ("a", "<f4"), ("b", "<f4"), ("obj", "<i4")]))
    want, _, _ = s.trace(o, d, 0.001, tmax)
    assert np.array_equal(got["obj"], want["prim"])
    hit = want["prim"] >= 0
    assert hit.mean() > 0.3
    for k in ("t", "a", "b"):
        assert np.array_equal(got[k][hit].view(np.uint32), want[k][hit].view(np.uint32))


def write_c5_spec(path):
    cfg = scenes.CONFIGS["C5"]
    c, m, dome = cfg["camera"], cfg["material"], cfg["lights"][0]
    dragon, buddha = scenes.proto_objs(cfg)   # C5's meshes (the full-size buddha stand-in)
    lines = [f"obj {dragon}", f"obj {buddha}", f"hdr {scenes.SKIES[dome['sky']]}",
             "camera " + " ".join(repr(float(x)) for x in (*c["eye"], *c["lookAt"], *c["up"], c["fov"])),
             "material " + " ".join(repr(float(x)) for x in (*m["kd"], m["specExp"], m["specAmt"])),
             "bg " + " ".join(repr(float(x)) for x in cfg["bg"]),
             f"dome {dome['power']!r} {dome['samples']} {dome['noise']!r}", f"env {cfg['env']['exposure']!r}"]
    Ms = scenes.instance_transforms(**cfg["instances"])
    lines += ["instance " + " ".join(repr(float(x)) for x in np.asarray(M, np.float32).reshape(16)) for M in Ms]
    open(path, "w").write("\n".join(lines) + "\n")
    return Ms


def write_instance_rays(path, Ms, n=3000, seed=5):
    """Rays from around the instances toward their origins (world-space
    translation of each ProxyObject), plus some toward the floor."""
    rng = np.random.default_rng(seed)
    centres = np.array([np.asarray(M, np.float32).reshape(4, 4)[:3, 3] for M in Ms], np.float32)
    k = rng.integers(0, len(centres), n)
    tgt = centres[k] + rng.normal(scale=0.4, size=(n, 3)).astype(np.float32) + np.array([0, 0.8, 0], np.float32)
    o = (tgt + rng.normal(scale=4.0, size=(n, 3)) + np.array([0, 3.0, 0])).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmax = np.where(rng.uniform(size=n) < 0.15, 3.0, 1e12).astype(np.float32)
    with open(path, "wb") as f:
        np.array([n], np.int32).tofile(f)
        o.tofile(f); d.tofile(f); tmax.tofile(f)
    return o, d, tmax


HIT_REC = np.dtype([("t", "<f4"), ("a", "<f4"), ("b", "<f4"), ("id", "<i4"), ("inst", "<i4")])


@pytest.mark.gpu
def test_shim_renders_c5_instances_dome_and_env_like_the_oracle(tmp_path):
    """BASELINE config 5 through the compiled bridge: ProxyObject::setupProxy over
    two loaded meshes, 64 ProxyObject instances, the floor, a DomeLight and the
    environment map from the reference's Arches_E_PineTree.hdr (RawImage /
    Texture), Scene::raytraceImage at 128x72 and Scene::trace on rays aimed at
    the instances (HitInfo::obj = the proxy's Object, m_proxy = the instance).
    Hit ids exact; float RGB within 1e-4 relative (double atan2 / acos / pow)."""
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    from helpers import config_scene
    W, H = 128, 72
    spec, rays, out8, outf, outh, rayhits = (str(tmp_path / n) for n in
                                             ("c5.txt", "rays.bin", "o.rgb8", "o.rgbf", "o.hits", "r.hits"))
    Ms = write_c5_spec(spec)
    o, d, tmax = write_instance_rays(rays, Ms)
    r = subprocess.run([BIN, "c5", spec, str(W), str(H), out8, outf, outh, rays, rayhits], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr + r.stdout
    _, Osc, cam = config_scene("C5")
    ref = Osc.render(cam, W, H, threads=8)
    hits = np.fromfile(outh, HIT_REC).reshape(H, W)
    assert np.array_equal(hits["id"], ref["hits"]["prim"])
    n_world = 65   # 64 instances + the floor triangle
    inst_px = ref["hits"]["prim"] >= n_world
    assert inst_px.sum() > 500
    assert (hits["inst"][inst_px] >= 0).all() and (hits["inst"][~inst_px] == -1).all()
    rgb = np.fromfile(outf, np.float32).reshape(H, W, 3)
    g, rf = rgb.astype(np.float64), ref["rgb"].astype(np.float64)
    assert not (np.abs(g - rf) > 1e-4 * np.abs(rf)).any()
    assert np.mean(rgb.view(np.uint32) == ref["rgb"].view(np.uint32)) > 0.99
    img = np.fromfile(out8, np.uint8).reshape(H, W, 3)
    same = np.all(rgb.view(np.uint32) == ref["rgb"].view(np.uint32), axis=-1)
    assert np.array_equal(img[same], ref["rgb8"][same])
    # Scene::trace on instance rays: ids (instance BLAS objects) and t / a / b exact
    got = np.fromfile(rayhits, HIT_REC)
    want, _, _ = Osc.trace(o, d, 0.001, tmax)
    assert np.array_equal(got["id"], want["prim"])
    hit = want["prim"] >= 0
    assert (want["prim"] >= n_world).sum() > 1000
    for k in ("t", "a", "b"):
        assert np.array_equal(got[k][hit].view(np.uint32), want[k][hit].view(np.uint32))


def test_c_abi_light_transparency_flag():
    """Light::setFastShadows(false): a point light's transparent-shadow walk
    (src/PointLight.cpp:49-70) never traces (it loops while sampleHit.t <
    distance, starting at t = distance), so the C-ABI takes it as a light that
    casts no shadow; rectangle / dome lights take the transparency walk (ABI 9,
    tests/test_transparent.py)."""
    from miro import _lib
    L = miro.lib()
    s = L.mrt_scene_create()
    try:
        l = _lib.mrt_light(0, _lib.f3((0, 1, 0)), _lib.f3((0, 0, 0)), _lib.f3((0, 0, 0)), _lib.f3((0, 0, 0)), 1.0, 1,
                           0.001, 1, -1, 1)
        assert L.mrt_scene_add_light(s, C.byref(l)) >= 0       # point light: no shadow ray, as the reference
        r = _lib.mrt_light(1, _lib.f3((0, 0, 0)), _lib.f3((0, 2, 0)), _lib.f3((1, 2, 0)), _lib.f3((0, 2, 1)), 1.0, 1,
                           0.001, 1, -1, 1)
        assert L.mrt_scene_add_light(s, C.byref(r)) >= 0
    finally:
        L.mrt_scene_destroy(s)
    p = miro.PointLight()
    p.setFastShadows(False)
    assert p._c().transparent_shadows == 1
