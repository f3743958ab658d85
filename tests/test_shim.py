"""The compiled reference-side C++ bridge (shim/miro_shim.cpp): reference-layout
types (16-B Vector3 arrays, TupleI3 indices, one Object per triangle) marshalled
into libmrt by Scene::preCalc, then Scene::raytraceImage and Scene::trace
(reference src/Scene.h:31-32).  The GPU test renders config C1 through the
binary and compares with the CPU oracle: 8-bit pixels and hit records exact."""
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
