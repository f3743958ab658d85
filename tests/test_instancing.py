"""ProxyObject instancing (reference src/ProxyObject.cpp, src/BVH.cpp:1305-1315,
src/Ray.cpp:27-31): the product (libmrt host build + HIP kernels) against the CPU
oracle.  CPU tests compare the BLAS and the world QBVH with proxies bit for bit;
GPU tests compare rendered frames (hit ids, t/a/b, float and 8-bit RGB, shadow
ray counts) and batched ray queries bit for bit."""
import numpy as np
import pytest

import miro
import oracle as O
from helpers import bits, camera, fixture_mesh


def rot_y(deg, s=1.0, t=(0.0, 0.0, 0.0)):
    a = np.radians(deg)
    c, n = np.cos(a), np.sin(a)
    return np.array([[c * s, 0, n * s, t[0]], [0, s, 0, t[1]], [-n * s, 0, c * s, t[2]], [0, 0, 0, 1]], np.float32)


def rot_x(deg, s=1.0, t=(0.0, 0.0, 0.0)):
    a = np.radians(deg)
    c, n = np.cos(a), np.sin(a)
    return np.array([[s, 0, 0, t[0]], [0, c * s, -n * s, t[1]], [0, n * s, c * s, t[2]], [0, 0, 0, 1]], np.float32)


FLOOR = (np.array([(-100, 0, -100), (0, 0, 100), (100, 0, -100)], np.float32), np.array([(0, 1, 0)] * 3, np.float32),
         np.array([(0, 1, 2)], np.uint32), np.array([(0, 1, 2)], np.uint32))


def instanced_pair(kind="lambert", transforms=None, lights=(("point", (10.0, 20.0, 10.0), 1000.0),),
                   blas_meshes=("teapot",), floor_first=True, spec=(1.0, 0.0)):
    """(product Scene, oracle scene): an optional world floor triangle and
    instances of one BLAS built from fixture meshes, in call order."""
    P = miro.Scene()
    Osc = O.OracleScene()
    pm = miro.Lambert((0.8, 0.7, 0.6)) if kind == "lambert" else miro.Blinn((0.8, 0.7, 0.6), specExp=spec[0],
                                                                           specAmt=spec[1])
    om = Osc.add_material(kind, kd=(0.8, 0.7, 0.6), specExp=spec[0], specAmt=spec[1])
    fm = miro.Lambert((0.5, 0.5, 0.5))
    ofm = Osc.add_material("lambert", kd=(0.5, 0.5, 0.5))
    transforms = transforms if transforms is not None else [rot_y(0, 1.0, (-3, 0, 0)), rot_y(40, 0.8, (0, 0.5, -2)),
                                                            rot_x(-30, 1.3, (3.5, 1.0, 0.5)), rot_y(200, 0.6, (0, 3, 1))]

    def floor():
        tm = miro.TriangleMesh()
        tm.setArrays(*FLOOR)
        miro.makeMeshObjs(P, tm, fm)
        Osc.add_mesh(*FLOOR, ofm)

    if floor_first:
        floor()
    objs, bvh = miro.Objects(), miro.BVH()
    ometa = []
    for name in blas_meshes:
        arrs = fixture_mesh(name)
        tm = miro.TriangleMesh()
        tm.setArrays(*arrs)
        objs.append((tm, pm))
        ometa.append(Osc.add_mesh(*arrs, om))
    bvh.objects = objs
    oblas = Osc.make_blas(ometa)
    for M in transforms:
        P.addObject(miro.ProxyObject(objs, bvh, miro.Matrix4x4(M)))
        Osc.add_instance(oblas, M)
    if not floor_first:
        floor()
    for kind_l, pos, power in lights:
        pl = miro.PointLight(); pl.setPosition(pos); pl.setPower(power)
        P.addLight(pl)
        Osc.add_point_light(pos, power)
    P.setBGColor((0.0, 0.0, 0.2))
    Osc.set_bg((0.0, 0.0, 0.2))
    P.preCalc()
    Osc.build()
    return P, Osc


CAM = dict(eye=(0.0, 4.0, 12.0), lookAt=(0.0, 1.0, 0.0), up=(0, 1, 0), fov=45.0)


def assert_same_arrays(a_list, b_list):
    for a, b in zip(a_list, b_list):
        a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
        assert a.shape == b.shape
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("floor_first", [True, False])
def test_blas_and_world_hierarchy_match_oracle(floor_first):
    P, Osc = instanced_pair(floor_first=floor_first)
    assert_same_arrays(P.blas_export(0), Osc.blas_export(0))
    info = Osc.qbvh_info()
    assert P.bvh_info["nodes"] == info["nodes"] and P.bvh_info["prims"] == info["prims"] == 1 + 4
    assert_same_arrays(P.bvh_export(), Osc.qbvh_export())


def test_blas_of_two_meshes_and_many_instances_match_oracle():
    ts = [rot_y(17 * i, 0.3 + 0.05 * (i % 5), (i % 8 - 4.0, 0.2 * (i // 8), -(i // 8) * 1.5)) for i in range(40)]
    P, Osc = instanced_pair(transforms=ts, blas_meshes=("teapot", "cornell_box"))
    assert_same_arrays(P.blas_export(0), Osc.blas_export(0))
    assert_same_arrays(P.bvh_export(), Osc.qbvh_export())


def test_blas_objects_are_reversed_per_mesh():
    """ProxyObject::setupProxy pushes a mesh's triangles last to first
    (src/ProxyObject.cpp:136-144): the BLAS leaf prims index that order."""
    P, Osc = instanced_pair(transforms=[np.eye(4, dtype=np.float32)])
    nt = len(fixture_mesh("teapot")[2])
    lp = P.blas_export(0)[3]
    ids = np.sort(lp[lp >= 0])
    assert np.array_equal(ids, np.arange(nt))


def test_instancing_errors_fail_loudly():
    import ctypes as C
    L = miro.lib()
    h = L.mrt_scene_create()
    try:
        ids = (C.c_int32 * 1)(0)
        assert L.mrt_scene_make_blas(h, ids, 1) == -1           # no such mesh
        m16 = (C.c_float * 16)(*np.eye(4, dtype=np.float32).ravel())
        assert L.mrt_scene_add_instance(h, 0, m16) == -1         # no such BLAS
    finally:
        L.mrt_scene_destroy(h)


# ---------------------------------------------------------------- GPU parity
gpu = pytest.mark.gpu


def render(P, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(CAM), img, want_hits=True)
    return img, hits


@gpu
@pytest.mark.parametrize("kind,W,H", [("lambert", 96, 72), ("blinn", 77, 53)])
def test_instanced_frame_matches_oracle(kind, W, H):
    if miro.device_count() < 1:
        pytest.fail("no HIP device visible")
    P, Osc = instanced_pair(kind)
    img, hits = render(P, W, H)
    ref = Osc.render(CAM, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"])
    inst_hits = ref["hits"]["prim"] >= P.bvh_info["prims"]
    assert inst_hits.sum() > 100
    hit = ref["hits"]["prim"] >= 0
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(hits[k][hit]), bits(ref["hits"][k][hit])), k
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
    assert np.array_equal(img.pixels, ref["rgb8"])


@gpu
def test_instanced_trace_batch_matches_oracle():
    if miro.device_count() < 1:
        pytest.fail("no HIP device visible")
    P, Osc = instanced_pair()
    rng = np.random.default_rng(5)
    n = 20000
    o = np.stack([rng.uniform(-6, 6, n), rng.uniform(0.2, 6, n), rng.uniform(4, 10, n)], 1).astype(np.float32)
    tgt = np.stack([rng.uniform(-5, 5, n), rng.uniform(0, 3, n), rng.uniform(-3, 2, n)], 1).astype(np.float32)
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    got = P.traceBatch(o, d, 0.001, 1e12)
    want, _, _ = Osc.trace(o, d, 0.001, 1e12)
    assert np.array_equal(got["prim"], want["prim"])
    hit = want["prim"] >= 0
    assert (want["prim"] >= P.bvh_info["prims"]).sum() > 1000
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(got[k][hit]), bits(want[k][hit])), k
    occl = P.traceBatch(o, d, 0.001, 1e12, any_hit=True)
    assert np.array_equal(occl["prim"] >= 0, hit)
