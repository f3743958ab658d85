"""ABI 4 additions (include/mrt.h): HitInfo identity (mrt_hit.inst,
mrt_scene_prim_object), 16-byte Vector3 mesh strides, emission setters, the
int32 hit-id guard, and mrt_render over several devices."""
import ctypes as C

import numpy as np
import pytest

import miro
from miro import _lib
from helpers import bits, camera, config_scene, fixture_mesh


def _mesh(L, h, v, n, vi, ni, mat, vs=3, ns=3):
    m = _lib.mrt_mesh(v.ctypes.data_as(C.POINTER(C.c_float)), n.ctypes.data_as(C.POINTER(C.c_float)),
                      vi.ctypes.data_as(C.POINTER(C.c_uint32)), ni.ctypes.data_as(C.POINTER(C.c_uint32)),
                      len(v), len(n), len(vi), vs, ns)
    return _lib.check(L.mrt_scene_add_mesh(h, C.byref(m), mat), "add_mesh")


def _scene(L):
    h = L.mrt_scene_create()
    mat = _lib.mrt_material(0, _lib.f3((1, 1, 1)), _lib.f3((0, 0, 0)), _lib.f3((1, 1, 1)), 1.0, 0.0,
                            _lib.f3((0, 0, 0)), 0.0)
    return h, _lib.check(L.mrt_scene_add_material(h, C.byref(mat)), "material")


def _export(L, h):
    info = _lib.mrt_bvh_info()
    _lib.check(L.mrt_scene_bvh_info(h, C.byref(info)), "info")
    nb = np.zeros((info.nodes, 24), np.float32); nc = np.zeros((info.nodes, 4), np.int32)
    lt = np.zeros((info.leaves, 36), np.float32); lp = np.zeros((info.leaves, 4), np.int32)
    fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int32)
    _lib.check(L.mrt_scene_bvh_export(h, nb.ctypes.data_as(fp), nc.ctypes.data_as(ip), lt.ctypes.data_as(fp),
                                      lp.ctypes.data_as(ip)), "export")
    return nb, nc, lt, lp


def test_vector3_stride_mesh_equals_packed_mesh():
    """TriangleMesh keeps 16-B Vector3s (src/Vector3.h:19): stride 4 hands them over as they are."""
    L = miro.lib()
    v, n, vi, ni = fixture_mesh("teapot")
    v4 = np.zeros((len(v), 4), np.float32); v4[:, :3] = v; v4[:, 3] = 7.0     # garbage in the pad
    n4 = np.zeros((len(n), 4), np.float32); n4[:, :3] = n; n4[:, 3] = -3.0
    out = []
    for vv, nn, s in ((v, n, 3), (v4, n4, 4)):
        h, mat = _scene(L)
        _mesh(L, h, np.ascontiguousarray(vv), np.ascontiguousarray(nn), vi, ni, mat, s, s)
        _lib.check(L.mrt_scene_build_bvh(h), "build")
        out.append(_export(L, h))
        L.mrt_scene_destroy(h)
    for a, b in zip(*out):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_bad_stride_is_rejected():
    L = miro.lib()
    v, n, vi, ni = fixture_mesh("cornell_box")
    h, mat = _scene(L)
    m = _lib.mrt_mesh(v.ctypes.data_as(C.POINTER(C.c_float)), n.ctypes.data_as(C.POINTER(C.c_float)),
                      vi.ctypes.data_as(C.POINTER(C.c_uint32)), ni.ctypes.data_as(C.POINTER(C.c_uint32)),
                      len(v), len(n), len(vi), 2, 3)
    assert L.mrt_scene_add_mesh(h, C.byref(m), mat) == -1
    L.mrt_scene_destroy(h)


def test_prim_object_names_mesh_triangle_and_instance():
    """HitInfo::obj (Object: m_mesh, m_index, src/Object.h:49-77) and m_proxy for every hit id."""
    L = miro.lib()
    h, mat = _scene(L)
    floor = (np.array([(-9, 0, -9), (0, 0, 9), (9, 0, -9)], np.float32), np.array([(0, 1, 0)] * 3, np.float32),
             np.array([(0, 1, 2)], np.uint32), np.array([(0, 1, 2)], np.uint32))
    m_floor = _mesh(L, h, *floor, mat)
    tv, tn, tvi, tni = fixture_mesh("teapot")
    m_tea = _mesh(L, h, tv, tn, tvi, tni, mat)
    m_box = _mesh(L, h, *fixture_mesh("cornell_box"), mat)
    ids = (C.c_int32 * 1)(m_tea)
    blas = _lib.check(L.mrt_scene_make_blas(h, ids, 1), "blas")
    eye = np.eye(4, dtype=np.float32)
    for k in range(3):
        M = eye.copy(); M[0, 3] = 3.0 * k
        _lib.check(L.mrt_scene_add_instance(h, blas, M.ctypes.data_as(C.POINTER(C.c_float))), "instance")
    _lib.check(L.mrt_scene_build_bvh(h), "build")
    me, tr, ins = C.c_int32(), C.c_int32(), C.c_int32()

    def obj(p):
        _lib.check(L.mrt_scene_prim_object(h, p, C.byref(me), C.byref(tr), C.byref(ins)), "prim_object")
        return me.value, tr.value, ins.value

    # world objects in add order: the floor, the box (the teapot went into the BLAS), then the 3 proxies
    assert obj(0) == (m_floor, 0, -1)
    assert obj(1) == (m_box, 0, -1) and obj(36) == (m_box, 35, -1)
    assert obj(37)[2] == 0 and obj(37)[0] == -1           # ProxyObject 0's own slot
    nt = len(tvi)
    base = 1 + 36 + 3
    # ProxyObject::setupMultiProxy: a mesh's triangles last to first
    assert obj(base) == (m_tea, nt - 1, 0)
    assert obj(base + nt - 1) == (m_tea, 0, 0)
    assert obj(base + nt) == (m_tea, nt - 1, 1)
    assert obj(base + 3 * nt - 1) == (m_tea, 0, 2)
    assert L.mrt_scene_prim_object(h, base + 3 * nt, C.byref(me), C.byref(tr), C.byref(ins)) == -1
    L.mrt_scene_destroy(h)


def test_hit_ids_beyond_int32_are_rejected():
    """A 201 x 201 proxy grid (src/main.cpp:37-51) of a big BLAS overflows int32 hit
    ids: the build refuses instead of wrapping."""
    L = miro.lib()
    h, mat = _scene(L)
    n = 256   # 2 * 256^2 = 131072 triangles
    g = np.stack(np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij"), -1).reshape(-1, 2).astype(np.float32)
    v = np.concatenate([g, np.zeros((len(g), 1), np.float32)], 1)
    v += np.random.default_rng(5).uniform(-1e-3, 1e-3, v.shape).astype(np.float32)
    idx = np.arange((n + 1) ** 2).reshape(n + 1, n + 1)
    a, b, c, d = idx[:-1, :-1], idx[1:, :-1], idx[1:, 1:], idx[:-1, 1:]
    f = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)]).astype(np.uint32)
    nrm = np.array([(0, 0, 1)], np.float32)
    mid = _mesh(L, h, np.ascontiguousarray(v), nrm, f, np.zeros_like(f), mat)
    blas = _lib.check(L.mrt_scene_make_blas(h, (C.c_int32 * 1)(mid), 1), "blas")
    need = (2 ** 31) // len(f) + 1
    M = np.eye(4, dtype=np.float32)
    for k in range(need):
        M[0, 3] = float(k % 256) * 300.0
        M[1, 3] = float(k // 256) * 300.0
        _lib.check(L.mrt_scene_add_instance(h, blas, M.ctypes.data_as(C.POINTER(C.c_float))), "instance")
    assert L.mrt_scene_build_bvh(h) == -1
    assert b"exceed 2^31" in L.mrt_last_error()
    L.mrt_scene_destroy(h)


def test_emission_setter_only_for_blinn():
    L = miro.lib()
    h, mat = _scene(L)                       # a Lambert material
    assert L.mrt_scene_set_material_emission(h, mat, 1.0, _lib.f3((1, 1, 1))) == -1
    assert L.mrt_scene_set_path_trace(h, 1, 0, 0) == -1 and L.mrt_scene_set_path_trace(h, 1, 65, 0) == -1
    assert L.mrt_scene_set_path_trace(h, 1, 10, 0) == 0
    L.mrt_scene_destroy(h)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("key,W,H,devices", [("C1", 96, 80, [0, 0]), ("C4", 128, 72, [0, 0, 0]),
                                              ("C5", 96, 64, [0, 0])])
def test_render_over_device_shares_equals_one_device(key, W, H, devices):
    """mrt_render_opts.devices: buckets b -> devices[b % n] (here shares of one GPU),
    gathered on the host -- bit-identical to the one-device frame."""
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    P, _, cam = config_scene(key)
    one = miro.Image(); one.resize(W, H)
    h1 = P.raytraceImage(camera(cam), one, want_hits=True)
    s1 = dict(P.last_stats)
    many = miro.Image(); many.resize(W, H)
    h2 = P.raytraceImage(camera(cam), many, want_hits=True, devices=devices)
    s2 = P.last_stats
    assert np.array_equal(bits(one.rgb), bits(many.rgb))
    assert np.array_equal(one.pixels, many.pixels)
    assert np.array_equal(h1, h2)
    assert s1["shadow_rays"] == s2["shadow_rays"]


@pytest.mark.gpu
def test_trace_reports_the_instance_of_a_hit():
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    P, _, cam = config_scene("C5")
    rng = np.random.default_rng(3)
    o = np.tile(np.array([[0.0, 10.0, 27.0]], np.float32), (4000, 1))
    d = rng.normal(size=(4000, 3)).astype(np.float32) * 0.15 + np.array([0.0, -0.35, -1.0], np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    got = P.traceBatch(o, d)
    hit = got["prim"] >= 0
    assert (got["inst"][hit] >= 0).sum() > 100
    for p, i in zip(got["prim"][hit][:300], got["inst"][hit][:300]):
        assert P.primObject(int(p))[2] == i
