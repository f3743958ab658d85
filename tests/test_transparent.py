"""Transparent shadows of rectangle / dome lights and per-material environment maps.

Light::setFastShadows(false) (src/Light.h:24) switches RectangleLight::sampleLight
(src/RectangleLight.cpp:93-116) and DomeLight::sampleLight (src/DomeLight.cpp:123-145)
from one any-hit shadow ray to a walk of closest-hit rays through every surface
on the way, attenuated by the hit material's refractAmt where the hit's
interpolated normal faces the ray.  sampleHit lives across that loop, so each
trace is bounded by the previous hit's t (the oracle and Shader::transmit keep
that).  Material::setEnvMap (src/Material.h:19) gives a Blinn material its own
map for missed reflection / refraction / GI rays (Material::getEnvironmentColor,
src/Material.cpp:44-64).

CPU: the oracle's walk against properties of the reference code (a pane of
glass passes refractAmt of the light, an opaque pane none; a point light's
walk never traces); the C-ABI accepts the flags.  GPU: libmrt against the
oracle, bit for bit (hits, RGB, 8-bit, shadow and secondary ray counts):
the fused direct kernel, the fused chain kernel, supersampling, a dome light,
instanced BLASes (object-space normals), and material environment maps on the
fused and the wavefront chain engines.  Parity against the reference binary
itself is unpinned (the reference does not build here)."""
import ctypes as C

import numpy as np
import pytest

import miro
from helpers import bits, camera, fixture_mesh, scene_pair
from miro import scenes

RECT = dict(type="rect", v1=(2.0, 5.4, -2.0), v2=(3.5, 5.4, -2.0), v3=(2.0, 5.4, -3.5), power=15.0, samples=3,
            noise=0.001)
GLASS_PANE = dict(kind="blinn", kd=(0.5, 0.6, 0.7), refractAmt=0.6, ior=1.3, specExp=8.0, specAmt=0.2)
OPAQUE_PANE = dict(kind="lambert", kd=(0.5, 0.6, 0.7))


def pane(y=3.5, x=(1.0, 4.5), z=(-4.5, -1.0), up=True):
    """A horizontal quad (two triangles) under the ceiling light, normals up or down."""
    v = np.array([(x[0], y, z[0]), (x[1], y, z[0]), (x[1], y, z[1]), (x[0], y, z[1])], np.float32)
    n = np.array([(0, 1 if up else -1, 0)] * 4, np.float32)
    i = np.array([(0, 2, 1), (0, 3, 2)] if up else [(0, 1, 2), (0, 2, 3)], np.uint32)
    return v, n, i, i


def cornell(material=None, lights=None, extra=None, subdivs=None, num_paths=1, env=None):
    cfg = dict(scenes.CONFIGS["C1"], material=material or dict(kind="lambert", kd=(0.8, 0.8, 0.8)))
    if env:
        cfg["env"] = env
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights or [dict(RECT, fast_shadows=False)],
                      extra=extra, subdivs=subdivs, num_paths=num_paths)


# ------------------------------------------------------------------ CPU: the oracle's walk
def test_oracle_glass_pane_passes_refract_amount_of_the_light():
    """The walk attenuates only at faces whose normal faces the shadow ray's
    reverse direction: a glass pane facing the floor passes refractAmt of the
    light, one facing the light passes all of it, fast shadows pass none; an
    opaque (Lambert, refractAmt 0) pane facing the floor stops it as fast
    shadows do."""
    W, H = 40, 30
    n_box = fixture_mesh("cornell_box")[2].shape[0]
    fr = {}
    for name, mat, up, fast in [("down_walk", GLASS_PANE, False, False), ("up_walk", GLASS_PANE, True, False),
                                ("fast", GLASS_PANE, False, True), ("opaque_walk", OPAQUE_PANE, False, False)]:
        _, O_, cam = cornell(lights=[dict(RECT, fast_shadows=fast)], extra=[(pane(up=up), mat)])
        fr[name] = O_.render(cam, W, H, threads=8)
    prim = fr["fast"]["hits"]["prim"]
    box = (prim >= 0) & (prim < n_box)            # pixels whose eye ray hits the box, not the pane
    lum = {k: v["rgb"].sum(-1)[box] for k, v in fr.items()}
    assert (lum["down_walk"] >= lum["fast"]).all() and (lum["up_walk"] >= lum["down_walk"]).all()
    assert lum["down_walk"].sum() > lum["fast"].sum() * 1.02
    assert lum["up_walk"].sum() > lum["down_walk"].sum() * 1.02
    assert np.array_equal(bits(fr["opaque_walk"]["rgb"])[box], bits(fr["fast"]["rgb"])[box])
    # every walk step is a traced (counted) ray
    assert fr["up_walk"]["shadow_rays"] > fr["fast"]["shadow_rays"]
    _, O1, _ = cornell(lights=[dict(RECT, fast_shadows=False)], extra=[(pane(up=False), GLASS_PANE)])
    assert np.array_equal(bits(fr["down_walk"]["rgb"]), bits(O1.render(cam, W, H, threads=1)["rgb"]))


def test_oracle_walk_without_occluders_equals_fast_shadows():
    """Nothing between the floor and the light: the walk's first trace misses, so
    the frame and the shadow-ray count equal the fast-shadow ones."""
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.8, 0.8, 0.8)))
    floor = [(pane(y=0.0, x=(-3, 3), z=(-3, 3)), dict(kind="lambert", kd=(0.7, 0.7, 0.7)))]
    light = dict(type="rect", v1=(-1.0, 4.0, -1.0), v2=(1.0, 4.0, -1.0), v3=(-1.0, 4.0, 1.0), power=20.0, samples=2,
                 noise=0.001)
    cam = dict(eye=(0.0, 3.0, 4.0), lookAt=(0.0, 0.0, 0.0), up=(0, 1, 0), fov=50.0)
    out = []
    for fast in (True, False):
        _, O_, _ = scene_pair(dict(cfg, camera=cam), extra=floor, lights=[dict(light, fast_shadows=fast)])
        out.append(O_.render(cam, 32, 24, threads=8))
    assert np.array_equal(bits(out[0]["rgb"]), bits(out[1]["rgb"]))
    assert out[0]["shadow_rays"] == out[1]["shadow_rays"]


def test_oracle_material_env_map_replaces_the_scene_map():
    """A mirror with its own map reflects that map where its reflection rays miss;
    the same map as the scene's (same exposure) gives the scene-map frame."""
    mirror = dict(kind="blinn", kd=(0.2, 0.2, 0.2), reflectAmt=1.0, ior=1.5)
    cfg = dict(scenes.CONFIGS["D1"], material=mirror, lights=[dict(type="point", pos=(10.0, 20.0, 10.0), power=800.0)])
    cam = cfg["camera"]
    _, Os, _ = scene_pair(cfg, obj=scenes.bunny_obj(), floor=True)
    _, Om, _ = scene_pair(dict(cfg, material=dict(mirror, env=dict(sky=(32, 16), exposure=2.0))), obj=scenes.bunny_obj(),
                          floor=True)
    _, Oq, _ = scene_pair(dict(cfg, material=dict(mirror, env=dict(cfg["env"]))), obj=scenes.bunny_obj(), floor=True)
    a, b, q = (o.render(cam, 40, 30, threads=8) for o in (Os, Om, Oq))
    assert a["secondary_rays"] == b["secondary_rays"] > 0
    assert not np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert np.array_equal(bits(a["rgb"]), bits(q["rgb"]))


def test_c_abi_accepts_transparent_lights_and_material_env_maps():
    from miro import _lib
    L = miro.lib()
    s = L.mrt_scene_create()
    try:
        r = _lib.mrt_light(1, _lib.f3((0, 0, 0)), _lib.f3((0, 2, 0)), _lib.f3((1, 2, 0)), _lib.f3((0, 2, 1)), 1.0, 1,
                           0.001, 1, -1, 1)
        assert L.mrt_scene_add_light(s, C.byref(r)) >= 0
        m = _lib.mrt_material(1, _lib.f3((1, 1, 1)), _lib.f3((0, 0, 0)), _lib.f3((1, 1, 1)), 1.0, 0.0,
                              _lib.f3((0, 0, 0)), 0.0)
        mid = L.mrt_scene_add_material(s, C.byref(m))
        assert mid >= 0
        rgb = np.ones((4, 8, 3), np.float32)
        t = L.mrt_scene_add_texture(s, rgb.ctypes.data_as(C.POINTER(C.c_float)), 8, 4)
        gray = np.ones((4, 8, 1), np.float32)
        g = L.mrt_scene_add_texture_typed(s, gray.ctypes.data_as(C.POINTER(C.c_float)), 8, 4, 1)
        assert L.mrt_scene_set_material_env_map(s, mid, t, 1.5) == 0
        assert L.mrt_scene_set_material_env_map(s, mid, -1, 1.0) == 0
        assert L.mrt_scene_set_material_env_map(s, mid, g, 1.0) == -1        # one channel: not a lat-long map
        assert L.mrt_scene_set_material_env_map(s, mid, t + 5, 1.0) == -1
        assert L.mrt_scene_set_material_env_map(s, mid + 1, t, 1.0) == -1
    finally:
        L.mrt_scene_destroy(s)


# ------------------------------------------------------------------ GPU parity
def need_gpu():
    if miro.device_count() < 1:
        pytest.skip("no HIP device")


def assert_same(P, O_, cam, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = O_.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "primary hit ids differ"
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"]), "8-bit RGB differs"
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    assert P.last_stats["secondary_rays"] == ref["secondary_rays"]
    return ref


@pytest.mark.gpu
def test_transparent_rect_light_opaque_scene_matches_oracle():
    """No refractive material: the fused direct kernel (no chain); back faces on the
    way let the light through, front faces stop it."""
    need_gpu()
    P, O_, cam = cornell(extra=[(pane(up=False), OPAQUE_PANE)])
    assert_same(P, O_, cam, 64, 48)


@pytest.mark.gpu
@pytest.mark.parametrize("up", [True, False], ids=["pane_up", "pane_down"])
def test_transparent_rect_light_through_glass_matches_oracle(up):
    """A glass pane (refractAmt 0.6) between the light and the floor: the fused
    chain kernel (the scene has refraction rays) with the walk in its shading."""
    need_gpu()
    P, O_, cam = cornell(lights=[dict(RECT, fast_shadows=False), dict(type="point", pos=(1.0, 3.0, -1.0), power=5.0)],
                         extra=[(pane(up=up), GLASS_PANE), (pane(y=2.0, x=(2.0, 3.0), z=(-3.0, -2.0)), GLASS_PANE)],
                         num_paths=2)
    ref = assert_same(P, O_, cam, 64, 48)
    assert ref["secondary_rays"] > 0


@pytest.mark.gpu
def test_transparent_rect_light_with_supersampling_matches_oracle():
    need_gpu()
    P, O_, cam = cornell(extra=[(pane(), GLASS_PANE)], subdivs=(1, 3, 0.01))
    assert_same(P, O_, cam, 48, 40)


@pytest.mark.gpu
def test_transparent_dome_light_matches_oracle():
    """Dome light over a glass bunny on a floor (the walk starts at MIRO_TMAX)."""
    need_gpu()
    cfg = dict(scenes.CONFIGS["D1"], material=dict(GLASS_PANE, kd=(0.6, 0.6, 0.6)))
    cfg["lights"] = [dict(l, fast_shadows=False, samples=3) if l["type"] == "dome" else l for l in cfg["lights"]]
    P, O_, cam = scene_pair(cfg, obj=scenes.bunny_obj(), floor=True)
    assert_same(P, O_, cam, 48, 36)


@pytest.mark.gpu
def test_transparent_shadows_through_instances_match_oracle():
    """Glass leaves in ProxyObject instances: the walk's hit normal is the BLAS
    mesh's, in object space (getInterpolatedNormal has no m_invTranspose)."""
    need_gpu()
    from test_textures import LEAF_CAM, LEAF_OBJ
    leaf = dict(kind="blinn", kd=(0.4, 0.8, 0.3), refractAmt=0.5, ior=1.2, specExp=6.0, specAmt=0.2)
    placed = []
    for i in range(5):
        a = 1.1 * i
        c, s = np.cos(a), np.sin(a)
        placed.append((0, np.array([[c * 0.6, 0, s * 0.6, 0.4 * np.cos(2.0 * i)], [0, 0.6, 0, 0.3 * (i % 3)],
                                    [-s * 0.6, 0, c * 0.6, 0.4 * np.sin(2.0 * i)], [0, 0, 0, 1]], np.float32)))
    lights = [dict(type="rect", v1=(-0.5, 3.0, -0.5), v2=(0.5, 3.0, -0.5), v3=(-0.5, 3.0, 0.5), power=20.0, samples=3,
                   noise=0.001, fast_shadows=False)]
    P, O_, _ = scene_pair(dict(scenes.CONFIGS["C1"], material=leaf), instances=([LEAF_OBJ], placed), lights=lights,
                          floor=True)
    ref = assert_same(P, O_, LEAF_CAM, 56, 56)
    assert (ref["hits"]["prim"] >= 0).mean() > 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("chain", [1, 0], ids=["chain_engine", "fused"])
def test_material_env_maps_match_oracle(chain):
    """Mirror, glass and a path-traced diffuse material, each with its own map, over
    a scene map: the wavefront chain engine (fold-time lookup of the parent
    material's map) and the fused chain kernel."""
    need_gpu()
    mirror = dict(kind="blinn", kd=(0.2, 0.2, 0.2), reflectAmt=0.9, ior=1.5, env=dict(sky=(32, 16), exposure=2.0))
    glass = dict(GLASS_PANE, refractAmt=0.9, env=dict(sky=(48, 24), exposure=0.5))
    cfg = dict(scenes.CONFIGS["C1"], material=mirror)
    L = miro.lib()
    try:
        assert L.mrt_set_tuning(b"chain", chain) == 0
        P, O_, cam = scene_pair(dict(cfg, env=dict(sky=(64, 32), exposure=0.7)), meshes=[fixture_mesh("cornell_box")],
                                extra=[(pane(y=2.0), glass)], num_paths=2)
        ref = assert_same(P, O_, cam, 64, 48)
        assert ref["secondary_rays"] > 0
        assert P.last_stats["chain"] == chain
        diffuse = dict(kind="blinn", kd=(0.7, 0.7, 0.7), env=dict(sky=(32, 16), exposure=3.0))
        P, O_, cam = scene_pair(dict(cfg, material=diffuse, env=dict(sky=(64, 32), exposure=1.0)),
                                meshes=[fixture_mesh("cornell_box")], path_trace=(3, True), num_paths=2)
        assert_same(P, O_, cam, 48, 36)
    finally:
        L.mrt_set_tuning(b"chain", 1)
