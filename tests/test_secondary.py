"""Blinn reflection and refraction rays (src/Blinn.cpp:91-335).

Blinn::shade picks, by Fresnel-weighted Russian roulette, either direct lighting
or one reflection / refraction ray (at most 5 bounces), carrying the ray's IOR
history (Ray::IORList, src/Ray.h:43-50).  The oracle restates that recursion
literally (oracle/mrt_oracle.c shade_blinn); the device runs it as a loop
(Shader::shade_path) and must be bit-identical.  CPU tests pin the oracle's
restatement by properties of the reference code (energy weights, bounce cap,
unchanged direct-only frames); against the reference binary itself parity is
statistical (its RNG pool is sequential), so it is unpinned.
"""
import numpy as np
import pytest

import miro
from helpers import bits, camera, fixture_mesh, scene_pair
from miro import scenes


def cornell(material, lights=None, subdivs=None):
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = material
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, subdivs=subdivs)


MIRROR = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=1.0, ior=1.5)
GLASS = dict(kind="blinn", kd=(0.6, 0.5, 0.4), refractAmt=1.0, ior=1.5)
GLOSSY = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=0.8, ior=1.5, specGloss=0.6, specExp=8.0, specAmt=0.3)
SHINY = dict(kind="blinn", kd=(0.6, 0.5, 0.4), specGloss=0.5, specExp=10.0, specAmt=0.5)   # gloss, no secondary rays
LEAF = dict(kind="blinn", kd=(0.3, 0.7, 0.2), translucency=0.6, specExp=6.0, specAmt=0.2)   # main.cpp:253
MIXED = dict(kind="blinn", kd=(0.6, 0.5, 0.4), ks=(0.9, 0.8, 0.7), reflectAmt=0.6, refractAmt=0.7, ior=1.33,
             specExp=12.0, specAmt=0.2)


def test_oracle_without_optics_spawns_no_secondary_rays():
    _, O_, cam = cornell(dict(kind="blinn", kd=(0.6, 0.5, 0.4)))
    assert O_.render(cam, 32, 24, threads=4)["secondary_rays"] == 0


@pytest.mark.parametrize("mat", [MIRROR, GLASS, MIXED])
def test_oracle_spawns_secondary_rays_and_stays_deterministic(mat):
    _, O_, cam = cornell(mat)
    a, b = O_.render(cam, 40, 30, threads=1), O_.render(cam, 40, 30, threads=8)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert a["secondary_rays"] == b["secondary_rays"] > 0
    # at most 5 bounces per shade call: <= 5 secondary rays per primary hit
    hits = int((a["hits"]["prim"] >= 0).sum())
    assert a["secondary_rays"] <= 5 * hits
    assert np.isfinite(a["rgb"]).all()


def test_oracle_black_mirror_frame_is_finite_and_non_negative():
    """kd = ka = 0: the direct branch is black; the reflection branch carries
    ks * (reflected colour) * rrWeightRecipSpec -- finite and non-negative."""
    _, O_, cam = cornell(dict(kind="blinn", kd=(0, 0, 0), reflectAmt=1.0, ior=1.5))
    ref = O_.render(cam, 16, 16, threads=4)
    assert ref["secondary_rays"] > 0
    assert (ref["rgb"] >= 0).all() and np.isfinite(ref["rgb"]).all()


def test_oracle_gloss_jitters_the_reflection_vector():
    """specGloss < 1 draws a cosine sample per shade (src/Blinn.cpp:166-171):
    the specular highlight moves, the frame stays deterministic."""
    _, O1, cam = cornell(dict(SHINY, specGloss=1.0))
    _, O2, _ = cornell(SHINY)
    a, b = O1.render(cam, 32, 24, threads=4), O2.render(cam, 32, 24, threads=4)
    assert not np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert np.array_equal(bits(b["rgb"]), bits(O2.render(cam, 32, 24, threads=1)["rgb"]))
    assert b["secondary_rays"] == 0


def leaf_floor(translucency):
    """Bunny stand-in + floor, one light above and one below the floor: the
    floor's back side (-normal) sees the lower light."""
    cfg = dict(scenes.CONFIGS["D1"])
    cfg.pop("env")
    cfg["material"] = dict(LEAF, translucency=translucency)
    lights = [dict(type="point", pos=(10.0, 20.0, 10.0), power=1000.0),
              dict(type="point", pos=(0.0, -5.0, 3.0), power=300.0)]
    return scene_pair(cfg, obj=scenes.bunny_obj(), floor=True, lights=lights)


def test_oracle_translucency_samples_the_back_side():
    """translucency > 0.01 adds one more sampleLight per light with -normal
    (src/Blinn.cpp:224-236): more shadow rays, a brighter floor."""
    _, O0, cam = leaf_floor(0.0)
    _, O1, _ = leaf_floor(0.6)
    a, b = O0.render(cam, 32, 24, threads=4), O1.render(cam, 32, 24, threads=4)
    assert b["shadow_rays"] > a["shadow_rays"]
    assert (b["rgb"] >= a["rgb"]).all() and (b["rgb"] > a["rgb"]).any()


def test_material_optics_are_validated():
    L = miro.lib()
    h = L.mrt_scene_create()
    try:
        from miro import _lib
        import ctypes as C
        m = _lib.mrt_material(1, (C.c_float * 3)(1, 1, 1), (C.c_float * 3)(0, 0, 0), (C.c_float * 3)(1, 1, 1), 1.0, 0.0)
        mid = L.mrt_scene_add_material(h, C.byref(m))
        assert L.mrt_scene_set_material_optics(h, mid, 0.5, 0.5, 1.5) == 0
        assert L.mrt_scene_set_material_gloss(h, mid, 0.5) == 0
        for bad in [(mid + 1, 0.5), (mid, -0.1), (mid, 1.5)]:
            assert L.mrt_scene_set_material_gloss(h, *bad) < 0
        for bad in [(mid + 1, 0.5, 0.5, 1.5), (mid, -1.0, 0.0, 1.5), (mid, 0.0, -1.0, 1.5), (mid, 0.0, 0.0, 0.0)]:
            assert L.mrt_scene_set_material_optics(h, *bad) < 0
    finally:
        L.mrt_scene_destroy(h)


# ---------------------------------------------------------------- GPU parity
def gpu_frame(P, cam, W, H, **kw):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True, **kw)
    return img, hits


def assert_same(P, O_, cam, W, H):
    img, hits = gpu_frame(P, cam, W, H)
    ref = O_.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "primary hit ids differ"
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"]), "8-bit RGB differs"
    assert P.last_stats["secondary_rays"] == ref["secondary_rays"]
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("mat", [MIRROR, GLASS, MIXED, GLOSSY], ids=["mirror", "glass", "mixed", "glossy"])
def test_secondary_rays_match_oracle(mat):
    P, O_, cam = cornell(mat)
    ref = assert_same(P, O_, cam, 72, 56)
    assert ref["secondary_rays"] > 0


@pytest.mark.gpu
def test_translucency_matches_oracle():
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=3, noise=0.001),
              dict(type="point", pos=(2.75, 2.0, -2.75), power=20.0)]
    P, O_, cam = cornell(LEAF, lights=lights)
    assert_same(P, O_, cam, 64, 48)
    P, O_, cam = leaf_floor(0.6)
    assert_same(P, O_, cam, 48, 40)


@pytest.mark.gpu
def test_gloss_without_secondary_rays_matches_oracle():
    P, O_, cam = cornell(SHINY)
    ref = assert_same(P, O_, cam, 64, 48)
    assert ref["secondary_rays"] == 0


@pytest.mark.gpu
def test_secondary_rays_with_area_light_environment_and_supersampling():
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=3, noise=0.001),
              dict(type="point", pos=(1.0, 3.0, -1.0), power=5.0)]
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = MIXED
    cfg["env"] = dict(sky=(64, 32), exposure=0.7)
    P, O_, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, subdivs=(1, 2, 0.01))
    assert_same(P, O_, cam, 48, 40)


@pytest.mark.gpu
def test_secondary_rays_on_the_bunny_with_a_dome_light():
    """Closed mesh (refraction in and out through the IOR history) lit by a dome."""
    cfg = dict(scenes.CONFIGS["D1"])
    cfg["material"] = dict(MIXED, kd=(0.8, 0.8, 0.8))
    P, O_, cam = scene_pair(cfg, obj=scenes.bunny_obj(), floor=True)
    assert_same(P, O_, cam, 40, 40)
