"""Dispersion (Material::m_disperse with Blinn m_ior[0..2], src/Blinn.cpp:169-185,275-301).

A ray that is not itself a refraction ray and picks refraction at a dispersive
Blinn material splits into three refraction rays, one per colour channel i,
through m_ior[i]; each child's colour is masked to its channel, a missed child
adds nothing, and only when no child hits does Lt take the environment along
the last direction computed (channel 2).  The split also changes the IOR rules
of the shade() call: outIOR = m_ior[0] for Fresnel and no pop on a back-face
hit.  The non-dispersive refraction reads m_ior[1] (src/Blinn.cpp:183), so the
reference's setIor(x) -- which sets m_ior[0] -- changes only dispersion.

The oracle restates the recursion literally (oracle/mrt_oracle.c shade_blinn);
the device walks the three-way tree depth first in the fused kernels
(Shader::shade_path, disp_child) and must be bit-identical.  The CPU tests pin
the restatement by an identity of the reference code: with three equal IORs and
children that land on Lambert surfaces (whose shading draws no random numbers),
the split's masked channels add up to the plain refraction exactly, with three
times the secondary rays.
"""
import numpy as np
import pytest

import miro
from helpers import bits, camera, fixture_mesh, scene_pair
from miro import scenes


def quad(z=1.0, lo=0.5, hi=5.0):
    """A two-triangle sheet at depth z facing the C1 camera (+z geometric normal)."""
    v = np.array([[lo, lo, z], [hi, lo, z], [hi, hi, z], [lo, hi, z]], np.float32)
    n = np.tile(np.array([[0, 0, 1]], np.float32), (4, 1))
    idx = np.array([[0, 1, 2], [0, 2, 3]], np.uint32)
    return v, n, idx, idx.copy()


SHEET = dict(kind="blinn", kd=(0.5, 0.5, 0.5), refractAmt=1.0, ior=1.5)
PRISM = dict(kind="blinn", kd=(0.2, 0.3, 0.3), reflectAmt=1.0, refractAmt=1.0, specExp=30.0,
             disperse=True, ior3=(1.57, 1.60, 1.62))          # src/Assignment3.h:169-177 (mat2)
FINAL = dict(kind="blinn", kd=(0.9, 0.9, 0.9), reflectAmt=1.0, refractAmt=1.0, specExp=30.0,
             disperse=True, ior3=(1.56, 1.5, 1.5))            # src/main.cpp:167-174: setIor(1.56f) sets m_ior[0]


def sheet_scene(sheet_mat, env=False, subdivs=None):
    """Lambert Cornell box behind a refracting sheet."""
    cfg = dict(scenes.CONFIGS["C1"])
    if env:
        cfg["env"] = dict(sky=(64, 32), exposure=0.7)
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], extra=[(quad(), sheet_mat)], subdivs=subdivs)


def test_blinn_setior_sets_one_component_and_refraction_reads_the_second():
    b = miro.Blinn(ior=1.5)
    b.setIor(1.56)                    # src/main.cpp:170 -- m_ior[0]
    assert b.m_ior == [1.56, 1.5, 1.5] and b.ior == 1.5
    b.setIor(1.7, 1)
    assert b.ior == pytest.approx(1.7)


@pytest.mark.parametrize("env", [False, True])
def test_oracle_equal_ior_dispersion_equals_plain_refraction(env):
    _, O0, cam = sheet_scene(SHEET, env=env)
    _, O1, _ = sheet_scene(dict(SHEET, disperse=True, ior3=(1.5, 1.5, 1.5)), env=env)
    a, b = O0.render(cam, 48, 40, threads=8), O1.render(cam, 48, 40, threads=8)
    assert a["secondary_rays"] > 0
    assert b["secondary_rays"] == 3 * a["secondary_rays"]
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert np.array_equal(a["rgb8"], b["rgb8"])


def test_oracle_dispersion_separates_the_channels():
    _, O0, cam = sheet_scene(dict(SHEET, disperse=True, ior3=(1.5, 1.5, 1.5)))
    _, O1, _ = sheet_scene(dict(SHEET, disperse=True, ior3=(1.3, 1.5, 1.9)))
    a, b = O0.render(cam, 48, 40, threads=8), O1.render(cam, 48, 40, threads=8)
    # channel 1 refracts through the same m_ior[1] (and Fresnel reads m_ior[0]: changed)
    assert not np.array_equal(bits(a["rgb"][..., 0]), bits(b["rgb"][..., 0]))
    assert not np.array_equal(bits(a["rgb"][..., 2]), bits(b["rgb"][..., 2]))
    # every split traces three children, which land on Lambert walls and spawn nothing
    assert a["secondary_rays"] % 3 == 0 and b["secondary_rays"] % 3 == 0 and b["secondary_rays"] > 0
    c = O1.render(cam, 48, 40, threads=1)
    assert np.array_equal(bits(b["rgb"]), bits(c["rgb"]))
    assert np.isfinite(b["rgb"]).all() and (b["rgb"] >= 0).all()


def test_oracle_dispersion_flag_off_ignores_the_other_iors():
    """m_disperse false: m_ior[0] / m_ior[2] are never read (src/Blinn.cpp:169-185)."""
    _, O0, cam = sheet_scene(SHEET)
    _, O1, _ = sheet_scene(dict(SHEET, ior3=(1.1, 1.5, 2.2)))
    a, b = O0.render(cam, 40, 32, threads=8), O1.render(cam, 40, 32, threads=8)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))


def test_dispersion_is_validated():
    import ctypes as C
    from miro import _lib
    L = miro.lib()
    h = L.mrt_scene_create()
    try:
        m = _lib.mrt_material(1, (C.c_float * 3)(1, 1, 1), (C.c_float * 3)(0, 0, 0), (C.c_float * 3)(1, 1, 1), 1.0, 0.0)
        mid = L.mrt_scene_add_material(h, C.byref(m))
        good = (C.c_float * 3)(1.5, 1.6, 1.7)
        assert L.mrt_scene_set_material_dispersion(h, mid, 1, good) == 0
        assert L.mrt_scene_set_material_dispersion(h, mid + 1, 1, good) < 0
        assert L.mrt_scene_set_material_dispersion(h, mid, 1, (C.c_float * 3)(1.5, 0.0, 1.7)) < 0
        assert L.mrt_scene_set_material_dispersion(h, mid, 1, None) < 0
    finally:
        L.mrt_scene_destroy(h)


# ---------------------------------------------------------------- GPU parity
def assert_same(P, O_, cam, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = O_.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "primary hit ids differ"
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"]), "8-bit RGB differs"
    assert P.last_stats["secondary_rays"] == ref["secondary_rays"]
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("mat", [dict(SHEET, disperse=True, ior3=(1.3, 1.5, 1.9)), PRISM, FINAL],
                         ids=["sheet", "prism", "final"])
def test_dispersive_sheet_matches_oracle(mat):
    P, O_, cam = sheet_scene(mat, env=True)
    ref = assert_same(P, O_, cam, 64, 48)
    assert ref["secondary_rays"] > 0


@pytest.mark.gpu
def test_dispersive_bunny_with_dome_light_matches_oracle():
    """Closed mesh: splits on entry, refraction children leave through back faces
    (no split: IS_REFRACT_RAY), reflections inside split again."""
    cfg = dict(scenes.CONFIGS["D1"])
    cfg["material"] = dict(PRISM, kd=(0.8, 0.8, 0.8))
    P, O_, cam = scene_pair(cfg, obj=scenes.bunny_obj(), floor=True)
    assert_same(P, O_, cam, 40, 40)


@pytest.mark.gpu
def test_dispersion_with_area_light_and_supersampling_matches_oracle():
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=3, noise=0.001),
              dict(type="point", pos=(1.0, 3.0, -1.0), power=5.0)]
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = dict(kind="lambert", kd=(1, 1, 1))
    cfg["env"] = dict(sky=(64, 32), exposure=0.7)
    P, O_, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, subdivs=(1, 3, 0.01),
                            extra=[(quad(), FINAL)])
    assert_same(P, O_, cam, 40, 32)
