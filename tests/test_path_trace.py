"""Path tracing and emission: Blinn::calculatePathTracing (reference
src/Blinn.cpp:39-89, called at :207-210 under Scene::m_pathTrace /
m_maxBounces, src/Scene.cpp:17-19) and Blinn's m_Le / m_lightEmitted
(src/Blinn.h:44-45,63-64; added at src/Blinn.cpp:335).

CPU tests pin the oracle's restatement on properties that follow from the
reference's arithmetic alone (no RNG): with m_maxBounces = 1 the path-tracing
term is the last-bounce direct light, so a Blinn point-light frame is exactly
doubled; m_Le adds to every Blinn result; an emitter seen directly returns
emitted * Le + Le.  GPU tests compare the HIP chain kernels with the oracle
(hit ids exact, ray counts exact, RGB within 1e-4 -- the GI cosine sample uses
libm cos / sin in double on both sides)."""
import numpy as np
import pytest

import miro
import oracle as O
from helpers import bits, camera, fixture_mesh, scene_pair

CORNELL_CAM = dict(eye=(2.75, 2.75, 5.0), lookAt=(2.75, 2.75, 0.0), up=(0, 1, 0), fov=55.0)
POINT = [dict(type="point", pos=(2.75, 5.0, -2.75), power=40.0)]
RECT = [dict(type="rect", v1=(2.0, 5.4, -2.0), v2=(3.5, 5.4, -2.0), v3=(2.0, 5.4, -3.5), power=6.0, samples=1,
             noise=0.001)]


def panel(y=5.45, x=(2.0, 3.5), z=(-3.5, -2.0)):
    """A ceiling light panel (two triangles facing down), as the sponza-light.obj
    mesh of makeSponzaScenePathTrace (src/assignment2.h:696-701)."""
    v = np.array([(x[0], y, z[0]), (x[1], y, z[0]), (x[1], y, z[1]), (x[0], y, z[1])], np.float32)
    n = np.array([(0, -1, 0)] * 4, np.float32)
    f = np.array([(0, 2, 1), (0, 3, 2)], np.uint32)
    return v, n, f, f.copy()


def cfg(kind="blinn", lights=POINT, **mat):
    return dict(camera=CORNELL_CAM, lights=lights, bg=(0.0, 0.0, 0.2), material=dict(kind=kind, kd=(0.7, 0.7, 0.7), **mat))


def oracle_render(c, W=48, H=48, **kw):
    _, Osc, cam = scene_pair(c, meshes=[fixture_mesh("cornell_box")], **kw)
    return Osc.render(cam, W, H, threads=4)


def test_last_bounce_path_tracing_doubles_a_point_light():
    """m_maxBounces = 1: giBounces 0 is not < 0, so calculatePathTracing samples the
    lights directly (isSecondary, rVec = 0): Ld = (0 + E*kd) + E*kd = 2 E*kd."""
    base = oracle_render(cfg())
    pt = oracle_render(cfg(), path_trace=(1, False))
    hit = base["hits"]["prim"] >= 0
    assert hit.mean() > 0.5
    assert np.array_equal(bits(pt["rgb"][hit]), bits(2.0 * base["rgb"][hit]))
    assert np.array_equal(bits(pt["rgb"][~hit]), bits(base["rgb"][~hit]))
    assert pt["shadow_rays"] == 2 * base["shadow_rays"] and pt["secondary_rays"] == 0


def test_emission_color_adds_to_every_blinn_result():
    le = (0.25, 0.5, 0.0)
    base = oracle_render(cfg())
    em = oracle_render(cfg(le=le))
    hit = base["hits"]["prim"] >= 0
    want = (base["rgb"][hit] + np.array(le, np.float32)).astype(np.float32)
    assert np.array_equal(bits(em["rgb"][hit]), bits(want))


def test_emitter_seen_directly_under_path_tracing():
    """No lights: an emitter hit returns Ld = 0 + emitted * Le, result (Ld)*1 + 0 + Le;
    every other surface is lit only by GI rays that reach the panel."""
    c = cfg(lights=[])
    _, Osc, cam = scene_pair(c, meshes=[fixture_mesh("cornell_box")], path_trace=(4, False),
                             extra=[(panel(), dict(kind="blinn", kd=(1, 1, 1), emitted=2.0, le=(1, 1, 1)))], num_paths=4)
    r = Osc.render(cam, 48, 48, threads=4)
    prim = r["hits"]["prim"]
    on_panel = prim >= 36            # the Cornell mesh has 36 triangles, the panel comes after it
    assert on_panel.any()
    assert np.all(r["rgb"][on_panel] == np.float32(3.0))
    walls = (prim >= 0) & ~on_panel
    assert (r["rgb"][walls] > 0).mean() > 0.05      # indirect light from the panel (4 paths, open box)
    assert r["secondary_rays"] > 0 and r["shadow_rays"] == 0


def test_path_traced_pixels_are_independent_of_the_render_window():
    c = cfg(lights=RECT, reflectAmt=0.3)
    _, Osc, cam = scene_pair(c, meshes=[fixture_mesh("cornell_box")], path_trace=(3, False), num_paths=2,
                             extra=[(panel(), dict(kind="blinn", kd=(1, 1, 1), emitted=1.5, le=(1, 1, 1)))])
    full = Osc.render(cam, 40, 30, threads=4)
    part = Osc.render(cam, 40, 30, rect=(7, 5, 31, 22), threads=2)
    assert np.array_equal(bits(full["rgb"][5:22, 7:31]), bits(part["rgb"][5:22, 7:31]))


# ------------------------------------------------------------------ GPU parity
def need_gpu():
    if miro.device_count() < 1:
        pytest.skip("no HIP device")


def assert_close(got, ref, rtol=1e-4):
    d = np.abs(got.astype(np.float64) - ref.astype(np.float64))
    tol = rtol * np.maximum(np.abs(ref.astype(np.float64)), 1e-3)
    bad = d > tol
    assert not bad.any(), f"{bad.sum()} channels beyond {rtol} (max {d.max()})"


PT_CASES = {
    "point_pt4": dict(c=cfg(), kw=dict(path_trace=(4, False), num_paths=2)),
    "rect_panel_reflect": dict(c=cfg(lights=RECT, reflectAmt=0.3, specExp=8.0, specAmt=0.25),
                               kw=dict(path_trace=(3, False), num_paths=4,
                                       extra=[(panel(), dict(kind="blinn", kd=(1, 1, 1), emitted=1.5, le=(1, 1, 1)))])),
    "panel_only_env": dict(c=dict(cfg(lights=[]), env=dict(sky=(64, 32), exposure=1.0)),
                           kw=dict(path_trace=(5, True), num_paths=3,
                                   extra=[(panel(), dict(kind="blinn", kd=(1, 1, 1), emitted=2.0, le=(1, 1, 1)))])),
    "glass_inside_ior": dict(c=cfg(refractAmt=0.8, reflectAmt=0.2, ior=1.4), kw=dict(num_paths=3)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(PT_CASES))
def test_path_trace_matches_oracle(case):
    need_gpu()
    spec = PT_CASES[case]
    P, Osc, cam = scene_pair(spec["c"], meshes=[fixture_mesh("cornell_box")], **spec["kw"])
    W, H = 64, 48
    if case == "glass_inside_ior":   # camera inside the box: back faces, popped IOR histories over the paths
        cam = dict(eye=(2.75, 2.75, -2.5), lookAt=(2.75, 2.0, -5.0), up=(0, 1, 0), fov=70.0)
    img = miro.Image(); img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = Osc.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"])
    assert_close(img.rgb, ref["rgb"])
    st = P.last_stats
    assert st["shadow_rays"] == ref["shadow_rays"]
    assert st["secondary_rays"] == ref["secondary_rays"]
    assert ref["secondary_rays"] > 0 or case == "none"


@pytest.mark.gpu
def test_emission_without_path_tracing_matches_oracle():
    need_gpu()
    c = cfg(le=(0.2, 0.1, 0.05))
    P, Osc, cam = scene_pair(c, meshes=[fixture_mesh("cornell_box")])
    img = miro.Image(); img.resize(64, 64)
    P.raytraceImage(camera(cam), img)
    ref = Osc.render(cam, 64, 64, threads=8)
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
    assert np.array_equal(img.pixels, ref["rgb8"])
