"""Depth of field: the lens of Camera::eyeRayAdaptive (reference
src/Camera.cpp:153-174; setAperture / setFocusPlane, src/Camera.h:38-42).

With m_aperture >= epsilon the camera ray starts on a disc of radius m_aperture
around the eye -- (u, v) rejection-sampled from the unit square mapped to
[-1, 1]^2 by 1.0 - 2 * getRand -- and passes through the focal point
m_focusPlane along the pinhole direction.  The disc draws follow the jitter and
time draws in the counter RNG (dims 3, 4, ...), on the device and in the oracle.

CPU tests pin the oracle's restatement by geometry: aperture 0 is the pinhole
frame bit for bit; a surface at the focus distance stays in focus (every lens
ray of a pixel meets the pinhole ray there), while one far from it blurs.  GPU
tests compare the HIP path with the oracle bit for bit (direct lighting, the
chain engine with mirrors, adaptive supersampling, environment-map misses)."""
import numpy as np
import pytest

import miro
from helpers import bits, camera, fixture_mesh, scene_pair
from miro import scenes

CAM = dict(eye=(2.75, 2.75, 5.0), lookAt=(2.75, 2.75, 0.0), up=(0, 1, 0), fov=55.0)
BACK_WALL = 5.0 + 5.59   # eye z to the Cornell box's back wall (z = -5.59)


def cornell(material=None, **kw):
    cfg = dict(scenes.CONFIGS["C1"])
    if material:
        cfg["material"] = material
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], **kw)


def test_zero_aperture_is_the_pinhole_frame():
    _, O_, _ = cornell()
    a = O_.render(CAM, 48, 40, threads=4)
    b = O_.render(dict(CAM, aperture=0.0, focusPlane=3.0), 48, 40, threads=4)
    c = O_.render(dict(CAM, aperture=0.0009, focusPlane=3.0), 48, 40, threads=4)   # below epsilon
    for r in (b, c):
        assert np.array_equal(bits(a["rgb"]), bits(r["rgb"]))
        assert np.array_equal(a["hits"]["prim"], r["hits"]["prim"])


def test_surface_at_the_focus_distance_stays_sharp():
    """The lens ray passes through the pinhole ray's point at the focus distance:
    focusing on the back wall keeps the wall's hit triangles (the view axis meets
    it at BACK_WALL); focusing near the camera blurs them."""
    _, O_, _ = cornell()
    W = H = 48
    pin = O_.render(CAM, W, H, threads=4)["hits"]["prim"]
    sharp = O_.render(dict(CAM, aperture=0.4, focusPlane=BACK_WALL), W, H, threads=4)["hits"]["prim"]
    blur = O_.render(dict(CAM, aperture=0.4, focusPlane=1.0), W, H, threads=4)["hits"]["prim"]
    centre = (slice(16, 32), slice(16, 32))   # the back wall around the view axis
    assert (sharp[centre] == pin[centre]).mean() > 0.9    # misses only along the wall's diagonal edge
    assert (blur != pin).mean() > 5 * (sharp != pin).mean()


def test_lens_draws_are_deterministic_and_seed_independent_of_threads():
    _, O_, _ = cornell()
    c = dict(CAM, aperture=0.3, focusPlane=6.0)
    a, b = O_.render(c, 40, 30, threads=1), O_.render(c, 40, 30, threads=8)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))


# ------------------------------------------------------------------ GPU parity
def need_gpu():
    if miro.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")


def gpu_vs_oracle(P, O_, cam, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = O_.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "primary hit ids differ"
    hit = ref["hits"]["prim"] >= 0
    assert np.array_equal(bits(hits["t"][hit]), bits(ref["hits"]["t"][hit]))
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"])
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    assert P.last_stats["secondary_rays"] == ref["secondary_rays"]
    return ref


DOF = dict(CAM, aperture=0.35, focusPlane=7.0)


@pytest.mark.gpu
def test_dof_direct_lighting_matches_oracle():
    need_gpu()
    P, O_, _ = cornell()
    gpu_vs_oracle(P, O_, DOF, 64, 48)
    P, O_, _ = cornell(dict(kind="blinn", kd=(0.6, 0.5, 0.4)),
                       lights=[dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5),
                                    power=15.0, samples=3, noise=0.001)], num_paths=2)
    gpu_vs_oracle(P, O_, DOF, 64, 48)


@pytest.mark.gpu
def test_dof_chain_engine_and_supersampling_match_oracle():
    need_gpu()
    mirror = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=0.7, refractAmt=0.3, ior=1.4)
    P, O_, _ = cornell(mirror)
    ref = gpu_vs_oracle(P, O_, DOF, 64, 48)
    assert ref["secondary_rays"] > 0
    P, O_, _ = cornell(subdivs=(1, 3, 0.01))
    gpu_vs_oracle(P, O_, DOF, 40, 32)


@pytest.mark.gpu
def test_dof_env_map_misses_use_the_lens_ray():
    need_gpu()
    cfg = dict(scenes.CONFIGS["C1"], env=dict(sky=(64, 32), exposure=0.8))
    P, O_, _ = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")])
    cam = dict(DOF, eye=(2.75, 2.75, 9.0))   # the box's open front: lens rays miss around the edges
    ref = gpu_vs_oracle(P, O_, cam, 64, 48)
    assert (ref["hits"]["prim"] < 0).any()
