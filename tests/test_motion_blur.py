"""Motion blur: MBObject (reference src/MBObject.h/.cpp, created by makeMBMeshObjs,
src/main.cpp:23,202) and its lanes in intersect4 (src/BVH.cpp:1316-1334).

An MBObject triangle has a time-0 mesh and a time-1 mesh of the same topology.
Its BVH box is the union of both triangle boxes; in a leaf packet it is a
checkOut lane whose triangle is formed per ray: A = time * A2 + (1 - time) * A1
(edges from the blended B and C).  Ray time is Camera::getTimeSample
(src/Camera.h:46, 1 - r^3 * shutterSpeed, counter-RNG dim 2), inherited by every
secondary and shadow ray of the camera ray -- except the translucency shadow
rays, which Blinn::shade casts at time .001 (src/Blinn.cpp:229).  Shading uses
the time-0 mesh (MBObject::getAllInfos).

CPU tests pin the oracle by geometry: with shutter 0 every ray has time 1, so a
moving mesh hits exactly like a static mesh at its time-1 vertices (same t, same
(a, b), same triangle ids); with equal meshes the frame is the static frame; with
a long shutter the hits spread over the swept region and stay inside it.  GPU
tests compare the HIP path with the oracle bit for bit (direct lighting, the
wavefront shadow pass, the chain engine with mirrors and path tracing,
translucency, adaptive supersampling, depth of field)."""
import os

import numpy as np
import pytest

import miro
from helpers import ROOT, bits, camera, fixture_mesh, scene_pair
from miro import scenes

CAM = dict(eye=(2.75, 2.75, 5.0), lookAt=(2.75, 2.75, 0.0), up=(0, 1, 0), fov=55.0)
BALL = dict(kind="lambert", kd=(0.2, 0.7, 0.3))


def sphere(center=(1.7, 1.6, -2.6), radius=0.8, nu=16, nv=10):
    """A UV sphere: (verts, normals, vidx, nidx) with per-vertex normals."""
    V, N = [], []
    for j in range(nv + 1):
        th = np.pi * j / nv
        for i in range(nu):
            ph = 2 * np.pi * i / nu
            n = np.array([np.sin(th) * np.cos(ph), np.cos(th), np.sin(th) * np.sin(ph)])
            N.append(n)
            V.append(np.asarray(center) + radius * n)
    F = []
    for j in range(nv):
        for i in range(nu):
            a, b = j * nu + i, j * nu + (i + 1) % nu
            c, d = a + nu, b + nu
            if j > 0:
                F.append((a, b, c))
            if j < nv - 1:
                F.append((b, d, c))
    V = np.asarray(V, np.float32)
    F = np.asarray(F, np.uint32)
    return V, np.asarray(N, np.float32), F, F.copy()


def moved(arrs, delta=(1.6, 0.5, 0.0)):
    return (arrs[0] + np.asarray(delta, np.float32)).astype(np.float32)


def cornell(moving=None, extra=None, **kw):
    return scene_pair(dict(scenes.CONFIGS["C1"]), meshes=[fixture_mesh("cornell_box")], moving=moving, extra=extra,
                      **kw)


def ball_ids(O_):
    """object ids of the ball: the Cornell box's triangles come first"""
    v, n, vi, ni = fixture_mesh("cornell_box")
    return len(vi)


def test_shutter_zero_hits_the_time_one_mesh_exactly():
    ball = sphere()
    v2 = moved(ball)
    _, Om, _ = cornell(moving=[(ball, v2, BALL)])
    _, Os, _ = cornell(extra=[((v2,) + ball[1:], BALL)])
    cam = dict(CAM, shutterSpeed=0.0)
    a, b = Om.render(cam, 96, 72, threads=4), Os.render(cam, 96, 72, threads=4)
    first = ball_ids(Om)
    # the ball's pixels (the two BVHs differ -- union boxes -- so ties between the
    # box's coplanar triangle pairs may resolve to the other triangle elsewhere)
    on = (a["hits"]["prim"] >= first) | (b["hits"]["prim"] >= first)
    assert on.sum() > 100   # the ball is in view
    assert np.array_equal(a["hits"]["prim"][on], b["hits"]["prim"][on])
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(a["hits"][k][on]), bits(b["hits"][k][on]))


def test_unmoving_mesh_renders_the_static_frame():
    ball = sphere()
    _, Om, _ = cornell(moving=[(ball, ball[0].copy(), BALL)])
    _, Os, _ = cornell(extra=[(ball, BALL)])
    cam = dict(CAM, shutterSpeed=0.0)
    a, b = Om.render(cam, 64, 48, threads=4), Os.render(cam, 64, 48, threads=4)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert np.array_equal(a["hits"]["prim"], b["hits"]["prim"])


def test_long_shutter_spreads_hits_over_the_swept_region():
    ball = sphere(radius=0.6)
    v2 = moved(ball, (2.2, 0.4, 0.0))   # the ends are 2.2 apart: a gap between the footprints
    _, Om, _ = cornell(moving=[(ball, v2, BALL)])
    _, O0, _ = cornell(extra=[(ball, BALL)])
    _, O1, _ = cornell(extra=[((v2,) + ball[1:], BALL)])
    W, H = 96, 72
    first = ball_ids(Om)
    blur = Om.render(dict(CAM, shutterSpeed=1.0), W, H, threads=8)["hits"]["prim"] >= first
    at0 = O0.render(dict(CAM, shutterSpeed=0.0), W, H, threads=8)["hits"]["prim"] >= first
    at1 = O1.render(dict(CAM, shutterSpeed=0.0), W, H, threads=8)["hits"]["prim"] >= first
    # hits outside both end positions (the middle of the sweep; time = 1 - r^3
    # favours the end) and inside each end's footprint
    assert (blur & ~at0 & ~at1).sum() > 20
    assert (blur & at0 & ~at1).sum() > 5 and (blur & at1 & ~at0).sum() > 5
    # every hit lies within the sweep: the rows / columns spanned by the two ends
    ys, xs = np.nonzero(at0 | at1)
    by, bx = np.nonzero(blur)
    assert by.min() >= ys.min() - 1 and by.max() <= ys.max() + 1
    assert bx.min() >= xs.min() - 1 and bx.max() <= xs.max() + 1


def test_time_draws_are_deterministic_across_threads():
    ball = sphere()
    _, Om, _ = cornell(moving=[(ball, moved(ball), BALL)])
    c = dict(CAM, shutterSpeed=0.7)
    a, b = Om.render(c, 40, 30, threads=1), Om.render(c, 40, 30, threads=8)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))


def test_motion_mesh_must_match_topology():
    P = miro.Scene()
    m1, m2 = miro.TriangleMesh(), miro.TriangleMesh()
    ball = sphere()
    m1.setArrays(*ball)
    m2.setArrays(ball[0][:-3], *ball[1:])
    miro.makeMBMeshObjs(P, m1, m2, miro.Lambert())
    with pytest.raises(miro.MRTError):
        P.preCalc()


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


MB = dict(CAM, shutterSpeed=1.0)


@pytest.mark.gpu
def test_motion_blur_direct_lighting_matches_oracle():
    need_gpu()
    ball = sphere()
    P, O_, _ = cornell(moving=[(ball, moved(ball), BALL)])
    ref = gpu_vs_oracle(P, O_, MB, 64, 48)
    assert (ref["hits"]["prim"] >= ball_ids(O_)).sum() > 50
    rect = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5),
                 power=15.0, samples=3, noise=0.001)]
    P, O_, _ = cornell(moving=[(ball, moved(ball), dict(kind="blinn", kd=(0.6, 0.5, 0.4)))], lights=rect,
                       num_paths=2)
    gpu_vs_oracle(P, O_, dict(CAM, shutterSpeed=0.5), 64, 48)


@pytest.mark.gpu
def test_motion_blur_chain_engine_and_translucency_match_oracle():
    need_gpu()
    ball = sphere()
    mirror = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=0.7, refractAmt=0.3, ior=1.4)
    P, O_, _ = cornell(moving=[(ball, moved(ball), mirror)])
    ref = gpu_vs_oracle(P, O_, MB, 64, 48)
    assert ref["secondary_rays"] > 0
    glow = dict(kind="blinn", kd=(0.6, 0.5, 0.4), translucency=0.5)
    P, O_, _ = cornell(moving=[(ball, moved(ball), glow)])
    gpu_vs_oracle(P, O_, MB, 64, 48)


@pytest.mark.gpu
def test_motion_blur_path_tracing_matches_oracle():
    need_gpu()
    ball = sphere()
    gi = dict(kind="blinn", kd=(0.2, 0.7, 0.3))   # Blinn::shade's calculatePathTracing casts the GI rays
    P, O_, _ = cornell(moving=[(ball, moved(ball), gi)], num_paths=2, path_trace=(2, False))
    ref = gpu_vs_oracle(P, O_, MB, 48, 40)
    assert ref["secondary_rays"] > 0


@pytest.mark.gpu
def test_motion_blur_supersampling_and_depth_of_field_match_oracle():
    need_gpu()
    ball = sphere()
    P, O_, _ = cornell(moving=[(ball, moved(ball), BALL)], subdivs=(1, 3, 0.01))
    gpu_vs_oracle(P, O_, MB, 40, 32)
    P, O_, _ = cornell(moving=[(ball, moved(ball), BALL)])
    gpu_vs_oracle(P, O_, dict(MB, aperture=0.3, focusPlane=7.0), 64, 48)


# ------------------------------------------- the reference's own MBObject pair
def cannonball_parts():
    """cannonBallT1 -> cannonBallT2 over the groundPlane (src/main.cpp:216-225),
    lit by a point light; fixture tests/golden/cannonball_mb.npz
    (tests/golden/make_fixtures.py motion)."""
    f = np.load(os.path.join(ROOT, "tests", "golden", "cannonball_mb.npz"))
    ball = (f["verts"], f["normals"], f["vidx"], f["nidx"])
    ground = (f["ground_verts"], f["ground_normals"], f["ground_vidx"], f["ground_nidx"])
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.5, 0.45, 0.4)),
               lights=[dict(type="point", pos=(2.0, 3.0, 2.0), power=60.0)])
    return cfg, ground, ball, f["verts2"]


def cannonball(mat=None, **kw):
    cfg, ground, ball, v2 = cannonball_parts()
    return scene_pair(cfg, meshes=[ground], moving=[(ball, v2, mat or BALL)], **kw)


BALL_CAM = dict(eye=(0.75, 0.62, 0.38), lookAt=(0.0, 0.5, 0.38), up=(0, 1, 0), fov=60.0)
N_GROUND = 32   # the ground plane's triangles come first


def test_cannonball_shutter_zero_is_the_time_one_mesh():
    cfg, ground, ball, v2 = cannonball_parts()
    _, Om, _ = cannonball()
    _, Os, _ = scene_pair(cfg, meshes=[ground], extra=[((v2,) + ball[1:], BALL)])
    cam = dict(BALL_CAM, shutterSpeed=0.0)
    a, b = Om.render(cam, 96, 72, threads=8), Os.render(cam, 96, 72, threads=8)
    on = (a["hits"]["prim"] >= N_GROUND) | (b["hits"]["prim"] >= N_GROUND)
    assert on.sum() > 200
    assert np.array_equal(a["hits"]["prim"][on], b["hits"]["prim"][on])
    assert np.array_equal(bits(a["hits"]["t"][on]), bits(b["hits"]["t"][on]))


@pytest.mark.gpu
def test_cannonball_motion_blur_matches_oracle():
    need_gpu()
    P, O_, _ = cannonball()
    ref = gpu_vs_oracle(P, O_, dict(BALL_CAM, shutterSpeed=1.0), 96, 72)
    assert (ref["hits"]["prim"] >= N_GROUND).sum() > 200
    shiny = dict(kind="blinn", kd=(0.01, 0.01, 0.01), reflectAmt=0.5, ior=1.8)   # cBallMat without specAmt
    P, O_, _ = cannonball(shiny, num_paths=2)
    ref = gpu_vs_oracle(P, O_, dict(BALL_CAM, shutterSpeed=0.6), 96, 72)
    assert ref["secondary_rays"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("chain", [False, True])
def test_motion_blur_under_a_dome_light_matches_oracle(chain):
    """A moving ball lit by a dome light: the dome's shadow rays take the lane-refill shadow
    kernel (frame path) or the chain levels (mirror material), whose steps must test the
    motion-blurred lanes at the ray's time, with no alpha map in the scene."""
    need_gpu()
    ball = sphere()
    dome = [dict(type="dome", sky=(64, 32), power=0.15, samples=3, noise=0.001)]
    mat = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=0.7, refractAmt=0.3, ior=1.4) if chain else BALL
    P, O_, _ = cornell(moving=[(ball, moved(ball), mat)], lights=dome)
    ref = gpu_vs_oracle(P, O_, MB, 48, 40)
    assert ref["shadow_rays"] > 0
    if chain:
        assert ref["secondary_rays"] > 0
