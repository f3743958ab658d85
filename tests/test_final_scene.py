"""Config FS: the reference's own final scene (makeFinalScene, src/main.cpp:132-670)
built from its data (assets/final) plus seeded stand-ins for the missing meshes.

CPU: the packed data matches its manifest; the transform helpers follow
Matrix4x4::rotate / rotateX..Z / scale / translate / operator*= (src/Matrix4x4.h);
the product's world QBVH over 42,178 ProxyObjects and the world meshes is
bit-identical to the oracle's; every BLAS too.
GPU: a frame at a small size with everything the script sets (adaptive 3..5,
dispersive MB glass, MB cannonball, DOF, dome light + environment, alpha-mapped
translucent leaves in proxies, normal maps, 40,401 grass proxies) against the
oracle: primary hit ids and t / a / b exact, shadow / secondary ray counts exact,
float RGB within north_star's 1e-4 relative per channel -- under the device's libm
convention and, at 160x88, under the reference's own (glibc sinf / cosf / powf)."""
import hashlib
import json
import os

import numpy as np
import pytest

import miro
from helpers import bits, camera, final_scene_pair
from miro import final_scene as F

CHAIN_SHADOW_STEP_DEFAULT = 0   # libmrt's default (csrc/mrt_device.hip g_chain_shadow_step)


def test_packed_data_matches_manifest():
    man = json.load(open(os.path.join(F.FINAL_DIR, "manifest.json")))
    assert len(man) == 43
    for name in ("groundPlane.obj", "flower02Body.obj", "sky.hdr", "FL30stm2.tga"):
        data = open(F.asset(name), "rb").read()
        assert len(data) == man[name]["bytes"]
        assert hashlib.sha256(data).hexdigest() == man[name]["sha256"]


def test_matrix_helpers_follow_the_reference():
    # rotate(angle, 0, 1, 0) sets the matrix: cos / sin in the (0,0) (0,2) (2,0) (2,2) slots, row order
    m = F._rotate(90.0, 0, 1, 0)
    assert abs(m[0, 0]) < 1e-6 and abs(m[0, 2] + 1) < 1e-6 and abs(m[2, 0] - 1) < 1e-6 and m[1, 1] == 1
    # rotateY agrees with rotate about y
    assert np.allclose(F._axis(33.0, "y"), F._rotate(33.0, 0, 1, 0), atol=1e-6)
    # scale touches the diagonal only; translate adds to column 4
    s = F._translate(F._scale(F._rotate(30.0, 0, 1, 0), 2, 3, 4), 1, 2, 3)
    r = F._rotate(30.0, 0, 1, 0)
    assert s[0, 0] == np.float32(r[0, 0] * np.float32(2)) and s[0, 2] == r[0, 2]
    assert tuple(s[:3, 3]) == (1, 2, 3)
    # the product is the DPPS one: exact for exactly representable values
    a = np.arange(16, dtype=np.float32).reshape(4, 4)
    assert np.array_equal(F._mul(a, np.eye(4, dtype=np.float32)), a)
    assert np.array_equal(F._mul(a, a), (a.astype(np.float64) @ a.astype(np.float64)).astype(np.float32))


def test_spec_counts_follow_the_script():
    sp = F.spec()
    n = {}
    for o in sp["objects"]:
        n[o.get("blas", "world")] = n.get(o.get("blas", "world"), 0) + 1
    assert n["grass"] == 201 * 201                      # makeProxyGrid
    assert n["fl02yellow"] == n["fl02white"] == 391     # makeFlowers: 391 each
    assert n["fl02pink"] == 392 and n["fl01"] == 4 and n["tree04"] == 1
    assert n["world"] == 5                              # explosion, cannonball, ground, tree03 body + leaves
    assert sp["subdivs"] == (3, 5, 0.01) and sp["dome"]["samples"] == 6 and sp["env"]["exposure"] == 1.5


def test_world_and_blas_hierarchies_match_oracle():
    P, O_, _ = final_scene_pair()
    po = O_.qbvh_info()
    assert P.bvh_info["nodes"] == po["nodes"] and P.bvh_info["leaves"] == po["leaves"]
    for a, b in zip(P.bvh_export(), O_.qbvh_export()):
        a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(160, 88), (97, 53)])
def test_final_scene_frame_matches_oracle(W, H):
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    P, O_, cam = final_scene_pair()
    img = miro.Image(); img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = O_.render(cam, W, H, threads=16)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "primary hit ids differ"
    hit = ref["hits"]["prim"] >= 0
    assert hit.mean() > 0.3
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(hits[k][hit]), bits(ref["hits"][k][hit]))
    st = P.last_stats
    assert st["primary_rays"] == ref["primary_rays"]          # eye rays of the adaptive passes
    assert st["shadow_rays"] == ref["shadow_rays"]
    assert st["secondary_rays"] == ref["secondary_rays"]
    g, r = img.rgb.astype(np.float64), ref["rgb"].astype(np.float64)
    bad = np.abs(g - r) > 1e-4 * np.abs(r)
    exact = float(np.mean(bits(img.rgb) == bits(ref["rgb"])))
    print(f"FS {W}x{H}: {int(bad.sum())} channels beyond 1e-4 relative, {exact:.6f} bit-exact, "
          f"{st['primary_rays'] / (W * H):.1f} eye rays/px, {st['secondary_rays']} secondary, {st['shadow_rays']} shadow")
    assert not bad.any()
    assert exact > 0.99
    if W == 160:   # the reference's own libm convention (glibc sinf / cosf / powf): the same 1e-4 bar
        import oracle as O
        rf = O_.render(cam, W, H, threads=16, want_hits=False, libm=O.LIBM_FLOAT)
        assert rf["shadow_rays"] == ref["shadow_rays"] and rf["secondary_rays"] == ref["secondary_rays"]
        r2 = rf["rgb"].astype(np.float64)
        bad2 = np.abs(g - r2) > 1e-4 * np.abs(r2)
        print(f"FS {W}x{H} vs the reference's libm convention: {int(bad2.sum())} channels beyond 1e-4 relative, "
              f"{float(np.mean(bits(img.rgb) == bits(rf['rgb']))):.6f} bit-exact")
        assert not bad2.any()


@pytest.mark.gpu
def test_final_scene_chain_shadow_schedules_give_identical_frames():
    """The chain levels' shadow rays of an instanced scene on the lane-refill kernel
    (chain_shadow_refill 1, deferred proxy walks), inside chain_trace with nested proxy
    walks (0) or inside chain_trace stepping with deferred proxy walks (chain_shadow_step 1):
    the same rays and answers, so the same frame, hit ids and ray counts."""
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    P, _, cam = final_scene_pair()
    L = miro.lib()
    out = []
    try:
        for refill, step in ((0, 0), (1, 0), (0, 1)):
            assert L.mrt_set_tuning(b"chain_shadow_refill", refill) == 0
            assert L.mrt_set_tuning(b"chain_shadow_step", step) == 0
            img = miro.Image(); img.resize(72, 40)
            hits = P.raytraceImage(camera(cam), img, want_hits=True)
            out.append((img, hits, dict(P.last_stats)))
    finally:
        L.mrt_set_tuning(b"chain_shadow_refill", 0)
        L.mrt_set_tuning(b"chain_shadow_step", CHAIN_SHADOW_STEP_DEFAULT)
    a, ha, sa = out[0]
    for b, hb, sb in out[1:]:
        assert np.array_equal(ha["prim"], hb["prim"])
        assert np.array_equal(bits(a.rgb), bits(b.rgb)) and np.array_equal(a.pixels, b.pixels)
        assert sa["shadow_rays"] == sb["shadow_rays"] and sa["secondary_rays"] == sb["secondary_rays"]
