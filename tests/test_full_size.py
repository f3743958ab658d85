"""Full-size frames of the BASELINE configs and of the secondary-ray configs against the
CPU oracle, and the traversal-stack spill / overflow path (MRT_ERR_OVERFLOW past 256
entries: 16 LDS + 240 HBM per lane, the reference's 256-entry stack, src/BVH.cpp:1133).

Every frame is compared whole (every row, every pixel), against the oracle under the
reference's own libm convention (oracle.LIBM_FLOAT: glibc's atan2f / acosf / sinf / cosf /
powf, which the device restates bit for bit, csrc/mrt_libm.h):
- hit ids, t, a, b and the shadow-ray (and secondary-ray) counts exact;
- float RGB and 8-bit RGB bit-exact;
- north_star's 1e-4 relative per channel (|got - ref| <= 1e-4 |ref|, no absolute floor)
  follows from that; the count beyond it is printed too."""
import ctypes as C

import numpy as np
import pytest

import miro
import oracle as O
from miro import _lib
from helpers import bits, camera, config_scene


def need_gpu():
    if miro.device_count() < 1:
        pytest.skip("no HIP device")


def close_frac(got, ref, rtol=1e-4):
    """Channels beyond rtol relative (north_star: 1e-4 relative per RGB channel, no floor)
    and the share of bit-identical channels."""
    g, r = got.astype(np.float64), ref.astype(np.float64)
    bad = np.abs(g - r) > rtol * np.abs(r)
    return int(bad.sum()), float((bits(got) == bits(ref)).mean())


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["C2", "C3", "C3L", "C4", "C5", "D1"])
def test_full_size_frame_matches_oracle(key):
    """Under the config's own tuning (bench.py's: C3's nested camera-ray walk, C2's 6-wave frame
    kernel; the others the library defaults), so every benched kernel form is compared here."""
    need_gpu()
    P, Osc, cam = config_scene(key)
    from miro import scenes
    W, H = scenes.CONFIGS[key]["W"], scenes.CONFIGS[key]["H"]
    img = miro.Image(); img.resize(W, H)
    tune = scenes.CONFIGS[key].get("tune", {})
    L = miro.lib()
    try:
        for k, v in tune.items():
            assert L.mrt_set_tuning(k.encode(), v) == 0
        hits = P.raytraceImage(camera(cam), img, want_hits=True)
    finally:
        for k in tune:
            assert L.mrt_set_tuning(k.encode(), {"walk_latch": 1, "frame1_waves": 7}[k]) == 0   # the defaults
    ref = Osc.render(cam, W, H, threads=16, libm=O.LIBM_FLOAT)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), f"{key}: primary hit ids differ"
    hit = ref["hits"]["prim"] >= 0
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(hits[k][hit]), bits(ref["hits"][k][hit])), f"{key}: hit {k} differs"
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    nbad, exact = close_frac(img.rgb, ref["rgb"])
    print(f"{key} {W}x{H} vs the reference's libm convention: {nbad} channels beyond 1e-4 relative, "
          f"{exact:.6f} of channels bit-exact, {int((img.pixels != ref['rgb8']).any(axis=2).sum())} 8-bit pixels differ")
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), f"{key}: float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"]), f"{key}: 8-bit RGB differs"


SECONDARY = {"R3": (1920, 1080), "G3": (1920, 1080), "P4": (512, 512)}


@pytest.mark.gpu
@pytest.mark.parametrize("key", sorted(SECONDARY))
def test_full_size_secondary_rays_vs_reference_libm(key):
    """The BASELINE-size frames of the secondary-ray configs (Fresnel's sin(acosf),
    src/Material.h:47-55; dispersion, src/Blinn.cpp:169-185; path tracing's cosine
    sampler cos / sin, src/Material.cpp:14-42) against the oracle under the reference's
    own libm convention (glibc's float overloads): hit ids / t / a / b, shadow and
    secondary ray counts exact, float and 8-bit RGB bit-exact.  (Round 5's device
    evaluated sinf / cosf / powf in double and rounded once; against glibc that left P4
    with 6 of 786,432 channels beyond 1e-4 at this size, profiles/r06_pytest_gpu_a.txt.)"""
    need_gpu()
    P, Osc, cam = config_scene(key)
    W, H = SECONDARY[key]
    img = miro.Image(); img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = Osc.render(cam, W, H, threads=16, libm=O.LIBM_FLOAT)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), f"{key}: primary hit ids differ"
    hit = ref["hits"]["prim"] >= 0
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(hits[k][hit]), bits(ref["hits"][k][hit])), f"{key}: hit {k} differs"
    nbad, exact = close_frac(img.rgb, ref["rgb"])
    st = P.last_stats
    print(f"{key} {W}x{H} vs the reference's libm convention: {nbad} channels beyond 1e-4 relative, "
          f"{exact:.6f} of channels bit-exact, {int((img.pixels != ref['rgb8']).any(axis=2).sum())} 8-bit pixels "
          f"differ; shadow rays {st['shadow_rays']} / {ref['shadow_rays']}, secondary rays "
          f"{st['secondary_rays']} / {ref['secondary_rays']} (device / oracle)")
    assert st["shadow_rays"] == ref["shadow_rays"] and st["secondary_rays"] == ref["secondary_rays"]
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), f"{key}: float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"])


def _chain_bvh(depth):
    """A QBVH for mrt_scene_bvh_import: a chain of `depth` nodes whose boxes
    contain everything; node k's slot 3 (the highest, visited next) is node k + 1
    and slots 0-2 are one small node L holding the scene's triangle packet, so a
    ray pushes three entries per chain node (3 * depth in all) and then visits L
    3 * depth times -- linear work, a stack as deep as we like."""
    big = np.array([-1e6] * 12 + [1e6] * 12, np.float32)
    L = depth
    nb = np.tile(big, (depth + 1, 1))
    nc = np.zeros((depth + 1, 4), np.int32)
    for k in range(depth):
        nc[k] = [L, L, L, k + 1 if k + 1 < depth else L]
    empty = np.iinfo(np.int32).min
    nc[L] = [~0, empty, empty, empty]
    return nb, nc


@pytest.mark.gpu
@pytest.mark.parametrize("depth,overflow", [(30, False), (85, False), (86, True)])
def test_traversal_stack_spill_and_overflow(depth, overflow):
    """depth 30: 90 entries -- past the 16 LDS entries into the HBM spill column,
    still exact; depth 85: 255 entries, the reference's 256-entry stack nearly full
    (src/BVH.cpp:1133), still exact; depth 86: 258 > 256 entries (where the
    reference writes past its stack) -> MRT_ERR_OVERFLOW, never a wrong answer or a
    fault."""
    need_gpu()
    L = miro.lib()
    P = miro.Scene()
    tm = miro.TriangleMesh()
    tri = np.array([(-1, -1, -5), (1, -1, -5), (0, 1, -5)], np.float32)
    tm.setArrays(tri, np.array([(0, 0, 1)] * 3, np.float32), np.array([(0, 1, 2)], np.uint32),
                 np.array([(0, 1, 2)], np.uint32))
    miro.makeMeshObjs(P, tm, miro.Lambert())
    P.preCalc()
    _, _, lt, lp = P.bvh_export()
    nb, nc = _chain_bvh(depth)
    fp, ip = C.POINTER(C.c_float), C.POINTER(C.c_int32)
    _lib.check(L.mrt_scene_bvh_import(P.handle, depth + 1, len(lt), nb.ctypes.data_as(fp), nc.ctypes.data_as(ip),
                                      lt.ctypes.data_as(fp), lp.ctypes.data_as(ip)), "import")
    o = np.zeros((256, 3), np.float32)
    d = np.tile(np.array([[0, 0, -1]], np.float32), (256, 1))
    if overflow:
        with pytest.raises(miro.MRTError, match="OVERFLOW"):
            P.traceBatch(o, d)
    else:
        got = P.traceBatch(o, d)
        assert (got["prim"] == 0).all() and np.allclose(got["t"], 5.0, rtol=1e-6)
