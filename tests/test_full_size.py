"""Full-size frames of the BASELINE configs against the CPU oracle (VERDICT r1:
C2, C4 and C5 were only compared at reduced sizes), and the traversal-stack
overflow path (MRT_ERR_OVERFLOW: 16 LDS + 80 HBM entries per lane).

Bars: hit ids exact everywhere; float RGB bit-exact for the configs without
libm (C2), within north_star's 1e-4 relative per channel where pow / atan2 / acos
enter (C4 specular, C5 dome + environment) -- |got - ref| <= 1e-4 |ref| with no
absolute floor, so an exact zero must stay zero -- with >99% of channels
bit-exact.  The count of channels beyond the bar is printed (0 required)."""
import ctypes as C

import numpy as np
import pytest

import miro
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
@pytest.mark.parametrize("key", ["C2", "C4", "C5"])
def test_full_size_frame_matches_oracle(key):
    need_gpu()
    P, Osc, cam = config_scene(key)
    from miro import scenes
    W, H = scenes.CONFIGS[key]["W"], scenes.CONFIGS[key]["H"]
    img = miro.Image(); img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = Osc.render(cam, W, H, threads=16)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), f"{key}: primary hit ids differ"
    hit = ref["hits"]["prim"] >= 0
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(hits[k][hit]), bits(ref["hits"][k][hit]))
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    if key == "C2":
        assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
        assert np.array_equal(img.pixels, ref["rgb8"])
    else:
        nbad, exact = close_frac(img.rgb, ref["rgb"])
        print(f"{key} {W}x{H}: {nbad} channels beyond 1e-4 relative, {exact:.6f} of channels bit-exact")
        assert nbad == 0 and exact > 0.99, (nbad, exact)


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
@pytest.mark.parametrize("depth,overflow", [(30, False), (40, True)])
def test_traversal_stack_spill_and_overflow(depth, overflow):
    """depth 30: 90 entries -- past the 16 LDS entries into the HBM spill column,
    still exact; depth 40: 120 > 96 entries -> MRT_ERR_OVERFLOW, never a wrong
    answer or a fault."""
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
