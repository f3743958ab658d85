"""Adaptive supersampling, Scene::adaptiveSampleScene (src/Scene.cpp:252-293).

CPU tests pin the oracle's restatement by properties of the reference loop
(sample counts per level, the min/max/noise stop rule, the 1-spp path left
unchanged).  GPU tests require libmrt's fused adaptive kernel to be
bit-identical to the oracle: same eye rays, same RNG streams, same running
mean and gamma-space stop test.  Parity against the reference's own frames is
statistical only (its MT19937 pool is sequential), so it is unpinned here.
"""
import numpy as np
import pytest

import miro
from helpers import bits, camera, config_scene, fixture_mesh, scene_pair
from miro import scenes


def sum_squares(n):
    return sum(k * k for k in range(1, n + 1))


def oracle_c1(subdivs, lights=None, kind="lambert"):
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = dict(kind=kind, kd=(0.7, 0.6, 0.5))
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, subdivs=subdivs)


@pytest.mark.parametrize("lo,hi", [(2, 2), (3, 3), (1, 4)])
def test_oracle_noise_zero_runs_every_level(lo, hi):
    """noise 0 never cuts off: every pixel takes 1 + 2^2 + ... + max^2 eye rays."""
    _, O_, cam = oracle_c1((lo, hi, 0.0))
    ref = O_.render(cam, 24, 16, threads=4)
    assert ref["primary_rays"] == 24 * 16 * (1 + sum_squares(hi) - 1)


def test_oracle_huge_noise_stops_after_level_two_unless_min_forces_more():
    """The loop runs level 2 at least once (max > 1); a threshold above any
    gamma difference stops it there, and min_subdivs forces further levels."""
    _, O_, cam = oracle_c1((1, 6, 1e9))
    assert O_.render(cam, 20, 12, threads=4)["primary_rays"] == 20 * 12 * 5
    _, O_, cam = oracle_c1((3, 6, 1e9))
    assert O_.render(cam, 20, 12, threads=4)["primary_rays"] == 20 * 12 * (1 + 4 + 9)


def test_oracle_one_subdiv_is_the_one_spp_frame():
    """min = max = 1 is the 1-spp path (the golden-fixture frames)."""
    _, O1, cam = oracle_c1((1, 1, 0.01))
    _, O0, _ = oracle_c1(None)
    a, b = O1.render(cam, 32, 24), O0.render(cam, 32, 24)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert a["primary_rays"] == 32 * 24


def test_oracle_adaptive_is_thread_independent_and_keeps_centre_hits():
    """Counter RNG keyed by (pixel, eye ray): the frame does not depend on the
    thread count; the hit record is the centre sample's (the 1-spp hit)."""
    _, O_, cam = oracle_c1((1, 3, 0.01))
    a, b = O_.render(cam, 40, 30, threads=1), O_.render(cam, 40, 30, threads=8)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))
    assert a["primary_rays"] == b["primary_rays"]
    assert 40 * 30 * 5 <= a["primary_rays"] <= 40 * 30 * 14
    _, O0, _ = oracle_c1(None)
    h0 = O0.render(cam, 40, 30)["hits"]
    assert np.array_equal(a["hits"]["prim"], h0["prim"])


def test_oracle_supersampled_mean_is_close_to_the_centre_sample():
    """Sub-samples jitter within the pixel: on the interior of the Cornell box
    the supersampled frame stays near the 1-spp frame (mean |diff| small), and
    edges differ (anti-aliasing happened)."""
    _, O_, cam = oracle_c1((2, 2, 0.0))
    _, O0, _ = oracle_c1(None)
    a, b = O_.render(cam, 64, 64, threads=8)["rgb"], O0.render(cam, 64, 64, threads=8)["rgb"]
    d = np.abs(a.astype(np.float64) - b)
    assert np.median(d) < 0.02
    assert (d.max(axis=2) > 0).mean() > 0.05


def test_subdiv_arguments_are_validated():
    from oracle import OracleScene
    s = OracleScene()
    for bad in [(0, 1, 0.01), (3, 2, 0.01), (1, 17, 0.01), (1, 2, -1.0)]:
        with pytest.raises(ValueError):
            s.set_subdivs(*bad)
    L = miro.lib()
    h = L.mrt_scene_create()
    try:
        assert L.mrt_scene_set_subdivs(h, 1, 4, 0.01) == 0
        for bad in [(0, 1, 0.01), (3, 2, 0.01), (1, 17, 0.01), (1, 2, -1.0)]:
            assert L.mrt_scene_set_subdivs(h, *bad) < 0
    finally:
        L.mrt_scene_destroy(h)


# ---------------------------------------------------------------- GPU parity
def gpu_render(P, cam, W, H, **kw):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True, **kw)
    return img, hits


def assert_same(P, O_, cam, W, H):
    img, hits = gpu_render(P, cam, W, H)
    ref = O_.render(cam, W, H, threads=8)
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"]), "8-bit RGB differs"
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "centre-sample hit ids differ"
    assert P.last_stats["primary_rays"] == ref["primary_rays"]
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    return P.last_stats


@pytest.mark.gpu
@pytest.mark.parametrize("kind,subdivs", [("lambert", (1, 3, 0.01)), ("blinn", (2, 4, 0.005)),
                                          ("lambert", (1, 4, 0.0)), ("blinn", (1, 1, 0.01))])
def test_adaptive_point_light_matches_oracle(kind, subdivs):
    P, O_, cam = oracle_c1(subdivs, kind=kind)
    st = assert_same(P, O_, cam, 72, 56)
    if subdivs[1] > 1:
        assert st["primary_rays"] > 72 * 56


@pytest.mark.gpu
def test_adaptive_area_light_and_paths_match_oracle():
    """RectangleLight draws come from each eye ray's own RNG stream."""
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=4, noise=0.001)]
    P, O_, cam = oracle_c1((1, 3, 0.01), lights=lights, kind="blinn")
    assert_same(P, O_, cam, 64, 48)


@pytest.mark.gpu
def test_adaptive_bunny_with_environment_matches_oracle():
    """Misses sample the environment map per eye ray (src/Scene.cpp:236-239)."""
    P, O_, cam = config_scene("D1", subdivs=(1, 3, 0.01))
    assert_same(P, O_, cam, 48, 48)


@pytest.mark.gpu
def test_adaptive_count_mode_is_exact():
    """The instrumented launch produces the same frame.  Its visit count covers
    eye rays (closest hit, as the oracle) plus any-hit shadow rays, which stop
    at the first occluder where the oracle's closest-hit shadow rays go on."""
    P, O_, cam = oracle_c1((1, 3, 0.01), kind="blinn")
    img, _ = gpu_render(P, cam, 40, 40, count_visits=True)
    ref = O_.render(cam, 40, 40, threads=8)
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
    assert ref["primary_node_visits"] < P.last_stats["node_visits"] <= ref["node_visits"]
    assert P.last_stats["primary_rays"] == ref["primary_rays"]


@pytest.mark.gpu
def test_adaptive_bucket_batch_equals_frame():
    """The multi-GPU path (32x32 buckets dealt to ranks, mrt_render_batch_async)
    renders adaptive frames bit-identically to the whole-frame launch."""
    torch = pytest.importorskip("torch")
    import ctypes as C
    from miro import _lib
    P, _, cam = oracle_c1((1, 3, 0.01), kind="blinn")
    W, H = 70, 45
    img, _ = gpu_render(P, cam, W, H)
    bpf = ((W + 31) // 32) * ((H + 31) // 32)
    order = np.random.default_rng(3).permutation(bpf).tolist()
    ids = torch.tensor(order, dtype=torch.int32, device="cuda")
    tiles = torch.zeros(bpf * 1024 * 3, dtype=torch.float32, device="cuda")
    frame = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    camc = (_lib.mrt_camera * 1)(camera(cam)._c())
    opts = _lib.mrt_render_opts(W, H, 0, 0, 0, 0, 0)
    L = miro.lib()
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(L.mrt_render_batch_async(P.handle, camc, 1, C.byref(opts), ids.data_ptr(), bpf, tiles.data_ptr(),
                                        None, stream), "batch")
    _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), bpf, tiles.data_ptr(), None, W, H, 1, frame.data_ptr(),
                                        None, P.handle, stream), "unpack")
    torch.cuda.synchronize()
    assert np.array_equal(bits(frame.cpu().numpy().reshape(H, W, 3)), bits(img.rgb))


@pytest.mark.gpu
@pytest.mark.parametrize("refill", [1, 32, 64])
def test_adaptive_pixel_refill_equals_tile_schedule(refill):
    """Lane refill (a lane takes the next pixel when its own has stopped) and the
    tile schedule give the same frame bit for bit: every pixel's eye rays, draws
    and running mean are the same, whichever lane runs them."""
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=3, noise=0.001)]
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = dict(kind="blinn", kd=(0.7, 0.6, 0.5), specExp=12.0, specAmt=0.3)
    P, _, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, subdivs=(1, 4, 0.004))
    L = miro.lib()
    try:
        assert L.mrt_set_tuning(b"adapt_refill", 0) == 0
        img0, hits0 = gpu_render(P, cam, 97, 61)
        st0 = P.last_stats
        assert L.mrt_set_tuning(b"adapt_refill", refill) == 0
        img1, hits1 = gpu_render(P, cam, 97, 61)
        st1 = P.last_stats
    finally:
        L.mrt_set_tuning(b"adapt_refill", 32)
    assert np.array_equal(hits0["prim"], hits1["prim"])
    assert np.array_equal(bits(img0.rgb), bits(img1.rgb))
    assert np.array_equal(img0.pixels, img1.pixels)
    assert st0["shadow_rays"] == st1["shadow_rays"] > 0
    assert st0["primary_rays"] == st1["primary_rays"]
