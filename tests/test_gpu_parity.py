"""GPU parity: the HIP path (libmrt.so through the C-ABI) against the CPU
oracle and the committed golden fixtures.  Integer outputs (hit ids, 8-bit
pixels) and floats (t, a, b, RGB) are compared bit-for-bit: the device follows
the reference's x86 numeric contract exactly (csrc/mrt_math.h)."""
import json
import os

import numpy as np
import pytest

import miro
import oracle as O
from conftest import GOLDEN
from helpers import bits, camera, config_scene, fixture_mesh, scene_pair
from miro import scenes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if miro.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")


def render(P, cam, W, H, **kw):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True, **kw)
    return img, hits


def assert_frame_equal(img, hits, ref):
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"]), "8-bit RGB differs"
    assert np.array_equal(hits["prim"], ref["prim"]), "primary hit ids differ"
    hit = ref["prim"] >= 0
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(hits[k][hit]), bits(ref[k][hit])), f"hit {k} differs"


def test_c1_cornell_matches_golden():
    P, _, cam = config_scene("C1")
    g = np.load(os.path.join(GOLDEN, "c1_cornell_256.npz"))
    img, hits = render(P, cam, 256, 256)
    assert_frame_equal(img, hits, {k: g[k] for k in g.files})
    meta = json.load(open(os.path.join(GOLDEN, "fixtures.json")))
    st = P.last_stats
    assert st["primary_rays"] == 256 * 256
    assert st["shadow_rays"] == meta["C1"]["shadow_rays"]


@pytest.mark.parametrize("key,W,H", [("C2", 128, 128), ("C3", 192, 108), ("C2", 200, 75), ("C3L", 192, 108)])
def test_configs_match_oracle(key, W, H):
    P, Osc, cam = config_scene(key)
    img, hits = render(P, cam, W, H, count_visits=True)
    ref = Osc.render(cam, W, H, threads=8)
    r = {"rgb": ref["rgb"], "rgb8": ref["rgb8"], "prim": ref["hits"]["prim"], "t": ref["hits"]["t"],
         "a": ref["hits"]["a"], "b": ref["hits"]["b"]}
    assert_frame_equal(img, hits, r)
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    # same traversal, node for node: primary-ray visit counts equal the oracle's
    # (shadow rays are any-hit on the device, closest-hit in the oracle)
    assert P.last_stats["primary_node_visits"] == ref["primary_node_visits"]
    assert P.last_stats["primary_leaf_visits"] == ref["primary_leaf_visits"]


def test_lambert_and_blinn_multi_light():
    cfg = dict(scenes.CONFIGS["C1"])
    lights = [dict(type="point", pos=(2.75, 5.0, -2.75), power=40.0), dict(type="point", pos=(1.0, 2.0, -1.0), power=10.0)]
    for kind in ("lambert", "blinn"):
        cfg["material"] = dict(kind=kind, kd=(0.8, 0.5, 0.25))
        P, Osc, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights)
        img, hits = render(P, cam, 96, 64)
        ref = Osc.render(cam, 96, 64)
        assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))


def test_point_light_transparent_shadows_match_oracle():
    """Light::setFastShadows(false) on a point light: the reference's walk never
    traces (src/PointLight.cpp:49-70), so the frame has no shadows; it equals the
    oracle's bit for bit and differs from the fast-shadow frame."""
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="blinn", kd=(0.8, 0.5, 0.25), specExp=10.0, specAmt=0.4))
    light = dict(type="point", pos=(2.75, 5.0, -2.75), power=40.0)
    P, Osc, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=[dict(light, fast_shadows=False)])
    img, hits = render(P, cam, 96, 64)
    ref = Osc.render(cam, 96, 64)
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
    assert P.last_stats["shadow_rays"] == 0
    P2, _, _ = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=[light])
    img2, _ = render(P2, cam, 96, 64)
    assert P2.last_stats["shadow_rays"] > 0 and not np.array_equal(bits(img.rgb), bits(img2.rgb))


def test_trace_batch_matches_oracle():
    arrs = fixture_mesh("explosion01")
    P, Osc, _ = scene_pair(scenes.CONFIGS["C1"] | {"material": dict(kind="lambert", kd=(1, 1, 1))}, meshes=[arrs])
    rng = np.random.default_rng(11)
    n = 20000
    tgt = arrs[0][rng.integers(0, len(arrs[0]), n)]
    o = (tgt + rng.normal(scale=1.5, size=(n, 3))).astype(np.float32)
    d = (tgt - o + rng.normal(scale=0.05, size=(n, 3))).astype(np.float32)
    tmax = np.full(n, 1e12, np.float32)
    got = P.traceBatch(o, d, 0.001, tmax)
    ref, _, _ = Osc.trace(o, d, 0.001, tmax)
    assert np.array_equal(got["prim"], ref["prim"])
    hit = ref["prim"] >= 0
    assert hit.mean() > 0.3
    for k in ("t", "a", "b"):
        assert np.array_equal(bits(got[k][hit]), bits(ref[k][hit]))
    # any-hit (shadow) queries: occlusion equals "closest hit before tmax"
    tm = rng.uniform(0.1, 3.0, n).astype(np.float32)
    occ = P.traceBatch(o, d, 0.001, tm, any_hit=True)
    assert np.array_equal(occ["prim"] >= 0, hit & (ref["t"] < tm))


def test_bucketed_render_equals_frame(tmp_path):
    torch = pytest.importorskip("torch")
    import ctypes as C
    from miro import _lib
    P, _, cam = config_scene("C2")
    W, H = 300, 200
    img, _ = render(P, cam, W, H)
    bx, by = (W + 31) // 32, (H + 31) // 32
    ids = torch.arange(bx * by, dtype=torch.int32, device="cuda").flip(0).contiguous()
    tiles = torch.zeros(len(ids) * 1024 * 3, dtype=torch.float32, device="cuda")
    frame = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
    frame8 = torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda")
    opts = _lib.mrt_render_opts(W, H, 0, 0, 0, 0, 0)
    c = camera(cam)._c()
    stream = torch.cuda.current_stream().cuda_stream
    L = miro.lib()
    _lib.check(L.mrt_render_buckets_async(P.handle, C.byref(c), C.byref(opts), ids.data_ptr(), len(ids),
                                          tiles.data_ptr(), stream), "buckets")
    _lib.check(L.mrt_unpack_buckets_async(ids.data_ptr(), len(ids), tiles.data_ptr(), W, H, frame.data_ptr(),
                                          frame8.data_ptr(), P.handle, stream), "unpack")
    torch.cuda.synchronize()
    assert np.array_equal(bits(frame.cpu().numpy().reshape(H, W, 3)), bits(img.rgb))
    assert np.array_equal(frame8.cpu().numpy().reshape(H, W, 3), img.pixels)


def test_edge_cases():
    # 1x1 frame, frame sizes not multiple of 8/32, rays parallel to axes (d == 0 -> 1e12)
    P, Osc, cam = config_scene("C1")
    for W, H in ((1, 1), (33, 17), (7, 65)):
        img, hits = render(P, cam, W, H)
        ref = Osc.render(cam, W, H)
        assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
    o = np.array([[2.75, 2.75, 5.0], [2.75, 2.75, 5.0], [-3, 2, -2]], np.float32)
    d = np.array([[0, 0, -1], [0, -1, 0], [1, 0, 0]], np.float32)
    got = P.traceBatch(o, d)
    ref, _, _ = Osc.trace(o, d, 0.001, 1e12)
    assert np.array_equal(got["prim"], ref["prim"])
    assert np.array_equal(bits(got["t"]), bits(ref["t"]))


@pytest.mark.parametrize("knobs", [dict(shade1=0, fast_box=0, sched=0, primary_waves=0),
                                   dict(shade1=1, fast_box=1, sched=1, primary_waves=6),
                                   dict(shade1=0, fast_box=1, sched=2, primary_waves=0),
                                   dict(shade1=1, fast_box=0, sched=3, primary_waves=6),
                                   dict(shade1=1, fast_box=1, sched=2, primary_waves=6, scalar_nodes=0),
                                   dict(shade1=1, fast_box=1, sched=2, primary_waves=8, scalar_nodes=1),
                                   dict(shade1=0, wavefront=0), dict(shade1=0, wavefront=1, fast_box=0),
                                   dict(fused=0, shade1=1), dict(fused=1, frame1_waves=5, sched=3),
                                   dict(fused=1, frame1_waves=8, fast_box=0), dict(fused=1, frame1_waves=1, sched=0),
                                   dict(fused=1, walk_exit=0), dict(fused=1, walk_exit=1),
                                   dict(fused=0, walk_exit=0, primary_waves=7), dict(fused=0, walk_exit=1, primary_waves=7),
                                   dict(fused=1, lds_nodes=1), dict(fused=1, lds_nodes=1, frame1_waves=8),
                                   dict(fused=1, walk_latch=0), dict(fused=1, walk_latch=1, sched=3),
                                   dict(fused=1, walk_latch=0, walk_exit=0)])
def test_every_kernel_path_is_exact(knobs):
    """Performance switches must not change a single bit (fused vs split shading,
    one-launch frame1_kernel vs primary + shade1 launches, hardware vs select box
    test, XCD schedule, occupancy build, the walk loop's exit form and latches)."""
    L = miro.lib()
    try:
        for k, v in knobs.items():
            assert L.mrt_set_tuning(k.encode(), v) == 0
        P, Osc, cam = config_scene("C2")
        img, hits = render(P, cam, 160, 120)
        ref = Osc.render(cam, 160, 120, threads=8)
        assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
        img_c, _ = render(P, cam, 160, 120, count_visits=True)
        assert P.last_stats["primary_node_visits"] == ref["primary_node_visits"]
        assert P.last_stats["primary_leaf_visits"] == ref["primary_leaf_visits"]
        assert np.array_equal(hits["prim"], ref["hits"]["prim"])
        assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    finally:
        for k, v in dict(shade1=1, fast_box=1, sched=2, primary_waves=7, scalar_nodes=7, wavefront=1, fused=1,
                         frame1_waves=7, walk_exit=1, walk_latch=1, lds_nodes=0).items():   # the library's defaults
            L.mrt_set_tuning(k.encode(), v)


@pytest.mark.parametrize("kind,paths", [("lambert", 1), ("blinn", 1), ("blinn", 3), ("lambert", 2)])
def test_rectangle_light_and_paths_match_oracle(kind, paths):
    """RectangleLight sampling (src/RectangleLight.cpp:42-136) with the counter RNG
    shared by device and oracle, several samples and Scene::m_numPaths > 1."""
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = dict(kind=kind, kd=(0.7, 0.6, 0.5))
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=4, noise=0.001),
              dict(type="point", pos=(1.0, 3.0, -1.0), power=5.0)]
    P, Osc, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, num_paths=paths)
    img, hits = render(P, cam, 80, 64)
    ref = Osc.render(cam, 80, 64)
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"]))
    assert np.array_equal(img.pixels, ref["rgb8"])
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]


def test_degenerate_rays_take_the_exact_path():
    """Rays with denormal direction components (1/d = inf) or origins on box
    planes must match the reference select semantics (exact box test)."""
    P, Osc, _ = config_scene("C1")
    o = np.array([[2.75, 2.75, 5.0], [0.0, 2.0, -2.0], [2.75, 0.0, -1.0], [1.0, 1.0, 1.0]], np.float32)
    d = np.array([[1e-42, 0.0, -1.0], [1.0, 1e-40, 0.0], [0.0, 1.0, -1e-39], [np.nan, 0.0, -1.0]], np.float32)
    got = P.traceBatch(o, d)
    ref, _, _ = Osc.trace(o, d, 0.001, 1e12)
    assert np.array_equal(got["prim"], ref["prim"])
    hit = ref["prim"] >= 0
    assert np.array_equal(bits(got["t"][hit]), bits(ref["t"][hit]))


def test_batch_render_equals_per_camera_frames():
    """mrt_render_batch_async: 3 cameras of a path in one launch pair, items
    shuffled and padded with duplicates (as dealt across ranks), float and
    8-bit tiles; frame f == mrt_render of camera f with seed default + f
    (a RectangleLight scene, so the per-frame seed matters)."""
    torch = pytest.importorskip("torch")
    import ctypes as C
    from miro import _lib
    cfg = dict(scenes.CONFIGS["C1"])
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=3, noise=0.001)]
    P, _, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights)
    W, H, F = 100, 70, 3
    cams = scenes.camera_path(cam, F, step_deg=5.0)
    bpf = ((W + 31) // 32) * ((H + 31) // 32)
    order = np.random.default_rng(7).permutation(bpf * F).tolist()
    order += order[:5]                                   # duplicates, like rank padding
    ids = torch.tensor(order, dtype=torch.int32, device="cuda")
    n = len(order)
    tiles = torch.zeros(n * 1024 * 3, dtype=torch.float32, device="cuda")
    tiles8 = torch.zeros(n * 1024 * 3, dtype=torch.uint8, device="cuda")
    frames = torch.zeros(F * H * W * 3, dtype=torch.float32, device="cuda")
    frames8 = torch.zeros(F * H * W * 3, dtype=torch.uint8, device="cuda")
    frames8_lut = torch.zeros(F * H * W * 3, dtype=torch.uint8, device="cuda")
    camc = (_lib.mrt_camera * F)(*[camera(c)._c() for c in cams])
    opts = _lib.mrt_render_opts(W, H, 0, 0, 0, 0, 0)
    L = miro.lib()
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(L.mrt_render_batch_async(P.handle, camc, F, C.byref(opts), ids.data_ptr(), n, tiles.data_ptr(),
                                        tiles8.data_ptr(), stream), "batch")
    _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), n, tiles.data_ptr(), tiles8.data_ptr(), W, H, F,
                                        frames.data_ptr(), frames8.data_ptr(), P.handle, stream), "unpack")
    _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), n, tiles.data_ptr(), None, W, H, F, None,
                                        frames8_lut.data_ptr(), P.handle, stream), "unpack lut")
    torch.cuda.synchronize()
    fr = frames.cpu().numpy().reshape(F, H, W, 3)
    fr8 = frames8.cpu().numpy().reshape(F, H, W, 3)
    assert np.array_equal(fr8, frames8_lut.cpu().numpy().reshape(F, H, W, 3))
    for f in range(F):
        img, _ = render(P, cams[f], W, H, seed=0x5EED + f)
        assert np.array_equal(bits(fr[f]), bits(img.rgb)), f
        assert np.array_equal(fr8[f], img.pixels), f
    # frame 0 at the default seed is the oracle-checked single-frame render
    img0, _ = render(P, cams[0], W, H)
    assert np.array_equal(bits(fr[0]), bits(img0.rgb))
    # bad arguments fail loudly
    assert L.mrt_render_batch_async(P.handle, camc, 17, C.byref(opts), ids.data_ptr(), n, tiles.data_ptr(), None,
                                    stream) == -1
    assert L.mrt_render_batch_async(P.handle, camc, F, C.byref(opts), ids.data_ptr(), n, None, None, stream) == -1


def assert_close_rgb(got, ref, rtol=1e-4):
    """north_star tolerance for configs with a libm pow (Blinn specAmt > 0):
    |got - ref| <= rtol * |ref| per channel (exact zeros must stay zero)."""
    g, r = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    bad = np.abs(g - r) > rtol * np.abs(r)
    assert not bad.any(), f"{bad.sum()} channels beyond {rtol} relative"
    return float(np.mean(bits(got) == bits(ref)))


@pytest.mark.parametrize("W,H", [(160, 90), (97, 61)])
def test_c4_area_light_16_paths_matches_oracle(W, H):
    """C4: RectangleLight, Scene::m_numPaths = 16, Blinn with a specular lobe.
    Hits, shadow-ray counts bit-exact; float RGB within 1e-4 relative (pow)."""
    P, Osc, cam = config_scene("C4")
    img, hits = render(P, cam, W, H)
    ref = Osc.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"])
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    exact = assert_close_rgb(img.rgb, ref["rgb"])
    assert exact > 0.99, exact
    same = np.all(bits(img.rgb) == bits(ref["rgb"]), axis=-1)
    assert np.array_equal(img.pixels[same], ref["rgb8"][same])


def dome_cfg(kind, samples, env=True):
    cfg = dict(scenes.CONFIGS["D1"])
    cfg["material"] = dict(kind=kind, kd=(0.8, 0.8, 0.8), specExp=20.0, specAmt=0.3)
    cfg["lights"] = [dict(type="dome", sky=(128, 64), power=0.15, samples=samples, noise=0.001)]
    cfg["env"] = dict(sky=(128, 64), exposure=1.5) if env else None
    return cfg


@pytest.mark.parametrize("kind,samples,W,H", [("lambert", 1, 96, 64), ("blinn", 6, 80, 60), ("blinn", 6, 33, 17)])
def test_dome_light_and_env_map_match_oracle(kind, samples, W, H):
    """DomeLight (Distribution1D importance sampling of the lat-long map, shadow
    rays to 1e12) + environment map on missed primary rays.  Hits and shadow-ray
    counts exact (the sampling runs on the same RNG draws); float RGB within 1e-4
    relative (atan2 / acos / pow in double on both sides)."""
    P, Osc, cam = scene_pair(dome_cfg(kind, samples), obj=scenes.bunny_obj(), floor=True)
    img, hits = render(P, cam, W, H)
    ref = Osc.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"])
    assert (ref["hits"]["prim"] < 0).any() and (ref["hits"]["prim"] >= 0).any()   # env and shaded pixels
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"] > 0
    exact = assert_close_rgb(img.rgb, ref["rgb"])
    assert exact > 0.99, exact


def test_env_map_without_lights_in_shadow_free_frame():
    """Environment lookup alone: every missed pixel equals the oracle's lookup
    bit for bit except where double atan2 / acos round differently."""
    cfg = dome_cfg("lambert", 1)
    cfg["lights"] = [dict(type="point", pos=(10.0, 20.0, 10.0), power=1000.0)]
    P, Osc, cam = scene_pair(cfg, obj=scenes.bunny_obj(), floor=False)
    img, hits = render(P, cam, 64, 48)
    ref = Osc.render(cam, 64, 48, threads=8)
    miss = ref["hits"]["prim"] < 0
    assert miss.sum() > 100
    exact = assert_close_rgb(img.rgb[miss], ref["rgb"][miss], rtol=1e-6)
    assert exact > 0.99, exact


def test_dome_light_batch_equals_frame():
    """The bucketed batch path shades dome lights and env misses as the frame path."""
    P, _, cam = scene_pair(dome_cfg("blinn", 2), obj=scenes.bunny_obj(), floor=True)
    img, _ = render(P, cam, 64, 64)
    import torch
    from miro import _lib
    import ctypes as C
    L = _lib.load()
    opts = _lib.mrt_render_opts(64, 64, 0, 0, 0, 0, 0)
    camc = (_lib.mrt_camera * 1)(camera(cam)._c())
    ids = torch.arange(4, dtype=torch.int32, device="cuda")
    tiles = torch.zeros(4 * 1024 * 3, dtype=torch.float32, device="cuda")
    frame = torch.zeros(64 * 64 * 3, dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    assert L.mrt_render_batch_async(P.handle, camc, 1, C.byref(opts), ids.data_ptr(), 4, tiles.data_ptr(), None,
                                    stream) == 0
    assert L.mrt_unpack_batch_async(ids.data_ptr(), 4, tiles.data_ptr(), None, 64, 64, 1, frame.data_ptr(), None,
                                    P.handle, stream) == 0
    torch.cuda.synchronize()
    assert np.array_equal(bits(frame.cpu().numpy().reshape(64, 64, 3)), bits(img.rgb))


def test_c5_instanced_dome_matches_oracle():
    """C5 (64 ProxyObjects of two BLASes + floor, DomeLight 6 samples, env map) at a
    small size: hit ids (instance encoding) and shadow-ray counts exact, float RGB
    within 1e-4 relative (double atan2 / acos / pow)."""
    P, Osc, cam = config_scene("C5")
    img, hits = render(P, cam, 96, 54)
    ref = Osc.render(cam, 96, 54, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"])
    assert (ref["hits"]["prim"] >= P.bvh_info["prims"]).sum() > 500   # instance hits
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"] > 0
    exact = assert_close_rgb(img.rgb, ref["rgb"])
    assert exact > 0.99, exact


def shadow_schedules(P, cam, W, H):
    """Frames of one scene under every shadow_kernel schedule (grid-stride, XCD
    bands, bands + lane refill) and child order (reference order, nearest first):
    the any-hit answers -- and so every bit of the frame and the ray counts -- must
    not depend on the schedule, the visit order or the deferred instance walks of
    the lane-refill step."""
    L = miro.lib()
    out = []
    try:
        for sched, near in ((0, 0), (1, 0), (1, 1), (2, 0), (2, 1)):   # near: nearest hit child first
            assert L.mrt_set_tuning(b"shadow_sched", sched) == 0
            assert L.mrt_set_tuning(b"near_first", near) == 0
            img, hits = render(P, cam, W, H)
            out.append((img, hits, P.last_stats))
    finally:
        L.mrt_set_tuning(b"shadow_sched", -1)
        L.mrt_set_tuning(b"near_first", -1)
    img0, hits0, st0 = out[0]
    for img, hits, st in out[1:]:
        assert np.array_equal(hits0["prim"], hits["prim"])
        assert np.array_equal(bits(img0.rgb), bits(img.rgb))
        assert np.array_equal(img0.pixels, img.pixels)
        assert st0["shadow_rays"] == st["shadow_rays"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("key,W,H", [("C4", 120, 68), ("D1", 96, 96), ("C5", 128, 72)])
def test_shadow_schedules_give_identical_frames(key, W, H):
    P, _, cam = config_scene(key)
    shadow_schedules(P, cam, W, H)


@pytest.mark.parametrize("key,W,H", [("C4", 120, 68), ("D1", 96, 96), ("C5", 96, 54)])
def test_wavefront_shadow_pass_equals_fused_kernel(key, W, H):
    """Kernel 2a/2b/2c (shadow rays written, traced any-hit in a separate launch,
    shading resolved) against the fused shading kernel: every bit of RGB, hits and
    the shadow-ray count, in frame mode and through the batched bucket path."""
    L = miro.lib()
    P, _, cam = config_scene(key)
    try:
        assert L.mrt_set_tuning(b"wavefront", 0) == 0
        img0, hits0 = render(P, cam, W, H)
        st0 = P.last_stats
        assert L.mrt_set_tuning(b"wavefront", 1) == 0
        img1, hits1 = render(P, cam, W, H)
        st1 = P.last_stats
    finally:
        L.mrt_set_tuning(b"wavefront", 1)
    assert np.array_equal(hits0["prim"], hits1["prim"])
    assert np.array_equal(bits(img0.rgb), bits(img1.rgb))
    assert np.array_equal(img0.pixels, img1.pixels)
    assert st0["shadow_rays"] == st1["shadow_rays"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("rect", [False, True])
def test_batch_grid_sizing_gives_identical_tiles(rect):
    """A small bucket batch (rank 3's share of an 8-way split) launched with grids sized for
    1, 2, 4 and 64 tiles per wave (tuning key batch_tpw): the same tiles, bit for bit -- the
    fused point-light kernel and the general shading path (rectangle light)."""
    torch = pytest.importorskip("torch")
    import ctypes as C
    from miro import _lib
    cfg = dict(scenes.CONFIGS["C1"])
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=2, noise=0.001)] if rect else None
    P, _, cam = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], **({"lights": lights} if rect else {}))
    W, H = 300, 200
    bpf = ((W + 31) // 32) * ((H + 31) // 32)
    mine = [i for i in range(bpf) if i % 8 == 3]
    ids = torch.tensor(mine, dtype=torch.int32, device="cuda")
    camc = (_lib.mrt_camera * 1)(camera(cam)._c())
    opts = _lib.mrt_render_opts(W, H, 0, 0, 0, 0, 0)
    L = miro.lib()
    stream = torch.cuda.current_stream().cuda_stream
    out = []
    try:
        for tpw in (1, 2, 4, 64):
            assert L.mrt_set_tuning(b"batch_tpw", tpw) == 0
            tiles = torch.zeros(len(mine) * 1024 * 3, dtype=torch.float32, device="cuda")
            _lib.check(L.mrt_render_batch_async(P.handle, camc, 1, C.byref(opts), ids.data_ptr(), len(mine),
                                                tiles.data_ptr(), None, stream), "batch")
            torch.cuda.synchronize()
            out.append(tiles.cpu().numpy())
    finally:
        assert L.mrt_set_tuning(b"batch_tpw", 2) == 0
    assert np.abs(out[0]).sum() > 0
    for o in out[1:]:
        assert np.array_equal(bits(o), bits(out[0]))


@pytest.mark.parametrize("key", ["C3", "C4", "C5", "R3", "A3", "G3"])
def test_batch_frames_equal_per_camera_frames(key):
    """mrt_render_batch_frames_async (ABI 10, the IPC split's render): a camera-path batch
    whose items come shuffled, with duplicates and ids past the batch, written straight
    into frame-layout buffers -- through every engine (one-light frame kernel, wavefront
    shadow pass, instanced dome light, chain engine for secondary rays, adaptive passes,
    dispersion); frame f equals a single-frame render of camera f with seed default + f,
    float and 8-bit, and no pixel outside the batch's items is touched (ragged size)."""
    torch = pytest.importorskip("torch")
    import ctypes as C
    from miro import _lib
    P, _, cam = config_scene(key)
    W, H, F = 100, 70, 2
    cams = scenes.camera_path(cam, F, step_deg=5.0)
    bpf = ((W + 31) // 32) * ((H + 31) // 32)
    order = np.random.default_rng(11).permutation(bpf * F).tolist()
    order += order[:3] + [bpf * F + 1]                 # duplicates and an id past the batch (skipped)
    ids = torch.tensor(order, dtype=torch.int32, device="cuda")
    frames = torch.full((F * H * W * 3,), -7.0, dtype=torch.float32, device="cuda")
    frames8 = torch.zeros(F * H * W * 3, dtype=torch.uint8, device="cuda")
    camc = (_lib.mrt_camera * F)(*[camera(c)._c() for c in cams])
    opts = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
    L = miro.lib()
    _lib.check(L.mrt_render_batch_frames_async(P.handle, camc, F, C.byref(opts), ids.data_ptr(), len(order),
                                               frames.data_ptr(), frames8.data_ptr(),
                                               torch.cuda.current_stream().cuda_stream), "batch frames")
    torch.cuda.synchronize()
    fr = frames.cpu().numpy().reshape(F, H, W, 3)
    fr8 = frames8.cpu().numpy().reshape(F, H, W, 3)
    for f in range(F):
        img, _ = render(P, cams[f], W, H, seed=0x5EED + f)
        assert np.array_equal(bits(fr[f]), bits(img.rgb)), (key, f)
        assert np.array_equal(fr8[f], img.pixels), (key, f)
