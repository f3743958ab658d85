"""The wavefront chain engine (csrc/mrt_chain.hip) against the fused chain kernel.

Scenes with Blinn reflection / refraction rays or path tracing (reference
src/Blinn.cpp:39-335) shade level by level: level 0 of every path, then per
level a compaction of the spawned children, their closest hits, the shading of
the level with its shadow rays written, traced any-hit and resolved, and finally
a per-pixel combine up each path's chain.  Every ray, RNG draw and add is the
fused kernel's (shade_kernel<REC>, which the oracle tests pin), so the frames
must agree bit for bit -- RGB, 8-bit RGB, hit ids and the shadow / secondary ray
counts -- in frame mode, through the batched bucket path (multi-GPU), and when
a frame is split into chunks of work items.
"""
import ctypes as C

import numpy as np
import pytest

import miro
from helpers import bits, camera, config_scene, fixture_mesh, scene_pair
from miro import _lib, scenes

pytestmark = pytest.mark.gpu

MIRROR = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=1.0, ior=1.5)
GLASS = dict(kind="blinn", kd=(0.6, 0.5, 0.4), refractAmt=1.0, ior=1.5)
MIXED = dict(kind="blinn", kd=(0.6, 0.5, 0.4), ks=(0.9, 0.8, 0.7), reflectAmt=0.6, refractAmt=0.7, ior=1.33,
             specExp=12.0, specAmt=0.2)
GLOSSY = dict(kind="blinn", kd=(0.6, 0.5, 0.4), reflectAmt=0.8, ior=1.5, specGloss=0.6, specExp=8.0, specAmt=0.3)
LEAF = dict(kind="blinn", kd=(0.3, 0.7, 0.2), translucency=0.6, specExp=6.0, specAmt=0.2)
RECT = dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0, samples=3,
            noise=0.001)
POINT = dict(type="point", pos=(2.75, 2.0, -2.75), power=20.0)


def panel(y=5.45, x=(2.0, 3.5), z=(-3.5, -2.0)):
    v = np.array([(x[0], y, z[0]), (x[1], y, z[0]), (x[1], y, z[1]), (x[0], y, z[1])], np.float32)
    n = np.array([(0, -1, 0)] * 4, np.float32)
    f = np.array([(0, 2, 1), (0, 3, 2)], np.uint32)
    return v, n, f, f.copy()


EMIT = dict(kind="blinn", kd=(1, 1, 1), emitted=1.5, le=(1, 1, 1))
PRISM = dict(kind="blinn", kd=(0.2, 0.3, 0.3), reflectAmt=1.0, refractAmt=1.0, specExp=30.0,
             disperse=True, ior3=(1.57, 1.60, 1.62))          # src/Assignment3.h:169-177 (mat2)
FINAL = dict(kind="blinn", kd=(0.9, 0.9, 0.9), reflectAmt=1.0, refractAmt=1.0, specExp=30.0,
             disperse=True, ior3=(1.56, 1.5, 1.5))            # src/main.cpp:167-174


def quad(z=1.0, lo=0.5, hi=5.0):
    """A two-triangle sheet at depth z facing the C1 camera (+z geometric normal)."""
    v = np.array([[lo, lo, z], [hi, lo, z], [hi, hi, z], [lo, hi, z]], np.float32)
    n = np.tile(np.array([[0, 0, 1]], np.float32), (4, 1))
    idx = np.array([[0, 1, 2], [0, 2, 3]], np.uint32)
    return v, n, idx, idx.copy()


def cornell(material, lights=None, **kw):
    cfg = dict(scenes.CONFIGS["C1"])
    cfg["material"] = material
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, **kw)


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if miro.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")


def tuned(**knobs):
    L = miro.lib()
    for k, v in knobs.items():
        assert L.mrt_set_tuning(k.encode(), v) == 0, k


def render(P, cam, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    return img, hits, dict(P.last_stats)


def both_engines(P, cam, W, H):
    try:
        tuned(chain=0)
        fused = render(P, cam, W, H)
        tuned(chain=1)
        chain = render(P, cam, W, H)
    finally:
        tuned(chain=1, chain_mb=8192)
    return fused, chain


def assert_same(a, b):
    (img0, hits0, st0), (img1, hits1, st1) = a, b
    assert np.array_equal(hits0["prim"], hits1["prim"])
    assert np.array_equal(bits(img0.rgb), bits(img1.rgb)), "float RGB differs"
    assert np.array_equal(img0.pixels, img1.pixels), "8-bit RGB differs"
    assert st0["shadow_rays"] == st1["shadow_rays"]
    assert st0["secondary_rays"] == st1["secondary_rays"]


CASES = {
    "mirror": lambda: cornell(MIRROR),
    "glass": lambda: cornell(GLASS),
    "mixed_rect_point": lambda: cornell(MIXED, lights=[RECT, POINT]),
    "glossy": lambda: cornell(GLOSSY),
    "leaf_translucent": lambda: cornell(LEAF, lights=[RECT, POINT]),
    "mixed_env_paths": lambda: scene_pair(dict(scenes.CONFIGS["C1"], material=MIXED, env=dict(sky=(64, 32), exposure=0.7)),
                                          meshes=[fixture_mesh("cornell_box")], num_paths=3),
    "pt_rect_panel": lambda: cornell(dict(kind="blinn", kd=(0.7, 0.7, 0.7), reflectAmt=0.3, specExp=8.0, specAmt=0.25),
                                     lights=[dict(RECT, samples=1)], path_trace=(3, False), num_paths=4,
                                     extra=[(panel(), EMIT)]),
    "pt_panel_env": lambda: scene_pair(dict(scenes.CONFIGS["C1"], lights=[], env=dict(sky=(64, 32), exposure=1.0),
                                            material=dict(kind="blinn", kd=(0.7, 0.7, 0.7))),
                                       meshes=[fixture_mesh("cornell_box")], path_trace=(5, True), num_paths=3,
                                       extra=[(panel(), dict(EMIT, emitted=2.0))]),
    "pt_point_nosample_env": lambda: scene_pair(dict(scenes.CONFIGS["C1"], env=dict(sky=(64, 32), exposure=1.0),
                                                     material=dict(kind="blinn", kd=(0.7, 0.7, 0.7))),
                                                meshes=[fixture_mesh("cornell_box")], path_trace=(4, False), num_paths=2),
    "dome_bunny_mixed": lambda: scene_pair(dict(scenes.CONFIGS["D1"], material=dict(MIXED, kd=(0.8, 0.8, 0.8))),
                                           obj=scenes.bunny_obj(), floor=True),
    # dispersive splits (three refraction children per split, folded per level)
    "disp_sheet_env": lambda: scene_pair(dict(scenes.CONFIGS["C1"], env=dict(sky=(64, 32), exposure=0.7)),
                                         meshes=[fixture_mesh("cornell_box")], extra=[(quad(), PRISM)]),
    "disp_cornell_mixed": lambda: cornell(dict(PRISM, kd=(0.6, 0.5, 0.4), ior3=(1.3, 1.5, 1.9)), lights=[RECT, POINT],
                                          num_paths=2),
    "disp_bunny_dome": lambda: scene_pair(dict(scenes.CONFIGS["D1"], material=dict(PRISM, kd=(0.8, 0.8, 0.8))),
                                          obj=scenes.bunny_obj(), floor=True),
    # adaptive supersampling as passes over the chain engine
    "adapt_mixed_rect": lambda: cornell(MIXED, lights=[RECT, POINT], subdivs=(1, 3, 0.01)),
    "adapt_glossy_paths": lambda: cornell(GLOSSY, num_paths=2, subdivs=(2, 3, 0.02)),
    "adapt_disp_env": lambda: scene_pair(dict(scenes.CONFIGS["C1"], env=dict(sky=(64, 32), exposure=0.7)),
                                         meshes=[fixture_mesh("cornell_box")], extra=[(quad(), FINAL)],
                                         subdivs=(1, 3, 0.01)),
    "adapt_pt_panel": lambda: cornell(dict(kind="blinn", kd=(0.7, 0.7, 0.7), reflectAmt=0.3), lights=[dict(RECT, samples=1)],
                                      path_trace=(3, False), extra=[(panel(), EMIT)], subdivs=(1, 2, 0.0)),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_chain_engine_equals_fused_kernel(case):
    P, _, cam = CASES[case]()
    W, H = (40, 40) if "dome" in case else (64, 48)
    fused, chain = both_engines(P, cam, W, H)
    assert_same(fused, chain)
    assert chain[2]["chain"] == 1 and fused[2]["chain"] == 0
    assert chain[2]["secondary_rays"] > 0 or case in ("leaf_translucent", "pt_point_nosample_env")
    if case.startswith("adapt"):   # eye rays per pixel beyond one: the passes refined
        assert chain[2]["primary_rays"] == fused[2]["primary_rays"] > W * H


@pytest.mark.parametrize("case", ["disp_cornell_mixed", "adapt_disp_env"])
def test_chain_tree_and_adaptive_chunks_equal_one_chunk(case):
    """Dispersive trees and adaptive passes with a 2-MB scratch budget (many
    chunks of units per pass) equal the one-chunk frame."""
    P, _, cam = CASES[case]()
    one = render(P, cam, 48, 40)
    try:
        tuned(chain_mb=2)
        many = render(P, cam, 48, 40)
    finally:
        tuned(chain_mb=8192)
    assert_same(one, many)


@pytest.mark.parametrize("case", ["disp_cornell_mixed", "adapt_disp_env", "pt_rect_panel", "adapt_mixed_rect"])
def test_chain_estimated_capacities_and_fallback_equal_worst_case(case):
    """Level capacities from the counts earlier chunks needed (chain_est) give the
    worst-case-sized frame; with the headroom cut to 1% every chunk outgrows a level
    and the fallback (the fused chain shading over the chunk's units) must give the
    same frame and ray counts -- in one chunk and in many."""
    P, _, cam = CASES[case]()
    try:
        tuned(chain_est=0)
        worst = render(P, cam, 48, 40)
        tuned(chain_est=1)
        render(P, cam, 48, 40)           # seeds this stream's estimates
        est = render(P, cam, 48, 40)
        tuned(chain_est_pct=1)
        fb = render(P, cam, 48, 40)
        tuned(chain_mb=2)
        fb_many = render(P, cam, 48, 40)
    finally:
        tuned(chain_est=1, chain_est_pct=125, chain_mb=8192)
    assert worst[2]["chain_fallbacks"] == 0 and est[2]["chain_fallbacks"] == 0
    assert fb[2]["chain_fallbacks"] >= 1 and fb_many[2]["chain_fallbacks"] >= 1
    for other in (est, fb, fb_many):
        assert_same(worst, other)
        assert other[2]["primary_rays"] == worst[2]["primary_rays"]


def test_chain_engine_on_instances_with_mirrors():
    """ProxyObject instances (nested BLAS traversal in the trace and shadow
    kernels, inverse-transpose normals in the shading) under reflection."""
    P, _, cam = config_scene("C5")
    L = miro.lib()
    mids = [m for m in range(8) if L.mrt_scene_set_material_optics(P.handle, m, 0.5, 0.2, 1.5) == 0]
    assert mids
    fused, chain = both_engines(P, cam, 96, 54)
    assert_same(fused, chain)
    assert chain[2]["secondary_rays"] > 500


def test_chain_chunks_equal_one_chunk():
    """A 1-MB scratch budget forces one chunk per few work items."""
    P, _, cam = cornell(MIXED, lights=[RECT, POINT], num_paths=2)
    one = render(P, cam, 70, 50)
    try:
        tuned(chain_mb=1)
        many = render(P, cam, 70, 50)
    finally:
        tuned(chain_mb=8192)
    assert_same(one, many)


def test_chain_batch_equals_frames():
    """The batched bucket path (multi-GPU work items) through the chain engine:
    every frame of a 2-camera batch equals its single-frame render."""
    torch = pytest.importorskip("torch")
    P, _, cam = cornell(MIXED, lights=[RECT, POINT])
    W, H, F = 70, 50, 2
    cams = scenes.camera_path(cam, F, step_deg=5.0)
    bpf = ((W + 31) // 32) * ((H + 31) // 32)
    order = np.random.default_rng(3).permutation(bpf * F).tolist()
    ids = torch.tensor(order, dtype=torch.int32, device="cuda")
    n = len(order)
    tiles = torch.zeros(n * 1024 * 3, dtype=torch.float32, device="cuda")
    frames = torch.zeros(F * H * W * 3, dtype=torch.float32, device="cuda")
    camc = (_lib.mrt_camera * F)(*[camera(c)._c() for c in cams])
    opts = _lib.mrt_render_opts(W, H, 0, 0, 0, 0, 0)
    L = miro.lib()
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(L.mrt_render_batch_async(P.handle, camc, F, C.byref(opts), ids.data_ptr(), n, tiles.data_ptr(),
                                        None, stream), "batch")
    _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), n, tiles.data_ptr(), None, W, H, F, frames.data_ptr(),
                                        None, P.handle, stream), "unpack")
    torch.cuda.synchronize()
    fr = frames.cpu().numpy().reshape(F, H, W, 3)
    for f in range(F):
        img = miro.Image()
        img.resize(W, H)
        P.raytraceImage(camera(cams[f]), img, seed=0x5EED + f)
        assert np.array_equal(bits(fr[f]), bits(img.rgb)), f


@pytest.mark.parametrize("case", ["pt_rect_panel", "adapt_mixed_rect", "disp_cornell_mixed", "mixed_env_paths"])
def test_odd_frame_sizes_match_oracle(case):
    """1x1, 33x17 and 7x65 frames -- partial 8x8 tiles and 32x32 buckets, fewer units than one
    wave, chain levels of a handful of entries -- through both engines against the oracle:
    hit ids and ray counts exact, RGB within the path-tracing tolerance (1e-4 relative, libm
    pow in Blinn's specular term; tests/test_path_trace.py)."""
    P, O, cam = CASES[case]()
    for W, H in ((1, 1), (33, 17), (7, 65)):
        ref = O.render(cam, W, H)
        for img, hits, st in both_engines(P, cam, W, H):
            assert np.array_equal(hits["prim"], ref["hits"]["prim"]), (W, H)
            assert st["shadow_rays"] == ref["shadow_rays"] and st["secondary_rays"] == ref["secondary_rays"], (W, H)
            g, r = img.rgb.astype(np.float64), ref["rgb"].astype(np.float64)
            assert not (np.abs(g - r) > 1e-4 * np.maximum(np.abs(r), 1e-3)).any(), (W, H)
