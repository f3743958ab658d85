"""Ray binning (csrc/mrt_bin.h) and the dome-light replay are schedule
changes only: which lane traces which ray, and whether kernel 2c sums recorded
dome samples or draws them again.  Every bit of every frame, the hit ids and the
ray counts must equal the unbinned / re-sampling run (which the oracle tests
pin).  The reference traces rays one at a time (src/Scene.cpp:90-174,
src/BVH.cpp:1112-1178), so no answer may depend on the order."""
import numpy as np
import pytest

import miro
from helpers import bits, camera, config_scene
from test_chain import CASES

KNOB_DEFAULTS = dict(bin=-1, bin_dbits=2, bin_obits=2, dome_replay=1, chain=1, chain_mb=8192, chain_bands=-1,
                     shadow_sched=-1, bin_inst=0, primary_inst_waves=5)


def tuned(**knobs):
    L = miro.lib()
    for k, v in knobs.items():
        assert L.mrt_set_tuning(k.encode(), v) == 0, k


def render(P, cam, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    return img, hits, dict(P.last_stats)


def runs(P, cam, W, H, variants):
    out = []
    try:
        for v in variants:
            tuned(**dict(KNOB_DEFAULTS, **v))
            out.append(render(P, cam, W, H))
    finally:
        tuned(**KNOB_DEFAULTS)
    return out


def assert_all_same(out):
    img0, hits0, st0 = out[0]
    for img, hits, st in out[1:]:
        assert np.array_equal(hits0["prim"], hits["prim"])
        assert np.array_equal(bits(img0.rgb), bits(img.rgb)), "float RGB differs"
        assert np.array_equal(img0.pixels, img.pixels), "8-bit RGB differs"
        assert st0["shadow_rays"] == st["shadow_rays"]
        assert st0["secondary_rays"] == st["secondary_rays"]


def test_bin_tuning_validates_key_bits():
    """Each key field has its range; the pair (2 dbits + 3 obits <= 12 bits, the
    LDS counting sort) is checked when a batch is binned."""
    L = miro.lib()
    try:
        assert L.mrt_set_tuning(b"bin", 8) != 0
        assert L.mrt_set_tuning(b"bin", -2) != 0
        assert L.mrt_set_tuning(b"bin_dbits", 7) != 0
        assert L.mrt_set_tuning(b"bin_obits", 5) != 0
        assert L.mrt_set_tuning(b"bin_dbits", 6) == 0
        assert L.mrt_set_tuning(b"bin_obits", 0) == 0
        assert L.mrt_set_tuning(b"dome_replay", 0) == 0
    finally:
        assert L.mrt_set_tuning(b"bin_obits", 2) == 0
        assert L.mrt_set_tuning(b"bin_dbits", 2) == 0
        assert L.mrt_set_tuning(b"dome_replay", 1) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("key,W,H", [("C4", 120, 68), ("D1", 96, 96), ("C5", 128, 72)])
def test_binned_shadow_pass_and_dome_replay_give_identical_frames(key, W, H):
    P, _, cam = config_scene(key)
    out = runs(P, cam, W, H, [dict(dome_replay=0, bin=0), dict(), dict(bin=1), dict(bin=1, bin_dbits=6, bin_obits=0),
                              dict(bin=1, bin_dbits=0, bin_obits=4), dict(bin=1, dome_replay=0), dict(bin=1, bin_inst=1), dict(bin=1, bin_inst=2)])
    assert out[0][2]["shadow_rays"] > 0
    assert_all_same(out)


@pytest.mark.gpu
def test_dome_replay_with_two_paths_and_a_point_light():
    """Several dome calls per pixel (num_paths 2) after a point light: the replay
    advances the RNG by the recorded draws, so the second path and light match."""
    P, _, cam = config_scene("D1", num_paths=2)
    out = runs(P, cam, 80, 80, [dict(dome_replay=0, bin=0), dict(), dict(bin=1)])
    assert_all_same(out)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["pt_rect_panel", "pt_panel_env", "mixed_env_paths", "disp_cornell_mixed",
                                  "dome_bunny_mixed", "adapt_pt_panel", "adapt_glossy_paths"])
def test_binned_chain_levels_give_identical_frames(case):
    P, _, cam = CASES[case]()
    W, H = (40, 40) if "dome" in case else (64, 48)
    out = runs(P, cam, W, H, [dict(bin=0), dict(), dict(bin=2), dict(bin=4), dict(bin=6),
                              dict(bin=6, bin_dbits=5, bin_obits=0)])
    assert_all_same(out)
    assert out[0][2]["secondary_rays"] > 0


@pytest.mark.gpu
def test_binned_chain_chunks_equal_one_chunk():
    """Binning per chunk of units (a 1-MB scratch budget): the device counts of
    each chunk's levels bound the binned batches."""
    P, _, cam = CASES["pt_rect_panel"]()
    out = runs(P, cam, 70, 50, [dict(bin=0), dict(bin=6, chain_mb=1)])
    assert_all_same(out)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["pt_rect_panel", "pt_panel_env", "mixed_rect_point", "disp_cornell_mixed",
                                  "adapt_mixed_rect", "leaf_translucent"])
def test_chain_trace_schedules_give_identical_frames(case):
    """The chain trace kernel's schedules -- grid-stride chunks and XCD-banded
    chunks, each binned and unbinned -- trace every ray with the same visits, so
    frames, hit ids and ray counts are identical."""
    P, _, cam = CASES[case]()
    out = runs(P, cam, 64, 48, [dict(bin=0, chain_bands=0), dict(bin=0, chain_bands=1), dict(bin=6, chain_bands=0),
                                dict(bin=6, chain_bands=1), dict(bin=2), dict(bin=4, chain_bands=1)])
    assert_all_same(out)



@pytest.mark.gpu
def test_instanced_primary_occupancy_targets_give_identical_frames():
    """The instanced primary kernel at 4 (no spills), 5, 6 waves and unbounded: the
    same nested walks, so the same frames, hit ids and ray counts."""
    P, _, cam = config_scene("C5")
    out = runs(P, cam, 96, 54, [dict(primary_inst_waves=w) for w in (5, 4, 6, 1)])
    assert_all_same(out)
