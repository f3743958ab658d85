"""Pins for the CPU oracle against measurements of the reference itself
(explosion01.obj -> 11,647 QBVH nodes / 23,365 leaves),
the loader facts and the committed golden fixtures."""
import json
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, REF_MODELS
from helpers import fixture_mesh


def test_explosion01_qbvh_matches_reference_counts():
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_mesh(*fixture_mesh("explosion01"), m)
    s.build()
    info = s.qbvh_info()
    assert info["prims"] == 86914
    assert info["nodes"] == 11647     # reference QBVH_Node::nodeCount
    assert info["leaves"] == 23365    # reference QBVH_Node::leafCount


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference models not present")
@pytest.mark.parametrize("name,rel", [("cornell_box", "cornell_box.obj"), ("teapot", "teapot.obj")])
def test_loader_fixture_reproducible(name, rel):
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_obj(os.path.join(REF_MODELS, rel), m)
    got = s.mesh_arrays(0)
    for a, b in zip(got, fixture_mesh(name)):
        assert np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))


def test_loader_scaling_in_fixture():
    v = fixture_mesh("cornell_box")[0]
    # every 5.5 coordinate in cornell_box.obj is loaded as 5.4999995 (x rcp_nr(1))
    assert (v == np.float32(5.4999995)).any() and not (v == np.float32(5.5)).any()


def test_c1_golden_frame_reproduced():
    meta = json.load(open(os.path.join(GOLDEN, "fixtures.json")))
    g = np.load(os.path.join(GOLDEN, "c1_cornell_256.npz"))
    from helpers import config_scene
    from miro import scenes
    cfg = scenes.CONFIGS["C1"]
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_mesh(*fixture_mesh("cornell_box"), m)
    s.add_point_light(cfg["lights"][0]["pos"], cfg["lights"][0]["power"])
    s.set_bg(cfg["bg"])
    s.build()
    r = s.render(cfg["camera"], 256, 256)
    assert np.array_equal(r["rgb"].view(np.uint32), g["rgb"].view(np.uint32))
    assert np.array_equal(r["rgb8"], g["rgb8"])
    assert np.array_equal(r["hits"]["prim"], g["prim"])
    assert r["shadow_rays"] == meta["C1"]["shadow_rays"]


def test_trace_closest_vs_any_hit_consistency():
    """Occlusion booleans from closest-hit queries with tMax = distance equal
    'some triangle accepted' -- the property the GPU's any-hit shadow rays rely on."""
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_mesh(*fixture_mesh("teapot"), m)
    s.build()
    rng = np.random.default_rng(3)
    o = rng.uniform(-6, 6, (2000, 3)).astype(np.float32)
    d = rng.normal(size=(2000, 3)).astype(np.float32)
    full, _, _ = s.trace(o, d, 0.001, 1e12)
    tmax = rng.uniform(0.5, 12, 2000).astype(np.float32)
    short, _, _ = s.trace(o, d, 0.001, tmax)
    hit_full_before = (full["prim"] >= 0) & (full["t"] < tmax)
    assert np.array_equal(hit_full_before, short["prim"] >= 0)
