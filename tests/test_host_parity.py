"""Host side of the product (libmrt.so loader + BVH builder, no GPU needed)
against the CPU oracle: bit-identical meshes and bit-identical QBVH arrays,
i.e. the device traverses the hierarchy the reference would build."""
import os

import numpy as np
import pytest

import miro
import oracle as O
from conftest import REF_MODELS
from helpers import fixture_mesh
from miro import scenes


def product_scene(obj=None, arrays=None, ctm=None):
    s = miro.Scene()
    tm = miro.TriangleMesh()
    if obj:
        tm.load(obj, ctm)
    else:
        tm.setArrays(*arrays)
    miro.makeMeshObjs(s, tm, miro.Lambert())
    s.preCalc()
    return s


def oracle_scene(obj=None, arrays=None, ctm=None):
    s = O.OracleScene()
    m = s.add_material("lambert")
    if obj:
        s.add_obj(obj, m, None if ctm is None else ctm.m)
    else:
        s.add_mesh(*arrays, m)
    s.build()
    return s


def assert_bits_equal(a, b):
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def assert_same_bvh(p, o):
    po = o.qbvh_info()
    assert p.bvh_info["nodes"] == po["nodes"] and p.bvh_info["leaves"] == po["leaves"]
    for a, b in zip(p.bvh_export(), o.qbvh_export()):
        assert_bits_equal(a, b)


OBJS = ["cornell_box.obj", "teapot.obj", "sphere2.obj", "Final/tree03Leaves.obj", "Final/explosion01.obj"]


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference models not present")
@pytest.mark.parametrize("rel", OBJS)
def test_loader_and_bvh_match_oracle_on_reference_models(rel):
    path = os.path.join(REF_MODELS, rel)
    p, o = product_scene(obj=path), oracle_scene(obj=path)
    for a, b in zip(p.mesh_arrays(0), o.mesh_arrays(0)):
        assert_bits_equal(a, b)
    assert_same_bvh(p, o)


@pytest.mark.skipif(not os.path.isdir(REF_MODELS), reason="reference models not present")
def test_loader_with_transform_matches_oracle():
    ctm = miro.Matrix4x4()
    ctm.m = np.array([[0.5, 0.1, 0.0, 1.0], [0.0, 2.0, 0.3, -2.0], [0.2, 0.0, 1.5, 0.5], [0.0, 0.0, 0.0, 1.0]], np.float32)
    path = os.path.join(REF_MODELS, "teapot.obj")
    p, o = product_scene(obj=path, ctm=ctm), oracle_scene(obj=path, ctm=ctm)
    for a, b in zip(p.mesh_arrays(0), o.mesh_arrays(0)):
        assert_bits_equal(a, b)


@pytest.mark.parametrize("name", ["cornell_box", "teapot", "explosion01"])
def test_bvh_from_fixture_arrays(name):
    arrs = fixture_mesh(name)
    assert_same_bvh(product_scene(arrays=arrs), oracle_scene(arrays=arrs))


def test_explosion01_counts_product():
    p = product_scene(arrays=fixture_mesh("explosion01"))
    assert p.bvh_info["nodes"] == 11647 and p.bvh_info["leaves"] == 23365
    # bench.py's scene_setup line reads the host build time recorded by preCalc
    assert p.bvh_build_ms > 0


@pytest.mark.parametrize("which", ["sponza", "bunny"])
def test_synthetic_scenes_match_oracle(which):
    path = scenes.sponza_obj() if which == "sponza" else scenes.bunny_obj()
    p, o = product_scene(obj=path), oracle_scene(obj=path)
    for a, b in zip(p.mesh_arrays(0), o.mesh_arrays(0)):
        assert_bits_equal(a, b)
    assert_same_bvh(p, o)


def test_obj_errors_fail_loudly(tmp_path):
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nv 1 0 0\nf 1 2 9\n")
    with pytest.raises(miro.MRTError):
        product_scene(obj=str(bad))
    with pytest.raises(miro.MRTError):
        product_scene(obj=str(tmp_path / "missing.obj"))


def test_empty_scene_build_fails():
    s = miro.Scene()
    with pytest.raises(miro.MRTError):
        s.preCalc()
