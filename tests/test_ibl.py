"""Image-based lighting inputs on the host (no GPU): the product's HDR loader and
DomeLight tables (libmrt.so host code) against the CPU oracle, and the oracle's
decoder pinned against an independent numpy decode of the RGBE bytes (the
reference's HDRLoader, src/hdrloader.cpp:29-190, ships no tests of its own).
The reference's own Images/*.hdr are decoded too when present."""
import glob
import os

import numpy as np
import pytest

import miro
import oracle as O
from hdr_files import HEADER, decode, rgbe_pattern, write_hdr
from miro import scenes

REF_IMAGES = "/root/reference/Images"


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def product_hdr(path):
    img = miro.RawImage()
    img.loadHDR(str(path))
    return img.m_rawData


@pytest.mark.parametrize("mode,W,H", [("rle", 64, 9), ("rle", 300, 3), ("flat", 64, 5), ("flat", 5, 4),
                                      ("oldrle", 40, 6), ("oldrle", 7, 3)])
def test_hdr_decoders_match_rgbe_bytes(tmp_path, mode, W, H):
    rgbe = rgbe_pattern(H, W, seed=W * 31 + H)
    p = tmp_path / f"t_{mode}_{W}.hdr"
    write_hdr(p, rgbe, mode)
    want = decode(rgbe)
    assert np.array_equal(bits(O.hdr_load(p)), bits(want))
    assert np.array_equal(bits(product_hdr(p)), bits(want))


def test_hdr_short_file_keeps_the_rows_read(tmp_path):
    rgbe = rgbe_pattern(6, 32, seed=7)
    p = tmp_path / "short.hdr"
    write_hdr(p, rgbe, "flat")
    data = p.read_bytes()
    p.write_bytes(data[:-40])   # the last flat scanline is cut: oldDecrunch hits EOF, the load stops there
    o, q = O.hdr_load(p), product_hdr(p)
    assert np.array_equal(bits(o), bits(q))
    assert np.array_equal(bits(o[:5]), bits(decode(rgbe[:5])))
    assert not o[5].any()


def test_hdr_malformed_inputs_fail_loudly(tmp_path):
    row8 = bytes([2, 2, 0, 8])
    cases = {
        "magic": b"#?RGBE\n\n-Y 1 +X 1\n" + bytes(4),
        "truncated_header": b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n",
        "long_header": b"#?RADIANCE\n" + b"#" * 300 + b"\n\n-Y 1 +X 1\n" + bytes(4),
        "orientation": HEADER + b"+Y 2 +X 2\n" + bytes(16),
        "run_past_line": HEADER + b"-Y 1 +X 8\n" + row8 + bytes([128 + 9, 5]),
        "literal_past_line": HEADER + b"-Y 1 +X 8\n" + row8 + bytes([9]) + bytes(9),
        "rle_cut_short": HEADER + b"-Y 2 +X 8\n" + row8 + bytes([128 + 8, 5]),   # EOF bytes read as runs
        "run_without_pixel": HEADER + b"-Y 1 +X 4\n" + bytes([1, 1, 1, 3]) + bytes(12),
    }
    for name, data in cases.items():
        p = tmp_path / f"{name}.hdr"
        p.write_bytes(data)
        with pytest.raises(miro.MRTError):
            product_hdr(p)
        with pytest.raises(RuntimeError):
            O.hdr_load(p)
    with pytest.raises(miro.MRTError):
        product_hdr(tmp_path / "missing.hdr")


@pytest.mark.skipif(not os.path.isdir(REF_IMAGES), reason="reference images not present")
def test_reference_hdr_images_decode_identically():
    paths = sorted(glob.glob(os.path.join(REF_IMAGES, "*.hdr")))
    assert paths
    for p in paths:
        o, q = O.hdr_load(p), product_hdr(p)
        assert np.array_equal(bits(o), bits(q)), p
        assert np.isfinite(o).all() and o.max() > 0, p
    sky = O.hdr_load(os.path.join(REF_IMAGES, "sky.hdr"))
    assert sky.shape == (500, 1000, 3)   # header "-Y 500 +X 1000"


def dome_product(rgb):
    s = miro.Scene()
    tm = miro.TriangleMesh()
    tm.createSingleTriangle()
    tm.setV1((0, 0, 0)); tm.setV2((1, 0, 0)); tm.setV3((0, 1, 0))
    miro.makeMeshObjs(s, tm, miro.Lambert())
    dl = miro.DomeLight()
    dl.setTexture(miro.Texture(miro.RawImage(rgb.shape[1], rgb.shape[0], rgb)))
    s.addLight(dl)
    s.preCalc()
    return s.dome_tables(0)


def dome_oracle(rgb):
    o = O.OracleScene()
    return o.dome_export(o.add_dome_light(o.add_texture(rgb), 1.0))


@pytest.mark.parametrize("W,H", [(96, 48), (64, 64), (7, 3)])
def test_dome_tables_match_oracle(W, H):
    rgb = scenes.sky_rgb(W, H)
    p, o = dome_product(rgb), dome_oracle(rgb)
    for k in O.DOME_KEYS:
        assert p[k].shape == o[k].shape, k
        assert np.array_equal(bits(p[k]), bits(o[k])), k
    # Distribution1D invariants: CDFs start at 0, are non-decreasing and end at 1
    assert p["cdf_u"][0] == 0 and p["cdf_u"][-1] == 1 and (np.diff(p["cdf_u"]) >= 0).all()
    assert (p["cdf_v"][:, 0] == 0).all() and (p["cdf_v"][:, -1] == 1).all()


@pytest.mark.skipif(not os.path.isdir(REF_IMAGES), reason="reference images not present")
def test_dome_tables_of_reference_sky_match_oracle():
    rgb = O.hdr_load(os.path.join(REF_IMAGES, "sky.hdr"))
    p, o = dome_product(rgb), dome_oracle(rgb)
    for k in O.DOME_KEYS:
        assert np.array_equal(bits(p[k]), bits(o[k])), k


def test_dark_dome_texture_is_rejected():
    with pytest.raises(miro.MRTError):
        dome_product(np.zeros((8, 16, 3), np.float32))


def test_oracle_lookup_dir_poles_and_seam():
    """getLookupXYZ3 corner cases stay in bounds: the poles (acos(+-1)), the
    u seam (atan2 = +-pi) and axis directions."""
    rgb = scenes.sky_rgb(32, 16)
    o = O.OracleScene()
    t = o.add_texture(rgb)
    dirs = np.array([[0, 1, 0], [0, -1, 0], [-1, 0, 0], [-1, 0, -0.0], [1, 0, 0], [0, 0, 1], [0, 0, -1]], np.float32)
    out = o.texture_lookup_dir(t, dirs)
    assert np.isfinite(out).all()
    assert out.min() >= 0 and out.max() <= rgb.max()
