"""x86 approximate-math contract (reference src/SSE.h:67-101)."""
import os
import platform
import struct
import subprocess

import numpy as np
import pytest

import miro
import oracle as O
from conftest import ROOT


def u(f):
    return struct.unpack("<I", struct.pack("<f", f))[0]


def is_intel():
    try:
        return "GenuineIntel" in open("/proc/cpuinfo").read()
    except OSError:
        return False


def test_known_answers():
    # rcpss(1) = 0x3F7FF000, one Newton step -> 0x3F7FFFFF
    assert u(O.x86_rcp(1.0)) == 0x3F7FF000
    assert u(O.rcp_nr(1.0)) == 0x3F7FFFFF
    assert u(miro.rcp_nr(1.0)) == 0x3F7FFFFF
    # loader scaling: 5.5 * rcp_nr(1) = 5.49999952 (SURVEY.md key finding 5)
    assert np.float32(5.5) * np.float32(O.rcp_nr(1.0)) == np.float32(5.4999995)


def test_specials():
    inf = float("inf")
    assert O.x86_rcp(0.0) == inf and O.x86_rcp(-0.0) == -inf
    assert O.x86_rcp(inf) == 0.0
    assert O.x86_rcp(1e-40) == inf                 # denormal input -> inf
    assert O.x86_rcp(3e38) == 0.0                  # result below FLT_MIN flushes
    assert np.isnan(O.x86_rsqrt(-1.0))
    assert O.x86_rsqrt(inf) == 0.0 and O.x86_rsqrt(0.0) == inf


def test_product_matches_oracle_random():
    rng = np.random.default_rng(7)
    bitsv = rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32)
    xs = bitsv.view(np.float32)
    for x in xs[:4000]:
        a, b = O.rcp_nr(float(x)), miro.rcp_nr(float(x))
        assert u(a) == u(b) or (np.isnan(a) and np.isnan(b))
        a, b = O.rsqrt_nr(float(x)), miro.rsqrt_nr(float(x))
        assert u(a) == u(b) or (np.isnan(a) and np.isnan(b))


def test_product_matches_oracle_specials():
    """Every exponent class of the select-chain emulation: zeros, denormals,
    smallest/largest normals, results that flush, infinities, NaNs, negatives."""
    pats = [0x00000000, 0x80000000, 0x00000001, 0x807FFFFF, 0x00400000, 0x00800000, 0x80800000,
            0x01000000, 0x3F800000, 0xBF800000, 0x3F7FFFFF, 0x7E800000, 0x7E7FFFFF, 0x7EFFFFFF, 0x7F000000,
            0x7F7FFFFF, 0xFF7FFFFF, 0x7F800000, 0xFF800000, 0x7FC00000, 0xFFC00001, 0x7F800001, 0x40490FDB]
    for e in range(256):                      # every exponent, two mantissas, both signs
        for m in (0, 0x5A5A5A):
            pats += [(e << 23) | m, 0x80000000 | (e << 23) | m]
    for p in pats:
        x = struct.unpack("<f", struct.pack("<I", p))[0]
        for fo, fp in ((O.rcp_nr, miro.rcp_nr), (O.rsqrt_nr, miro.rsqrt_nr), (O.x86_rcp, None)):
            if fp is None:
                continue
            a, b = fo(x), fp(x)
            assert u(a) == u(b) or (np.isnan(a) and np.isnan(b)), hex(p)


@pytest.mark.skipif(not is_intel() or platform.machine() != "x86_64", reason="tables are Intel RCPSS/RSQRTSS")
def test_tables_match_live_instructions(tmp_path):
    """Re-derive the tables from live RCPSS/RSQRTSS and compare with the committed
    data (strided sweep here; tools/gen_x86_tables.c without --stride is exhaustive)."""
    exe = tmp_path / "gen"
    subprocess.check_call(["gcc", "-O2", "-msse4.1", "-o", str(exe), os.path.join(ROOT, "tools", "gen_x86_tables.c")])
    out = tmp_path / "t.inc"
    subprocess.check_call([str(exe), str(out), "--stride", "1031"])
    committed = open(os.path.join(ROOT, "rendering-algorithms-raytracer_amd", "csrc", "x86_approx_tables.inc")).read()
    body = lambda s: s[s.index("MRT_TABLE_QUAL"):]
    assert body(out.read_text()) == body(committed)
