"""The C-ABI library loads and exports every symbol include/mrt.h declares
(no compute calls: this runs on hosts without a GPU)."""
import ctypes
import os
import re

import miro
from conftest import ROOT
from miro import _lib


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "mrt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mrt_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = miro.lib()
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert L.mrt_abi_version() == 10


def test_errors_are_reported_not_raised():
    L = miro.lib()
    assert L.mrt_scene_build_bvh(None) == -1          # MRT_ERR_INVALID, no exception
    assert b"null" in L.mrt_last_error()


def test_chain_tuning_keys_validate():
    """The chain engine's capacity switches (round 4): estimates on / off, the
    headroom percentage in range, the scratch budget in range; bad values are
    rejected with an error, not clamped."""
    L = miro.lib()
    try:
        assert L.mrt_set_tuning(b"chain_est", 0) == 0
        assert L.mrt_set_tuning(b"chain_est", 1) == 0
        assert L.mrt_set_tuning(b"chain_est_pct", 0) != 0
        assert L.mrt_set_tuning(b"chain_est_pct", 200000) != 0
        assert L.mrt_set_tuning(b"chain_est_pct", 150) == 0
        assert L.mrt_set_tuning(b"chain_mb", 0) != 0
        assert L.mrt_set_tuning(b"bin_inst", 3) != 0
        assert L.mrt_set_tuning(b"bin_inst", 2) == 0
    finally:
        assert L.mrt_set_tuning(b"chain_est_pct", 125) == 0
        assert L.mrt_set_tuning(b"bin_inst", 0) == 0
        assert L.mrt_set_tuning(b"chain_est", 1) == 0


def test_batch_tiles_per_wave_key_validates():
    """batch_tpw (tiles per wave a bucket-batch launch is sized for): 1..64, bad values rejected."""
    L = miro.lib()
    try:
        assert L.mrt_set_tuning(b"batch_tpw", 0) != 0
        assert L.mrt_set_tuning(b"batch_tpw", 65) != 0
        assert L.mrt_set_tuning(b"batch_tpw", 1) == 0
    finally:
        assert L.mrt_set_tuning(b"batch_tpw", 2) == 0


def test_walk_tuning_keys_validate():
    """Traversal switches: walk_exit (0 two exits, 1 one exit -- the default; round 6 removed
    the per-scene probe, -1), walk_latch (0 nested, 1 one latch -- the default), lds_nodes
    (0 / 1), scalar_nodes (bit mask 0..7); bad values rejected with an error; the walk info
    entry rejects a null scene."""
    L = miro.lib()
    try:
        for k, good, bad in ((b"walk_exit", (0, 1), (-1, 2)), (b"walk_latch", (0, 1), (-1, 2)),
                             (b"lds_nodes", (0, 1), (-1, 2)),
                             (b"scalar_nodes", (0, 7), (-1, 8))):
            for v in good:
                assert L.mrt_set_tuning(k, v) == 0, (k, v)
            for v in bad:
                assert L.mrt_set_tuning(k, v) != 0, (k, v)
        assert L.mrt_scene_walk_info(None, None, None) != 0
    finally:
        for k, v in ((b"walk_exit", 1), (b"walk_latch", 1), (b"lds_nodes", 0), (b"scalar_nodes", 7)):
            assert L.mrt_set_tuning(k, v) == 0
