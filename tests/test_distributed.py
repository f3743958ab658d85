"""Multi-rank tiling + gather on CPU (gloo, world_size 2 and 3).  The per-rank
renderer is the CPU oracle (test infrastructure) rendering each bucket; the code
under test is the product's tiling / padding / gather / unpack logic
(miro/tiles.py), which must reproduce the single-rank frame bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from miro import scenes, tiles


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_scene():
    import oracle as O
    from helpers import fixture_mesh
    cfg = scenes.CONFIGS["C1"]
    s = O.OracleScene()
    m = s.add_material("lambert")
    s.add_mesh(*fixture_mesh("cornell_box"), m)
    s.add_point_light(cfg["lights"][0]["pos"], cfg["lights"][0]["power"])
    s.set_bg(cfg["bg"])
    s.build()
    return s, cfg["camera"]


def _render_buckets(s, cam, ids, W, H):
    bx, _ = tiles.bucket_grid(W, H)
    out = np.zeros((len(ids), 32, 32, 3), np.float32)
    for slot, b in enumerate(ids):
        x0, y0 = (b % bx) * 32, (b // bx) * 32
        r = s.render(cam, W, H, rect=(x0, y0, x0 + 32, y0 + 32), want_hits=False)
        h, w = min(32, H - y0), min(32, W - x0)
        out[slot, :h, :w] = r["rgb"][y0:y0 + h, x0:x0 + w]
    return out


def _worker(rank, world, port, W, H, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        import conftest  # noqa: F401  (paths)
        s, cam = _oracle_scene()
        nb = np.prod(tiles.bucket_grid(W, H))
        ids = tiles.padded_buckets(int(nb), world, rank)
        t = torch.from_numpy(_render_buckets(s, cam, ids, W, H).reshape(-1))
        got = tiles.gather_tiles(t, world, rank, dist)
        if rank == 0:
            frame = np.zeros((H, W, 3), np.float32)
            for r in range(world):
                tiles.unpack_tiles_numpy(tiles.padded_buckets(int(nb), world, r), got[r].numpy(), W, H, frame)
            np.save(result_path, frame)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_multi_rank_frame_equals_single_rank(tmp_path, world):
    W, H = 100, 70          # ragged: last bucket row/column partially outside the frame
    path = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, path), nprocs=world, start_method="spawn")
    frame = np.load(path)
    s, cam = _oracle_scene()
    ref = s.render(cam, W, H, want_hits=False)["rgb"]
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))


def test_bucket_assignment_covers_frame_once():
    nb = int(np.prod(tiles.bucket_grid(1920, 1080)))
    assert nb == 60 * 34
    for world in (1, 2, 4, 8):
        seen = sorted(b for r in range(world) for b in tiles.rank_buckets(nb, world, r))
        assert seen == list(range(nb))
        lens = {len(tiles.padded_buckets(nb, world, r)) for r in range(world)}
        assert lens == {(nb + world - 1) // world}
