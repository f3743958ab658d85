"""Bucket tiling across ranks + the frame-end gather.

The reference renders 32x32 buckets (src/Miro.h:55) in a dynamic OpenMP loop
(src/Scene.cpp:90-174).  Across GPUs the buckets are dealt statically,
bucket b -> rank b mod N, which interleaves them over the image (load balance
for interior scenes) and makes the result independent of N: every pixel is a
pure function of (scene, camera, pixel, seed).  Each rank renders its buckets
into a packed tile buffer (bucket-major, 32*32*3 floats per bucket); one
collective gather brings the equal-sized buffers to rank 0 (RCCL over xGMI on
the GPU box, gloo in the CPU tests), which scatters them into the frame.
"""
from __future__ import annotations

from typing import List

import numpy as np

BUCKET = 32


def bucket_grid(W: int, H: int):
    """(buckets_x, buckets_y) of the reference's bucket grid (src/Scene.cpp:90-95)."""
    return (W + BUCKET - 1) // BUCKET, (H + BUCKET - 1) // BUCKET


def rank_buckets(nb: int, world: int, rank: int) -> List[int]:
    return list(range(rank, nb, world))


def padded_buckets(nb: int, world: int, rank: int) -> List[int]:
    """This rank's bucket ids padded (by repeating its last id) to the common
    length ceil(nb / world), so every rank contributes an equal-sized buffer."""
    mine = rank_buckets(nb, world, rank)
    per = (nb + world - 1) // world
    if not mine:
        raise ValueError("more ranks than buckets")
    return mine + [mine[-1]] * (per - len(mine))


def gather_tiles(tiles, world: int, rank: int, dist):
    """Gather every rank's tile buffer on rank 0 (torch.distributed.gather; the
    nccl backend is RCCL and issues one send/recv pair per peer, so all xGMI
    links into rank 0 carry 1/N of the frame concurrently)."""
    if world == 1:
        return [tiles]
    out = [tiles.new_empty(tiles.shape) for _ in range(world)] if rank == 0 else None
    dist.gather(tiles, out, dst=0)
    return out


def unpack_tiles_numpy(ids, tiles, W: int, H: int, frame=None):
    """Host reference of mrt_unpack_buckets_async (used by CPU tests)."""
    bx, _ = bucket_grid(W, H)
    frame = np.zeros((H, W, 3), np.float32) if frame is None else frame
    t = np.asarray(tiles, np.float32).reshape(-1, BUCKET, BUCKET, 3)
    for slot, b in enumerate(ids):
        x0, y0 = (b % bx) * BUCKET, (b // bx) * BUCKET
        h, w = min(BUCKET, H - y0), min(BUCKET, W - x0)
        frame[y0:y0 + h, x0:x0 + w] = t[slot, :h, :w]
    return frame
