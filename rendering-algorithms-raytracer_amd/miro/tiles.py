"""Bucket tiling across ranks + the frame-end gather.

Frame batches: a step may render several frames of one size (a camera path).
Items are id = frame * buckets_per_frame + bucket, dealt id -> rank id mod N
over the whole batch, rendered in ONE launch pair per rank
(mrt_render_batch_async) and gathered once per step.  BatchPipeline keeps
`depth` tile buffers (one HIP stream each), so the gather of step k overlaps the
renders of the next steps and several steps' launches are in flight at once.

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

import contextlib
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


def padded_items(n: int, world: int, rank: int) -> List[int]:
    """This rank's item ids (i mod world == rank) padded with -1 to the common
    length ceil(n / world): the gather buffers have equal sizes, the renders skip
    the padding (they see only the unpadded list) and the unpack ignores id -1
    (its frame index is past the batch), so no work is done or counted twice."""
    mine = rank_buckets(n, world, rank)
    return mine + [-1] * (-(-n // world) - len(mine))


def split_items(n: int, world: int, rank: int):
    """The split of an n-item step used by bench.py and the gloo tests: (this
    rank's items id mod world, unpadded -- what it renders; every rank's items
    padded with -1 to ceil(n / world), concatenated in rank order -- the layout
    of the gathered buffer that rank 0 unpacks; that common length)."""
    all_ids = [i for r in range(world) for i in padded_items(n, world, r)]
    return rank_buckets(n, world, rank), all_ids, -(-n // world)


def batch_items(buckets_per_frame: int, n_frames: int, world: int, rank: int) -> List[int]:
    """This rank's item ids (frame * buckets_per_frame + bucket) of a batch,
    padded by repeating its last id to ceil(total / world) (equal gather sizes;
    a repeated item rewrites the same pixels with the same values)."""
    return padded_buckets(buckets_per_frame * n_frames, world, rank)


class BatchPipeline:
    """Per-step render -> gather(rank 0) -> unpack, over `depth` buffers.

    render(items, out_tiles) enqueues this rank's items into out_tiles;
    unpack(all_items, gathered, b) assembles the batch on rank 0 from ONE buffer
    holding every rank's tiles in rank order (all_items is the matching
    concatenation of the ranks' item lists).  new_tiles(k) allocates k ranks'
    worth of tiles.  Both callables are injected so the same pipeline drives
    libmrt on the GPU (RCCL) and the CPU oracle in the gloo tests.

    Step k writes buffer k % depth; before step k + depth reuses it, the gather
    of step k is waited on (work.wait() orders the compute stream after the
    collective on nccl; it blocks on gloo).  Rank 0 unpacks step k after
    enqueuing the render of step k + 1, so its next render is not queued behind
    the collective.  With `streams` (one torch.cuda.Stream per buffer; their
    number sets `depth`), everything of buffer b runs on streams[b]: up to
    `depth` steps' launches are in flight on the device at once, as the N = 1
    frame path keeps its frames in flight, so one share's launch tail overlaps
    the next share's start.  unpack gets the buffer index, so rank 0 can keep
    one output per buffer."""

    def __init__(self, world, rank, dist, items, all_items, new_tiles, render, unpack, streams=None, depth=2):
        self.world, self.rank, self.dist = world, rank, dist
        self.items, self.all_items = items, all_items
        self.render, self.unpack = render, unpack
        self.streams = streams
        self.depth = len(streams) if streams else max(1, depth)
        self.tiles = [new_tiles(1) for _ in range(self.depth)]
        self.recv = [new_tiles(world) for _ in range(self.depth)] if (rank == 0 and world > 1) else None
        self.work = [None] * self.depth
        self.pending = None      # (work, buffer) of the step rank 0 has not unpacked yet
        self.k = 0

    def _on(self, b):
        if self.streams is None:
            return contextlib.nullcontext()
        import torch
        return torch.cuda.stream(self.streams[b])

    def step(self):
        b = self.k % self.depth
        with self._on(b):
            if self.work[b] is not None:
                self.work[b].wait()
                self.work[b] = None
            self.render(self.items, self.tiles[b])
            if self.world == 1:
                self.unpack(self.all_items, self.tiles[b], b)
            else:
                outs = list(self.recv[b].chunk(self.world)) if self.rank == 0 else None
                w = self.dist.gather(self.tiles[b], outs, dst=0, async_op=True)
                self.work[b] = w
        if self.world > 1:
            self._drain()
            if self.rank == 0:
                self.pending = (w, b)
        self.k += 1

    def _drain(self):
        if self.pending is not None:
            w, pb = self.pending
            with self._on(pb):
                w.wait()
                self.unpack(self.all_items, self.recv[pb], pb)
            self.pending = None

    def flush(self):
        """Finish every outstanding gather / unpack (end of the timed region)."""
        self._drain()
        for i in range(self.depth):
            if self.work[i] is not None:
                with self._on(i):
                    self.work[i].wait()
                self.work[i] = None


class FramePipeline:
    """Per-step render straight into rank 0's frames -> one frame-end barrier.

    The frames live on rank 0 (`depth` buffers); every rank has them mapped
    (mrt_ipc_export / mrt_ipc_open on the GPU: rank r's pixels cross xGMI as the
    kernel stores them) and render(b) enqueues this rank's buckets of the step
    straight into buffer b (mrt_render_batch_frames_async) -- no tile buffers, no
    gather, no unpack.  barrier() is a stream-ordered collective (an all-reduce of
    one int, async) that completes once every rank's render of the step has
    completed, i.e. when rank 0's frame b is whole.  consume(b), on rank 0 only
    and optional, runs on buffer b's stream once its frame is whole (e.g. a copy
    out, a display).

    Ordering, with streams (one per buffer): step k renders into b = k % depth on
    streams[b] after the barrier of step k - depth + 1 has completed, and rank 0
    joins barrier j only after consume(j - 1) has run.  So that barrier implies
    that every rank finished step k - depth + 1 and that rank 0 consumed step
    k - depth, the last user of buffer b.  Up to depth - 1 steps' launches are in
    flight at once.  Without streams (gloo on the CPU) every call completes in
    order and the same code runs."""

    def __init__(self, world, rank, render, barrier, consume=None, streams=None, depth=2):
        self.world, self.rank = world, rank
        self.render, self.barrier, self.consume = render, barrier, consume
        self.streams = streams
        self.depth = len(streams) if streams else max(2, depth)
        if self.depth < 2:
            raise ValueError("FramePipeline needs at least 2 buffers")
        self.works = {}          # step -> barrier work
        self.consumed = -1       # last step rank 0 consumed
        self.ev = None           # rank 0: event after the last consume (GPU streams)
        self.k = 0

    def _on(self, b):
        if self.streams is None:
            return contextlib.nullcontext()
        import torch
        return torch.cuda.stream(self.streams[b])

    def _consume(self, j):
        """rank 0: step j's frame is whole after its barrier; consume it on its stream."""
        with self._on(j % self.depth):
            w = self.works.get(j)
            if w is not None:
                w.wait()
            if self.consume is not None:
                self.consume(j % self.depth)
            if self.streams is not None:
                import torch
                self.ev = torch.cuda.Event()
                self.ev.record()
        self.consumed = j

    def step(self):
        k, d = self.k, self.depth
        b = k % d
        if self.rank == 0 and self.consume is not None and k >= 1 and self.consumed < k - 1:
            self._consume(k - 1)
        with self._on(b):
            w = self.works.pop(k - d + 1, None)
            if w is not None:
                w.wait()
            self.render(b)
            if self.rank == 0 and self.ev is not None:   # barrier k only after consume(k - 1)
                import torch
                torch.cuda.current_stream().wait_event(self.ev)
            self.works[k] = self.barrier()
        self.k += 1

    def flush(self):
        """Every outstanding step whole (and consumed on rank 0)."""
        if self.rank == 0 and self.consume is not None:
            for j in range(self.consumed + 1, self.k):
                self._consume(j)
        for j, w in sorted(self.works.items()):
            if w is None:   # (a share rendered alone: no barrier)
                continue
            with self._on(j % self.depth):
                w.wait()
        self.works.clear()
