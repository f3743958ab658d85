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


def _batch_worker(rank, world, port, W, H, n_frames, steps, result_path, host_dist=False):
    """Each step renders a batch of n_frames cameras (shifted by the step index,
    so a buffer mix-up between steps shows) through BatchPipeline.  host_dist: the
    collectives through bench.py's _HostDist (its one-GPU rehearsal adapter)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = dist
    if host_dist:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        D = bench._HostDist(dist, torch)
        t = torch.tensor([float(rank + 1)])
        D.all_reduce(t)
        assert t.item() == world * (world + 1) / 2
        t = torch.tensor([float(rank)])
        D.all_reduce(t, op=D.ReduceOp.MAX)
        assert t.item() == world - 1
        D.barrier()
    try:
        s, cam = _oracle_scene()
        bx, by = tiles.bucket_grid(W, H)
        bpf = bx * by
        items = tiles.batch_items(bpf, n_frames, world, rank)
        all_items = [i for r in range(world) for i in tiles.batch_items(bpf, n_frames, world, r)]
        path = scenes.camera_path(cam, n_frames + steps, step_deg=4.0)
        state = {"render": 0, "unpack": 0}
        outs = []

        def render(ids, out):
            k = state["render"]
            state["render"] += 1
            t = out.view(-1, 32, 32, 3)
            for slot, i in enumerate(ids):
                f, b = divmod(i, bpf)
                x0, y0 = (b % bx) * 32, (b // bx) * 32
                r = s.render(path[k + f], W, H, rect=(x0, y0, x0 + 32, y0 + 32), want_hits=False)
                h, w = min(32, H - y0), min(32, W - x0)
                t[slot, :h, :w] = torch.from_numpy(r["rgb"][y0:y0 + h, x0:x0 + w])

        def unpack(ids, gathered, b):
            state["unpack"] += 1
            frames = np.zeros((n_frames, H, W, 3), np.float32)
            t = gathered.view(-1, 32, 32, 3).numpy()
            for slot, i in enumerate(ids):
                f, b = divmod(i, bpf)
                x0, y0 = (b % bx) * 32, (b // bx) * 32
                h, w = min(32, H - y0), min(32, W - x0)
                frames[f, y0:y0 + h, x0:x0 + w] = t[slot, :h, :w]
            outs.append(frames)

        per = len(items)
        pipe = tiles.BatchPipeline(world, rank, D, items, all_items,
                                   lambda k: torch.zeros(k * per * 1024 * 3, dtype=torch.float32), render, unpack)
        for _ in range(steps):
            pipe.step()
        pipe.flush()
        if rank == 0:
            np.save(result_path, np.stack(outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,host_dist", [(2, False), (3, False), (2, True)])
def test_batch_pipeline_frames_equal_single_rank(tmp_path, world, host_dist):
    W, H, n_frames, steps = 70, 40, 2, 3
    path = str(tmp_path / "frames.npy")
    mp.start_processes(_batch_worker, args=(world, _free_port(), W, H, n_frames, steps, path, host_dist),
                       nprocs=world, start_method="spawn")
    got = np.load(path)
    assert got.shape == (steps, n_frames, H, W, 3)
    s, cam = _oracle_scene()
    cams = scenes.camera_path(cam, n_frames + steps, step_deg=4.0)
    for k in range(steps):
        for f in range(n_frames):
            ref = s.render(cams[k + f], W, H, want_hits=False)["rgb"]
            assert np.array_equal(got[k, f].view(np.uint32), ref.view(np.uint32)), (k, f)


def test_batch_items_cover_every_frame_once():
    bpf = 60 * 34
    for world in (1, 2, 4, 8):
        for n_frames in (1, world):
            got = sorted(i for r in range(world) for i in set(tiles.batch_items(bpf, n_frames, world, r)))
            assert got == list(range(bpf * n_frames))
            lens = {len(tiles.batch_items(bpf, n_frames, world, r)) for r in range(world)}
            assert len(lens) == 1


def test_camera_path_starts_at_config_camera():
    cam = scenes.CONFIGS["C3"]["camera"]
    path = scenes.camera_path(cam, 4)
    assert path[0] == cam
    eye = np.array(cam["eye"])
    d0 = np.array(cam["lookAt"]) - eye
    for f, c in enumerate(path):
        assert c["eye"] == cam["eye"]
        d = np.array(c["lookAt"]) - eye
        assert abs(np.linalg.norm(d) - np.linalg.norm(d0)) < 1e-9
        cosang = np.dot(d[[0, 2]], d0[[0, 2]]) / (np.linalg.norm(d[[0, 2]]) * np.linalg.norm(d0[[0, 2]]))
        assert abs(np.degrees(np.arccos(min(1.0, cosang))) - 2.5 * f) < 1e-6


def test_padded_items_cover_once_with_minus_one_padding():
    for n in (1, 7, 60 * 34, 2 * 60 * 34 + 5):
        for world in (1, 2, 3, 8):
            if world > n:
                continue
            lists = [tiles.padded_items(n, world, r) for r in range(world)]
            assert {len(x) for x in lists} == {-(-n // world)}
            real = sorted(i for x in lists for i in x if i >= 0)
            assert real == list(range(n))
            for r, x in enumerate(lists):   # padding only at the end, -1 only
                k = len(tiles.rank_buckets(n, world, r))
                assert all(i == -1 for i in x[k:]) and all(i >= 0 for i in x[:k])


def test_bench_refuses_a_world_size_that_differs_from_gpus():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3 but --gpus 2" in r.stderr


def _libmrt_worker(rank, world, port, key, W, H, result_path):
    """One rank of a multi-process render on one GPU: this rank's 32x32 buckets
    (id mod world) through libmrt's batch path, host copies gathered over gloo,
    rank 0 scatters them with libmrt's unpack kernel."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ctypes as C
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path.insert(0, here)
        import conftest  # noqa: F401  (paths)
        import miro
        from miro import _lib
        from helpers import config_scene, camera
        torch.cuda.set_device(0)
        P, _, cam = config_scene(key)
        L = miro.lib()
        bx, by = tiles.bucket_grid(W, H)
        bpf = bx * by
        mine = tiles.rank_buckets(bpf, world, rank)
        per = -(-bpf // world)
        d_items = torch.tensor(mine, dtype=torch.int32, device="cuda")
        d_tiles = torch.zeros(per * 1024 * 3, dtype=torch.float32, device="cuda")
        opts = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
        camc = (_lib.mrt_camera * 1)(camera(cam)._c())
        s = torch.cuda.current_stream().cuda_stream
        _lib.check(L.mrt_render_batch_async(P.handle, camc, 1, C.byref(opts), d_items.data_ptr(), len(mine),
                                            d_tiles.data_ptr(), None, s), "render batch")
        host = d_tiles.cpu()
        got = [torch.zeros_like(host) for _ in range(world)] if rank == 0 else None
        dist.gather(host, got, dst=0)
        if rank == 0:
            allt = torch.cat(got).cuda()
            ids = torch.tensor([i for r in range(world) for i in tiles.padded_items(bpf, world, r)], dtype=torch.int32,
                               device="cuda")
            frame = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
            _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), len(ids), allt.data_ptr(), None, W, H, 1,
                                                frame.data_ptr(), None, P.handle, s), "unpack")
            np.save(result_path, frame.cpu().numpy().reshape(H, W, 3))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("key,world,W,H", [("C3", 2, 200, 120), ("C4", 3, 130, 70), ("C5", 2, 160, 90)])
def test_libmrt_multi_process_frame_equals_single_process(tmp_path, key, world, W, H):
    """the N > 1 path on libmrt end to end under a process group --
    several processes share cuda:0, each renders its buckets through
    mrt_render_batch_async, gloo gathers, the frame equals one mrt_render."""
    import miro
    from helpers import config_scene, camera
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    path = str(tmp_path / "frame.npy")
    mp.start_processes(_libmrt_worker, args=(world, _free_port(), key, W, H, path), nprocs=world,
                       start_method="spawn")
    frame = np.load(path)
    P, _, cam = config_scene(key)
    img = miro.Image(); img.resize(W, H)
    P.raytraceImage(camera(cam), img)
    assert np.array_equal(frame.view(np.uint32), img.rgb.view(np.uint32))


def _split_worker(rank, world, port, W, H, steps, result_path, depth=2):
    """bench.py's N > 1 headline path on the CPU: ONE frame per step, its buckets
    dealt id mod N (tiles.split_items: unpadded renders, -1-padded gather layout),
    float tiles gathered to rank 0 through BatchPipeline (`depth` buffers, as
    bench.py keeps --inflight of them), rank 0 unpacks; the renderer is the oracle
    (the code under test is the split)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, cam = _oracle_scene()
        bx, by = tiles.bucket_grid(W, H)
        bpf = bx * by
        mine, all_ids, per = tiles.split_items(bpf, world, rank)
        path = scenes.camera_path(cam, steps, step_deg=4.0)
        state = {"render": 0}
        outs = []

        def render(ids, out):
            k = state["render"]
            state["render"] += 1
            assert list(ids) == mine
            t = out.view(-1, 32, 32, 3)
            for slot, b in enumerate(ids):
                x0, y0 = (b % bx) * 32, (b // bx) * 32
                r = s.render(path[k], W, H, rect=(x0, y0, x0 + 32, y0 + 32), want_hits=False)
                h, w = min(32, H - y0), min(32, W - x0)
                t[slot, :h, :w] = torch.from_numpy(r["rgb"][y0:y0 + h, x0:x0 + w])

        def unpack(ids, gathered, b):
            assert len(ids) == world * per
            frame = np.zeros((H, W, 3), np.float32)
            t = gathered.view(-1, 32, 32, 3).numpy()
            for slot, i in enumerate(ids):
                if i < 0:          # padding of a rank with fewer buckets
                    continue
                x0, y0 = (i % bx) * 32, (i // bx) * 32
                h, w = min(32, H - y0), min(32, W - x0)
                frame[y0:y0 + h, x0:x0 + w] = t[slot, :h, :w]
            outs.append(frame)

        pipe = tiles.BatchPipeline(world, rank, dist, mine, all_ids,
                                   lambda k: torch.zeros(k * per * 1024 * 3, dtype=torch.float32), render, unpack,
                                   depth=depth)
        assert len(pipe.tiles) == depth
        for _ in range(steps):
            pipe.step()
        pipe.flush()
        if rank == 0:
            np.save(result_path, np.stack(outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,depth", [(2, 2), (3, 2), (2, 4)])
def test_single_frame_split_pipeline_equals_single_rank(tmp_path, world, depth):
    """The headline N > 1 split (bench.py --split frame) reproduces the single-rank
    frames bit for bit, step after step (ragged frame: 7 buckets over 2 / 3 ranks),
    with 2 or 4 buffers in flight (depth 4: 6 steps, so every buffer is reused)."""
    W, H = 70, 40
    steps = 3 if depth == 2 else 6
    path = str(tmp_path / "frames.npy")
    mp.start_processes(_split_worker, args=(world, _free_port(), W, H, steps, path, depth), nprocs=world,
                       start_method="spawn")
    got = np.load(path)
    assert got.shape == (steps, H, W, 3)
    s, cam = _oracle_scene()
    cams = scenes.camera_path(cam, steps, step_deg=4.0)
    for k in range(steps):
        ref = s.render(cams[k], W, H, want_hits=False)["rgb"]
        assert np.array_equal(got[k].view(np.uint32), ref.view(np.uint32)), k


def test_split_items_layout():
    for n in (7, 60 * 34, 120 * 68):
        for world in (1, 2, 3, 8):
            per_rank = [tiles.split_items(n, world, r) for r in range(world)]
            all_ids, per = per_rank[0][1], per_rank[0][2]
            assert all(p[1] == all_ids and p[2] == per for p in per_rank)
            assert len(all_ids) == world * per
            for r, (mine, _, _) in enumerate(per_rank):
                assert all_ids[r * per:r * per + len(mine)] == mine     # rank r's slots, in order
            assert sorted(i for i in all_ids if i >= 0) == list(range(n))


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["C3", "C4"])
def test_split_path_at_one_gpu_equals_frame_path(key):
    """bench.py's split path (tiles.split_items + BatchPipeline + libmrt batch
    render into float tiles + unpack) at N = 1 equals the whole-frame path bit
    for bit (float RGB and 8-bit)."""
    import ctypes as C
    import miro
    from miro import _lib
    from helpers import config_scene, camera
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 200, 120
    P, _, cam = config_scene(key)
    img = miro.Image(); img.resize(W, H)
    P.raytraceImage(camera(cam), img)
    L = miro.lib()
    bx, by = tiles.bucket_grid(W, H)
    mine, all_ids, per = tiles.split_items(bx * by, 1, 0)
    items = torch.tensor(mine, dtype=torch.int32, device="cuda")
    all_items = torch.tensor(all_ids, dtype=torch.int32, device="cuda")
    camc = (_lib.mrt_camera * 1)(camera(cam)._c())
    opts = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
    K = 4   # buffers / streams in flight, as bench.py --inflight
    out_f = [torch.zeros(H * W * 3, dtype=torch.float32, device="cuda") for _ in range(K)]
    out_8 = [torch.zeros(H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(K)]

    def render(ids, out):
        _lib.check(L.mrt_render_batch_async(P.handle, camc, 1, C.byref(opts), ids.data_ptr(), len(mine),
                                            out.data_ptr(), None, torch.cuda.current_stream().cuda_stream), "render")

    def unpack(ids, gathered, b):
        _lib.check(L.mrt_unpack_batch_async(ids.data_ptr(), len(ids), gathered.data_ptr(), None, W, H, 1,
                                            out_f[b].data_ptr(), out_8[b].data_ptr(), P.handle,
                                            torch.cuda.current_stream().cuda_stream), "unpack")

    pipe = tiles.BatchPipeline(1, 0, None, items, all_items,
                               lambda k: torch.zeros(k * per * 1024 * 3, dtype=torch.float32, device="cuda"),
                               render, unpack, streams=[torch.cuda.Stream() for _ in range(K)])
    for _ in range(2 * K + 1):
        pipe.step()
    pipe.flush()
    torch.cuda.synchronize()
    for b in range(K):
        assert np.array_equal(out_f[b].cpu().numpy().reshape(H, W, 3).view(np.uint32), img.rgb.view(np.uint32))
        assert np.array_equal(out_8[b].cpu().numpy().reshape(H, W, 3), img.pixels)


def _frame_pipeline_worker(rank, world, port, W, H, steps, depth, result_path):
    """FramePipeline on the CPU: rank 0's `depth` frames are a shared memory-mapped
    file (the stand-in for the IPC mapping), every rank writes its buckets of a
    step straight into frame k % depth, the barrier is a gloo all-reduce, and rank
    0 consumes (copies out) each frame once it is whole; the renderer is the oracle."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, cam = _oracle_scene()
        bx, by = tiles.bucket_grid(W, H)
        mine = tiles.rank_buckets(bx * by, world, rank)
        frames = np.lib.format.open_memmap(result_path + ".frames", mode="r+", dtype=np.float32,
                                           shape=(depth, H, W, 3))
        cams = scenes.camera_path(cam, steps, step_deg=4.0)
        state = {"k": 0}
        outs = []

        def render(b):
            k = state["k"]
            state["k"] += 1
            for i in mine:
                x0, y0 = (i % bx) * 32, (i // bx) * 32
                r = s.render(cams[k], W, H, rect=(x0, y0, x0 + 32, y0 + 32), want_hits=False)
                h, w = min(32, H - y0), min(32, W - x0)
                frames[b, y0:y0 + h, x0:x0 + w] = r["rgb"][y0:y0 + h, x0:x0 + w]
            frames.flush()

        def barrier():
            return dist.all_reduce(torch.zeros(1), async_op=True)

        def consume(b):
            outs.append(np.array(frames[b]))

        pipe = tiles.FramePipeline(world, rank, render, barrier, consume if rank == 0 else None, depth=depth)
        for _ in range(steps):
            pipe.step()
        pipe.flush()
        if rank == 0:
            np.save(result_path, np.stack(outs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,depth", [(2, 2), (3, 3)])
def test_frame_pipeline_direct_writes_equal_single_rank(tmp_path, world, depth):
    """bench.py's IPC split (--assemble ipc): ranks write their buckets straight into
    rank 0's frames, one barrier per step, rank 0 consumes each frame when whole --
    every consumed frame equals the single-rank render of its camera, with buffers
    reused (steps > depth) and a ragged bucket grid."""
    W, H = 70, 40
    steps = 5
    path = str(tmp_path / "frames.npy")
    np.lib.format.open_memmap(path + ".frames", mode="w+", dtype=np.float32, shape=(depth, H, W, 3)).flush()
    mp.start_processes(_frame_pipeline_worker, args=(world, _free_port(), W, H, steps, depth, path), nprocs=world,
                       start_method="spawn")
    got = np.load(path)
    assert got.shape == (steps, H, W, 3)
    s, cam = _oracle_scene()
    for k, c in enumerate(scenes.camera_path(cam, steps, step_deg=4.0)):
        ref = s.render(c, W, H, want_hits=False)["rgb"]
        assert np.array_equal(got[k].view(np.uint32), ref.view(np.uint32)), k


def _ipc_worker(rank, world, port, key, W, H, steps, K, result_path):
    """libmrt's IPC split on ONE device: rank 0 allocates the frames, exports them
    (mrt_ipc_export), every other process maps them (mrt_ipc_open) and renders its
    buckets of K camera-path frames per step straight into them
    (mrt_render_batch_frames_async); a gloo all-reduce after each rank's stream
    has drained is the frame-end barrier; rank 0 copies every whole step out."""
    import ctypes as C
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import conftest  # noqa: F401  (paths)
        import miro
        from miro import _lib
        from helpers import config_scene, camera
        torch.cuda.set_device(0)
        P, _, cam = config_scene(key)
        L = miro.lib()
        depth = 2
        bpf = int(np.prod(tiles.bucket_grid(W, H)))
        mine = tiles.rank_buckets(bpf * K, world, rank)
        d_items = torch.tensor(mine, dtype=torch.int32, device="cuda")
        if rank == 0:
            own = [(torch.full((K * H * W * 3,), -1.0, dtype=torch.float32, device="cuda"),
                    torch.zeros(K * H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(depth)]
            hs = []
            for f, f8 in own:
                for t in (f, f8):
                    h = _lib.mrt_ipc_handle()
                    _lib.check(L.mrt_ipc_export(C.c_void_p(t.data_ptr()), C.byref(h)), "ipc export")
                    hs.append(bytes(h))
            obj = [hs]
        else:
            obj = [None]
        dist.broadcast_object_list(obj, src=0)
        ptrs, opened = [], []
        for i in range(depth):
            if rank == 0:
                ptrs.append((own[i][0].data_ptr(), own[i][1].data_ptr()))
                continue
            pair = []
            for j in range(2):
                h = _lib.mrt_ipc_handle.from_buffer_copy(obj[0][2 * i + j])
                p = C.c_void_p()
                _lib.check(L.mrt_ipc_open(C.byref(h), 0, C.byref(p)), "ipc open")
                pair.append(p.value)
                opened.append(p.value)
            ptrs.append(tuple(pair))
        opts = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
        state = {"k": 0}
        outs = []

        def render(b):
            k = state["k"]
            state["k"] += 1
            cams = [camera(c)._c() for c in scenes.camera_path(cam, K * steps, step_deg=3.0)[k * K:(k + 1) * K]]
            cc = (_lib.mrt_camera * K)(*cams)
            _lib.check(L.mrt_render_batch_frames_async(P.handle, cc, K, C.byref(opts), d_items.data_ptr(), len(mine),
                                                       ptrs[b][0], ptrs[b][1],
                                                       torch.cuda.current_stream().cuda_stream), "render frames")

        def barrier():
            torch.cuda.current_stream().synchronize()
            return dist.all_reduce(torch.zeros(1), async_op=True)

        def consume(b):
            outs.append((own[b][0].cpu().numpy().reshape(K, H, W, 3), own[b][1].cpu().numpy().reshape(K, H, W, 3)))

        pipe = tiles.FramePipeline(world, rank, render, barrier, consume if rank == 0 else None, depth=depth)
        for _ in range(steps):
            pipe.step()
        pipe.flush()
        torch.cuda.synchronize()
        dist.barrier()
        for p in opened:
            _lib.check(L.mrt_ipc_close(C.c_void_p(p)), "ipc close")
        if rank == 0:
            np.save(result_path, np.stack([o[0] for o in outs]))
            np.save(result_path + "8.npy", np.stack([o[1] for o in outs]))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("key,world,W,H,K", [("C3", 2, 200, 120, 1), ("C4", 3, 130, 70, 2), ("C5", 2, 160, 90, 2)])
def test_ipc_split_frames_equal_single_process(tmp_path, key, world, W, H, K):
    """every rank of the split writes its buckets into rank 0's
    frames through an IPC mapping (processes sharing cuda:0 here; xGMI peers on a
    node), no gather and no unpack.  Every frame of every step equals one
    mrt_render_frame_async of its camera (seed + f within a step), float and 8-bit,
    with frame buffers reused across steps."""
    import ctypes as C
    import miro
    from miro import _lib
    from helpers import config_scene, camera
    if miro.device_count() < 1:
        pytest.skip("no HIP device")
    steps = 3
    path = str(tmp_path / "frames.npy")
    mp.start_processes(_ipc_worker, args=(world, _free_port(), key, W, H, steps, K, path), nprocs=world,
                       start_method="spawn")
    got, got8 = np.load(path), np.load(path + "8.npy")
    assert got.shape == (steps, K, H, W, 3)
    P, _, cam = config_scene(key)
    L = miro.lib()
    cams = scenes.camera_path(cam, K * steps, step_deg=3.0)
    f = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
    f8 = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    for k in range(steps):
        for j in range(K):
            o = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0x5EED + j)
            cc = camera(cams[k * K + j])._c()
            _lib.check(L.mrt_render_frame_async(P.handle, C.byref(cc), C.byref(o), f.data_ptr(), f8.data_ptr(), None),
                       "render")
            torch.cuda.synchronize()
            ref, ref8 = f.cpu().numpy().reshape(H, W, 3), f8.cpu().numpy().reshape(H, W, 3)
            assert np.array_equal(got[k, j].view(np.uint32), ref.view(np.uint32)), (k, j)
            assert np.array_equal(got8[k, j], ref8), (k, j)
