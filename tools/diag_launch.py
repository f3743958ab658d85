"""Host cost of mrt_render_frame_async on C3 and the timeline of a 20-frame
timed region (4 streams): per-call host microseconds, and GPU completion times
of each frame (events), to separate fixed start / drain cost from the per-frame
rate."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import miro  # noqa: E402
from miro import _lib, scenes  # noqa: E402

scene, cam, cfg = scenes.build_config("C3")
W, H = cfg["W"], cfg["H"]
L = miro.lib()
K = 4
streams = [torch.cuda.Stream() for _ in range(K)]
fr = [torch.empty(H * W * 3, dtype=torch.float32, device="cuda") for _ in range(K)]
fr8 = [torch.empty(H * W * 3, dtype=torch.uint8, device="cuda") for _ in range(K)]
camc = cam._c()
o = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)


def launch(i):
    _lib.check(L.mrt_render_frame_async(scene.handle, C.byref(camc), C.byref(o), fr[i % K].data_ptr(),
                                        fr8[i % K].data_ptr(), streams[i % K].cuda_stream), "render")


for i in range(10):
    launch(i)
torch.cuda.synchronize()
for trial in range(3):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    host = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(streams[0])
    for i in range(20):
        th = time.perf_counter()
        launch(i)
        host.append((time.perf_counter() - th) * 1e6)
        evs[i + 1].record(streams[i % K])
    t_issue = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) * 1e3
    done = [evs[0].elapsed_time(e) for e in evs[1:]]
    print(f"trial {trial}: host us/launch median {np.median(host):.1f} max {max(host):.1f}; issue {t_issue:.2f} ms, "
          f"wall {t_all:.2f} ms; frame done (ms from start): " + " ".join(f"{d:.2f}" for d in done))
