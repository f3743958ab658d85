"""Feasibility: do consecutive frames on two HIP streams overlap (the tail of
one frame's persistent launches with the start of the next)?  Two copies of
the C3 scene (separate device scratch) alternate frames over 1 or 2 streams."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import torch  # noqa: E402
import miro  # noqa: E402
from miro import _lib, scenes  # noqa: E402


def main():
    L = miro.lib()
    sa, cam, cfg = scenes.build_config("C3")
    sb, _, _ = scenes.build_config("C3")
    W, H = cfg["W"], cfg["H"]
    camc = cam._c()
    o = _lib.mrt_render_opts(W, H, 0, 0, 1, 0, 0)
    bufs = [(torch.empty(H * W * 3, dtype=torch.float32, device="cuda"),
             torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")) for _ in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run(n, nstreams, nscenes):
        t0 = time.perf_counter()
        for i in range(n):
            s = (sa, sb)[i % nscenes]
            st = streams[i % nstreams]
            f, f8 = bufs[i % 2]
            _lib.check(L.mrt_render_frame_async(s.handle, C.byref(camc), C.byref(o), f.data_ptr(), f8.data_ptr(),
                                                st.cuda_stream), "render")
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for _ in range(2):
        run(20, 1, 1); run(20, 2, 2)
    for rep in range(3):
        print("1 stream 1 scene  %.4f ms/frame" % run(60, 1, 1))
        print("1 stream 2 scenes %.4f ms/frame" % run(60, 1, 2))
        print("2 streams 2 scenes %.4f ms/frame" % run(60, 2, 2), flush=True)


if __name__ == "__main__":
    main()
