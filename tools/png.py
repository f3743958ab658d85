"""Minimal PNG writer (stdlib only) for eyeballing renders."""
import struct
import zlib

import numpy as np


def write_png(path, rgb8):
    """rgb8: (H, W, 3) uint8 with row 0 = TOP."""
    h, w, _ = rgb8.shape
    raw = b"".join(b"\x00" + rgb8[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    data += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(data)


def write_frame(path, rgb8_bottom_up):
    """Frame with row 0 = bottom (reference Image convention, src/Image.cpp:137-154)."""
    write_png(path, np.ascontiguousarray(rgb8_bottom_up[::-1]))
