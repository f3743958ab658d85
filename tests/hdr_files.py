"""Radiance .hdr writer for the loader tests (test infrastructure).

Encodes float RGB as RGBE bytes and writes them in the three scanline layouts
HDRLoader::load reads (reference src/hdrloader.cpp:118-190): flat, old-style
(1,1,1,n) repeat runs, and new-style per-channel run-length coding.  `decode`
is the independent expectation for the reference's convertComponent
((v / 256) * 2^(e - 128), every exponent byte, e = 0 included)."""
import numpy as np

HEADER = b"#?RADIANCE\n# written by tests/hdr_files.py\nFORMAT=32-bit_rle_rgbe\n\n"


def to_rgbe(rgb):
    """float (H, W, 3) -> uint8 (H, W, 4), the usual frexp encoding."""
    rgb = np.asarray(rgb, np.float64)
    m = rgb.max(axis=-1)
    out = np.zeros(rgb.shape[:-1] + (4,), np.uint8)
    nz = m > 1e-32
    mant, ex = np.frexp(m[nz])
    scale = mant * 256.0 / m[nz]
    out[nz, :3] = np.clip(np.floor(rgb[nz] * scale[:, None]), 0, 255).astype(np.uint8)
    out[nz, 3] = np.clip(ex + 128, 0, 255).astype(np.uint8)
    return out


def decode(rgbe):
    e = rgbe[..., 3].astype(np.int32) - 128
    scale = np.ldexp(np.float32(1.0), e).astype(np.float32)
    return (rgbe[..., :3].astype(np.float32) / np.float32(256.0)) * scale[..., None]


def _rle_channel(vals):
    out = bytearray()
    i, n = 0, len(vals)
    while i < n:
        run = 1
        while i + run < n and run < 127 and vals[i + run] == vals[i]:
            run += 1
        if run >= 3:
            out += bytes([128 + run, vals[i]])
            i += run
            continue
        lit = []
        j = i
        while j < n and len(lit) < 128:
            if j + 2 < n and vals[j] == vals[j + 1] == vals[j + 2]:
                break
            lit.append(vals[j])
            j += 1
        out += bytes([len(lit)]) + bytes(lit)
        i = j
    return bytes(out)


def _old_runs(row):
    W = len(row)
    buf = bytearray()
    x = 0
    while x < W:
        px = bytes(row[x])
        buf += px
        x += 1
        run = 0
        while x + run < W and run < 255 and bytes(row[x + run]) == px:
            run += 1
        if run >= 2:
            buf += bytes([1, 1, 1, run])
            x += run
    return bytes(buf)


def write_hdr(path, rgbe, mode="rle", header=HEADER):
    """mode: "rle" (new style, 8 <= W < 32768), "flat" or "oldrle"."""
    H, W = rgbe.shape[:2]
    with open(path, "wb") as f:
        f.write(header)
        f.write(b"-Y %d +X %d\n" % (H, W))
        for y in range(H):
            row = rgbe[y]
            if mode == "flat":
                f.write(row.tobytes())
            elif mode == "oldrle":
                f.write(_old_runs(row))
            else:
                f.write(bytes([2, 2, W >> 8, W & 255]))
                for ch in range(4):
                    f.write(_rle_channel(row[:, ch].tolist()))


def rgbe_pattern(H, W, seed):
    """RGBE test pattern with long runs, bright and dim texels, and no pixel the
    old-style reader would take for a run marker or a new-style line start."""
    rng = np.random.default_rng(seed)
    rgb = rng.gamma(1.0, 1.0, (H, W, 3)) * rng.choice([0.01, 1.0, 50.0], (H, W, 1))
    rgb[:, W // 3:W // 2] = rgb[:, W // 3:W // 3 + 1]
    e = to_rgbe(rgb)
    marker = (e[..., 0] == 1) & (e[..., 1] == 1) & (e[..., 2] == 1)
    e[marker, 0] = 3
    e[..., 0][e[..., 0] == 2] = 3
    return e
