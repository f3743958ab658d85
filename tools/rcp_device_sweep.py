"""The device's rcp_nr (RCPSS emulation + the Newton step, csrc/mrt_math.h, run through
mrt_debug_libm fn 2) against an independent numpy restatement of RCPSS on every float bit
pattern (2^32 inputs, in 16 chunks of 2^28).  The restatement reads the captured table
(csrc/x86_approx_tables.inc, full 32-bit entries) and applies the exponent rule directly:

    normal x (exponent e in 1..252): sign | (253 - e) << 23 | the entry's mantissa bits
    e >= 253 or +-inf: +-0;  zero / denormal: +-inf;  NaN: the input, quieted

then rcp_nr = (2r) - (x (r r)) in float32 (src/SSE.h:67-86; numpy float32 arithmetic is
IEEE single, no FMA).  NaN outputs are compared as NaN (payloads are not).  Needs a GPU:

    python tools/rcp_device_sweep.py > profiles/<round>_rcp_device_sweep.txt"""
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rendering-algorithms-raytracer_amd"))
import miro  # noqa: E402


def rcp_table():
    src = open(os.path.join(ROOT, "rendering-algorithms-raytracer_amd", "csrc", "x86_approx_tables.inc")).read()
    body = src[src.index("MRT_RCP_TABLE[2048]"):src.index("MRT_RSQRT_TABLE")]
    vals = [int(v, 16) for v in re.findall(r"0x([0-9a-fA-F]+)u", body)]
    assert len(vals) == 2048
    return np.array(vals, np.uint32)


def reference(u, T):
    a = u & np.uint32(0x7FFFFFFF)
    s = u & np.uint32(0x80000000)
    e = (a >> np.uint32(23)).astype(np.int64)
    t = T[(a >> np.uint32(12)) & np.uint32(0x7FF)]
    normal = s | (((253 - e) & 0xFF).astype(np.uint32) << np.uint32(23)) | (t & np.uint32(0x7FFFFF))
    r = np.where((e >= 1) & (e <= 252), normal, np.uint32(0))
    r = np.where(e >= 253, s, r)
    r = np.where(e == 0, s | np.uint32(0x7F800000), r)
    r = np.where(a > np.uint32(0x7F800000), u | np.uint32(0x00400000), r)
    x = u.view(np.float32)
    rf = r.view(np.float32)
    with np.errstate(all="ignore"):
        return (np.float32(2.0) * rf) - (x * (rf * rf))


def main():
    if miro.device_count() < 1:
        print("no HIP device")
        return 2
    T = rcp_table()
    chunk = 1 << 28
    total = bad = 0
    t0 = time.time()
    for c in range(1 << 32 >> 28):
        u = np.arange(c * chunk, (c + 1) * chunk, dtype=np.uint64).astype(np.uint32)
        got = miro.debug_libm("rcp_nr", u.view(np.float32))
        ref = reference(u, T)
        same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
        nb = int((~same).sum())
        if nb:
            i = int(np.flatnonzero(~same)[0])
            print(f"chunk {c}: {nb} mismatches, first input 0x{int(u[i]):08x}: device 0x{int(got.view(np.uint32)[i]):08x} "
                  f"reference 0x{int(ref.view(np.uint32)[i]):08x}", flush=True)
        bad += nb
        total += len(u)
        print(f"chunk {c:2d} done ({total} inputs, {bad} mismatches, {time.time() - t0:.0f} s)", flush=True)
    print(f"checked {total} mismatches {bad}")
    return 0 if bad == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
