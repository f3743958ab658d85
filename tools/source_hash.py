"""SHA-256 (first 16 hex digits) of the sources libmrt.so is built from: the
device and host code under rendering-algorithms-raytracer_amd/csrc, the C-ABI
header and the Makefile.  The Makefile embeds it in the library as
`mrt_source_hash`; build(), smoke() and bench.py compare it with the sources
beside the library, so a stale prebuilt libmrt.so is reported, not used
silently."""
import glob
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def files():
    pkg = os.path.join(ROOT, "rendering-algorithms-raytracer_amd")
    fs = sorted(glob.glob(os.path.join(pkg, "csrc", "*")))
    fs = [f for f in fs if os.path.isfile(f) and f.rsplit(".", 1)[-1] in ("hip", "h", "cpp", "inc")]
    return fs + [os.path.join(ROOT, "include", "mrt.h"), os.path.join(pkg, "Makefile")]


def source_hash():
    h = hashlib.sha256()
    for f in files():
        h.update(os.path.relpath(f, ROOT).encode())
        h.update(b"\0")
        h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_hash() + "\n")
