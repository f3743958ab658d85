"""Per-kernel resources of a built HIP object (VGPR / SGPR / LDS / scratch per
lane / spills), read from the gfx950 code object's metadata notes:

    python3 tools/kmeta.py rendering-algorithms-raytracer_amd/lib/build/mrt_device.o [regex]

No GPU needed (the same numbers rocprofv3's kernel trace reports per dispatch)."""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def kernels(obj):
    with tempfile.TemporaryDirectory() as t:
        fat, co = os.path.join(t, "fat.bin"), os.path.join(t, "dev.co")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", obj], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{B}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    rows, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s+- \.agpr_count:", line)
        if m:
            cur = {}
            rows.append(cur)
        m = re.match(r"\s+\.(\w+):\s+(\S+)", line)
        if m and cur is not None:
            cur.setdefault(m.group(1), m.group(2))
    return rows


def main():
    obj = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    for r in kernels(obj):
        name = r.get("name", "?")
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if pat and not (re.search(pat, name) or pat in dm):
            continue
        dm = dm.replace("mrt::", "").replace("(RenderParams)", "").replace("void ", "")
        print("%-60s vgpr %4s sgpr %4s lds %6s scratch %5s vspill %4s" % (
            dm[:60], r.get("vgpr_count"), r.get("sgpr_count"), r.get("group_segment_fixed_size"),
            r.get("private_segment_fixed_size"), r.get("vgpr_spill_count")))


if __name__ == "__main__":
    main()
