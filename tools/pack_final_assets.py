"""Pack the input data of the reference's final scene (makeFinalScene,
/root/reference/src/main.cpp:132-670) that the snapshot holds into
assets/final/ as xz-compressed copies, with a manifest (size and sha256 of each
original).  Data only -- models, textures, light probes; no reference source.
Run here (the reference tree is not on the GPU box); miro/scenes.py unpacks the
files into the scene cache on first use.

Missing from the snapshot (/root/reference/.MISSING_LARGE_BLOBS) and generated as
stand-ins by scenes.py instead: Models/Final/tree01Body.obj, tree01Leaves.obj,
tree02Body.obj, tree03Body.obj, tree04Body.obj, tree04Leaves.obj,
Models/testGrass2.obj and Textures/hdrvfx_nyany_1_n2_v101_Bg.tga (the
environment map; its companion hdrvfx_nyany_1_n2_v101_Ref.hdr, which the
snapshot holds, stands in for it).

    python3 tools/pack_final_assets.py [/root/reference]
"""
import hashlib
import json
import lzma
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "assets", "final")

FILES = [
    # geometry (Models/Final): MBObject pairs, the ground, tree leaves, flowers
    "Models/Final/explosion01.obj", "Models/Final/explosion02.obj",
    "Models/Final/cannonBallT1.obj", "Models/Final/cannonBallT2.obj",
    "Models/Final/groundPlane.obj", "Models/Final/tree02Leaves.obj", "Models/Final/tree03Leaves.obj",
    "Models/Final/flower01BigLeaves.obj", "Models/Final/flower01Body.obj", "Models/Final/flower01Bulbs01.obj",
    "Models/Final/flower01Bulbs02.obj", "Models/Final/flower01Bulbs03.obj", "Models/Final/flower01Petals.obj",
    "Models/Final/flower01Pistils.obj", "Models/Final/flower01SmallLeaves.obj",
    "Models/Final/flower02Body.obj", "Models/Final/flower02Bulb.obj", "Models/Final/flower02Leaves.obj",
    "Models/Final/flower02Petals.obj",
    # textures (colour, alpha and normal maps)
    "Textures/grassblade2.tga", "Textures/ground-dirt-texture.tga", "Textures/bw2.tga",
    "Textures/AL04brk.tga", "Textures/AL04aut.tga", "Textures/ML16lef1.tga", "Textures/ML16brk.tga",
    "Textures/AL17brk.tga", "Textures/AL17aut.tga", "Textures/grass-color-23.tga", "Textures/bud-yellow-1.tga",
    "Textures/bud-yellow-1-bump_NRM.tga", "Textures/grass-color-18.tga", "Textures/petal-pink-02.tga",
    "Textures/petal-yellow-1.tga", "Textures/petal-white-3.tga", "Textures/FL30lef1.tga", "Textures/FL30stm1.tga",
    "Textures/FL30flo1.tga", "Textures/FL30pet1.tga", "Textures/FL30stm2.tga", "Textures/FL30lef2.tga",
    # light probes: the dome light's sky, and the stand-in for the missing environment map
    "Images/sky.hdr", "Textures/hdrvfx_nyany_1_n2_v101_Ref.hdr",
]


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    os.makedirs(OUT, exist_ok=True)
    manifest = {}
    for rel in FILES:
        data = open(os.path.join(ref, rel), "rb").read()
        name = os.path.basename(rel)
        with open(os.path.join(OUT, name + ".xz"), "wb") as f:
            f.write(lzma.compress(data, preset=9 | lzma.PRESET_EXTREME))
        manifest[name] = {"source": rel, "bytes": len(data), "sha256": hashlib.sha256(data).hexdigest()}
    json.dump(manifest, open(os.path.join(OUT, "manifest.json"), "w"), indent=1, sort_keys=True)
    print(f"{len(manifest)} files -> {OUT}")


if __name__ == "__main__":
    main()
