"""Texture maps and alpha-mapped any-hit (reference src/RawImage.cpp:16-188,
src/Texture.cpp:12-125, src/TriangleMeshLoad.cpp:99-214, src/TriangleMesh.cpp:105-148,
src/Ray.cpp:33-47, src/Lambert.cpp:32-36, src/Blinn.cpp:114-142,
src/BVH.cpp:1397-1445).

Inputs are the reference's own assets: Textures/Tree_03_Leaves.tga (the
Assignment 3 leaf colour + alpha map, src/Assignment3.h:59-72, committed as
assets/Tree_03_Leaves.tga) and Models/leaf_test.obj (tests/golden/).

CPU tests pin the loaders three ways (libmrt's host loader, the oracle and an
independent numpy decode of the file bytes following RawImage::loadTGA /
loadPPM must agree bit for bit) and the oracle's alpha test by properties of
the reference code (an opaque map equals no map; a transparent map removes the
triangles from every ray, shadow rays included; every primary hit on a leaf has
alpha >= 0.5 at its texture coordinates).  GPU tests compare the HIP path with
the oracle bit for bit: colour / normal / specular / reflect maps (direct and
chain engine), alpha-mapped leaves (primary, shadow and secondary rays, batched
ray queries) and the OBJ texture-coordinate path."""
import os

import numpy as np
import pytest

import miro
import oracle as O
from helpers import ROOT, bits, camera, fixture_mesh, scene_pair
from miro import scenes

LEAF_TGA = os.path.join(ROOT, "assets", "Tree_03_Leaves.tga")
LEAF_OBJ = os.path.join(ROOT, "tests", "golden", "leaf_test.obj")
CAM = dict(eye=(2.75, 2.75, 5.0), lookAt=(2.75, 2.75, 0.0), up=(0, 1, 0), fov=55.0)


# ------------------------------------------------------------------ loaders
def numpy_tga(path):
    """RawImage::loadTGA from the bytes: 18-byte header, rows flipped, colour
    through Image::gamma_to_linear / 32768, alpha / 255, B <-> R."""
    raw = np.fromfile(path, np.uint8)
    w, h, depth = int(raw[12]) | int(raw[13]) << 8, int(raw[14]) | int(raw[15]) << 8, int(raw[16])
    mode = depth // 8
    img = raw[18:18 + w * h * mode].reshape(h, w, mode)[::-1]
    g2l = np.array([int(float(np.power(np.float32(i) / np.float32(255.0), np.float32(2.2))) * 32768.0 + 0.5)
                    for i in range(256)], np.uint16)
    out = (g2l[img].astype(np.float32) / np.float32(32768.0)).astype(np.float32)
    if mode == 4:
        out[..., 3] = img[..., 3].astype(np.float32) / np.float32(255.0)
    if mode >= 3:
        out[..., [0, 2]] = out[..., [2, 0]]
    return out


def test_tga_loader_matches_the_oracle_and_a_numpy_decode():
    img = miro.RawImage()
    img.loadImage(LEAF_TGA)
    ref, typ = O.image_load(LEAF_TGA)
    assert typ == miro.TEX_RGBA == img.m_imageType and img.m_rawData.shape == (512, 512, 4)
    assert np.array_equal(bits(img.m_rawData), bits(ref))
    npy = numpy_tga(LEAF_TGA)
    assert np.array_equal(bits(npy), bits(ref))
    a = ref[..., 3]
    assert (a == 0).mean() > 0.1 and (a == 1).mean() > 0.1   # a real cut-out map


def test_ppm_loader_skips_comments_and_scales_bytes(tmp_path):
    rng = np.random.default_rng(3)
    pix = rng.integers(0, 256, (7, 5, 3), dtype=np.uint8)
    p = tmp_path / "t.ppm"
    p.write_bytes(b"P6\n# made by a test\n5 7\n# max\n255\n" + pix.tobytes())
    img = miro.RawImage()
    img.loadImage(str(p))
    ref, typ = O.image_load(str(p))
    assert typ == miro.TEX_RGB
    want = (pix.astype(np.float32) / np.float32(255)).astype(np.float32)
    assert np.array_equal(bits(img.m_rawData), bits(want))
    assert np.array_equal(bits(ref), bits(want))


def test_unsupported_images_fail_loudly(tmp_path):
    p = tmp_path / "rle.tga"
    hdr = bytearray(18)
    hdr[2] = 10          # RLE true colour: RawImage::loadTGA accepts types 2 / 3 only
    hdr[12:14] = (4, 0); hdr[14:16] = (4, 0); hdr[16] = 24
    p.write_bytes(bytes(hdr) + bytes(48))
    with pytest.raises(miro.MRTError):
        miro.RawImage().loadImage(str(p))
    with pytest.raises(RuntimeError):
        O.image_load(str(p))


def test_obj_texture_coordinates_load_like_the_oracle():
    lines = [l.split() for l in open(LEAF_OBJ) if l.startswith("vt ")]
    vt = np.array([(float(a[1]), float(a[2])) for a in lines], np.float32)
    P, Osc, _ = scene_pair(dict(scenes.CONFIGS["C1"], material=dict(kind="blinn", kd=(1, 1, 1))),
                           meshes=[fixture_mesh("cornell_box")], extra=[(LEAF_OBJ, dict(kind="blinn", kd=(1, 1, 1)))])
    L = miro.lib()
    import ctypes as C
    n = C.c_int32()
    assert L.mrt_scene_mesh_texcoords(P.handle, 1, C.byref(n), None, None) == 0
    uv = np.zeros((n.value, 2), np.float32)
    ti = np.zeros((2, 3), np.uint32)
    L.mrt_scene_mesh_texcoords(P.handle, 1, C.byref(n), uv.ctypes.data_as(C.POINTER(C.c_float)),
                               ti.ctypes.data_as(C.POINTER(C.c_uint32)))
    ouv, oti = Osc.texcoords(1)
    assert np.array_equal(bits(uv), bits(vt)) and np.array_equal(bits(ouv), bits(vt))
    assert np.array_equal(ti, oti) and ti.max() < len(vt)


# ------------------------------------------------------------------ scenes
def leaf_quads(n=6, seed=5):
    """n textured quads (two triangles each, uv over the whole map) floating in
    the Cornell box, facing the camera at seeded offsets and tilts."""
    rng = np.random.default_rng(seed)
    V, N, F, T, UV = [], [], [], [], []
    for q in range(n):
        c = np.array([rng.uniform(1.0, 4.5), rng.uniform(1.0, 4.5), rng.uniform(-4.5, -1.0)], np.float32)
        s = np.float32(rng.uniform(0.6, 1.3))
        tilt = rng.uniform(-0.5, 0.5)
        ex = np.array([np.cos(tilt), 0, np.sin(tilt)], np.float32) * s
        ey = np.array([0, 1, 0], np.float32) * s
        nrm = np.cross(ex, ey); nrm /= np.linalg.norm(nrm)
        b = len(V)
        V += [c - ex - ey, c + ex - ey, c + ex + ey, c - ex + ey]
        N += [nrm] * 4
        UV += [(0, 0), (1, 0), (1, 1), (0, 1)]
        F += [(b, b + 1, b + 2), (b, b + 2, b + 3)]
    V, N, UV = np.array(V, np.float32), np.array(N, np.float32), np.array(UV, np.float32)
    F = np.array(F, np.uint32)
    return V, N, F, F.copy(), UV, F.copy()


def leaf_image():
    return O.image_load(LEAF_TGA)


def wall_uv(arrs, scale_=5.5):
    """planar texture coordinates for the Cornell mesh (x, y) / 5.5 + z / 11"""
    v = arrs[0]
    uv = np.stack([v[:, 0] / scale_ + v[:, 2] / (2 * scale_), v[:, 1] / scale_], 1).astype(np.float32)
    return tuple(arrs) + (uv, arrs[2].copy())


def leaves_scene(alpha=True, lights=None, leaf_mat=None, **kw):
    img, typ = leaf_image()
    maps = dict(color=(img, typ))
    if alpha:
        maps["alpha"] = (img, typ)
    mat = dict(kind="blinn", kd=(1, 1, 1), translucency=0.4, maps=maps, **(leaf_mat or {}))
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.8, 0.8, 0.8)))
    return scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], lights=lights, extra=[(leaf_quads(), mat)], **kw)


def synthetic_maps(seed=9, W=64, H=48):
    rng = np.random.default_rng(seed)
    color = rng.uniform(0.1, 0.9, (H, W, 3)).astype(np.float32)
    normal = np.concatenate([rng.uniform(-0.3, 0.3, (H, W, 2)), rng.uniform(0.8, 1.0, (H, W, 1))], 2).astype(np.float32)
    spec = rng.uniform(0.0, 1.0, (H, W)).astype(np.float32)
    refl = rng.uniform(0.2, 1.0, (H, W, 3)).astype(np.float32)
    return dict(color=(color, miro.TEX_RGB), normal=(normal, miro.TEX_RGB), specular=(spec, miro.TEX_GRAY),
                reflect=(refl, miro.TEX_RGB))


# ------------------------------------------------------------------ oracle properties
def test_opaque_alpha_map_equals_no_alpha_map():
    img, typ = leaf_image()
    opaque = img.copy(); opaque[..., 3] = 1.0
    _, Oa, cam = leaves_scene(alpha=False)
    mat = dict(kind="blinn", kd=(1, 1, 1), translucency=0.4, maps=dict(color=(img, typ), alpha=(opaque, typ)))
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.8, 0.8, 0.8)))
    _, Ob, _ = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], extra=[(leaf_quads(), mat)])
    a, b = Oa.render(CAM, 48, 40, threads=4), Ob.render(CAM, 48, 40, threads=4)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"])) and np.array_equal(a["hits"]["prim"], b["hits"]["prim"])


def test_transparent_alpha_map_removes_the_leaves_from_every_ray():
    img, typ = leaf_image()
    clear = img.copy(); clear[..., 3] = 0.0
    mat = dict(kind="blinn", kd=(1, 1, 1), maps=dict(color=(img, typ), alpha=(clear, typ)))
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.8, 0.8, 0.8)))
    _, Oc, _ = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], extra=[(leaf_quads(), mat)])
    _, Onone, _ = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")])
    a, b = Oc.render(CAM, 48, 40, threads=4), Onone.render(CAM, 48, 40, threads=4)
    assert np.array_equal(bits(a["rgb"]), bits(b["rgb"]))          # no leaf pixels, no leaf shadows
    assert np.array_equal(a["hits"]["prim"], b["hits"]["prim"])


def test_leaf_hits_lie_on_opaque_texels():
    _, Osc, _ = leaves_scene()
    r = Osc.render(CAM, 64, 48, threads=4)
    prim = r["hits"]["prim"]
    on = prim >= 36                                              # the 36 Cornell triangles come first
    assert on.mean() > 0.02
    img, _ = leaf_image()
    H, W = img.shape[:2]
    quads_uv = np.array([[(0, 0), (1, 0), (1, 1)], [(0, 0), (1, 1), (0, 1)]], np.float32)
    a, b = r["hits"]["a"][on], r["hits"]["b"][on]
    tri = (prim[on] - 36) % 2
    t = quads_uv[tri]
    c = 1 - a - b
    u = t[:, 0, 0] * c + t[:, 1, 0] * a + t[:, 2, 0] * b
    v = t[:, 0, 1] * c + t[:, 1, 1] * a + t[:, 2, 1] * b
    # bilinear alpha (Texture::getLookupAlpha) in float64: >= 0.5 up to rounding
    py, px = (1 - v) * H, u * W
    x1, y1 = np.floor(px).astype(int), np.floor(py).astype(int)
    dx, dy = px - x1, py - y1
    A = img[..., 3]
    g = lambda x, y: A[y % H, x % W]
    alpha = ((g(x1, y1) * (1 - dx) + g(x1 + 1, y1) * dx) * (1 - dy) + (g(x1, y1 + 1) * (1 - dx) + g(x1 + 1, y1 + 1) * dx) * dy)
    assert (alpha >= 0.5 - 1e-5).all()


# ------------------------------------------------------------------ GPU parity
def need_gpu():
    if miro.device_count() < 1:
        pytest.fail("no HIP device visible (GPU tests must run on the MI355X box)")


def gpu_vs_oracle(P, Osc, cam, W, H):
    img = miro.Image()
    img.resize(W, H)
    hits = P.raytraceImage(camera(cam), img, want_hits=True)
    ref = Osc.render(cam, W, H, threads=8)
    assert np.array_equal(hits["prim"], ref["hits"]["prim"]), "primary hit ids differ"
    hit = ref["hits"]["prim"] >= 0
    assert np.array_equal(bits(hits["t"][hit]), bits(ref["hits"]["t"][hit]))
    assert np.array_equal(bits(img.rgb), bits(ref["rgb"])), "float RGB differs"
    assert np.array_equal(img.pixels, ref["rgb8"])
    assert P.last_stats["shadow_rays"] == ref["shadow_rays"]
    assert P.last_stats["secondary_rays"] == ref["secondary_rays"]
    return ref


@pytest.mark.gpu
def test_alpha_mapped_leaves_match_oracle():
    need_gpu()
    P, Osc, _ = leaves_scene()
    ref = gpu_vs_oracle(P, Osc, CAM, 96, 72)
    assert (ref["hits"]["prim"] >= 36).mean() > 0.02
    rect = dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0, samples=3,
                noise=0.001)
    P, Osc, _ = leaves_scene(lights=[rect, dict(type="point", pos=(2.75, 2.0, -0.5), power=10.0)], num_paths=2)
    gpu_vs_oracle(P, Osc, CAM, 64, 48)


@pytest.mark.gpu
def test_alpha_leaves_under_reflection_chain_and_ray_queries():
    need_gpu()
    P, Osc, _ = leaves_scene(leaf_mat=dict(reflectAmt=0.5, refractAmt=0.3, ior=1.3))
    ref = gpu_vs_oracle(P, Osc, CAM, 64, 48)
    assert ref["secondary_rays"] > 0
    rng = np.random.default_rng(4)
    n = 4000
    o = np.tile(np.array([[2.75, 2.75, 4.5]], np.float32), (n, 1)) + rng.normal(0, 0.2, (n, 3)).astype(np.float32)
    d = (np.array([2.75, 2.75, -4.0], np.float32) + rng.normal(0, 1.5, (n, 3)).astype(np.float32) - o)
    got = P.traceBatch(o, d, 0.001, 1e12)
    want, _, _ = Osc.trace(o, d, 0.001, 1e12)
    assert np.array_equal(got["prim"], want["prim"])
    hit = want["prim"] >= 0
    assert np.array_equal(bits(got["t"][hit]), bits(want["t"][hit]))
    tm = rng.uniform(0.5, 9.0, n).astype(np.float32)
    occ = P.traceBatch(o, d, 0.001, tm, any_hit=True)
    assert np.array_equal(occ["prim"] >= 0, hit & (want["t"] < tm))


@pytest.mark.gpu
def test_colour_normal_specular_reflect_maps_match_oracle():
    need_gpu()
    maps = synthetic_maps()
    walls = wall_uv(fixture_mesh("cornell_box"))
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.7, 0.7, 0.7), maps=dict(color=maps["color"])))
    blinn = dict(kind="blinn", kd=(0.5, 0.5, 0.5), specExp=12.0, specAmt=0.6, maps=maps)
    # direct lighting (Lambert colour map on the box, Blinn maps on the leaves' quads)
    quads = leaf_quads(4, seed=11)
    P, Osc, _ = scene_pair(cfg, extra=[(walls, cfg["material"]), (quads, blinn)])
    gpu_vs_oracle(P, Osc, CAM, 64, 48)
    # with reflection (chain engine; the reflect map scales localReflectAmt)
    P, Osc, _ = scene_pair(cfg, extra=[(walls, cfg["material"]), (quads, dict(blinn, reflectAmt=1.0, ior=3.0))])
    ref = gpu_vs_oracle(P, Osc, CAM, 64, 48)
    assert ref["secondary_rays"] > 0


@pytest.mark.gpu
def test_obj_leaf_with_alpha_map_matches_oracle():
    need_gpu()
    img, typ = leaf_image()
    leaf = dict(kind="blinn", kd=(1, 1, 1), maps=dict(color=(img, typ), alpha=(img, typ)))
    cfg = dict(scenes.CONFIGS["C1"], material=dict(kind="lambert", kd=(0.8, 0.8, 0.8)))
    P, Osc, _ = scene_pair(cfg, meshes=[fixture_mesh("cornell_box")], extra=[(LEAF_OBJ, leaf)])
    cam = dict(eye=(0.0, 3.0, 0.5), lookAt=(0.0, 0.0, 0.0), up=(0, 0, -1), fov=60.0)
    ref = gpu_vs_oracle(P, Osc, cam, 64, 64)
    assert ((ref["hits"]["prim"] >= 36) & (ref["hits"]["prim"] < 38)).any()


@pytest.mark.gpu
def test_alpha_leaves_shadow_schedules_give_identical_frames():
    """The lane-refill any-hit step of special-leaf scenes (anyhit_step_inst)
    applies the alpha test like the traversal of the other schedules."""
    from test_gpu_parity import shadow_schedules
    lights = [dict(type="rect", v1=(3.0, 5.4, -2.5), v2=(3.0, 5.4, -3.0), v3=(2.5, 5.4, -2.5), power=15.0,
                   samples=4, noise=0.001)]
    P, _, cam = leaves_scene(lights=lights)
    shadow_schedules(P, cam, 64, 48)


# ------------------------------------------------------------------ alpha inside instances
def leaf_instances(alpha_img, lights=None):
    """The leaf OBJ as a ProxyObject BLAS with an alpha-mapped material, six
    overlapping instances at three heights (the reference's tree proxies carry
    alpha-mapped leaves inside their BLAS, src/main.cpp:240-274)."""
    img, typ = leaf_image()
    leaf = dict(kind="blinn", kd=(1, 1, 1), translucency=0.4, specExp=8.0, specAmt=0.3,
                maps=dict(color=(img, typ), alpha=(alpha_img, typ)))
    cfg = dict(scenes.CONFIGS["C1"], material=leaf)
    placed = []
    for i in range(6):
        a = 0.9 * i
        c, s = np.cos(a), np.sin(a)
        sc = 0.55 + 0.05 * i
        placed.append((0, np.array([[c * sc, 0, s * sc, 0.45 * np.cos(2.1 * i)], [0, sc, 0, 0.25 * (i % 3)],
                                    [-s * sc, 0, c * sc, 0.45 * np.sin(2.1 * i)], [0, 0, 0, 1]], np.float32)))
    lights = lights or [dict(type="point", pos=(0.5, 4.0, 0.5), power=30.0),
                        dict(type="rect", v1=(-0.5, 3.0, -0.5), v2=(0.5, 3.0, -0.5), v3=(-0.5, 3.0, 0.5), power=20.0,
                             samples=3, noise=0.001)]
    return scene_pair(cfg, instances=([LEAF_OBJ], placed), lights=lights)


LEAF_CAM = dict(eye=(0.0, 3.0, 0.5), lookAt=(0.0, 0.0, 0.0), up=(0, 0, -1), fov=60.0)


def test_transparent_alpha_removes_instanced_leaves():
    img, _ = leaf_image()
    clear = img.copy(); clear[..., 3] = 0.0
    _, Oc, _ = leaf_instances(clear)
    r = Oc.render(LEAF_CAM, 40, 40, threads=4)
    assert (r["hits"]["prim"] < 0).all()
    _, Oo, _ = leaf_instances(img)
    assert (Oo.render(LEAF_CAM, 40, 40, threads=4)["hits"]["prim"] >= 0).mean() > 0.05


def test_opaque_alpha_on_instanced_leaves_hits_every_quad_pixel():
    """An opaque map keeps every instanced quad; the real map cuts holes through
    which some rays reach a lower leaf or nothing."""
    img, _ = leaf_image()
    opaque = img.copy(); opaque[..., 3] = 1.0
    _, Oo, _ = leaf_instances(opaque)
    _, Oa, _ = leaf_instances(img)
    a, b = Oo.render(LEAF_CAM, 48, 48, threads=4), Oa.render(LEAF_CAM, 48, 48, threads=4)
    ha, hb = a["hits"]["prim"] >= 0, b["hits"]["prim"] >= 0
    assert (hb <= ha).all() and hb.sum() < ha.sum()
    assert not np.array_equal(a["hits"]["t"][hb], b["hits"]["t"][hb])   # some rays pass a hole to a lower leaf


@pytest.mark.gpu
def test_alpha_leaves_inside_instances_match_oracle():
    need_gpu()
    img, _ = leaf_image()
    P, Osc, _ = leaf_instances(img)
    ref = gpu_vs_oracle(P, Osc, LEAF_CAM, 64, 64)
    assert (ref["hits"]["prim"] >= 0).mean() > 0.05


@pytest.mark.gpu
def test_alpha_leaves_inside_instances_shadow_schedules_give_identical_frames():
    from test_gpu_parity import shadow_schedules
    img, _ = leaf_image()
    P, _, _ = leaf_instances(img)
    shadow_schedules(P, LEAF_CAM, 48, 48)
