"""ctypes wrapper for the CPU oracle (oracle/_build/libmrt_oracle.so).

TEST INFRASTRUCTURE ONLY.  Importable only from tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg.  The oracle is the checker, never the product.
PARITY UNPINNED against reference outputs (see mrt_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmrt_oracle.so")
_lib = None


# libm convention of the oracle's restated sin / cos / pow calls (oro_set_libm, oro_ibl.h):
#   "float"  -- the float overloads the reference's source resolves to under g++
#               (sin(acosf(x)) -> sinf, pow(float, float) -> powf, cos/sin of floats ->
#               cosf/sinf; src/Material.h:51, src/Blinn.cpp:219, src/Material.cpp:41), glibc
#               here: the reference's own calls;
#   "double" -- the same functions evaluated in double and rounded once (round 5's
#               device convention; tools/libm_parity.py measures how far it moves a
#               frame).
# atan2 / acos (src/Texture.cpp:82-93, the acosf of src/Material.h:51) are glibc's
# atan2f / acosf in both.  The HIP device restates all five glibc functions bit for
# bit (csrc/mrt_libm.h; since round 6 sinf / cosf / powf too), so it equals "float".
LIBM_FLOAT, LIBM_DOUBLE = "float", "double"
_default_libm = LIBM_FLOAT


def set_default_libm(mode):
    """Convention for render / texture_lookup_dir calls that do not name one; returns the previous."""
    global _default_libm
    if mode not in (LIBM_FLOAT, LIBM_DOUBLE):
        raise ValueError(mode)
    prev, _default_libm = _default_libm, mode
    return prev


def _apply_libm(mode):
    mode = mode or _default_libm
    if mode not in (LIBM_FLOAT, LIBM_DOUBLE):
        raise ValueError(mode)
    lib().oro_set_libm(1 if mode == LIBM_FLOAT else 0)


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = C.CDLL(_LIB_PATH)
        _declare(_lib)
    return _lib


class Material(C.Structure):
    _fields_ = [("type", C.c_int), ("kd", C.c_float * 3), ("ka", C.c_float * 3), ("ks", C.c_float * 3),
                ("specExp", C.c_float), ("specAmt", C.c_float),
                ("reflect", C.c_float), ("refract", C.c_float), ("ior", C.c_float), ("gloss", C.c_float),
                ("translucency", C.c_float), ("le", C.c_float * 3), ("emitted", C.c_float), ("sample_env", C.c_int),
                ("disperse", C.c_int), ("ior3", C.c_float * 3)]


class Light(C.Structure):
    _fields_ = [("type", C.c_int), ("pos", C.c_float * 3), ("v1", C.c_float * 3), ("v2", C.c_float * 3),
                ("v3", C.c_float * 3), ("power", C.c_float), ("samples", C.c_int),
                ("noiseThreshold", C.c_float), ("castShadows", C.c_int), ("texture", C.c_int),
                ("transparent", C.c_int)]


class Camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("up", C.c_float * 3), ("lookAt", C.c_float * 3), ("fov", C.c_float),
                ("aperture", C.c_float), ("focusPlane", C.c_float), ("shutterSpeed", C.c_float)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("a", C.c_float), ("b", C.c_float), ("prim", C.c_int32)]


HIT_DTYPE = np.dtype([("t", "<f4"), ("a", "<f4"), ("b", "<f4"), ("prim", "<i4")])

_fp = C.POINTER(C.c_float)
_u32p = C.POINTER(C.c_uint32)
_i32p = C.POINTER(C.c_int32)
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)


def _declare(L):
    L.oro_scene_create.restype = C.c_void_p
    L.oro_scene_destroy.argtypes = [C.c_void_p]
    L.oro_scene_add_obj.argtypes = [C.c_void_p, C.c_char_p, _fp, C.c_int]
    L.oro_scene_add_mesh.argtypes = [C.c_void_p, C.c_int, _fp, C.c_int, _fp, C.c_int, _u32p, _u32p, C.c_int]
    L.oro_mesh_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.oro_mesh_export.argtypes = [C.c_void_p, C.c_int, _fp, _fp, _u32p, _u32p]
    L.oro_scene_add_material.argtypes = [C.c_void_p, C.POINTER(Material)]
    L.oro_scene_add_light.argtypes = [C.c_void_p, C.POINTER(Light)]
    L.oro_scene_set_bg.argtypes = [C.c_void_p, C.c_float, C.c_float, C.c_float]
    L.oro_scene_set_num_paths.argtypes = [C.c_void_p, C.c_int]
    L.oro_scene_set_path_trace.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
    L.oro_scene_set_subdivs.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_float]
    L.oro_scene_build.argtypes = [C.c_void_p]
    L.oro_qbvh_info.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 6
    L.oro_qbvh_export.argtypes = [C.c_void_p, _fp, _i32p, _fp, _i32p]
    L.oro_set_libm.argtypes = [C.c_int]
    L.oro_trace.argtypes = [C.c_void_p, C.c_size_t, _fp, _fp, _fp, _fp, C.c_void_p, _u32p, _u32p]
    L.oro_render.argtypes = [C.c_void_p, C.POINTER(Camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                             _fp, _u8p, C.c_void_p, _u32p, _u64p, C.c_int]
    for n in ("oro_x86_rcp", "oro_x86_rsqrt", "oro_rcp_nr", "oro_rsqrt_nr"):
        getattr(L, n).argtypes = [C.c_float]
        getattr(L, n).restype = C.c_float
    L.oro_gamma_table.argtypes = [_u8p]
    L.oro_rand.argtypes = [C.c_uint32] * 4
    L.oro_rand.restype = C.c_float
    L.oro_hdr_info.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.oro_hdr_load.argtypes = [C.c_char_p, _fp, C.c_int, C.c_int]
    L.oro_scene_add_texture.argtypes = [C.c_void_p, _fp, C.c_int, C.c_int]
    L.oro_image_info.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.oro_image_load.argtypes = [C.c_char_p, _fp, C.c_int, C.c_int]
    L.oro_scene_add_texture_typed.argtypes = [C.c_void_p, _fp, C.c_int, C.c_int, C.c_int]
    L.oro_scene_set_material_maps.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    L.oro_mesh_set_texcoords.argtypes = [C.c_void_p, C.c_int, C.c_int, _fp, _u32p]
    L.oro_mesh_texcoords.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), _fp, _u32p]
    L.oro_mesh_set_motion.argtypes = [C.c_void_p, C.c_int, _fp]
    L.oro_scene_set_env_map.argtypes = [C.c_void_p, C.c_int, C.c_float]
    L.oro_scene_set_material_env_map.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_float]
    L.oro_dome_info.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.oro_dome_export.argtypes = [C.c_void_p, C.c_int] + [_fp] * 9
    L.oro_texture_lookup_dir.argtypes = [C.c_void_p, C.c_int, C.c_int, _fp, _fp]
    L.oro_scene_make_blas.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    L.oro_scene_add_instance.argtypes = [C.c_void_p, C.c_int, _fp]
    L.oro_blas_info.argtypes = [C.c_void_p, C.c_int] + [C.POINTER(C.c_int)] * 3
    L.oro_blas_export.argtypes = [C.c_void_p, C.c_int, _fp, _i32p, _fp, _i32p]


DOME_KEYS = ("cdf_u", "func_u", "cdf_v", "func_v", "func_int", "cos_u", "sin_u", "cos_v", "sin_v")


def dome_shapes(nu, nv):
    return {"cdf_u": (nu + 1,), "func_u": (nu,), "cdf_v": (nu, nv + 1), "func_v": (nu, nv), "func_int": (nu + 1,),
            "cos_u": (nu + 1,), "sin_u": (nu + 1,), "cos_v": (nv + 1,), "sin_v": (nv + 1,)}


def hdr_load(path):
    """HDRLoader::load restated: (H, W, 3) float32, row 0 = top.  Raises on error."""
    L = lib()
    w, h = C.c_int(), C.c_int()
    r = L.oro_hdr_info(str(path).encode(), C.byref(w), C.byref(h))
    if r != 0:
        raise RuntimeError(f"oracle HDR header rejected ({r}): {path}")
    rgb = np.zeros((h.value, w.value, 3), np.float32)
    r = L.oro_hdr_load(str(path).encode(), _p(rgb, _fp), w.value, h.value)
    if r != 0:
        raise RuntimeError(f"oracle HDR load rejected ({r}): {path}")
    return rgb


TEX_CHANNELS = {0: 3, 1: 1, 3: 3, 4: 4}   # RawImage types: HDR, GRAYSCALE, RGB, RGBA


def image_load(path):
    """RawImage::loadImage restated (TGA / PPM / HDR): (data (H, W, channels) float32, type)."""
    L = lib()
    w, h, t = C.c_int(), C.c_int(), C.c_int()
    r = L.oro_image_info(str(path).encode(), C.byref(w), C.byref(h), C.byref(t))
    if r != 0:
        raise RuntimeError(f"oracle image header rejected ({r}): {path}")
    data = np.zeros((h.value, w.value, TEX_CHANNELS[t.value]), np.float32)
    r = L.oro_image_load(str(path).encode(), _p(data, _fp), w.value, h.value)
    if r != 0:
        raise RuntimeError(f"oracle image load rejected ({r}): {path}")
    return data, t.value


def _p(a, t):
    return a.ctypes.data_as(t)


def _v3(x):
    return (C.c_float * 3)(*[float(v) for v in x])


class OracleScene:
    """Scene builder mirroring the reference scene scripts (src/assignment2.h)."""

    def __init__(self):
        self.L = lib()
        self.h = self.L.oro_scene_create()
        self.n_lights = 0

    def __del__(self):
        try:
            if self.h:
                self.L.oro_scene_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def add_material(self, kind="lambert", kd=(1, 1, 1), ka=(0, 0, 0), ks=(1, 1, 1), specExp=1.0, specAmt=0.0,
                     reflectAmt=0.0, refractAmt=0.0, ior=1.5, specGloss=1.0, translucency=0.0, le=(0, 0, 0),
                     emitted=0.0, sampleEnv=True, disperse=False, ior3=None):
        """Lambert / Blinn (src/Blinn.h:11-22 defaults: ior 1.5, no reflection / refraction;
        setLightEmittedColor / setLightEmittedIntensity -> le / emitted; Material::setSampleEnv).
        ior is m_ior[1] (the non-dispersive refraction); disperse / ior3 = m_disperse and
        m_ior[0..2] (default: ior three times, as the Blinn constructor sets them)."""
        i3 = (ior, ior, ior) if ior3 is None else tuple(ior3)
        m = Material(0 if kind == "lambert" else 1, _v3(kd), _v3(ka), _v3(ks), specExp, specAmt,
                     reflectAmt, refractAmt, ior, specGloss, translucency, _v3(le), emitted, int(bool(sampleEnv)),
                     int(bool(disperse)), _v3(i3))
        return self.L.oro_scene_add_material(self.h, C.byref(m))

    def add_obj(self, path, material, ctm=None):
        ctm_p = None
        if ctm is not None:
            arr = np.ascontiguousarray(np.asarray(ctm, np.float32).reshape(16))
            ctm_p = _p(arr, _fp)
        r = self.L.oro_scene_add_obj(self.h, path.encode(), ctm_p, material)
        if r < 0:
            raise RuntimeError(f"oracle OBJ load failed ({r}): {path}")
        return r

    def add_mesh(self, verts, normals, vidx, nidx, material):
        v = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
        n = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
        vi = np.ascontiguousarray(vidx, np.uint32).reshape(-1, 3)
        ni = np.ascontiguousarray(nidx, np.uint32).reshape(-1, 3)
        r = self.L.oro_scene_add_mesh(self.h, len(v), _p(v, _fp), len(n), _p(n, _fp), len(vi),
                                      _p(vi, _u32p), _p(ni, _u32p), material)
        if r < 0:
            raise RuntimeError("oracle add_mesh failed")
        return r

    def mesh_arrays(self, mesh):
        nv, nn, nt = C.c_int(), C.c_int(), C.c_int()
        self.L.oro_mesh_info(self.h, mesh, C.byref(nv), C.byref(nn), C.byref(nt))
        v = np.zeros((nv.value, 3), np.float32)
        n = np.zeros((nn.value, 3), np.float32)
        vi = np.zeros((nt.value, 3), np.uint32)
        ni = np.zeros((nt.value, 3), np.uint32)
        self.L.oro_mesh_export(self.h, mesh, _p(v, _fp), _p(n, _fp), _p(vi, _u32p), _p(ni, _u32p))
        return v, n, vi, ni

    def add_point_light(self, pos, power, cast_shadows=True):
        l = Light()
        l.type = 0
        l.pos = _v3(pos)
        l.power = power
        l.samples = 1
        l.noiseThreshold = 0.001
        l.castShadows = int(cast_shadows)
        l.texture = -1
        self.n_lights += 1
        return self.L.oro_scene_add_light(self.h, C.byref(l))

    def add_rect_light(self, v1, v2, v3, power, samples=1, noise=0.001, cast_shadows=True, fast_shadows=True):
        """fast_shadows False: Light::setFastShadows(false), the transparency walk of
        src/RectangleLight.cpp:93-116."""
        l = Light()
        l.transparent = 0 if fast_shadows else 1
        l.type = 1
        l.v1, l.v2, l.v3 = _v3(v1), _v3(v2), _v3(v3)
        l.power = power
        l.samples = samples
        l.noiseThreshold = noise
        l.castShadows = int(cast_shadows)
        l.texture = -1
        self.n_lights += 1
        return self.L.oro_scene_add_light(self.h, C.byref(l))

    def add_texture_typed(self, data, type_):
        a = np.ascontiguousarray(data, np.float32)
        r = self.L.oro_scene_add_texture_typed(self.h, _p(a, _fp), a.shape[1], a.shape[0], int(type_))
        if r < 0:
            raise RuntimeError("oracle add_texture_typed failed")
        return r

    def set_material_maps(self, material, color=-1, normal=-1, specular=-1, reflect=-1, refract=-1, alpha=-1):
        m = (C.c_int * 6)(color, normal, specular, reflect, refract, alpha)
        if self.L.oro_scene_set_material_maps(self.h, material, m) != 0:
            raise RuntimeError("oracle set_material_maps failed")

    def set_texcoords(self, mesh, uv, tidx):
        uv = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
        ti = np.ascontiguousarray(tidx, np.uint32).reshape(-1, 3)
        if self.L.oro_mesh_set_texcoords(self.h, mesh, len(uv), _p(uv, _fp), _p(ti, _u32p)) != 0:
            raise RuntimeError("oracle set_texcoords failed")

    def set_motion(self, mesh, verts2):
        v = np.ascontiguousarray(verts2, np.float32).reshape(-1, 3)
        if self.L.oro_mesh_set_motion(self.h, mesh, _p(v, _fp)) != 0:
            raise RuntimeError("oracle set_motion failed")

    def texcoords(self, mesh):
        n = C.c_int()
        self.L.oro_mesh_texcoords(self.h, mesh, C.byref(n), None, None)
        nv, nn, nt = C.c_int(), C.c_int(), C.c_int()
        self.L.oro_mesh_info(self.h, mesh, C.byref(nv), C.byref(nn), C.byref(nt))
        uv = np.zeros((n.value, 2), np.float32)
        ti = np.zeros((nt.value if n.value else 0, 3), np.uint32)
        if n.value:
            self.L.oro_mesh_texcoords(self.h, mesh, C.byref(n), _p(uv, _fp), _p(ti, _u32p))
        return uv, ti

    def add_texture(self, rgb):
        a = np.ascontiguousarray(rgb, np.float32)
        r = self.L.oro_scene_add_texture(self.h, _p(a, _fp), a.shape[1], a.shape[0])
        if r < 0:
            raise RuntimeError("oracle add_texture failed")
        return r

    def add_dome_light(self, texture, power, samples=1, noise=0.001, fast_shadows=True):
        """DomeLight: setTexture(texture) + setPower (m_Gain) + setSamples (fast_shadows
        False: the transparency walk of src/DomeLight.cpp:123-145)."""
        l = Light()
        l.transparent = 0 if fast_shadows else 1
        l.type = 2
        l.power = power
        l.samples = samples
        l.noiseThreshold = noise
        l.castShadows = 1
        l.texture = int(texture)
        r = self.L.oro_scene_add_light(self.h, C.byref(l))
        if r < 0:
            raise RuntimeError(f"oracle dome light rejected ({r})")
        self.n_lights += 1
        return r

    def make_blas(self, meshes):
        """ProxyObject::setupMultiProxy + BVH::build over mesh ids (they leave the world)."""
        ids = (C.c_int * len(meshes))(*[int(m) for m in meshes])
        r = self.L.oro_scene_make_blas(self.h, ids, len(meshes))
        if r < 0:
            raise RuntimeError(f"oracle BLAS build failed ({r})")
        return r

    def add_instance(self, blas, m):
        m16 = np.ascontiguousarray(np.asarray(m, np.float32).reshape(16))
        r = self.L.oro_scene_add_instance(self.h, int(blas), _p(m16, _fp))
        if r < 0:
            raise RuntimeError("oracle add_instance failed")
        return r

    def blas_export(self, blas):
        n, l, p = C.c_int(), C.c_int(), C.c_int()
        if self.L.oro_blas_info(self.h, int(blas), C.byref(n), C.byref(l), C.byref(p)) != 0:
            raise RuntimeError("bad BLAS id")
        nb = np.zeros((n.value, 24), np.float32)
        nc = np.zeros((n.value, 4), np.int32)
        lt = np.zeros((l.value, 36), np.float32)
        lp = np.zeros((l.value, 4), np.int32)
        self.L.oro_blas_export(self.h, int(blas), _p(nb, _fp), _p(nc, _i32p), _p(lt, _fp), _p(lp, _i32p))
        return nb, nc, lt, lp

    def set_env_map(self, texture, exposure=1.0):
        if self.L.oro_scene_set_env_map(self.h, int(texture), float(exposure)) != 0:
            raise RuntimeError("oracle set_env_map failed")

    def set_material_env_map(self, material, texture, exposure=1.0):
        """Material::setEnvMap + m_envExposure (src/Material.h:19,41-42)."""
        if self.L.oro_scene_set_material_env_map(self.h, int(material), int(texture), float(exposure)) != 0:
            raise RuntimeError("oracle set_material_env_map failed")

    def dome_export(self, light):
        nu, nv = C.c_int(), C.c_int()
        if self.L.oro_dome_info(self.h, light, C.byref(nu), C.byref(nv)) != 0:
            raise RuntimeError("not a dome light")
        out = {k: np.zeros(s, np.float32) for k, s in dome_shapes(nu.value, nv.value).items()}
        self.L.oro_dome_export(self.h, light, *[_p(out[k], _fp) for k in DOME_KEYS])
        return out

    def texture_lookup_dir(self, texture, dirs, libm=None):
        _apply_libm(libm)
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        out = np.zeros_like(d)
        if self.L.oro_texture_lookup_dir(self.h, int(texture), len(d), _p(d, _fp), _p(out, _fp)) != 0:
            raise RuntimeError("bad texture")
        return out

    def set_bg(self, rgb):
        self.L.oro_scene_set_bg(self.h, *[float(x) for x in rgb])

    def set_num_paths(self, n):
        self.L.oro_scene_set_num_paths(self.h, int(n))

    def set_path_trace(self, enable=True, max_bounces=10, sample_env=False):
        """Scene::m_pathTrace / m_maxBounces / setSampleEnv (src/Scene.h:40-64)."""
        if self.L.oro_scene_set_path_trace(self.h, int(bool(enable)), int(max_bounces), int(bool(sample_env))) != 0:
            raise ValueError("need 1 <= max_bounces <= 64")

    def set_subdivs(self, min_subdivs, max_subdivs, noise=0.01):
        """Scene::setMinSubdivs / setMaxSubdivs / setNoise (src/Scene.h:42-55)."""
        if self.L.oro_scene_set_subdivs(self.h, int(min_subdivs), int(max_subdivs), float(noise)) != 0:
            raise ValueError("need 1 <= min_subdivs <= max_subdivs <= 16 and noise >= 0")

    def build(self):
        r = self.L.oro_scene_build(self.h)
        if r != 0:
            raise RuntimeError(f"oracle BVH build failed ({r})")

    def qbvh_info(self):
        vals = [C.c_int() for _ in range(6)]
        self.L.oro_qbvh_info(self.h, *[C.byref(v) for v in vals])
        keys = ("nodes", "leaves", "prims", "bin_nodes", "bin_leaves", "max_depth")
        return {k: v.value for k, v in zip(keys, vals)}

    def qbvh_export(self):
        info = self.qbvh_info()
        nb = np.zeros((info["nodes"], 24), np.float32)
        nc = np.zeros((info["nodes"], 4), np.int32)
        lt = np.zeros((info["leaves"], 36), np.float32)
        lp = np.zeros((info["leaves"], 4), np.int32)
        self.L.oro_qbvh_export(self.h, _p(nb, _fp), _p(nc, _i32p), _p(lt, _fp), _p(lp, _i32p))
        return nb, nc, lt, lp

    def trace(self, o, d, tmin, tmax):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        tmin = np.ascontiguousarray(np.broadcast_to(np.float32(tmin), (n,)) if np.ndim(tmin) == 0 else tmin, np.float32)
        tmax = np.ascontiguousarray(np.broadcast_to(np.float32(tmax), (n,)) if np.ndim(tmax) == 0 else tmax, np.float32)
        out = np.zeros(n, HIT_DTYPE)
        nv = np.zeros(n, np.uint32)
        lv = np.zeros(n, np.uint32)
        r = self.L.oro_trace(self.h, n, _p(o, _fp), _p(d, _fp), _p(tmin, _fp), _p(tmax, _fp),
                             out.ctypes.data, _p(nv, _u32p), _p(lv, _u32p))
        if r != 0:
            raise RuntimeError(f"oracle trace failed ({r})")
        return out, nv, lv

    def render(self, cam, W, H, rect=None, threads=1, want_hits=True, libm=None):
        """cam: dict(eye, lookAt, up, fov[, aperture, focusPlane, shutterSpeed]).  Returns dict of numpy arrays.
        libm: LIBM_FLOAT / LIBM_DOUBLE (None: the module default, set_default_libm)."""
        _apply_libm(libm)
        c = Camera(_v3(cam["eye"]), _v3(cam.get("up", (0, 1, 0))), _v3(cam["lookAt"]), float(cam["fov"]),
                   float(cam.get("aperture", 0.0)), float(cam.get("focusPlane", 1.0)),
                   float(cam.get("shutterSpeed", 0.001)))
        x0, y0, x1, y1 = rect if rect is not None else (0, 0, W, H)
        rgb = np.zeros((H, W, 3), np.float32)
        rgb8 = np.zeros((H, W, 3), np.uint8)
        hits = np.zeros((H, W), HIT_DTYPE) if want_hits else None
        shadow = np.zeros((H, W), np.uint32)
        counters = np.zeros(7, np.uint64)
        r = self.L.oro_render(self.h, C.byref(c), W, H, x0, y0, x1, y1, _p(rgb, _fp), _p(rgb8, _u8p),
                              hits.ctypes.data if hits is not None else None, _p(shadow, _u32p),
                              _p(counters, _u64p), int(threads))
        if r != 0:
            raise RuntimeError(f"oracle render failed ({r})")
        return {"rgb": rgb, "rgb8": rgb8, "hits": hits, "shadow": shadow,
                "primary_rays": int(counters[0]), "shadow_rays": int(counters[1]),
                "node_visits": int(counters[2]), "leaf_visits": int(counters[3]),
                "primary_node_visits": int(counters[4]), "primary_leaf_visits": int(counters[5]),
                "secondary_rays": int(counters[6])}


def libm_eval(fn, x, y=None):
    """glibc acosf(x) ("acos"), atan2f(y, x) ("atan2"), sinf / cosf(x) ("sin" / "cos") or
    powf(x, y) ("pow"), elementwise."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, np.float32)
    out = np.empty_like(x)
    L = lib()
    L.oro_libm_eval.argtypes = [C.c_int, C.c_size_t, _fp, _fp, _fp]
    if L.oro_libm_eval({"acos": 0, "atan2": 1, "sin": 3, "cos": 4, "pow": 5}[fn], len(x), _p(x, _fp), _p(y, _fp), _p(out, _fp)) != 0:
        raise ValueError(fn)
    return out


def x86_rcp(x):
    return lib().oro_x86_rcp(float(x))


def x86_rsqrt(x):
    return lib().oro_x86_rsqrt(float(x))


def rcp_nr(x):
    return lib().oro_rcp_nr(float(x))


def rsqrt_nr(x):
    return lib().oro_rsqrt_nr(float(x))


def gamma_table():
    t = np.zeros(32769, np.uint8)
    lib().oro_gamma_table(_p(t, _u8p))
    return t
