"""miro -- host-side mirror of the reference's scene API over libmrt.so.

Names, argument meaning and call order follow the reference scene scripts
(reference src/assignment2.h, src/Scene.h, src/Camera.h, src/Light.h):

    scene = Scene(); cam = Camera(); img = Image(); img.resize(512, 512)
    scene.setBGColor(Vector3(0, 0, 0.2))
    cam.setEye(Vector3(8, 1.5, 1)); cam.setLookAt(Vector3(0, 2.5, -1))
    cam.setUp(Vector3(0, 1, 0)); cam.setFOV(55)
    light = PointLight(); light.setPosition(Vector3(0, 10, 0)); light.setPower(200)
    scene.addLight(light)
    mesh = TriangleMesh(); mesh.load("sponza.obj"); makeMeshObjs(scene, mesh, Blinn(Vector3(1)))
    scene.preCalc()                    # BVH::build
    scene.raytraceImage(cam, img)      # 1 spp primary + shadow rays on the GPU

Everything that computes runs in libmrt.so (HIP kernels for gfx950); this
module only marshals data.  Missing library -> MRTError, no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import time
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import MRTError, check, f3

__all__ = ["Vector3", "Matrix4x4", "TriangleMesh", "Lambert", "Blinn", "PointLight", "RectangleLight",
           "DomeLight", "RawImage", "Texture", "Objects", "BVH", "ProxyObject",
           "Camera", "Image", "Scene", "Ray", "HitInfo", "makeMeshObjs", "MRTError", "lib", "device_count",
           "rcp_nr", "rsqrt_nr"]

lib = _lib.load


def device_count() -> int:
    return int(lib().mrt_device_count())


def rcp_nr(x: float) -> float:
    return float(lib().mrt_rcp_nr(float(x)))


def rsqrt_nr(x: float) -> float:
    return float(lib().mrt_rsqrt_nr(float(x)))


def debug_libm(fn: str, x, y=None):
    """The device's acosf(x) ("acos") / atan2f(y, x) ("atan2") / sinf(x) ("sin") / cosf(x)
    ("cos") / powf(x, y) ("pow") / rcp_nr(x) ("rcp_nr") (numerics probe)."""
    import numpy as np
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(np.zeros_like(x) if y is None else y, np.float32)
    out = np.empty_like(x)
    _lib.check(lib().mrt_debug_libm({"acos": 0, "atan2": 1, "rcp_nr": 2, "sin": 3, "cos": 4, "pow": 5}[fn], x.ctypes.data, y.ctypes.data, len(x),
                                    out.ctypes.data), "mrt_debug_libm")
    return out


class Vector3(tuple):
    """Plain 3-tuple with the reference's constructors: Vector3(s) or Vector3(x, y, z)."""

    def __new__(cls, *a):
        if len(a) == 1 and np.ndim(a[0]) == 0:
            a = (a[0], a[0], a[0])
        elif len(a) == 1:
            a = tuple(a[0])
        if len(a) != 3:
            raise ValueError("Vector3 needs 1 or 3 components")
        return super().__new__(cls, (float(a[0]), float(a[1]), float(a[2])))

    x = property(lambda s: s[0])
    y = property(lambda s: s[1])
    z = property(lambda s: s[2])


class Matrix4x4:
    """Row-major 4x4 (m11..m44), src/Matrix4x4.h.  Only used as a load-time ctm."""

    def __init__(self, m=None):
        self.m = np.eye(4, dtype=np.float32) if m is None else np.asarray(m, np.float32).reshape(4, 4).copy()

    def setIdentity(self):
        self.m = np.eye(4, dtype=np.float32)

    def translate(self, x, y, z):  # setColumn4(Vector4(x,y,z,0) + column4), src/Matrix4x4.h:751-754
        self.m[0, 3] = np.float32(x) + self.m[0, 3]
        self.m[1, 3] = np.float32(y) + self.m[1, 3]
        self.m[2, 3] = np.float32(z) + self.m[2, 3]

    def scale(self, x, y, z):  # src/Matrix4x4.h:757-762
        self.m[0, 0] *= np.float32(x)
        self.m[1, 1] *= np.float32(y)
        self.m[2, 2] *= np.float32(z)


class TriangleMesh:
    """TriangleMesh (src/TriangleMesh.h).  load() keeps the path; the OBJ is parsed
    by libmrt's loader (src/TriangleMeshLoad.cpp semantics) at Scene.preCalc()."""

    def __init__(self):
        self.path: Optional[str] = None
        self.ctm: Optional[np.ndarray] = None
        self.verts = self.normals = self.vidx = self.nidx = None

    def load(self, file, ctm: Optional[Matrix4x4] = None) -> bool:
        self.path = str(file)
        self.ctm = None if ctm is None else np.ascontiguousarray(ctm.m, np.float32)
        return True

    def createSingleTriangle(self):  # src/TriangleMesh.cpp:11-42
        self.verts = np.zeros((3, 3), np.float32)
        self.normals = np.zeros((3, 3), np.float32)
        self.vidx = np.array([[0, 1, 2]], np.uint32)
        self.nidx = np.array([[0, 1, 2]], np.uint32)

    def setArrays(self, verts, normals, vidx, nidx):
        self.verts = np.ascontiguousarray(verts, np.float32).reshape(-1, 3)
        self.normals = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
        self.vidx = np.ascontiguousarray(vidx, np.uint32).reshape(-1, 3)
        self.nidx = np.ascontiguousarray(nidx, np.uint32).reshape(-1, 3)

    def setTexCoords(self, uv, tidx):
        """m_texCoords ((u, v) per texture coordinate) / m_texCoordIndices (3 per triangle)."""
        self.uv = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
        self.tidx = np.ascontiguousarray(tidx, np.uint32).reshape(-1, 3)

    uv = tidx = None

    def setV1(self, v): self.verts[0] = v
    def setV2(self, v): self.verts[1] = v
    def setV3(self, v): self.verts[2] = v
    def setN1(self, n): self.normals[0] = n
    def setN2(self, n): self.normals[1] = n
    def setN3(self, n): self.normals[2] = n


class _Maps:
    """Material::setColorMap / setAlphaMap / setNormalMap / setSpecularMap /
    setReflectMap / setRefractMap (src/Material.h:20-25): Texture objects."""
    colorMap = normalMap = specularMap = reflectMap = refractMap = alphaMap = None

    def setColorMap(self, t): self.colorMap = t
    def setNormalMap(self, t): self.normalMap = t
    def setSpecularMap(self, t): self.specularMap = t
    def setReflectMap(self, t): self.reflectMap = t
    def setRefractMap(self, t): self.refractMap = t
    def setAlphaMap(self, t): self.alphaMap = t

    def _maps(self):
        return (self.colorMap, self.normalMap, self.specularMap, self.reflectMap, self.refractMap, self.alphaMap)

    # Material::setEnvMap / m_envExposure (src/Material.h:19,41-42): the map a missed
    # reflection / refraction / GI ray of a Blinn material takes (getEnvironmentColor,
    # src/Material.cpp:44-64); None = the scene's
    envMap = None
    envExposure = 1.0

    def setEnvMap(self, t): self.envMap = t
    def setEnvExposure(self, x): self.envExposure = float(x)


class Lambert(_Maps):
    """Lambert(kd = Vector3(1), ka = Vector3(0)), src/Lambert.h:11-13."""

    def __init__(self, kd=Vector3(1), ka=Vector3(0)):
        self.kd, self.ka = Vector3(kd), Vector3(ka)

    def setKd(self, kd): self.kd = Vector3(kd)
    def setKa(self, ka): self.ka = Vector3(ka)

    def setSampleEnv(self, b): self.sampleEnv = bool(b)          # Material::setSampleEnv (src/Material.h:27)

    sampleEnv = True

    def _c(self):
        return _lib.mrt_material(0, f3(self.kd), f3(self.ka), f3((1, 1, 1)), 1.0, 0.0, f3((0, 0, 0)), 0.0)


class Blinn(_Maps):
    """Blinn(kd, ka, ks, kt, ior, specExp, specAmt, reflectAmt, refractAmt) defaults of
    src/Blinn.h:11-22: direct lighting plus Fresnel-weighted reflection / refraction
    rays (src/Blinn.cpp:91-335), glossy reflection vectors, translucency, emission
    (setLightEmittedIntensity / setLightEmittedColor), path tracing (Scene.setPathTrace)
    texture maps (colour, normal, specular, reflect, refract, alpha) and dispersion
    (m_disperse with m_ior[0..2]: one refraction ray per colour channel).  As in the
    reference, setIor(ior, i) sets m_ior[i] and the non-dispersive refraction reads
    m_ior[1] (src/Blinn.cpp:183), so setIor(x) alone changes only dispersion."""

    def __init__(self, kd=Vector3(1), ka=Vector3(0), ks=Vector3(1), kt=Vector3(0), ior=1.5,
                 specExp=1.0, specAmt=0.0, reflectAmt=0.0, refractAmt=0.0, specGloss=1.0):
        self.kd, self.ka, self.ks, self.kt = Vector3(kd), Vector3(ka), Vector3(ks), Vector3(kt)
        self.m_ior = [float(ior)] * 3      # src/Blinn.cpp:25-27
        self.m_disperse = False            # Material::m_disperse (src/Material.cpp:6)
        self.specExp, self.specAmt = float(specExp), float(specAmt)
        self.reflectAmt, self.refractAmt = float(reflectAmt), float(refractAmt)
        self.specGloss = float(specGloss)
        self.translucency = 0.0
        self.lightEmitted = 0.0          # the Blinn ctor forces 0 (src/Blinn.cpp:28-29)
        self.Le = Vector3(0)
        self.sampleEnv = True            # Material::m_sampleEnv (src/Material.cpp:6)

    def setLightEmittedIntensity(self, le): self.lightEmitted = float(le)   # src/Blinn.h:44
    def setLightEmittedColor(self, c): self.Le = Vector3(c)                 # src/Blinn.h:45
    def setSampleEnv(self, b): self.sampleEnv = bool(b)                     # src/Material.h:27

    def setTranslucency(self, t): self.translucency = float(t)   # src/Material.h:30

    def setReflectGloss(self, g): self.specGloss = float(g)    # src/Blinn.h:42

    def setReflectAmt(self, a): self.reflectAmt = float(a)     # src/Blinn.h:41
    def setRefractAmt(self, a): self.refractAmt = float(a)     # src/Material.h:32
    def setIor(self, ior, i=0):                                # src/Blinn.h:38
        self.m_ior[i] = float(ior)

    @property
    def ior(self):                                             # the refraction IOR: m_ior[1] (src/Blinn.cpp:183)
        return self.m_ior[1]

    def setKd(self, v): self.kd = Vector3(v)
    def setKa(self, v): self.ka = Vector3(v)
    def setKs(self, v): self.ks = Vector3(v)
    def setSpecExp(self, e): self.specExp = float(e)
    def setSpecAmt(self, a): self.specAmt = float(a)

    def _c(self):
        return _lib.mrt_material(1, f3(self.kd), f3(self.ka), f3(self.ks), self.specExp, self.specAmt, f3(self.Le),
                                 self.lightEmitted)


class _Light:
    def __init__(self):  # Light::Light, src/Light.h:15-19
        self.color = Vector3(0)
        self.power = 0.0
        self.samples = 1
        self.castShadows = True
        self.fastShadows = True           # src/Light.h:16; False: a point light casts no shadow (its walk never traces), rect / dome lights walk through refractive hits
        self.noiseThreshold = 0.001

    def setColor(self, c): self.color = Vector3(c)
    def setPower(self, p): self.power = float(p)
    def setSamples(self, n): self.samples = int(n)
    def setCastShadows(self, c): self.castShadows = bool(c)
    def setFastShadows(self, c): self.fastShadows = bool(c)
    def setNoiseThreshold(self, t): self.noiseThreshold = float(t)


class PointLight(_Light):
    def __init__(self):
        super().__init__()
        self.position = Vector3(0)

    def setPosition(self, v): self.position = Vector3(v)

    def _c(self, texture=-1):
        return _lib.mrt_light(0, f3(self.position), f3((0, 0, 0)), f3((0, 0, 0)), f3((0, 0, 0)), self.power,
                              self.samples, self.noiseThreshold, int(self.castShadows), -1, int(not self.fastShadows))


class RectangleLight(_Light):
    def __init__(self):
        super().__init__()
        self.v1 = self.v2 = self.v3 = Vector3(0)

    def setVertices(self, v1, v2, v3):
        self.v1, self.v2, self.v3 = Vector3(v1), Vector3(v2), Vector3(v3)

    def _c(self, texture=-1):
        return _lib.mrt_light(1, f3((0, 0, 0)), f3(self.v1), f3(self.v2), f3(self.v3), self.power,
                              self.samples, self.noiseThreshold, int(self.castShadows), -1, int(not self.fastShadows))


TEX_HDR, TEX_GRAY, TEX_RGB, TEX_RGBA = 0, 1, 3, 4   # RawImage ImageType (floats per texel 3, 1, 3, 4)
_CHANNELS = {TEX_HDR: 3, TEX_GRAY: 1, TEX_RGB: 3, TEX_RGBA: 4}


class RawImage:
    """RawImage (src/RawImage.h:9-30): float texels in m_rawData order (row 0 =
    the top row for .hdr; TGA rows flipped as loadTGA does).  RawImage(w, h, data,
    type) wraps an array; loadImage decodes .tga / .ppm / .hdr in libmrt."""

    def __init__(self, w=0, h=0, data=None, imageType=TEX_HDR):
        self.m_width, self.m_height, self.m_imageType = int(w), int(h), int(imageType)
        self.m_rawData = None if data is None else np.ascontiguousarray(data, np.float32).reshape(
            self.m_height, self.m_width, _CHANNELS[self.m_imageType])

    def loadImage(self, filename):  # src/RawImage.cpp:16-26 (by extension)
        ext = str(filename).rsplit(".", 1)[-1]
        if ext in ("hdr", "HDR"):
            return self.loadHDR(filename)
        L = lib()
        w, h, t = C.c_int32(), C.c_int32(), C.c_int32()
        check(L.mrt_image_info(str(filename).encode(), C.byref(w), C.byref(h), C.byref(t)), f"image {filename}")
        data = np.zeros((h.value, w.value, _CHANNELS[t.value]), np.float32)
        check(L.mrt_image_load(str(filename).encode(), data.ctypes.data_as(C.POINTER(C.c_float)), w.value, h.value),
              f"image {filename}")
        self.m_width, self.m_height, self.m_imageType, self.m_rawData = w.value, h.value, t.value, data
        return True

    def loadHDR(self, filename):  # src/RawImage.cpp:29-32 -> HDRLoader::load
        L = lib()
        w, h = C.c_int32(), C.c_int32()
        check(L.mrt_hdr_info(str(filename).encode(), C.byref(w), C.byref(h)), f"HDR {filename}")
        data = np.zeros((h.value, w.value, 3), np.float32)
        check(L.mrt_hdr_load(str(filename).encode(), data.ctypes.data_as(C.POINTER(C.c_float)), w.value, h.value),
              f"HDR {filename}")
        self.m_width, self.m_height, self.m_rawData = w.value, h.value, data
        return True


class Texture:
    """Texture(RawImage) (src/Texture.h:9-28): a material map, or a lat-long map
    for DomeLight and Scene.setEnvMap."""

    def __init__(self, image: RawImage):
        self.m_image = image

    def getWidth(self): return self.m_image.m_width
    def getHeight(self): return self.m_image.m_height


class DomeLight(_Light):
    """DomeLight (src/DomeLight.h:44-62): setTexture, setPower (= m_Gain, default
    1), setSamples, setNoiseThreshold.  Importance-sampled from the texture."""

    def __init__(self):
        super().__init__()
        self.power = 1.0
        self.texture = None

    def setTexture(self, t): self.texture = t

    def _c(self, texture=-1):
        return _lib.mrt_light(2, f3((0, 0, 0)), f3((0, 0, 0)), f3((0, 0, 0)), f3((0, 0, 0)), self.power,
                              self.samples, self.noiseThreshold, int(self.castShadows), int(texture),
                              int(not self.fastShadows))


class Camera:
    """Camera setters of src/Camera.h:26-45 (fov in degrees, like setFOV), with the
    lens of eyeRayAdaptive: setAperture / setFocusPlane (depth of field,
    src/Camera.cpp:153-174) and setShutterSpeed (getTimeSample, src/Camera.h:44-46)."""

    def __init__(self):
        self.eye, self.lookAt, self.up, self.fov = Vector3(0), Vector3(0, 0, -1), Vector3(0, 1, 0), 45.0
        self.aperture, self.focusPlane, self.shutterSpeed = 0.0, 1.0, 0.001   # src/Camera.cpp:21-23

    def setEye(self, v): self.eye = Vector3(v)
    def setLookAt(self, v): self.lookAt = Vector3(v)
    def setUp(self, v): self.up = Vector3(v)
    def setFOV(self, f): self.fov = float(f)
    def setAperture(self, a): self.aperture = float(a)
    def setFocusPlane(self, f): self.focusPlane = float(f)
    def setShutterSpeed(self, s): self.shutterSpeed = float(s)

    def _c(self):
        return _lib.mrt_camera(f3(self.eye), f3(self.lookAt), f3(self.up), self.fov, self.aperture, self.focusPlane,
                               self.shutterSpeed)


class Image:
    """Image (src/Image.h): 8-bit RGB, row 0 = bottom, plus the float RGB frame
    before Image::Map (`rgb`) for parity checks."""

    def __init__(self):
        self.resize(1, 1)

    def resize(self, w, h):
        self.m_width, self.m_height = int(w), int(h)
        self.rgb = np.zeros((self.m_height, self.m_width, 3), np.float32)
        self.pixels = np.zeros((self.m_height, self.m_width, 3), np.uint8)

    def width(self): return self.m_width
    def height(self): return self.m_height

    def writePPM(self, path):  # src/Image.cpp:137-154 (rows flipped)
        with open(path, "wb") as f:
            f.write(b"P6\n%d %d\n255\n" % (self.m_width, self.m_height))
            f.write(np.ascontiguousarray(self.pixels[::-1]).tobytes())


class Ray:
    def __init__(self, o, d):
        self.o, self.d = Vector3(o), Vector3(d)


class HitInfo:
    """HitInfo (src/Ray.h:185-200); obj is the global triangle id (-1 = none)."""

    def __init__(self, t=1e12, a=0.0, b=0.0, obj=-1):
        self.t, self.a, self.b, self.obj = float(t), float(a), float(b), int(obj)


HIT_DTYPE = np.dtype([("t", "<f4"), ("a", "<f4"), ("b", "<f4"), ("prim", "<i4"), ("inst", "<i4")])


def makeMeshObjs(scene: "Scene", mesh: TriangleMesh, material):
    """One Object per triangle, in mesh order (the reference's missing helper)."""
    scene.addMesh(mesh, material)


def _mesh_vertices(mesh: TriangleMesh) -> np.ndarray:
    """The vertices of a TriangleMesh: its arrays, or its OBJ parsed by libmrt's
    loader (through a scratch scene)."""
    if mesh.path is None:
        return mesh.verts
    L = lib()
    h = L.mrt_scene_create()
    try:
        ctm = mesh.ctm.ctypes.data_as(C.POINTER(C.c_float)) if mesh.ctm is not None else None
        mid = check(L.mrt_scene_add_material(h, C.byref(Lambert()._c())), "add_material")
        mesh_id = check(L.mrt_scene_add_obj(h, mesh.path.encode(), ctm, mid), f"load {mesh.path}")
        nv, nn, nt = C.c_int32(), C.c_int32(), C.c_int32()
        check(L.mrt_scene_mesh_info(h, mesh_id, C.byref(nv), C.byref(nn), C.byref(nt)), "mesh_info")
        v = np.zeros((nv.value, 3), np.float32)
        n = np.zeros((nn.value, 3), np.float32)
        vi = np.zeros((nt.value, 3), np.uint32)
        ni = np.zeros((nt.value, 3), np.uint32)
        check(L.mrt_scene_mesh_export(h, mesh_id, v.ctypes.data_as(C.POINTER(C.c_float)),
                                      n.ctypes.data_as(C.POINTER(C.c_float)), vi.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      ni.ctypes.data_as(C.POINTER(C.c_uint32))), "mesh_export")
        return v
    finally:
        L.mrt_scene_destroy(h)


def makeMBMeshObjs(scene: "Scene", mesh: TriangleMesh, mesh2: TriangleMesh, material):
    """makeMBMeshObjs (src/main.cpp:23, :202): one MBObject(material, mesh, mesh2, i)
    per triangle (src/MBObject.cpp:7-11) -- mesh at time 0, mesh2 (same topology)
    at time 1; a ray of time t meets the blend t * mesh2 + (1 - t) * mesh."""
    # mesh2 rides on this entry only: other entries of the same TriangleMesh
    # (makeMeshObjs) stay static, as their Objects are plain Objects
    scene._meshes.append((mesh, material, mesh2))


class Objects(list):
    """Objects (std::vector<Object*>) of a proxy: (mesh, material) pairs here."""


class BVH:
    """A ProxyObject's BVH (src/BVH.h:113-154); built in libmrt at Scene.preCalc()."""

    def __init__(self):
        self.objects = None


class ProxyObject:
    """ProxyObject(objects, bvh, Matrix4x4) (src/ProxyObject.h, src/ProxyObject.cpp:5-12):
    one instance of a shared BVH under a transform.  setupProxy / setupMultiProxy
    fill the Objects and BVH as the reference's static helpers do
    (src/ProxyObject.cpp:131-167); Scene.addObject adds the instance."""

    def __init__(self, objects, bvh, t=None):
        self.objects, self.bvh = objects, bvh
        self.matrix = (t if t is not None else Matrix4x4()).m.copy()

    @staticmethod
    def setupProxy(mesh, mat, objects, bvh):
        objects.append((mesh, mat))
        bvh.objects = objects

    @staticmethod
    def setupMultiProxy(meshes, numObjs, mats, objects, bvh):
        for j in range(numObjs):
            objects.append((meshes[j], mats[j]))
        bvh.objects = objects


class Scene:
    """Scene (src/Scene.h).  Objects are whole meshes here; object ids inside a
    HitInfo are global triangle indices in insertion order."""

    def __init__(self, device: int = 0):
        self._meshes: List[tuple] = []   # (mesh, material) / (mesh, material, time-1 mesh) / (ProxyObject, None)
        self._lights: List[_Light] = []
        self.bg = Vector3(0)
        self.m_numPaths = 1
        self.m_pathTrace = False         # src/Scene.cpp:17-19
        self.m_maxBounces = 10
        self.m_sampleLightFromEnv = False   # never initialised by the reference's Scene ctor
        self.m_minSubdivs = 1            # src/Scene.cpp:20-22
        self.m_maxSubdivs = 1
        self.m_noiseThreshold = 0.01
        self.m_envMap = None
        self.m_envExposure = 1.0
        self.device = int(device)
        self._h = None
        self.bvh_info = None

    # -- construction (src/Scene.h:17-28)
    def addMesh(self, mesh, material): self._meshes.append((mesh, material))
    def addObject(self, proxy): self._meshes.append((proxy, None))   # Scene::addObject (a ProxyObject)
    def addLight(self, light): self._lights.append(light)
    def setBGColor(self, c): self.bg = Vector3(c)
    def setNumPaths(self, p): self.m_numPaths = int(p)
    def setPathTrace(self, pt): self.m_pathTrace = bool(pt)        # src/Scene.h:40
    def setMaxBounces(self, mb): self.m_maxBounces = int(mb)       # src/Scene.h:48
    def maxBounces(self): return self.m_maxBounces
    def setSampleEnv(self, b): self.m_sampleLightFromEnv = bool(b)  # src/Scene.h:57
    # adaptive supersampling, Scene::adaptiveSampleScene (src/Scene.h:42-55, src/Scene.cpp:252-293)
    def setMinSubdivs(self, r): self.m_minSubdivs = int(r)
    def minSubdivs(self): return self.m_minSubdivs
    def setMaxSubdivs(self, r): self.m_maxSubdivs = int(r)
    def maxSubdivs(self): return self.m_maxSubdivs
    def setNoise(self, n): self.m_noiseThreshold = float(n)
    def noise(self): return self.m_noiseThreshold
    def setEnvMap(self, t): self.m_envMap = t                    # src/Scene.h:23
    def setEnvExposure(self, e): self.m_envExposure = float(e)   # src/Scene.h:24

    def __del__(self):
        try:
            if self._h:
                lib().mrt_scene_destroy(self._h)
                self._h = None
        except Exception:
            pass

    @property
    def handle(self):
        if self._h is None:
            raise MRTError("call preCalc() first")
        return self._h

    def preCalc(self):
        """Scene::preCalc -> BVH::build (host side of libmrt)."""
        L = lib()
        if self._h:
            L.mrt_scene_destroy(self._h)
        self._h = L.mrt_scene_create()
        mats = {}
        mat_objs = {}

        def add_mesh(mesh, mat):
            if id(mat) not in mats:
                mat_objs[id(mat)] = mat
                m = mat._c()
                mats[id(mat)] = check(L.mrt_scene_add_material(self._h, C.byref(m)), "add_material")
                if isinstance(mat, Blinn):
                    check(L.mrt_scene_set_material_optics(self._h, mats[id(mat)], mat.reflectAmt, mat.refractAmt,
                                                          mat.ior), "material optics")
                    check(L.mrt_scene_set_material_gloss(self._h, mats[id(mat)], mat.specGloss), "material gloss")
                    if mat.m_disperse:
                        i3 = (C.c_float * 3)(*mat.m_ior)
                        check(L.mrt_scene_set_material_dispersion(self._h, mats[id(mat)], 1, i3), "dispersion")
                    check(L.mrt_scene_set_material_translucency(self._h, mats[id(mat)], mat.translucency),
                          "material translucency")
                check(L.mrt_scene_set_material_sample_env(self._h, mats[id(mat)], int(mat.sampleEnv)), "sampleEnv")
            mid = mats[id(mat)]
            if mesh.path is not None:
                ctm = mesh.ctm.ctypes.data_as(C.POINTER(C.c_float)) if mesh.ctm is not None else None
                return check(L.mrt_scene_add_obj(self._h, mesh.path.encode(), ctm, mid), f"load {mesh.path}")
            v, n, vi, ni = mesh.verts, mesh.normals, mesh.vidx, mesh.nidx
            mm = _lib.mrt_mesh(v.ctypes.data_as(C.POINTER(C.c_float)), n.ctypes.data_as(C.POINTER(C.c_float)),
                               vi.ctypes.data_as(C.POINTER(C.c_uint32)), ni.ctypes.data_as(C.POINTER(C.c_uint32)),
                               len(v), len(n), len(vi), v.shape[1] if v.ndim == 2 else 3, n.shape[1] if n.ndim == 2 else 3)
            mesh_id = check(L.mrt_scene_add_mesh(self._h, C.byref(mm), mid), "add_mesh")
            if mesh.uv is not None:
                check(L.mrt_scene_mesh_set_texcoords(self._h, mesh_id, mesh.uv.ctypes.data_as(C.POINTER(C.c_float)),
                                                     len(mesh.uv), mesh.tidx.ctypes.data_as(C.POINTER(C.c_uint32))),
                      "texcoords")
            return mesh_id

        def set_motion(mesh_id, mesh2):
            v2 = np.ascontiguousarray(_mesh_vertices(mesh2), np.float32).reshape(-1, 3)
            nv = C.c_int32()
            check(L.mrt_scene_mesh_info(self._h, mesh_id, C.byref(nv), C.byref(C.c_int32()), C.byref(C.c_int32())),
                  "mesh_info")
            if len(v2) != nv.value:
                raise MRTError(f"motion mesh has {len(v2)} vertices, the time-0 mesh {nv.value}")
            check(L.mrt_scene_set_mesh_motion(self._h, mesh_id, v2.ctypes.data_as(C.POINTER(C.c_float))), "mesh motion")

        blas = {}   # BVH object -> BLAS id (built once, shared by its instances)
        self.blas_build_ms = 0.0
        self.blas_prims = 0
        self.blas_ids = blas
        for entry in self._meshes:
            item, mat = entry[0], entry[1]
            if not isinstance(item, ProxyObject):
                mesh_id = add_mesh(item, mat)
                if len(entry) > 2:   # makeMBMeshObjs: MBObjects of this entry only
                    set_motion(mesh_id, entry[2])
                continue
            key = id(item.bvh)
            if key not in blas:
                ids = (C.c_int32 * len(item.bvh.objects))(*[add_mesh(m, mt) for m, mt in item.bvh.objects])
                t0 = time.perf_counter()
                blas[key] = check(L.mrt_scene_make_blas(self._h, ids, len(ids)), "BLAS build")
                self.blas_build_ms += (time.perf_counter() - t0) * 1e3
                n, lv, p = C.c_int32(), C.c_int32(), C.c_int32()
                check(L.mrt_scene_blas_info(self._h, blas[key], C.byref(n), C.byref(lv), C.byref(p)), "blas_info")
                self.blas_prims += p.value
            m16 = np.ascontiguousarray(item.matrix, np.float32).reshape(16)
            check(L.mrt_scene_add_instance(self._h, blas[key], m16.ctypes.data_as(C.POINTER(C.c_float))), "instance")
        tex_ids = {}

        def tex_id(t):
            if t is None:
                return -1
            if id(t) not in tex_ids:
                img = t.m_image
                if img.m_rawData is None:
                    raise MRTError("texture image has no data (loadImage first)")
                a = np.ascontiguousarray(img.m_rawData, np.float32)
                tex_ids[id(t)] = check(L.mrt_scene_add_texture_typed(self._h, a.ctypes.data_as(C.POINTER(C.c_float)),
                                                                     img.m_width, img.m_height,
                                                                     getattr(img, "m_imageType", TEX_HDR)), "add_texture")
            return tex_ids[id(t)]

        for key, mid in mats.items():   # Material::set*Map
            mat = mat_objs[key]
            maps = mat._maps() if isinstance(mat, _Maps) else (None,) * 6
            if any(m is not None for m in maps):
                arr = (C.c_int32 * 6)(*[tex_id(m) for m in maps])
                check(L.mrt_scene_set_material_maps(self._h, mid, arr), "material maps")
            if getattr(mat, "envMap", None) is not None:
                check(L.mrt_scene_set_material_env_map(self._h, mid, tex_id(mat.envMap), mat.envExposure),
                      "material env map")

        for light in self._lights:
            lc = light._c(tex_id(getattr(light, "texture", None)))
            check(L.mrt_scene_add_light(self._h, C.byref(lc)), "add_light")
        if self.m_envMap is not None:
            check(L.mrt_scene_set_env_map(self._h, tex_id(self.m_envMap), self.m_envExposure), "env map")
        check(L.mrt_scene_set_background(self._h, f3(self.bg)), "bg")
        check(L.mrt_scene_set_num_paths(self._h, self.m_numPaths), "num_paths")
        check(L.mrt_scene_set_path_trace(self._h, int(self.m_pathTrace), self.m_maxBounces,
                                         int(self.m_sampleLightFromEnv)), "path trace")
        check(L.mrt_scene_set_subdivs(self._h, self.m_minSubdivs, self.m_maxSubdivs, self.m_noiseThreshold), "subdivs")
        t0 = time.perf_counter()
        check(L.mrt_scene_build_bvh(self._h), "BVH build")
        self.bvh_build_ms = (time.perf_counter() - t0) * 1e3   # host BVH::build wall time
        info = _lib.mrt_bvh_info()
        check(L.mrt_scene_bvh_info(self._h, C.byref(info)), "bvh_info")
        self.bvh_info = {k: getattr(info, k) for k, _ in info._fields_}
        return self.bvh_info

    def mesh_arrays(self, mesh_id: int):
        L = lib()
        nv, nn, nt = C.c_int32(), C.c_int32(), C.c_int32()
        check(L.mrt_scene_mesh_info(self.handle, mesh_id, C.byref(nv), C.byref(nn), C.byref(nt)), "mesh_info")
        v = np.zeros((nv.value, 3), np.float32)
        n = np.zeros((nn.value, 3), np.float32)
        vi = np.zeros((nt.value, 3), np.uint32)
        ni = np.zeros((nt.value, 3), np.uint32)
        check(L.mrt_scene_mesh_export(self.handle, mesh_id, v.ctypes.data_as(C.POINTER(C.c_float)),
                                      n.ctypes.data_as(C.POINTER(C.c_float)), vi.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      ni.ctypes.data_as(C.POINTER(C.c_uint32))), "mesh_export")
        return v, n, vi, ni

    def dome_tables(self, light: int):
        """DomeLight::setTexture tables of light `light` (host arrays of libmrt)."""
        L = lib()
        nu, nv = C.c_int32(), C.c_int32()
        check(L.mrt_scene_dome_info(self.handle, int(light), C.byref(nu), C.byref(nv)), "dome_info")
        nu, nv = nu.value, nv.value
        shapes = {"cdf_u": (nu + 1,), "func_u": (nu,), "cdf_v": (nu, nv + 1), "func_v": (nu, nv),
                  "func_int": (nu + 1,), "cos_u": (nu + 1,), "sin_u": (nu + 1,), "cos_v": (nv + 1,),
                  "sin_v": (nv + 1,)}
        out = {k: np.zeros(s, np.float32) for k, s in shapes.items()}
        check(L.mrt_scene_dome_export(self.handle, int(light),
                                      *[out[k].ctypes.data_as(C.POINTER(C.c_float)) for k in shapes]), "dome_export")
        return out

    def blas_export(self, blas: int):
        L = lib()
        n, l, p = C.c_int32(), C.c_int32(), C.c_int32()
        check(L.mrt_scene_blas_info(self.handle, int(blas), C.byref(n), C.byref(l), C.byref(p)), "blas_info")
        nb = np.zeros((n.value, 24), np.float32)
        nc = np.zeros((n.value, 4), np.int32)
        lt = np.zeros((l.value, 36), np.float32)
        lp = np.zeros((l.value, 4), np.int32)
        check(L.mrt_scene_blas_export(self.handle, int(blas), nb.ctypes.data_as(C.POINTER(C.c_float)),
                                      nc.ctypes.data_as(C.POINTER(C.c_int32)), lt.ctypes.data_as(C.POINTER(C.c_float)),
                                      lp.ctypes.data_as(C.POINTER(C.c_int32))), "blas_export")
        return nb, nc, lt, lp

    def bvh_export(self):
        info = self.bvh_info
        nb = np.zeros((info["nodes"], 24), np.float32)
        nc = np.zeros((info["nodes"], 4), np.int32)
        lt = np.zeros((info["leaves"], 36), np.float32)
        lp = np.zeros((info["leaves"], 4), np.int32)
        check(lib().mrt_scene_bvh_export(self.handle, nb.ctypes.data_as(C.POINTER(C.c_float)),
                                         nc.ctypes.data_as(C.POINTER(C.c_int32)),
                                         lt.ctypes.data_as(C.POINTER(C.c_float)),
                                         lp.ctypes.data_as(C.POINTER(C.c_int32))), "bvh_export")
        return nb, nc, lt, lp

    # -- rendering (src/Scene.cpp:85-217)
    def raytraceImage(self, cam: Camera, img: Image, count_visits=False, want_hits=False, seed=0, devices=None):
        """devices: HIP device ordinals to deal the 32x32 buckets over (bucket b ->
        devices[b % n], mrt_render_opts.devices; one device may repeat)."""
        W, H = img.width(), img.height()
        opts = _lib.mrt_render_opts(W, H, self.device, int(count_visits), 1, int(want_hits), seed)
        if devices:
            dev_arr = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            opts.devices, opts.n_devices = dev_arr, len(devices)
        hits = np.zeros((H, W), HIT_DTYPE) if want_hits else None
        c = cam._c()
        check(lib().mrt_render(self.handle, C.byref(c), C.byref(opts), img.rgb.ctypes.data_as(C.POINTER(C.c_float)),
                               img.pixels.ctypes.data_as(C.POINTER(C.c_uint8)),
                               hits.ctypes.data if hits is not None else None), "raytraceImage")
        self.last_stats = self.stats()
        return hits

    def walk_info(self):
        """The walk of this scene's last one-light frame: {"lds_nodes": 1 (LDS top-node walk),
        0 (plain), -1 (none yet); "walk_exits": 1 or 2 (the walk loop's form: one exit unless
        tuning "walk_exit" 0 asks for the two-exit loop)}."""
        ln, wx = C.c_int32(-1), C.c_int32(-1)
        check(lib().mrt_scene_walk_info(self.handle, C.byref(ln), C.byref(wx)), "walk_info")
        return {"lds_nodes": int(ln.value), "walk_exits": int(wx.value)}

    def stats(self):
        st = _lib.mrt_stats()
        check(lib().mrt_scene_last_stats(self.handle, C.byref(st)), "stats")
        return {k: getattr(st, k) for k, _ in st._fields_}

    def wave_log(self, launch: int):
        """Per-wave records of the last count-mode render (diagnostics):
        array (waves, 60): start, end (device wall-clock ticks), tiles, node
        visits, then per tile (first 28) tile id << 40 | start tick & (2^40 - 1),
        then per tile its dequeue time in ticks;
        for launch 0 (primary) or 1 (shade); plus the clock rate (kHz)."""
        L = lib()
        out = np.zeros((1 << 16, 60), np.uint64)
        n = check(L.mrt_debug_wave_log(self.handle, int(launch), out.ctypes.data, len(out)), "wave_log")
        return out[:n].copy(), int(L.mrt_device_wall_clock_khz(self.handle))

    # -- ray queries (src/Scene.cpp:295-298)
    def traceBatch(self, o, d, tmin=0.001, tmax=1e12, any_hit=False):
        o = np.ascontiguousarray(o, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(d, np.float32).reshape(-1, 3)
        n = len(o)
        tmin = np.ascontiguousarray(np.broadcast_to(np.asarray(tmin, np.float32), (n,)))
        tmax = np.ascontiguousarray(np.broadcast_to(np.asarray(tmax, np.float32), (n,)))
        out = np.zeros(n, HIT_DTYPE)
        fp = C.POINTER(C.c_float)
        check(lib().mrt_trace(self.handle, o.ctypes.data_as(fp), d.ctypes.data_as(fp), tmin.ctypes.data_as(fp),
                              tmax.ctypes.data_as(fp), n, int(any_hit), out.ctypes.data), "trace")
        return out

    def primObject(self, prim: int):
        """HitInfo::obj / m_proxy of a hit id: (mesh id, triangle index, instance or -1)."""
        m, t, i = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().mrt_scene_prim_object(self.handle, int(prim), C.byref(m), C.byref(t), C.byref(i)), "prim_object")
        return m.value, t.value, i.value

    def trace(self, hitInfo: HitInfo, ray: Ray, tMin=0.001) -> bool:
        """Scene::trace(threadID, HitInfo&, const Ray&, tMin): hitInfo.t is tMax in, t out."""
        r = self.traceBatch([ray.o], [ray.d], tMin, hitInfo.t)[0]
        if r["prim"] < 0:
            return False
        hitInfo.t, hitInfo.a, hitInfo.b, hitInfo.obj = float(r["t"]), float(r["a"]), float(r["b"]), int(r["prim"])
        return True
