// miro_shim.h -- the reference-side C++ bridge to libmrt (include/mrt.h).
//
// These are stand-in declarations with the reference's memory layout and member
// names (not its code): what a maintainer of bitfrozen/rendering-algorithms-
// raytracer would keep, with Scene::preCalc / raytraceImage / trace
// re-implemented on top of the C-ABI.  They cover exactly what the bridge reads:
//   Vector3        16 B: x y z + pad            (src/Vector3.h:19)
//   TriangleMesh   m_vertices / m_normals (Vector3 arrays), m_vertexIndices /
//                  m_normalIndices (TupleI3), m_numTris (src/TriangleMesh.h:27-49)
//   Object         m_material, m_mesh, m_index: one triangle (src/Object.h:49-77)
//   Lambert/Blinn  material parameters (src/Lambert.h, src/Blinn.h:59-70,
//                  src/Material.h:30-44)
//   PointLight /   src/PointLight.h, src/RectangleLight.h, src/Light.h:14-46
//   RectangleLight
//   Camera         eye / lookAt / up / fov (src/Camera.h:26-45)
//   Image          8-bit RGB pixels, row 0 = bottom (src/Image.h:7-40)
//   HitInfo        obj, m_proxy, t, a, b (src/Ray.h:185-200)
//   Scene          addObject / addLight / preCalc / raytraceImage / trace
//                  (src/Scene.h:17-37)
// Everything the GPU computes goes through mrt_* calls in miro_shim.cpp.
#pragma once
#include <stdint.h>

#include <vector>

#include "../include/mrt.h"

namespace miro {

struct alignas(16) Vector3 {
    float x = 0.f, y = 0.f, z = 0.f, pad = 1.f;   // the __dummy lane of the reference's SSE union
    Vector3() = default;
    Vector3(float s) : x(s), y(s), z(s) {}
    Vector3(float a, float b, float c) : x(a), y(b), z(c) {}
};
static_assert(sizeof(Vector3) == 16, "Vector3 is one SSE register in the reference");

struct TupleI3 {
    uint32_t x, y, z;
};

struct TriangleMesh {
    Vector3* m_normals = nullptr;
    Vector3* m_vertices = nullptr;
    TupleI3* m_normalIndices = nullptr;
    TupleI3* m_vertexIndices = nullptr;
    uint32_t m_numTris = 0;
};

struct Material {
    bool m_disperse = false;   // src/Material.h:45 (read by Blinn::shade only)
    virtual ~Material() = default;
};
struct Lambert : Material {
    Vector3 m_kd{1.f}, m_ka{0.f};
    explicit Lambert(const Vector3& kd = Vector3(1.f), const Vector3& ka = Vector3(0.f)) : m_kd(kd), m_ka(ka) {}
};
struct Blinn : Material {
    Vector3 m_kd{1.f}, m_ka{0.f}, m_ks{1.f};
    float m_ior[3] = {1.5f, 1.5f, 1.5f};
    float m_specExp = 1.f, m_specAmt = 0.f, m_reflectAmt = 0.f, m_refractAmt = 0.f, m_specGloss = 1.f;
    float m_lightEmitted = 0.f, m_translucency = 0.f;
    Vector3 m_Le{0.f};
    bool m_sampleEnv = true;
    explicit Blinn(const Vector3& kd = Vector3(1.f)) : m_kd(kd) {}
};

struct Light {
    float m_power = 0.f;
    int m_numSamples = 1;
    bool m_castShadows = true;
    float m_noiseThreshold = 0.001f;
    virtual ~Light() = default;
};
struct PointLight : Light {
    Vector3 m_position;
};
struct RectangleLight : Light {
    Vector3 m_v1, m_v2, m_v3;
};

struct Object {
    const Material* m_material = nullptr;
    TriangleMesh* m_mesh = nullptr;
    uint32_t m_index = 0;
    Object(const Material* m, TriangleMesh* mesh, uint32_t i) : m_material(m), m_mesh(mesh), m_index(i) {}
};
using Objects = std::vector<Object*>;
using Lights = std::vector<Light*>;

struct Camera {
    Vector3 m_eye, m_lookAt{0.f, 0.f, -1.f}, m_up{0.f, 1.f, 0.f};
    float m_fov = 45.f;
    float m_focusPlane = 1.0f, m_aperture = 0.0f, m_shutterSpeed = 0.001f;   // src/Camera.cpp:21-23
};

struct Image {
    struct Pixel {
        unsigned char r, g, b;
    };
    std::vector<Pixel> m_pixels;
    int m_width = 0, m_height = 0;
    void resize(int w, int h) {
        m_width = w;
        m_height = h;
        m_pixels.assign((size_t)w * h, Pixel{0, 0, 0});
    }
};

struct Ray {
    float o[4] = {0, 0, 0, 1}, d[4] = {0, 0, 1, 0};
};

struct ProxyObject;  // instancing is exposed as an instance index here
struct HitInfo {
    Object* obj = nullptr;
    ProxyObject* m_proxy = nullptr;
    int32_t m_instance = -1;   // the ProxyObject's instance index (mrt_hit.inst)
    float t = 1e12f, a = 0.f, b = 0.f;
};

class Scene {
   public:
    Scene() = default;
    ~Scene();
    void addObject(Object* o) { m_objects.push_back(o); }
    void addLight(Light* l) { m_lights.push_back(l); }
    void setBGColor(const Vector3& c) { m_BGColor = c; }
    // Scene::preCalc -> BVH::build: marshals the objects (in order, so hit ids
    // are object indices), materials and lights into an mrt_scene and builds it.
    // Returns 0 or an MRT_ERR_* code (mrt_last_error() has the message).
    int preCalc();
    // Scene::raytraceImage: 1 spp (or adaptive) frame on the GPU, written into img.
    int raytraceImage(Camera* cam, Image* img);
    // Scene::trace: closest hit, hitInfo.t = tMax in / t out, obj = the hit Object*.
    bool trace(unsigned int threadID, HitInfo& hitInfo, const Ray& ray, float tMin = 0.001f) const;
    // Scene::trace over n rays in one launch (the form GPU callers should use).
    int traceBatch(const Ray* rays, HitInfo* hits, size_t n, float tMin = 0.001f) const;

    bool m_pathTrace = false;
    int m_numPaths = 1, m_minSubdivs = 1, m_maxSubdivs = 1, m_maxBounces = 10;
    float m_noiseThreshold = 0.01f;
    // buckets b -> m_devices[b % n] (mrt_render_opts.devices); empty = device 0
    std::vector<int32_t> m_devices;

   protected:
    Objects m_objects;
    Lights m_lights;
    Vector3 m_BGColor{0.f};
    mrt_scene* m_gpu = nullptr;
};

}  // namespace miro
