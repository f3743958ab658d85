// miro_shim.h -- the reference-side C++ bridge to libmrt (include/mrt.h).
//
// These are stand-in declarations with the reference's memory layout and member
// names (not its code): what a maintainer of bitfrozen/rendering-algorithms-
// raytracer would keep, with Scene::preCalc / raytraceImage / trace
// re-implemented on top of the C-ABI.  They cover exactly what the bridge reads:
//   Vector3        16 B: x y z + pad            (src/Vector3.h:19)
//   TriangleMesh   m_vertices / m_normals (Vector3 arrays), m_vertexIndices /
//                  m_normalIndices / m_texCoordIndices (TupleI3), m_texCoords
//                  (16-B VectorR2), m_numTris (src/TriangleMesh.h:27-49)
//   Object         m_material, m_mesh, m_index: one triangle (src/Object.h:49-77)
//   MBObject       + m_mesh_t2 (src/MBObject.h:10-25)
//   ProxyObject    m_objects, m_BVH, the 4x4 transform; setupProxy /
//                  setupMultiProxy (src/ProxyObject.h, src/ProxyObject.cpp:5-12,131-167)
//   Lambert/Blinn  material parameters and the Material maps / env map
//                  (src/Lambert.h, src/Blinn.h:59-70, src/Material.h:19-45)
//   RawImage /     m_rawData, m_width, m_height, m_imageType; loadImage
//   Texture        (src/RawImage.h, src/Texture.h)
//   PointLight /   src/PointLight.h, src/RectangleLight.h, src/DomeLight.h:45-64,
//   RectangleLight src/Light.h:14-46 (m_fastShadows)
//   / DomeLight
//   Camera         eye / lookAt / up / fov / lens / shutter (src/Camera.h:26-45)
//   Image          8-bit RGB pixels, row 0 = bottom (src/Image.h:7-40)
//   HitInfo        obj, m_proxy, t, a, b (src/Ray.h:185-200)
//   Scene          addObject / addLight / setEnvMap / preCalc / raytraceImage /
//                  trace (src/Scene.h:17-37)
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
struct alignas(16) VectorR2 {   // ALIGN_SSE struct VectorR2 {float x, y;} (src/TriangleMesh.h:32-35)
    float x, y;
};
static_assert(sizeof(VectorR2) == 16, "VectorR2 is 16-byte aligned in the reference");

// Matrix4x4 (src/Matrix4x4.h): row-major m[row][col], identity by default.
struct Matrix4x4 {
    float m[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
};

struct TriangleMesh {
    Vector3* m_normals = nullptr;
    Vector3* m_vertices = nullptr;
    VectorR2* m_texCoords = nullptr;
    TupleI3* m_normalIndices = nullptr;
    TupleI3* m_vertexIndices = nullptr;
    TupleI3* m_texCoordIndices = nullptr;
    uint32_t m_numTris = 0;
    // TriangleMesh::load(file, ctm) (src/TriangleMeshLoad.cpp:50-214) through
    // libmrt's loader, which restates the reference's bit for bit; the arrays
    // are owned by this mesh.  Returns false when the file cannot be loaded.
    bool load(const char* file, const Matrix4x4& ctm = Matrix4x4());
    // TriangleMesh::createSingleTriangle + setV1..3 / setN1..3 (src/TriangleMesh.cpp:11-42)
    void createSingleTriangle();
    void setV1(const Vector3& v) { m_vertices[0] = v; }
    void setV2(const Vector3& v) { m_vertices[1] = v; }
    void setV3(const Vector3& v) { m_vertices[2] = v; }
    void setN1(const Vector3& n) { m_normals[0] = n; }
    void setN2(const Vector3& n) { m_normals[1] = n; }
    void setN3(const Vector3& n) { m_normals[2] = n; }

    std::vector<Vector3> m_vstore, m_nstore;   // storage of loaded / created meshes
    std::vector<VectorR2> m_tstore;
    std::vector<TupleI3> m_vistore, m_nistore, m_tistore;
};

// RawImage (src/RawImage.h): float pixels, m_imageType channels per texel.
enum ImageType { RGB, RGBA, GRAYSCALE, HDR };   // src/RawImage.h:4-9
struct RawImage {
    float* m_rawData = nullptr;
    int m_width = 0, m_height = 0;
    ImageType m_imageType = RGB;
    RawImage() = default;
    RawImage(int w, int h, float* data, ImageType t) : m_rawData(data), m_width(w), m_height(h), m_imageType(t) {}
    // RawImage::loadImage by extension (.tga / .ppm / .hdr, src/RawImage.cpp:16-188)
    // through libmrt's restated loaders; false when the file cannot be read.
    bool loadImage(const char* filename);
    std::vector<float> m_store;
};
struct Texture {
    RawImage* m_image = nullptr;
    Texture() = default;
    explicit Texture(RawImage* image) : m_image(image) {}
};

struct Material {
    Texture* m_colorMap = nullptr;
    Texture* m_alphaMap = nullptr;
    Texture* m_specularMap = nullptr;
    Texture* m_reflectMap = nullptr;
    Texture* m_refractMap = nullptr;
    Texture* m_normalMap = nullptr;
    Texture* m_envMap = nullptr;      // Material::setEnvMap (mrt_scene_set_material_env_map)
    float m_envExposure = 1.f;
    bool m_sampleEnv = true;
    float m_translucency = 0.f;
    bool m_disperse = false;          // src/Material.h:45 (read by Blinn::shade only)
    void setColorMap(Texture* t) { m_colorMap = t; }
    void setAlphaMap(Texture* t) { m_alphaMap = t; }
    void setNormalMap(Texture* t) { m_normalMap = t; }
    void setSpecularMap(Texture* t) { m_specularMap = t; }
    void setReflectMap(Texture* t) { m_reflectMap = t; }
    void setRefractMap(Texture* t) { m_refractMap = t; }
    void setEnvMap(Texture* t) { m_envMap = t; }
    void setEnvExposure(float e) { m_envExposure = e; }
    void setSampleEnv(bool b) { m_sampleEnv = b; }
    void setTranslucency(float t) { m_translucency = t; }
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
    float m_lightEmitted = 0.f;
    Vector3 m_Le{0.f};
    explicit Blinn(const Vector3& kd = Vector3(1.f)) : m_kd(kd) {}
};

struct Light {
    float m_power = 0.f;
    int m_numSamples = 1;
    bool m_castShadows = true;
    bool m_fastShadows = true;   // src/Light.h:16 (false: a point light casts no shadow, its walk never traces; rect / dome walk through refractive hits)
    float m_noiseThreshold = 0.001f;
    void setPower(float f) { m_power = f; }
    void setSamples(int n) { m_numSamples = n; }
    void setCastShadows(bool c) { m_castShadows = c; }
    void setFastShadows(bool c) { m_fastShadows = c; }
    void setNoiseThreshold(float t) { m_noiseThreshold = t; }
    virtual ~Light() = default;
};
struct PointLight : Light {
    Vector3 m_position;
};
struct RectangleLight : Light {
    Vector3 m_v1, m_v2, m_v3;
};
struct DomeLight : Light {   // src/DomeLight.h:45-64: m_lightMap, m_Gain (setPower)
    Texture* m_lightMap = nullptr;
    float m_Gain = 1.f;
    void setTexture(Texture* t) { m_lightMap = t; }
    void setPower(float f) { m_Gain = f; }
};

struct Object {
    const Material* m_material = nullptr;
    TriangleMesh* m_mesh = nullptr;
    uint32_t m_index = 0;
    Object() = default;
    Object(const Material* m, TriangleMesh* mesh, uint32_t i) : m_material(m), m_mesh(mesh), m_index(i) {}
    void setMesh(TriangleMesh* m) { m_mesh = m; }
    void setIndex(uint32_t i) { m_index = i; }
    void setMaterial(const Material* m) { m_material = m; }
    virtual ~Object() = default;
};
using Objects = std::vector<Object*>;
using Lights = std::vector<Light*>;

// MBObject(material, mesh, mesh_t2, i) (src/MBObject.cpp:7-11): a ray of time t
// meets t * mesh_t2 + (1 - t) * mesh.
struct MBObject : Object {
    TriangleMesh* m_mesh_t2 = nullptr;
    MBObject(const Material* m, TriangleMesh* mesh, TriangleMesh* mesh2, uint32_t i) : Object(m, mesh, i), m_mesh_t2(mesh2) {}
};

// A proxy's hierarchy: BVH::build(Objects*) records the objects; libmrt builds
// the tree when the first instance of it reaches Scene::preCalc.
struct BVH {
    Objects* m_objects = nullptr;
    void build(Objects* objs) { m_objects = objs; }
};

struct ProxyObject : Object {
    Objects* m_objects = nullptr;
    BVH* m_BVH = nullptr;
    Matrix4x4 m_transform;
    ProxyObject(Objects* m = nullptr, BVH* b = nullptr, const Matrix4x4& t = Matrix4x4())
        : m_objects(m), m_BVH(b), m_transform(t) {}
    // src/ProxyObject.cpp:131-167: one Object per triangle, each mesh's triangles
    // last to first, then BVH::build.  (The Object arrays live as long as the
    // program, as in the reference.)
    static void setupProxy(TriangleMesh* mesh, const Material* mat, Objects* m, BVH* b);
    static void setupMultiProxy(TriangleMesh* mesh[], int numObjs, const Material* mat[], Objects* m, BVH* b);
};

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

struct HitInfo {
    Object* obj = nullptr;
    ProxyObject* m_proxy = nullptr;   // the instance a BLAS object was hit through (obj is then its Object)
    int32_t m_instance = -1;          // that ProxyObject's instance index (mrt_hit.inst)
    float t = 1e12f, a = 0.f, b = 0.f;
};

class Scene {
   public:
    Scene() = default;
    ~Scene();
    void addObject(Object* o) { m_objects.push_back(o); }
    void addLight(Light* l) { m_lights.push_back(l); }
    void setBGColor(const Vector3& c) { m_BGColor = c; }
    void setEnvMap(Texture* t) { m_envMap = t; }                 // src/Scene.h:23
    void setEnvExposure(float e) { m_envExposure = e; }          // src/Scene.h:24
    const Texture* getEnvMap() const { return m_envMap; }
    // Scene::preCalc -> BVH::build: marshals the objects (in order, so hit ids
    // are object indices), the proxies' BVHs (one per shared BVH) and their
    // instances, materials with their maps, textures and lights into an
    // mrt_scene and builds it.  Returns 0 or an MRT_ERR_* code (mrt_last_error()
    // has the message).
    int preCalc();
    // Scene::raytraceImage: the frame on the GPU, written into img.
    int raytraceImage(Camera* cam, Image* img);
    // Scene::trace: closest hit, hitInfo.t = tMax in / t out; obj = the hit Object*
    // (for an instance hit: the proxy's Object, with m_proxy the ProxyObject).
    bool trace(unsigned int threadID, HitInfo& hitInfo, const Ray& ray, float tMin = 0.001f) const;
    // Scene::trace over n rays in one launch (the form GPU callers should use).
    int traceBatch(const Ray* rays, HitInfo* hits, size_t n, float tMin = 0.001f) const;

    bool m_pathTrace = false;
    int m_numPaths = 1, m_minSubdivs = 1, m_maxSubdivs = 1, m_maxBounces = 10;
    float m_noiseThreshold = 0.01f;
    // buckets b -> m_devices[b % n] (mrt_render_opts.devices); empty = device 0
    std::vector<int32_t> m_devices;
    // the float frame (before Image::Map) and primary hits of the last
    // raytraceImage, kept when m_keepFrame is set (parity checks)
    bool m_keepFrame = false;
    std::vector<float> m_lastRGB;
    std::vector<HitInfo> m_lastHits;

   protected:
    void to_hit(const mrt_hit& r, HitInfo& h) const;
    Objects m_objects;
    Lights m_lights;
    Vector3 m_BGColor{0.f};
    Texture* m_envMap = nullptr;
    float m_envExposure = 1.f;
    mrt_scene* m_gpu = nullptr;
    // instance i of the C-ABI: its ProxyObject and the first hit id of its BLAS objects
    std::vector<ProxyObject*> m_instProxy;
    std::vector<int32_t> m_instBase;
};

}  // namespace miro
