// mrt_types.h -- scene data as it lives in HBM (shared host/device layout).
#pragma once
#include <stdint.h>

namespace mrt {

// 4-wide node, one 128-B line.  SoA boxes exactly as QBVH_Node
// (reference src/BVH.h:83-109): minX[4] minY[4] minZ[4] maxX[4] maxY[4] maxZ[4].
// child[i] >= 0: inner node index; child[i] == INT32_MIN: empty slot;
// otherwise ~child[i] is a leaf-packet index.  The device copy keeps its slot kinds
// in pad[0] (slot_kinds, mrt_kernels.h).
struct alignas(16) QNode {
    float box[24];
    int32_t child[4];
    uint32_t pad[4];
};
static_assert(sizeof(QNode) == 128, "QNode must be one 128-B line");

// 4-triangle packet, TriCache4 (src/BVH.h:37-50): A, e0 = B-A, e1 = C-A (SoA),
// plus global prim ids (-1 = empty lane).  160 B.
struct alignas(16) QLeaf {
    float t[36];
    int32_t prim[4];
};
static_assert(sizeof(QLeaf) == 160, "QLeaf must be 160 B");

// Device copy of a packet: per-triangle AoS (Ax Ay Az e0x e0y e0z e1x e1y e1z)
// so one lane walks its packet a triangle at a time; prim = -1 ends the packet.
struct alignas(16) DLeaf {
    float tri[4][9];
    int32_t prim[4];
};
static_assert(sizeof(DLeaf) == 160, "DLeaf must be 160 B");

static constexpr int32_t kEmptySlot = (int32_t)0x80000000u;

// A ProxyObject on the device (src/ProxyObject.cpp:76-95, src/Ray.cpp:27-31).
struct alignas(16) DevInstance {
    float inv[16];       // ProxyMatrix::m_inverse, row-major: rays into object space
    float inv_t[12];     // m_invTranspose rows 0-2 (4 floats each): normals back to world space
    int32_t root;        // the BLAS root in the scene's node array
    int32_t hit_base;    // hit id of BLAS object 0
    int32_t shade_base;  // PrimShade index of BLAS object 0
    int32_t pad;
};
static_assert(sizeof(DevInstance) == 128, "DevInstance is 128 B");

// Per-triangle shading record: global vertex / normal indices + material.
struct alignas(16) PrimShade {
    uint32_t v[3];
    uint32_t mat;
    uint32_t n[3];
    uint32_t pad;
};
static_assert(sizeof(PrimShade) == 32, "PrimShade is 32 B");

struct DevMaterial {
    int32_t type;
    float kd[3], ka[3], ks[3];
    float spec_exp, spec_amt;
    float reflect, refract;  // Blinn m_reflectAmt / m_refractAmt (src/Blinn.h:62, src/Material.h:73)
    float ior;               // Blinn m_ior[1] (src/Blinn.cpp:25-27): the non-dispersive refraction (src/Blinn.cpp:183)
    float gloss;             // Blinn m_specGloss (src/Blinn.h:42,65): < 1 jitters the reflection vector
    float translucency;      // Material::m_translucency (src/Material.h:30,44): > 0.01 lights the back side
    float le[3];             // Blinn m_Le (src/Blinn.h:64): added to every shade() result (src/Blinn.cpp:335)
    float emitted;           // Blinn m_lightEmitted (src/Blinn.h:63): path-tracing emitter intensity
    int32_t sample_env;      // Material::m_sampleEnv (src/Material.h:43; default true)
    int32_t emitter;         // host-derived: emitted > 0 || le.x + le.y + le.z > 0 (src/Blinn.cpp:47)
    // Material m_colorMap, m_normalMap, m_specularMap, m_reflectMap, m_refractMap,
    // m_alphaMap (src/Material.h:20-25,35-40): texture ids, -1 = none
    int32_t maps[6];
    // Material::m_disperse + Blinn m_ior[0..2] (src/Material.h:45, src/Blinn.h:59):
    // a ray that is not a refraction ray splits into one refraction ray per channel
    int32_t disperse;
    float ior3[3];
    // Material::m_envMap / m_envExposure (src/Material.h:19,41-42): the map a missed
    // reflection / refraction / GI ray of this material takes (-1: the scene's)
    int32_t env;
    float env_exposure;
};
enum { kMapColor = 0, kMapNormal = 1, kMapSpecular = 2, kMapReflect = 3, kMapRefract = 4, kMapAlpha = 5 };

// A material-map texture on the device (Texture + RawImage, src/Texture.h)
struct DevTexture {
    const float* data;   // W*H*channels floats, RawImage m_rawData order
    int32_t W, H, type;  // type: kTexHDR 0 (3 floats), kTexGray 1, kTexRGB 3, kTexRGBA 4
    int32_t pad;
};

struct DevLight {
    int32_t type;
    float pos[3], v1[3], v2[3], v3[3];
    float power;        // point: m_power; rect: power * rsqrt_nr(area^2) (setPower); dome: m_Gain
    int32_t samples;
    float noise;
    int32_t cast_shadows;
    int32_t dome;       // dome light: index of its DevDome tables (-1 otherwise)
    int32_t transparent;   // rect / dome: Light::m_fastShadows false, the transparency walk (fused kernels)
};

// DomeLight::setTexture products in HBM (src/DomeLight.cpp:8-78): the lat-long
// texture (nu x nv texels, row 0 = top), a Distribution1D over u of the column
// integrals, one over v per column (nu x (nv+1) CDF, row-major by column), and
// the sin / cos tables of the sampled angles.
struct DevDome {
    const float* tex;
    const float* cdf_u;      // nu + 1
    const float* func_u;     // nu
    const float* cdf_v;      // nu * (nv + 1)
    const float* func_v;     // nu * nv
    const float* inv_int_v;  // nu
    const float* cos_u;      // nu + 1
    const float* sin_u;
    const float* cos_v;      // nv + 1
    const float* sin_v;
    float inv_int_u;
    int32_t nu, nv;
    const float* rad;        // (nu + 1) x (nv + 1) x 4: texture lookup of each table direction, row iv
    const int32_t* guide_u;  // nu + 1: CDF guide table of cdf_u (mrt_texture.h dist_sample_guided)
    const int32_t* guide_v;  // nu * (nv + 1): one per column's cdf_v
};

// Camera basis hoisted to the host (bit-identical to the per-ray recompute of
// Camera::eyeRayAdaptive, src/Camera.cpp:116-137).
struct CamParams {
    float eye[3], u[3], v[3], w[3];
    float left, right, bottom, top;
    int32_t W, H;
    float aperture, focus;   // Camera::m_aperture / m_focusPlane (depth of field, src/Camera.cpp:155-174)
    float shutter;           // Camera::m_shutterSpeed (getTimeSample, src/Camera.h:46)
};

static constexpr int kMaxLights = 8;
static constexpr int kMaxBatch = 16;   // cameras (frames) per batched bucket launch (kernel argument)
static constexpr int kMaxMaterials = 64;
static constexpr int kMaxTextures = 64;   // the final scene (config FS) maps 22 textures + 2 light probes

}  // namespace mrt
