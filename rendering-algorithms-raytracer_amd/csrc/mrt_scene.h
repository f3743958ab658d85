// mrt_scene.h -- internal scene object behind the opaque mrt_scene handle.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mrt.h"
#include "mrt_math.h"
#include "mrt_types.h"

namespace mrt {

// Packed x86 approximation tables (host copies; uploaded to the device).
const uint16_t* host_rcp_table();
const uint16_t* host_rsqrt_table();
const uint8_t* host_gamma_lut();  // 32769 entries, Image::generateGammaTables
const float* host_gamma_float_lut();  // Image::linear_to_gammaF, 32769 entries

struct Mesh {
    std::vector<v3> verts, normals;
    std::vector<uint32_t> vidx, nidx;
    int material = 0;
    // TriangleMesh m_texCoords (u, v pairs) / m_texCoordIndices (empty: none), and
    // the per-normal tangent frame TriangleMesh::preCalc derives from them
    std::vector<float> uv;
    std::vector<uint32_t> tidx;
    std::vector<v3> tan, btan;
    // MBObject m_mesh_t2 vertices (motion blur, src/MBObject.cpp): empty = static
    std::vector<v3> verts2;
    int32_t nt() const { return (int32_t)(vidx.size() / 3); }
};

// RawImage types (src/RawImage.h ImageType): floats per texel 3 (HDR), 1, 3, 4
enum { kTexHDR = 0, kTexGray = 1, kTexRGB = 3, kTexRGBA = 4 };
inline int tex_channels(int type) { return type == kTexGray ? 1 : type == kTexRGBA ? 4 : 3; }

struct Texture {                // RawImage (src/RawImage.h): W*H*channels floats (m_rawData order)
    std::vector<float> rgb;
    int32_t W = 0, H = 0;
    int32_t type = kTexHDR;
};

struct DomeTables {             // DomeLight::setTexture (src/DomeLight.cpp:8-78)
    int32_t tex = -1, nu = 0, nv = 0;
    std::vector<float> func_u, cdf_u, func_v, cdf_v, int_v, inv_int_v, cos_u, sin_u, cos_v, sin_v;
    float int_u = 0.f, inv_int_u = 0.f;
    // derived lookup tables of the device sampler (not reference state):
    // rad = the lat-long lookup of every table direction (iu, iv) in 0..nu x 0..nv,
    // 4 floats per cell; guide_u / guide_v = CDF guide tables (guide_table)
    std::vector<float> rad;
    std::vector<int32_t> guide_u, guide_v;
};

// A ProxyObject's BVH (ProxyObject::setupMultiProxy, src/ProxyObject.cpp:149-167):
// objects are the meshes in order, each mesh's triangles last to first.
struct Blas {
    std::vector<int32_t> meshes;
    std::vector<int32_t> obj_mesh, obj_tri;
    std::vector<QNode> nodes;
    std::vector<QLeaf> leaves;
};

// ProxyObject + ProxyMatrix (src/ProxyObject.cpp:5-12, src/ProxyMatrix.cpp:3-8)
struct Instance {
    float m[16], inv[16], inv_t[16];  // m_transform, m_inverse, m_invTranspose (row-major)
    float box[6];                     // ProxyObject::getAABB: min xyz, max xyz
    int32_t blas;
    int32_t hit_base;                 // hit id of its BLAS object 0 (set by build_qbvh)
};

struct DeviceState;  // defined in mrt_device.hip

struct Scene {
    std::vector<Mesh> meshes;
    std::vector<DevMaterial> materials;
    std::vector<DevLight> lights;
    std::vector<Texture> textures;
    std::vector<DomeTables> domes;
    int32_t env_tex = -1;           // Scene::m_envMap (-1: background colour)
    float env_exposure = 1.f;       // Scene::m_envExposure
    float bg[3] = {0.f, 0.f, 0.f};
    int num_paths = 1;
    // Scene::m_pathTrace / m_maxBounces / m_sampleLightFromEnv (src/Scene.cpp:17-19)
    bool path_trace = false;
    int max_bounces = 10;
    bool sample_env = false;
    // Scene::m_minSubdivs / m_maxSubdivs / m_noiseThreshold (src/Scene.cpp:20-22)
    int min_subdivs = 1, max_subdivs = 1;
    float noise_threshold = 0.01f;
    // world object groups in add order: mesh id (>= 0) or ~instance id
    std::vector<int32_t> groups;
    std::vector<int32_t> mesh_blas;   // per mesh: owning BLAS, -1 = world geometry
    std::vector<Blas> blas;
    std::vector<Instance> instances;

    int32_t push_mesh(Mesh&& m) {
        meshes.push_back(std::move(m));
        mesh_blas.push_back(-1);
        groups.push_back((int32_t)meshes.size() - 1);
        built = false;
        dev_dirty = true;
        return (int32_t)meshes.size() - 1;
    }

    // objects in scene order (makeMeshObjs): global prim id -> (mesh, tri)
    std::vector<int32_t> obj_mesh, obj_tri, obj_inst;  // obj_inst >= 0: a ProxyObject
    // QBVH
    std::vector<QNode> nodes;
    std::vector<QLeaf> leaves;
    mrt_bvh_info info{};
    bool built = false;

    // device replicas (one per HIP device used, mrt_render_opts.devices); `dev` is
    // the one the last call used.  dev_dirty: the host scene changed, every
    // replica is re-uploaded on its next use.
    std::vector<DeviceState*> devs;
    DeviceState* dev = nullptr;
    bool dev_dirty = true;
    mrt_stats last{};
    // the last call was a multi-device mrt_render: `last` already holds the summed
    // counters of its shares (last_rc: MRT_ERR_OVERFLOW if a share overflowed)
    bool stats_final = false;
    int last_rc = 0;
};

// host_build.cpp
int load_obj(const char* path, const float* ctm16, Mesh& out, std::string& err);
int build_qbvh(Scene& s, std::string& err);
int make_blas(Scene& s, const int32_t* meshes, int n_meshes, std::string& err);
int add_instance(Scene& s, int32_t blas, const float* m16, std::string& err);
// host_texture.cpp
int load_hdr(const char* path, int& W, int& H, std::vector<float>* rgb, std::string& err);
int build_dome(const Texture& t, DomeTables& d, std::string& err);
// RawImage::loadImage (TGA / PPM / HDR by extension); data == nullptr: size + type only
int load_image(const char* path, int& W, int& H, int& type, std::vector<float>* data, std::string& err);
// TriangleMesh::preCalc's tangent frame (src/TriangleMesh.cpp:105-148)
void mesh_tangents(Mesh& m);

void set_error(const std::string& msg);

}  // namespace mrt

struct mrt_scene {
    mrt::Scene impl;
};
