/*
 * mrt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the reference (bitfrozen/rendering-algorithms-raytracer)
 * hot path: OBJ load -> binned-SAH BVH -> QBVH collapse -> stack traversal ->
 * 4-wide Moller-Trumbore -> Lambert/Blinn direct shading + PointLight /
 * RectangleLight shadow rays -> gamma-LUT tone map.  Every function cites the
 * reference file:line it restates.
 *
 * It is the CHECKER for the MI355X product (rendering-algorithms-raytracer_amd/),
 * never part of it: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * PARITY UNPINNED against reference outputs: the reference cannot be compiled in
 * this image without stand-ins for headers the image lacks (<GL/glut.h>,
 * <Windows.h>; reference src/OpenGL.h:13, src/Scene.cpp:8) and it ships no tests,
 * golden images or fixtures.  What IS pinned: the x86 RCPSS/RSQRTSS emulation
 * (exhaustively, all 2^32 inputs, against live instructions), the OBJ-loader
 * scaling facts and the QBVH node/leaf counts measured from the reference in
 * SURVEY.md (tests/test_oracle_pins.py).
 */
#ifndef MRT_ORACLE_H
#define MRT_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oro_scene oro_scene;

enum { ORO_LAMBERT = 0, ORO_BLINN = 1 };
enum { ORO_POINT_LIGHT = 0, ORO_RECT_LIGHT = 1, ORO_DOME_LIGHT = 2 };

typedef struct {
    int type;               /* ORO_LAMBERT / ORO_BLINN                        */
    float kd[3], ka[3], ks[3];
    float specExp, specAmt; /* Blinn only (reference src/Blinn.h:11-22)       */
    float reflect, refract; /* Blinn m_reflectAmt / m_refractAmt               */
    float ior;              /* Blinn m_ior (src/Blinn.cpp:25-27)                */
    float gloss;            /* Blinn m_specGloss (src/Blinn.h:42,65)           */
    float translucency;     /* Material::m_translucency (src/Material.h:30,44) */
    float le[3];            /* Blinn m_Le (src/Blinn.h:64), added to shade()   */
    float emitted;          /* Blinn m_lightEmitted (src/Blinn.h:63)           */
    int sample_env;         /* Material::m_sampleEnv (src/Material.h:43)       */
    int disperse;           /* Material::m_disperse (src/Material.h:45)        */
    float ior3[3];          /* Blinn m_ior[0..2] (src/Blinn.h:59): dispersion  */
} oro_material;

typedef struct {
    int type;               /* ORO_POINT_LIGHT / ORO_RECT_LIGHT               */
    float pos[3];           /* point light position                            */
    float v1[3], v2[3], v3[3]; /* rect light parallelogram                     */
    float power;            /* as passed to setPower()                         */
    int samples;            /* rect light samples (Light::m_numSamples)        */
    float noiseThreshold;   /* Light::m_noiseThreshold (default epsilon)       */
    int castShadows;
    int texture;            /* dome light: texture id (oro_scene_add_texture)  */
    int transparent;        /* Light::setFastShadows(false): rect / dome lights walk
                               through refractive hits (0 = fast shadows)       */
} oro_light;

typedef struct {
    float eye[3], up[3], lookAt[3];
    float fov;              /* degrees, as setFOV()                            */
    float aperture, focusPlane;   /* Camera::m_aperture / m_focusPlane (DOF)   */
    float shutterSpeed;     /* Camera::m_shutterSpeed (getTimeSample)          */
} oro_camera;

typedef struct {
    float t, a, b;
    int32_t prim;           /* -1 on miss                                      */
} oro_hit;

/* mesh-level helpers ------------------------------------------------------- */
/* Load an OBJ exactly as TriangleMesh::loadObj (src/TriangleMeshLoad.cpp:99-214).
 * ctm: 16 floats row-major (m11..m44) or NULL for identity.
 * Returns a mesh handle index inside the scene (>=0) or negative on error. */
int oro_scene_add_obj(oro_scene* s, const char* path, const float* ctm, int material);
/* Raw triangle mesh (TriangleMesh::createSingleTriangle-style: no ctm, no rcp). */
int oro_scene_add_mesh(oro_scene* s, int nv, const float* verts, int nn, const float* normals,
                       int nt, const uint32_t* vidx, const uint32_t* nidx, int material);
int oro_mesh_info(const oro_scene* s, int mesh, int* nv, int* nn, int* nt);
int oro_mesh_export(const oro_scene* s, int mesh, float* verts, float* normals,
                    uint32_t* vidx, uint32_t* nidx);

oro_scene* oro_scene_create(void);
void oro_scene_destroy(oro_scene* s);
int oro_scene_add_material(oro_scene* s, const oro_material* m);
int oro_scene_add_light(oro_scene* s, const oro_light* l);
void oro_scene_set_bg(oro_scene* s, float r, float g, float b);
/* libm convention of Fresnel's sin, Blinn's pow and the cosine sampler's cos / sin:
 * 1 (default) = the float overloads the reference's source calls (glibc sinf / powf /
 * cosf), 0 = the same functions in double, rounded once (the device's convention).
 * atan2 / acos are glibc's atan2f / acosf either way (oro_ibl.h).  Process-wide;
 * returns the previous setting. */
int oro_set_libm(int float_overloads);
void oro_scene_set_num_paths(oro_scene* s, int n);
/* Scene::m_pathTrace / m_maxBounces / m_sampleLightFromEnv (src/Scene.h:40-64) */
int oro_scene_set_path_trace(oro_scene* s, int enable, int max_bounces, int sample_env);
/* Scene::setMinSubdivs / setMaxSubdivs / setNoise (src/Scene.h:42-55); 0 = OK */
int oro_scene_set_subdivs(oro_scene* s, int min_subdivs, int max_subdivs, float noise);
/* Scene::preCalc -> BVH::build (src/Scene.cpp:62-79, src/BVH.cpp:457-575). */
int oro_scene_build(oro_scene* s);
/* ProxyObject instancing (src/ProxyObject.cpp:5-95,131-167).  oro_scene_make_blas
 * builds a proxy BVH from whole meshes (ProxyObject::setupMultiProxy: meshes in
 * order, each one's triangles last to first); those meshes leave the world
 * object list.  oro_scene_add_instance adds one ProxyObject (row-major 4x4) to
 * the world objects, in add order with the world meshes.  Hit ids: world
 * objects 0..n-1 (a proxy's own id never hits), then instance i's BLAS objects
 * at n + (sum of the BLAS sizes of instances < i) + BLAS object index. */
int oro_scene_make_blas(oro_scene* s, const int* meshes, int n_meshes);
int oro_scene_add_instance(oro_scene* s, int blas, const float* m16);
int oro_blas_info(const oro_scene* s, int blas, int* n_nodes, int* n_leaves, int* n_prims);
int oro_blas_export(const oro_scene* s, int blas, float* node_boxes, int32_t* node_child, float* leaf_tris,
                    int32_t* leaf_prims);

/* Canonical QBVH export (preorder node numbering, leaf numbering = nodeNum). */
int oro_qbvh_info(const oro_scene* s, int* n_nodes, int* n_leaves, int* n_prims,
                  int* bin_nodes, int* bin_leaves, int* max_depth);
int oro_qbvh_export(const oro_scene* s, float* node_boxes /*24/node*/, int32_t* node_child /*4/node*/,
                    float* leaf_tris /*36/leaf*/, int32_t* leaf_prims /*4/leaf*/);

/* Scene::trace for a batch (closest hit; reference src/BVH.cpp:1112-1178). */
int oro_trace(const oro_scene* s, size_t n, const float* o /*3n*/, const float* d /*3n*/,
              const float* tmin, const float* tmax, oro_hit* out,
              uint32_t* node_visits, uint32_t* leaf_visits);

/* Render rows [y0,y1) x columns [x0,x1) of a W x H frame (row 0 = bottom),
 * Scene::adaptiveSampleScene (src/Scene.cpp:252-293; 1 spp unless
 * oro_scene_set_subdivs raised the subdivisions), Blinn reflection /
 * refraction rays (src/Blinn.cpp:238-330) for materials with reflect / refract.
 * rgb: W*H*3 floats (before Image::Map), rgb8: W*H*3 (after Map), hit: W*H
 * primary hit records, shadow: W*H bitmask of occluded lights, may be NULL.
 * counters[7] (nullable) += {primary rays, shadow rays, node visits, leaf visits,
 *                            primary-ray node visits, primary-ray leaf visits,
 *                            reflection + refraction rays}.
 * n_threads > 1 uses OpenMP over rows (the oracle is deterministic per pixel). */
int oro_render(const oro_scene* s, const oro_camera* cam, int W, int H,
               int x0, int y0, int x1, int y1,
               float* rgb, uint8_t* rgb8, oro_hit* hit, uint32_t* shadow,
               uint64_t* counters, int n_threads);

/* image-based lighting (src/hdrloader.cpp, src/Texture.cpp, src/DomeLight.*) -- */
/* HDRLoader::load: header only (sizes), then W*H*3 floats, row 0 = top.
 * 0 on success, negative on error (oro_ibl.c lists the rejected inputs). */
int oro_hdr_info(const char* path, int* w, int* h);
int oro_hdr_load(const char* path, float* rgb, int w, int h);
/* RawImage + Texture: copies W*H*3 floats (row 0 = top); returns texture id. */
int oro_scene_add_texture(oro_scene* s, const float* rgb, int w, int h);
/* RawImage::loadImage (TGA / PPM / HDR): size and type (0 HDR, 1 gray, 3 RGB, 4 RGBA), then
 * w*h*channels floats in RawImage m_rawData order */
int oro_image_info(const char* path, int* w, int* h, int* type);
int oro_image_load(const char* path, float* data, int w, int h);
/* a texture of any RawImage type (channels per texel: 1, 3, 4; 0 = HDR, 3) */
int oro_scene_add_texture_typed(oro_scene* s, const float* data, int w, int h, int type);
/* Material maps: color, normal, specular, reflect, refract, alpha (texture id or -1) */
int oro_scene_set_material_maps(oro_scene* s, int material, const int maps[6]);
/* TriangleMesh m_texCoords (ntc x 2 floats) / m_texCoordIndices (nt x 3) of a mesh */
int oro_mesh_set_texcoords(oro_scene* s, int mesh, int ntc, const float* uv, const uint32_t* tidx);
int oro_mesh_texcoords(const oro_scene* s, int mesh, int* ntc, float* uv, uint32_t* tidx);
/* MBObject (src/MBObject.cpp): every triangle of the mesh moves from its vertices
 * (time 0) to verts2 (time 1, nv x 3 floats) over the camera's time sample */
int oro_mesh_set_motion(oro_scene* s, int mesh, const float* verts2);
/* Scene::setEnvMap + setEnvExposure (src/Scene.h:23-24); texture -1 clears. */
int oro_scene_set_env_map(oro_scene* s, int texture, float exposure);
/* Material::setEnvMap + m_envExposure (src/Material.h:19,41-42): a Blinn
 * material's missed reflection / refraction / GI rays take this map instead of
 * the scene's (Material::getEnvironmentColor, src/Material.cpp:44-64); -1 clears */
int oro_scene_set_material_env_map(oro_scene* s, int material, int texture, float exposure);
/* DomeLight::setTexture tables of light `light` (src/DomeLight.cpp:8-78):
 * cdf_u[nu+1], func_u[nu], cdf_v[nu*(nv+1)], func_v[nu*nv], func_int[nu+1]
 * (column integrals, then the u integral), cos_u/sin_u[nu+1], cos_v/sin_v[nv+1]. */
int oro_dome_info(const oro_scene* s, int light, int* nu, int* nv);
int oro_dome_export(const oro_scene* s, int light, float* cdf_u, float* func_u, float* cdf_v, float* func_v,
                    float* func_int, float* cos_u, float* sin_u, float* cos_v, float* sin_v);
/* Texture::getLookupXYZ3 of texture `tex` for n directions (3n floats in/out). */
int oro_texture_lookup_dir(const oro_scene* s, int tex, int n, const float* dirs, float* out);

/* numerics probes (for tests) */
float oro_x86_rcp(float x);
/* glibc acosf(x) (fn 0) / atan2f(y, x) (fn 1) over n inputs; 0 = ok */
int oro_libm_eval(int fn, size_t n, const float* x, const float* y, float* out);
float oro_x86_rsqrt(float x);
float oro_rcp_nr(float x);
float oro_rsqrt_nr(float x);
void oro_gamma_table(uint8_t* lut32769);
/* counter-based RNG used in place of the reference's global MT pool.  Keys:
 * skey = eye-ray sample * 1024 + path, dim = (chain level + 1) << 24 | k for the
 * k-th draw of one shade() call (the camera ray's draws are dims 0-2). */
float oro_rand(uint32_t pixel, uint32_t sample, uint32_t dim, uint32_t seed);

#ifdef __cplusplus
}
#endif
#endif
