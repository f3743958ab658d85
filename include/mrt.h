/*
 * mrt.h -- C-ABI of the MI355X ray engine (libmrt.so).
 *
 * Drop-in boundary for the hot path of bitfrozen/rendering-algorithms-raytracer
 * ("Miro"): per-pixel ray generation -> QBVH traversal -> Moller-Trumbore ->
 * Lambert/Blinn shade + shadow rays.  Plain C types only (no torch / HIP types in
 * the signatures; streams are passed as void*).  Every entry point cites the
 * reference interface it replaces (paths relative to the reference repo).
 *
 * Conventions
 *  - Return value: 0 (MRT_OK) or a negative MRT_ERR_* code; mrt_last_error()
 *    gives a thread-local message.  No C++ exception crosses this ABI
 *    (reference: bool returns + printf, src/TriangleMeshLoad.cpp:53-57).
 *  - Ownership: the library copies every input array; the caller keeps its
 *    buffers.  The scene owns its device memory; mrt_scene_destroy frees all
 *    (reference: Scene never frees Objects, src/Scene.h:17-21).
 *  - Frames are W*H, row 0 = bottom (reference src/Image.cpp:78-87,137-154).
 *  - Numerics are the reference's x86 SSE contract:
 *    hit t/a/b/prim and float RGB are bit-identical to the CPU restatement.
 */
#ifndef MRT_H
#define MRT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRT_ABI_VERSION 10

enum {
    MRT_OK = 0,
    MRT_ERR_INVALID = -1,   /* bad argument / handle                              */
    MRT_ERR_IO = -2,        /* file could not be read / parsed                    */
    MRT_ERR_HIP = -3,       /* HIP runtime failure (device, alloc, launch)        */
    MRT_ERR_BUILD = -4,     /* BVH build failed (degenerate input)                */
    MRT_ERR_NOT_BUILT = -5, /* scene used before mrt_scene_build_bvh              */
    MRT_ERR_OVERFLOW = -6,  /* traversal stack overflow detected on the device    */
    MRT_ERR_NO_DEVICE = -7  /* no HIP device visible                              */
};

enum { MRT_LAMBERT = 0, MRT_BLINN = 1 };                 /* src/Lambert.h, src/Blinn.h */
enum { MRT_POINT_LIGHT = 0, MRT_RECT_LIGHT = 1, MRT_DOME_LIGHT = 2 }; /* src/Light.h:9 lightType_t */

typedef struct mrt_scene mrt_scene;

/* Material as data (replaces virtual Material::shade, src/Material.h:18). */
typedef struct {
    int32_t type;            /* MRT_LAMBERT | MRT_BLINN                               */
    float kd[3], ka[3], ks[3];
    float spec_exp, spec_amt;/* Blinn m_specExp / m_specAmt (src/Blinn.h:59-61)       */
    float le[3];             /* Blinn m_Le, setLightEmittedColor (src/Blinn.h:45,64):
                                added to every Blinn shade() result (src/Blinn.cpp:335) */
    float emitted;           /* Blinn m_lightEmitted, setLightEmittedIntensity
                                (src/Blinn.h:44,63): with path tracing, a GI ray that
                                reaches this surface returns emitted * le
                                (src/Blinn.cpp:46-51).  Both 0 = not an emitter
                                (the Blinn ctor forces 0, src/Blinn.cpp:28-29)     */
} mrt_material;

/* Light as data (replaces virtual Light::sampleLight, src/Light.h:35). */
typedef struct {
    int32_t type;            /* MRT_POINT_LIGHT | MRT_RECT_LIGHT | MRT_DOME_LIGHT      */
    float pos[3];            /* PointLight::setPosition                                */
    float v1[3], v2[3], v3[3];/* RectangleLight::setVertices                           */
    float power;             /* Light::setPower (area scaling applied internally);
                                DomeLight::setPower = m_Gain                           */
    int32_t samples;         /* Light::setSamples                                      */
    float noise_threshold;   /* Light::setNoiseThreshold (default 0.001)               */
    int32_t cast_shadows;    /* Light::setCastShadows (a dome light always casts)      */
    int32_t texture;         /* MRT_DOME_LIGHT: DomeLight::setTexture, a texture id of
                                mrt_scene_add_texture (-1 for the other lights)        */
    int32_t transparent_shadows; /* 1 = Light::setFastShadows(false) (src/Light.h:24).
                                Point light: its walk (src/PointLight.cpp:49-70) starts
                                with sampleHit.t = distance and loops while t < distance,
                                so it never traces -- the light casts no shadow, as the
                                reference.  Rectangle / dome lights: the transparency
                                walk of src/RectangleLight.cpp:93-116 / src/DomeLight.cpp:
                                123-145 (closest-hit rays through every hit, attenuated
                                by refractAmt at front faces; ABI 9), rendered by the
                                fused kernels.  0 (zero-initialised) = m_fastShadows
                                true, the reference default (ABI 7)                   */
} mrt_light;

/* Camera (src/Camera.h:26-45): eye, lookAt, up, vertical FOV in degrees, and
 * the lens of Camera::eyeRayAdaptive (src/Camera.cpp:153-174; ABI 5):
 * aperture < 0.001 (epsilon) is a pinhole; otherwise rays start on a
 * rejection-sampled disc of radius aperture and pass through the point at
 * distance focus_plane along the pinhole direction (setAperture / setFocusPlane,
 * reference defaults 0 and 1).  shutter_speed scales getTimeSample's
 * time = 1 - r^3 * shutter_speed (src/Camera.h:44-46, default 0.001), the ray
 * time of motion-blurred objects. */
typedef struct {
    float eye[3], look_at[3], up[3];
    float fov_deg;
    float aperture, focus_plane, shutter_speed;
} mrt_camera;

/* Raw triangle mesh (TriangleMesh arrays, src/TriangleMesh.h:36-47).  The
 * reference keeps vertices and normals as 16-byte Vector3 (src/Vector3.h:19,
 * x y z + pad): pass vert_stride = normal_stride = 4 to hand those arrays over
 * without repacking; 0 (or 3) = packed x y z. */
typedef struct {
    const float* verts;      /* nv*vert_stride floats                                   */
    const float* normals;    /* nn*normal_stride floats                                 */
    const uint32_t* vidx;    /* nt*3 vertex indices (TupleI3 m_vertexIndices)           */
    const uint32_t* nidx;    /* nt*3 normal indices (TupleI3 m_normalIndices)           */
    int32_t nv, nn, nt;
    int32_t vert_stride, normal_stride;  /* floats per vertex / normal: 0 or 3 packed, 4 Vector3 */
} mrt_mesh;

typedef struct {             /* HitInfo (src/Ray.h:185-200)                            */
    float t, a, b;
    int32_t prim;            /* global object id in scene order, -1 = miss (or, for an
                                any-hit query, 1 = occluded); mrt_scene_prim_object
                                maps it to (mesh, triangle, instance) = HitInfo::obj  */
    int32_t inst;            /* HitInfo::m_proxy: ProxyObject instance of the hit,
                                -1 = a world triangle (or a miss)                      */
} mrt_hit;

typedef struct {
    int32_t nodes, leaves, prims;       /* QBVH nodes / 4-triangle leaf packets / tris */
    int32_t bin_nodes, bin_leaves;      /* binary BVH before the 4-wide collapse       */
    int32_t max_depth;
    double build_ms;
    uint64_t device_bytes;              /* node + leaf + shading arrays in HBM         */
} mrt_bvh_info;

typedef struct {
    int32_t width, height;   /* frame size                                              */
    int32_t device;          /* HIP device ordinal                                      */
    int32_t count_visits;    /* 1: instrumented launch (node/leaf visit counters)       */
    int32_t want_rgb8;       /* 1: also write tone-mapped 8-bit RGB (Image::Map)        */
    int32_t want_hits;       /* 1: also write primary mrt_hit per pixel (debug/parity)  */
    uint32_t seed;           /* stochastic configs only (counter RNG stream)            */
    /* mrt_render only: render on several HIP devices of this process.  The 32x32
     * buckets of src/Scene.cpp:90-95 are dealt bucket b -> devices[b mod n] (a
     * device may appear more than once), each device renders its share from its
     * own scene replica, and the tiles are gathered into the caller's frame.  The
     * result is bit-identical to a one-device render.  NULL / 0 = `device` only. */
    const int32_t* devices;
    int32_t n_devices;
} mrt_render_opts;

typedef struct {
    uint64_t primary_rays, shadow_rays;
    uint64_t node_visits, leaf_visits;   /* all rays; valid when count_visits was set   */
    uint64_t primary_node_visits, primary_leaf_visits; /* primary-ray launch share     */
    uint64_t primary_hits;               /* primary rays that hit geometry               */
    uint64_t primary_wave_steps;         /* count mode: sum over tiles of the max node
                                            visits of a lane (x64 = issued lane-steps)   */
    uint64_t primary_uniform_visits;     /* count mode: primary node visits made in wave
                                            steps where all active lanes were on one node */
    float kernel_ms;                     /* device time of the last frame (all launches)*/
    float primary_ms, shade_ms;          /* per launch: primary rays / shade + shadows  */
    int32_t max_stack;                   /* deepest traversal stack seen (count mode)   */
    /* count mode, per launch of the persistent render kernels (device wall clock):
     * span = first wave start -> last wave end, ramp = spread of wave starts,
     * tail = spread of wave ends (time the launch runs below full occupancy)   */
    float primary_span_us, primary_ramp_us, primary_tail_us;
    float shade_span_us, shade_ramp_us, shade_tail_us;
    uint64_t secondary_rays;             /* Blinn reflection / refraction / GI rays traced */
    /* count mode, wavefront shadow_kernel: wave loop steps and node visits (lane
     * utilisation = shadow_node_visits / (64 * shadow_wave_steps)) */
    uint64_t shadow_wave_steps, shadow_node_visits;
    /* 1: the frame ran as ONE launch (frame1_kernel: camera rays, closest hits,
     * shading and shadow rays fused; one point light, one path); primary_ms is
     * then the whole frame and shade_ms ~0 (ABI 7) */
    int32_t fused;
    /* 1: the frame's shading ran the wavefront chain engine (secondary rays,
     * dispersive splits, path tracing; with adaptive supersampling as passes
     * over it) rather than one fused kernel (ABI 7) */
    int32_t chain;
    /* chain engine: the per-stream chunk budget its last frame was cut to (bytes,
     * at most the mrt_set_tuning("chain_mb") cap, 80% of the free memory and the
     * stream's share of 80% of the device) and the chunks it ran (ABI 8) */
    uint64_t chain_budget_bytes;
    uint32_t chain_chunks;
    /* chunks whose level counts outgrew the capacities estimated from earlier chunks
     * on the stream (mrt_set_tuning "chain_est"): their units were rendered again by
     * the fused chain shading -- same frame, slower (ABI 9) */
    int32_t chain_fallbacks;
} mrt_stats;

const char* mrt_last_error(void);
int mrt_abi_version(void);
/* Number of visible HIP devices (0 when none); never initialises a context. */
int mrt_device_count(void);

/* ---- scene construction: Scene::addObject/addLight/preCalc (src/Scene.h:17-28) */
mrt_scene* mrt_scene_create(void);
void mrt_scene_destroy(mrt_scene* s);
/* returns material id >= 0 */
int mrt_scene_add_material(mrt_scene* s, const mrt_material* m);
/* returns light id >= 0 */
int mrt_scene_add_light(mrt_scene* s, const mrt_light* l);
/* TriangleMesh::load(file, ctm) + makeMeshObjs (src/TriangleMeshLoad.cpp:50-214).
 * ctm16: row-major 4x4 or NULL (identity).  Returns mesh id >= 0. */
int mrt_scene_add_obj(mrt_scene* s, const char* path, const float* ctm16, int material);
/* Raw mesh (TriangleMesh::createSingleTriangle + setV1..3 / setN1..3, src/TriangleMesh.cpp:11-42). */
int mrt_scene_add_mesh(mrt_scene* s, const mrt_mesh* mesh, int material);
int mrt_scene_mesh_info(const mrt_scene* s, int mesh, int32_t* nv, int32_t* nn, int32_t* nt);
int mrt_scene_mesh_export(const mrt_scene* s, int mesh, float* verts, float* normals,
                          uint32_t* vidx, uint32_t* nidx);
/* TriangleMesh m_texCoords / m_texCoordIndices of a mesh added with
 * mrt_scene_add_mesh (OBJ files load their vt lines): n_texcoords (u, v) pairs
 * and 3 indices per triangle.  HitInfo::getAllInfos interpolates (u, v) and the
 * tangent frame TriangleMesh::preCalc derives (src/Ray.cpp:33-47,
 * src/TriangleMesh.cpp:105-148); without texture coordinates (u, v) = (a, b). */
int mrt_scene_mesh_set_texcoords(mrt_scene* s, int mesh, const float* uv, int32_t n_texcoords, const uint32_t* tidx);
int mrt_scene_mesh_texcoords(const mrt_scene* s, int mesh, int32_t* n_texcoords, float* uv, uint32_t* tidx);
/* MBObject(material, mesh, mesh_t2, i) for every triangle of `mesh`
 * (src/MBObject.cpp:7-11, src/MBObject.h): verts2 = m_mesh_t2's vertices,
 * n_vertices x 3 floats, same topology.  A ray of time t meets
 * t*verts2 + (1-t)*verts; shading uses the time-0 mesh.  World meshes only
 * (instanced BLAS meshes stay static, as in the reference). */
int mrt_scene_set_mesh_motion(mrt_scene* s, int mesh, const float* verts2);
/* Scene::setBGColor (src/Scene.h:37) */
int mrt_scene_set_background(mrt_scene* s, const float rgb[3]);
/* Scene::m_numPaths (src/Scene.h:61): shade() calls per primary hit */
int mrt_scene_set_num_paths(mrt_scene* s, int num_paths);
/* Blinn::setReflectAmt / Material::setRefractAmt / Blinn::setIor (src/Blinn.h:38-41,
 * src/Material.h:32; Blinn ctor defaults 0, 0, 1.5, src/Blinn.h:11-22): reflection and refraction rays of Blinn::shade (src/Blinn.cpp:238-330),
 * Fresnel-weighted Russian roulette, at most 5 bounces, IOR history per ray.
 * No effect on Lambert materials. */
int mrt_scene_set_material_optics(mrt_scene* s, int material, float reflect_amt, float refract_amt, float ior);
/* (ior is m_ior[1]: it also replaces the middle IOR of mrt_scene_set_material_dispersion,
 * as the reference keeps one m_ior[3] array.) */
/* Material::m_disperse + Blinn::setIor(ior, i) for i = 0..2 (src/Material.h:45,
 * src/Blinn.h:38,59; ABI 6).  `ior` replaces all three m_ior; ior[1] is also the
 * optics IOR above (the non-dispersive refraction reads m_ior[1], src/Blinn.cpp:183).
 * With disperse set, a ray that is not itself a refraction ray and refracts at
 * this material splits into three refraction rays through ior[0], ior[1], ior[2],
 * each child's colour masked to its channel (src/Blinn.cpp:169-173,275-301). */
int mrt_scene_set_material_dispersion(mrt_scene* s, int material, int disperse, const float ior[3]);
/* Blinn::setReflectGloss (src/Blinn.h:42; default 1): below 1 the reflection
 * vector is blended with a cosine-distributed sample
 * (Material::getCosineDistributedSamples, src/Material.cpp:14-41; src/Blinn.cpp:166-171). */
int mrt_scene_set_material_gloss(mrt_scene* s, int material, float gloss);
/* Material::setTranslucency (src/Material.h:30; default 0): above 0.01 a Blinn
 * material also samples every light from the back side (-normal) and adds
 * translucency * light * kd (src/Blinn.cpp:224-236), as the reference's leaf
 * materials do (src/main.cpp:253, src/Assignment3.h:70). */
int mrt_scene_set_material_translucency(mrt_scene* s, int material, float translucency);
/* Blinn::setLightEmittedIntensity / setLightEmittedColor after the material was
 * added (same fields as mrt_material.emitted / le). */
int mrt_scene_set_material_emission(mrt_scene* s, int material, float emitted, const float le[3]);
/* Material::setSampleEnv (src/Material.h:27; default true): a path-tracing GI ray
 * that misses takes the environment colour only when both this flag and the
 * scene's (mrt_scene_set_path_trace) are set (src/Blinn.cpp:70-73). */
int mrt_scene_set_material_sample_env(mrt_scene* s, int material, int sample_env);
/* Scene::m_pathTrace / m_maxBounces / setSampleEnv (src/Scene.h:40,48,57-64;
 * defaults false, 10; the reference never initialises m_sampleLightFromEnv, read
 * here as false): Blinn::calculatePathTracing (src/Blinn.cpp:39-89) adds one
 * cosine-distributed GI ray per direct-lighting shade() while the ray's GI bounce
 * count is below max_bounces - 1, and samples the lights directly at the last
 * bounce.  1 <= max_bounces <= 64. */
int mrt_scene_set_path_trace(mrt_scene* s, int enable, int max_bounces, int sample_env);
/* Scene::setMinSubdivs / setMaxSubdivs / setNoise (src/Scene.h:42-55; defaults
 * 1, 1, 0.01 at src/Scene.cpp:20-22): adaptive supersampling of
 * Scene::adaptiveSampleScene (src/Scene.cpp:252-293).  With both counts 1 a
 * frame is one ray per pixel; otherwise levels 2.. of n x n jittered sub-samples
 * run until the gamma-space change is below noise (at least up to min_subdivs,
 * at most max_subdivs).  1 <= min_subdivs <= max_subdivs <= 16. */
int mrt_scene_set_subdivs(mrt_scene* s, int min_subdivs, int max_subdivs, float noise_threshold);
/* ---- images and image-based lighting -------------------------------------
 * HDRLoader::load (src/hdrloader.cpp:29-97, via RawImage::loadImage/loadHDR,
 * src/RawImage.cpp:16-32): mrt_hdr_info reads the header, mrt_hdr_load decodes
 * into caller memory, width*height*3 floats, row 0 = the top (first) scanline. */
int mrt_hdr_info(const char* path, int32_t* width, int32_t* height);
int mrt_hdr_load(const char* path, float* rgb, int32_t width, int32_t height);
/* new RawImage(w, h, data, HDR) + new Texture(image) (src/RawImage.cpp:9-14,
 * src/Texture.h:13): copies width*height*3 floats (row 0 = top).  Returns the
 * texture id (<= 16 per scene). */
int mrt_scene_add_texture(mrt_scene* s, const float* rgb, int32_t width, int32_t height);
/* RawImage::loadImage (src/RawImage.cpp:16-188) by extension: .tga (uncompressed
 * 8/24/32-bit, rows flipped, colour through Image::gamma_to_linear, alpha / 255,
 * B/R swapped), .ppm (P6, bytes / 255) or .hdr.  type: MRT_TEX_HDR (3 floats per
 * texel), MRT_TEX_GRAY (1), MRT_TEX_RGB (3), MRT_TEX_RGBA (4); data holds
 * width*height*channels floats in RawImage m_rawData order (ABI 5). */
enum { MRT_TEX_HDR = 0, MRT_TEX_GRAY = 1, MRT_TEX_RGB = 3, MRT_TEX_RGBA = 4 };
int mrt_image_info(const char* path, int32_t* width, int32_t* height, int32_t* type);
int mrt_image_load(const char* path, float* data, int32_t width, int32_t height);
/* new RawImage(w, h, data, type) + new Texture(image) for any RawImage type
 * (Texture::getPixel per type, src/Texture.cpp:100-125).  Returns the texture id. */
int mrt_scene_add_texture_typed(mrt_scene* s, const float* data, int32_t width, int32_t height, int32_t type);
/* Material::setColorMap / setNormalMap / setSpecularMap / setReflectMap /
 * setRefractMap / setAlphaMap (src/Material.h:20-25): maps[6] texture ids in that
 * order, -1 = none.  Lambert uses the colour map (src/Lambert.cpp:32-36); Blinn all
 * of them (src/Blinn.cpp:114-142); an alpha map makes intersect4 skip a
 * triangle whose alpha at the hit is below 0.5 (src/BVH.cpp:1397-1445), for
 * closest-hit and shadow rays.  Alpha maps apply to world (non-instanced) meshes. */
int mrt_scene_set_material_maps(mrt_scene* s, int material, const int32_t maps[6]);
/* Scene::setEnvMap + Scene::setEnvExposure (src/Scene.h:23-24): primary rays
 * that miss return the lat-long lookup x exposure instead of the background
 * (src/Scene.cpp:236-239).  texture = -1 clears. */
int mrt_scene_set_env_map(mrt_scene* s, int32_t texture, float exposure);
/* Material::setEnvMap + m_envExposure (src/Material.h:19,41-42; ABI 9): a Blinn
 * material's missed reflection / refraction / path-tracing GI rays take this map
 * x exposure instead of the scene's (Material::getEnvironmentColor,
 * src/Material.cpp:44-64).  An RGB / HDR texture id, or -1 = the scene's. */
int mrt_scene_set_material_env_map(mrt_scene* s, int material, int32_t texture, float exposure);
/* Importance tables of dome light `light` (DomeLight::setTexture,
 * src/DomeLight.cpp:8-78), for inspection: cdf_u[nu+1], func_u[nu],
 * cdf_v[nu*(nv+1)], func_v[nu*nv], func_int[nu+1] (column integrals, then the u
 * integral), cos_u/sin_u[nu+1], cos_v/sin_v[nv+1]. */
int mrt_scene_dome_info(const mrt_scene* s, int32_t light, int32_t* nu, int32_t* nv);
int mrt_scene_dome_export(const mrt_scene* s, int32_t light, float* cdf_u, float* func_u, float* cdf_v,
                          float* func_v, float* func_int, float* cos_u, float* sin_u, float* cos_v, float* sin_v);

/* ---- instancing: ProxyObject (src/ProxyObject.cpp:5-95,131-167) -----------
 * mrt_scene_make_blas builds a proxy BVH from meshes already added
 * (ProxyObject::setupMultiProxy: the meshes in order, each mesh's triangles last
 * to first, then BVH::build); those meshes leave the world object list.  Returns
 * the BLAS id.  mrt_scene_add_instance adds one ProxyObject (row-major 4x4
 * m_transform; ProxyMatrix derives the inverse and inverse transpose); it joins
 * the world objects in call order with the world meshes.  Hit ids (mrt_hit.prim):
 * world objects 0..n-1 (mrt_bvh_info.prims = n; a proxy's own slot never hits),
 * then instance i's BLAS objects at n + (BLAS sizes of the instances before i) +
 * BLAS object index.  blas_info/export give a BLAS's canonical QBVH arrays
 * (same layout as mrt_scene_bvh_export). */
int mrt_scene_make_blas(mrt_scene* s, const int32_t* meshes, int32_t n_meshes);
int mrt_scene_add_instance(mrt_scene* s, int32_t blas, const float* m16);
int mrt_scene_blas_info(const mrt_scene* s, int32_t blas, int32_t* nodes, int32_t* leaves, int32_t* prims);
int mrt_scene_blas_export(const mrt_scene* s, int32_t blas, float* node_boxes, int32_t* node_child,
                          float* leaf_tris, int32_t* leaf_prims);

/* Scene::preCalc -> BVH::build (src/Scene.cpp:62-79, src/BVH.cpp:457-575):
 * binned SAH, 4-wide collapse, host-side; then uploads to the device lazily. */
int mrt_scene_build_bvh(mrt_scene* s);
int mrt_scene_bvh_info(const mrt_scene* s, mrt_bvh_info* info);
/* HitInfo::obj / m_proxy of a hit id (mrt_hit.prim): the Object's mesh id and
 * triangle index (Object::m_mesh / m_index, src/Object.h:49-77) and the
 * ProxyObject instance (-1 = a world triangle).  Valid after mrt_scene_build_bvh. */
int mrt_scene_prim_object(const mrt_scene* s, int32_t prim, int32_t* mesh, int32_t* tri, int32_t* inst);
/* Canonical QBVH arrays: node_boxes[24*nodes] (minX4 minY4 minZ4 maxX4 maxY4 maxZ4),
 * node_child[4*nodes] (>=0 inner node, ~leaf for a leaf slot, INT32_MIN empty),
 * leaf_tris[36*leaves] (Ax4 Ay4 Az4 e0x4 e0y4 e0z4 e1x4 e1y4 e1z4),
 * leaf_prims[4*leaves] (-1 empty).  (QBVH_Node / TriCache4, src/BVH.h:37-109) */
int mrt_scene_bvh_export(const mrt_scene* s, float* node_boxes, int32_t* node_child,
                         float* leaf_tris, int32_t* leaf_prims);
/* Replace the built hierarchy with given canonical arrays (identical-BVH tests). */
int mrt_scene_bvh_import(mrt_scene* s, int32_t nodes, int32_t leaves, const float* node_boxes,
                         const int32_t* node_child, const float* leaf_tris, const int32_t* leaf_prims);
/* Copy the scene to device `device` (done implicitly by render/trace). */
int mrt_scene_upload(mrt_scene* s, int device);

/* ---- frame entry: Scene::raytraceImage(Camera*, Image*) (src/Scene.cpp:85-217).
 * Synchronous, host buffers: rgb (W*H*3 floats, before Map) and rgb8 (W*H*3,
 * after Image::Map; nullable); hits (W*H, nullable).  1 spp primary + shadow. */
int mrt_render(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts,
               float* rgb, uint8_t* rgb8, mrt_hit* hits);

/* ---- bucketed device render for multi-GPU tiling (src/Scene.cpp:90-174 buckets).
 * Renders the 32x32 buckets listed in d_buckets (device int32 ids, row-major
 * bucket grid) into d_tiles: n_buckets * 32*32*3 floats, bucket-major, pixels
 * row-major inside a bucket (pixels outside the frame left untouched).
 * Everything is enqueued on `stream` (hipStream_t, NULL = default); returns
 * without synchronising.  Device pointers come from the caller (e.g. torch). */
int mrt_render_buckets_async(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts,
                             const int32_t* d_buckets, int32_t n_buckets, float* d_tiles,
                             void* stream);
/* Scatter bucket tiles into a W*H*3 float frame (and optional W*H*3 rgb8). */
int mrt_unpack_buckets_async(const int32_t* d_buckets, int32_t n_buckets, const float* d_tiles,
                             int32_t width, int32_t height, float* d_frame, uint8_t* d_frame8,
                             const mrt_scene* s_for_lut, void* stream);
/* ---- batched bucket render: several frames (cameras) in one launch pair.
 * Same bucket loop (src/Scene.cpp:90-174) over a batch of n_cams <= 16 frames of
 * one size (e.g. a camera path, or one frame's buckets dealt across GPUs).
 * d_items: device int32 ids, id = frame * buckets_per_frame + bucket, with
 * buckets_per_frame = ceil(W/32) * ceil(H/32); an id whose frame is >= n_cams
 * renders with the last camera.  Frame f uses RNG seed (opts->seed or the
 * default) + f, so it equals an mrt_render of camera f with that seed.
 * Outputs (either may be NULL, not both), slot-major like mrt_render_buckets_async:
 * d_tiles n_items*1024*3 floats; d_tiles8 n_items*1024*3 bytes (Image::Map). */
int mrt_render_batch_async(mrt_scene* s, const mrt_camera* cams, int32_t n_cams, const mrt_render_opts* opts,
                           const int32_t* d_items, int32_t n_items, float* d_tiles, uint8_t* d_tiles8,
                           void* stream);
/* Scatter batch tiles into n_frames consecutive W*H frames (frame f at offset
 * f*W*H*3).  d_frames needs d_tiles; d_frames8 copies d_tiles8 or, when it is
 * NULL, maps d_tiles through the scene's gamma LUT.  Items of frames >= n_frames
 * are skipped. */
int mrt_unpack_batch_async(const int32_t* d_items, int32_t n_items, const float* d_tiles, const uint8_t* d_tiles8,
                           int32_t width, int32_t height, int32_t n_frames, float* d_frames, uint8_t* d_frames8,
                           const mrt_scene* s_for_lut, void* stream);
/* ---- the batch render written straight into frames (ABI 10): the same items and
 * launches as mrt_render_batch_async, but each pixel goes to its place in n_cams
 * consecutive W*H frames (frame f at offset f*W*H*3 of d_frames / d_frames8, either
 * may be NULL, not both); pixels outside the frame and items of frames >= n_cams
 * write nothing.  With the frames of another process mapped by mrt_ipc_open, every
 * rank of the multi-GPU split writes its buckets into rank 0's frame directly: the
 * frame is complete when every rank's launch is (a stream-ordered barrier), with no
 * gather and no unpack (src/Scene.cpp:90-174's bucket loop, one image for all). */
int mrt_render_batch_frames_async(mrt_scene* s, const mrt_camera* cams, int32_t n_cams, const mrt_render_opts* opts,
                                  const int32_t* d_items, int32_t n_items, float* d_frames, uint8_t* d_frames8,
                                  void* stream);
/* Device memory shared between processes (hipIpcGetMemHandle / hipIpcOpenMemHandle):
 * mrt_ipc_export describes the allocation holding d_ptr (any pointer into a device
 * allocation, e.g. a torch tensor's data) and d_ptr's offset in it; mrt_ipc_open maps
 * it in this process for `device` (peer access enabled) and returns the same byte;
 * mrt_ipc_close unmaps a pointer mrt_ipc_open returned.  The handle is plain bytes
 * (send it to the other ranks over any channel). */
typedef struct {
    uint8_t handle[64];
    uint64_t offset, size;
} mrt_ipc_handle;
int mrt_ipc_export(const void* d_ptr, mrt_ipc_handle* out);
int mrt_ipc_open(const mrt_ipc_handle* h, int device, void** d_ptr);
int mrt_ipc_close(void* d_ptr);
/* Whole frame straight into device buffers (N = 1 fast path, no tiles). */
int mrt_render_frame_async(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts,
                           float* d_rgb, uint8_t* d_rgb8, void* stream);

/* ---- batched ray query: Scene::trace / BVH::intersect (src/Scene.cpp:295-298,
 * src/BVH.cpp:1112-1178).  o,d: n*3 floats; tmin,tmax: n floats.  any_hit=1
 * stops at the first accepted triangle (shadow rays; occlusion result is
 * identical to the reference's closest-hit shadow traversal). */
int mrt_trace(mrt_scene* s, const float* o, const float* d, const float* tmin, const float* tmax,
              size_t n, int any_hit, mrt_hit* out);
int mrt_trace_async(mrt_scene* s, const float* d_o, const float* d_d, const float* d_tmin,
                    const float* d_tmax, size_t n, int any_hit, mrt_hit* d_out, void* stream);

/* The walk of the scene's last one-light frame on its current device: *lds_nodes = 1
 * when it ran the LDS top-node walk (tuning "lds_nodes"), 0 when not, -1 before any;
 * *walk_exits = the walk loop's form of the frame / primary kernels, 1 (one exit: a
 * stack overflow empties the stack and leaves at the pop test; the default) or 2 (a
 * second exit on overflow; tuning "walk_exit" 0).  Both forms give the same bits. */
int mrt_scene_walk_info(const mrt_scene* s, int32_t* lds_nodes, int32_t* walk_exits);

/* Counters of the last render on this scene (ray counts, visits, kernel time). */
int mrt_scene_last_stats(const mrt_scene* s, mrt_stats* out);

/* Performance A/B switches (no effect on results; defaults in brackets).  Each key is
 * either selected by a default path or exercised by the GPU tests (round 6 removed the
 * rest, with their kernel instantiations; their A/B records stay in profiles/):
 * "fast_box" 0/[1] (hardware min/max slab test when its finiteness precondition holds),
 * "scalar_nodes" 0..[7] (bit 0 scalar fetch of wave-uniform nodes, bit 1 of wave-uniform
 * triangles, bit 2 octant-ordered box test), "walk_exit" 0/[1] (the frame / primary
 * kernels' walk loop: two exits, one exit), "walk_latch" 0/[1] (the frame kernel's
 * camera-ray walk: nested latches, one latch), "lds_nodes" [0]/1 (the frame kernel's LDS
 * top-node walk), "sched" 0..3 [2] (tile schedule: static grid-stride, static XCD bands,
 * dynamic interleaved, dynamic banded; see TileSched), "fused" 0/[1] (one-launch frame
 * kernel for one point light), "shade1" 0/[1] (specialised shading kernel for one point
 * light and one path), "frame1_waves" 1/5/6/[7]/8 and "primary_waves" 0/6/[7]/8 and
 * "primary_inst_waves" 1/4/[5]/6 (occupancy targets), "wavefront" 0/[1] (gen / shadow /
 * resolve passes instead of the fused shading kernel), "shadow_sched" [-1]..2 (wavefront
 * shadow rays: auto, grid-stride, XCD bands, bands + lane refill), "near_first" [-1]..1
 * (any-hit walks descend into the nearest hit child first), "dome_replay" 0/[1] (the
 * dome-light resolve pass sums the recorded samples), "bin" [-1] / 0..7 (ray binning
 * before tracing: bit 0 the wavefront shadow pass, bit 1 the chain levels' closest-hit
 * entries, bit 2 their shadow rays; -1 auto), "bin_dbits" 0..6 [2] / "bin_obits" 0..4 [2]
 * (binning key: direction and origin cells per axis as powers of two, 2 dbits + 3 obits
 * <= 12), "bin_inst" [0]..2 (instance-major shadow-ray bin keys), "chain" 0/[1] (the
 * wavefront chain engine for secondary rays), "chain_bands" [-1]..1 (XCD-banded chain
 * trace queue; -1: on for binned levels), "chain_est" 0/[1] / "chain_est_pct" [125] /
 * "chain_mb" [8192] (chain level capacities and scratch budget), "chain_shadow_step"
 * [0]/1 and "chain_shadow_refill" [0]/1 (instanced chain levels' shadow walks),
 * "adapt_refill" 0..64 [32] (adaptive pixel refill), "batch_tpw" 1..64 [2] (tiles per
 * wave a bucket batch smaller than the persistent grid is launched for), "wave_log"
 * [0]/1 (timing-only wave log, diagnostics).  Process-wide. */
int mrt_set_tuning(const char* key, int value);

/* Diagnostics: per-wave records of the last count-mode render (count_visits = 1)
 * for launch 0 (primary rays) or 1 (shading + shadow rays): 60 x uint64 per wave
 * {start, end (device wall clock ticks), tiles processed, node visits, then for the
 * wave's first 28 tiles: tile id << 40 | low 40 bits of the tick it started, then
 * for the same tiles the ticks their dequeue (tile-queue atomics) took}.
 * Returns the number of waves copied (<= max_waves). */
int mrt_debug_wave_log(const mrt_scene* s, int launch, uint64_t* out, int32_t max_waves);
/* Device wall-clock rate (kHz) of the scene's device, for the ticks above. */
int mrt_device_wall_clock_khz(const mrt_scene* s);

/* Numerics probes (x86 RCPSS/RSQRTSS emulation + one Newton step, SSE.h:67-101). */
/* The device's acosf(x) (fn 0) / atan2f(y, x) (fn 1) / sinf(x) (fn 3) / cosf(x) (fn 4) /
 * powf(x, y) (fn 5) over n host inputs (a kernel on the current device; glibc's code
 * restated, csrc/mrt_libm.h), or its rcp_nr(x) (fn 2: the RCPSS emulation and Newton step
 * of every triangle test; y unused). */
int mrt_debug_libm(int fn, const float* x, const float* y, size_t n, float* out);
float mrt_rcp_nr(float x);
float mrt_rsqrt_nr(float x);

#ifdef __cplusplus
}
#endif
#endif /* MRT_H */
