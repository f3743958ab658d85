// mrt_shader.h -- device shading code shared by the kernel translation units
// (mrt_device.hip: frame kernels + host; mrt_rec.hip: the fused chain and
// adaptive kernels; mrt_chain.hip: the wavefront chain kernels).  Included
// after mrt_kernels.h / mrt_scene.h / mrt_texture.h inside namespace mrt.
#pragma once
#include <hip/hip_runtime.h>

#include "mrt_kernels.h"
#include "mrt_scene.h"
#include "mrt_texture.h"

namespace mrt {

enum { CTR_SHADOW = 0, CTR_NODES = 1, CTR_LEAVES = 2, CTR_MAXSP = 3, CTR_OVERFLOW = 4, CTR_NODES_P = 5, CTR_LEAVES_P = 6, CTR_HITS = 7,
       CTR_WAVE_STEPS_P = 8, CTR_UNIFORM_P = 9,
       // count mode, per launch (primary at CTR_TP, shade at CTR_TS): wave start/end
       // wall clocks as ~min start, max start, ~min end, max end (zero-initialised maxima)
       CTR_TP = 10, CTR_TS = 14,
       CTR_RAYS_P = 18,  // eye rays traced (adaptive supersampling; otherwise one per pixel)
       CTR_SECONDARY = 19,  // Blinn reflection / refraction rays
       CTR_WAVE_STEPS_S = 20, CTR_NODES_S = 21,  // count mode, shadow_kernel: wave loop steps, node visits
       CTR_FALLBACK = 22,  // chain chunks that outgrew an estimated level capacity (rendered by the fallback)
       CTR_N = 23 };
static constexpr int kMaxBlocksPerCU = 8;
// wave log record: start, end, tiles, node visits, then (tile id << 40 | start tick) of the first kLogTiles
// tiles, then the wall-clock ticks each of those tiles' dequeue took
static constexpr int kLogTiles = 28;
static constexpr int kLogWords = 4 + 2 * kLogTiles;  // 256-thread blocks: 8 waves per SIMD at most
// counter block: CTR_N u64 statistics, then four launches x 8 work counters x 128 B
// (primary, shade / gen, resolve, shadow_kernel's per-XCD ray queues); cleared per launch
// with one hipMemsetAsync, whose length is a multiple of 256 B so the runtime fills it with
// one kernel (an odd length costs a second fill launch for the tail)
#ifndef MRT_CTR_ODD
static constexpr size_t kCtrBytes = (CTR_N * sizeof(unsigned long long) + 4 * 8 * 128 + 255) / 256 * 256;
#else   // A/B build: round 3's unpadded length
static constexpr size_t kCtrBytes = CTR_N * sizeof(unsigned long long) + 4 * 8 * 128;
#endif
// Shadow rays of the general shading path, wavefront style (ShadowMode): kernel
// 2a runs the shading code and writes every shadow ray to its slot, kernel 2b
// traces all of them any-hit (few registers, full occupancy), kernel 2c runs the
// same shading code again with the occlusion bits.  Same rays, same order, same
// arithmetic as the fused kernel, which keeps the whole shading state live
// across each traversal.
enum ShadowMode { kFused = 0, kGen = 1, kResolve = 2 };
static constexpr int kMaxWaveShadow = 64;  // rays per pixel beyond this use the fused kernel
static constexpr int kMaxLevelsP1 = 64;     // chain levels + 1 (kMaxChainLevels = 63)

struct RenderParams {
    const QNode* nodes;
    const DLeaf* leaves;
    const PrimShade* prims;
    const float4* verts;
    const float4* normals;
    const DevMaterial* mats;
    const DevLight* lights;
    const DevDome* domes;    // dome-light tables (DevLight::dome)
    const DevInstance* insts;  // ProxyObjects (instanced scenes)
    // material maps (src/Material.h:20-25): map textures, per-prim texture-coordinate
    // indices (w = the mesh has texture coordinates), (u, v) pairs, per-normal tangents
    const DevTexture* texs;
    const uint4* puv;
    const float2* uvs;
    const float4* tans;
    const float4* btans;
    int32_t has_maps;          // some material has a colour / normal / specular / reflect / refract map
    int32_t n_insts, n_world;  // instances; world objects (instance hit ids start here)
    const float* env;        // environment map (nullable), env_w x env_h RGB, row 0 = top
    float4* ray_o;           // wavefront shadow rays: slot * max_shadow + j -> origin, tMax
    float4* ray_d;           //   direction
    uint8_t* occl;           //   1 = occluded (kernel 2b)
    uint8_t* nrays;          //   rays of each output slot (kernel 2a)
    int32_t max_shadow;      //   rays per pixel at most (num_paths x light samples)
    int32_t env_w, env_h;
    float env_exposure;
    const uint16_t* tables;  // rcp[2048] | rsqrt[2048]
    const uint8_t* gamma;
    const float* gammaF;     // Image::linear_to_gammaF (adaptive supersampling stop test)
    int32_t min_subdivs, max_subdivs;
    float noise;             // Scene::m_noiseThreshold
    int32_t* gstack;
    uint32_t gstride;        // total threads in the launch
    unsigned long long* ctr;
    unsigned long long* wave_log;  // count mode: kLogWords per wave (this launch), see mrt_debug_wave_log
    CamParams cam[kMaxBatch];    // frame mode: cam[0]; batch mode: one camera per frame
    float bg[3];
    int32_t n_lights, num_paths;
    int32_t path_trace, max_bounces, sample_env;  // Scene::m_pathTrace / m_maxBounces / sampleEnv
    float* lvl;                  // REC kernels: chain level records, (level * lvl_words + w) * gstride + thread
    int32_t lvl_words;           //   words per level record
    uint32_t seed;
    int32_t fast_box;            // node boxes finite && tuning allows the hardware min/max box test
    int32_t sched;               // tile schedule (TileSched)
    int32_t n_waves;             // waves in this launch
    int32_t refill_min;          // adaptive_kernel: 0 tile schedule, > 0 pixel refill at this many idle lanes
    int32_t near_first;          // any-hit walks take the nearest hit child first (their answer is order-free)
    int32_t cus;                 // compute units (slot of a persistent block = blockIdx / cus)
    int32_t scalar_nodes;        // scalar fetch of wave-uniform nodes
    unsigned int* queue;         // 8 tile counters, 32 words apart (sched >= 2)
    // work: 8x8 tiles
    int32_t tiles_x, n_tiles;    // frame mode: tiles_x = ceil(W/8)
    const int32_t* buckets;      // bucket mode: bucket ids (row-major bucket grid)
    int32_t buckets_x;           // ceil(W/32)
    int32_t buckets_per_frame;   // bucket mode: id = frame * buckets_per_frame + bucket
    int32_t n_cams;              // bucket mode: frames (cameras) in the batch
    int32_t mode;                // 0 frame, 1 buckets
    int32_t frame_out;           // buckets: outputs are n_cams consecutive W*H frames, not tiles (store_rgb)
    float* out_rgb;              // frame: W*H*3; buckets: n_buckets*1024*3, or n_cams*W*H*3 with frame_out (nullable)
    uint8_t* out_rgb8;           // same slots as out_rgb (nullable)
    float4* hits;                // per slot: t, a, b, prim bits (kernel 1 -> kernel 2)
    // wavefront chain engine (mrt_chain.hip; REC scenes on the frame / bucket
    // path): chain level k's entries are [ch_lofs[k], ch_lofs[k + 1]) of every
    // per-entry array (capacity of level k = ch_lofs[k + 1] - ch_lofs[k]);
    // two-array fields hold level k's first array at 2 * lofs and its second at
    // 2 * lofs + capacity (coalesced SoA per level)
    float4* ch_ray;              // origin | path id bits; direction | state bits
    float4* ch_ior;              // IOR history 1..4; 5..7 | parent entry bits
    float4* ch_hit;              // closest hit (t, a, b, prim bits)
    float* ch_rec;               // lvl_words per entry: the level record of a spawning entry
    float4* ch_val;              // the entry's value (rgb) | kVal* flags
    uint32_t* ch_map;            // ch_split per entry: dense entry of the child spawned from that slot
    float4* ch_sp;               // [4][ch_spcap]: the current level's spawned children, sparse (entry * split + i)
    uint8_t* ch_flag;            // [ch_spcap]: spawned (ch_sp slot valid)
    uint32_t* ch_cnt;            // [level]: entries (level 0: unused, the chunk's paths)
    uint32_t ch_spcap;           // sparse spawn slots
    int32_t ch_split;            // spawn slots per entry: 3 where dispersive splits can occur, else 1
    int32_t ch_level;            // the level a chain launch works on
    int32_t ch_skip_shadow;      // chain_trace: the previous level's shadow rays run in a launch of their own
    int32_t ch_levels;           // levels allocated
    uint32_t ch_lofs[kMaxLevelsP1 + 1];
    // work units of the chain engine: one eye ray of a pixel.  Without a unit
    // list, unit u is lane u & 63 of work item u >> 6 with the centre sample
    // (adapt_n <= 1); adaptive pass n >= 2: unit u is sample (i, j) = ((u % n^2) / n,
    // u % n) of pixel units[u / n^2] (item << 6 | lane).  A chunk covers units
    // [unit_base, unit_base + n_units) of the pass.
    const uint32_t* units;
    const uint32_t* unit_cnt;    // device count of `units` (pixels), or null: units_total units
    uint32_t units_total;
    uint32_t unit_base, n_units;
    int32_t adapt_n;             // adaptive supersampling pass (level) n; 0: no adaptive supersampling
    float4* uhits;               // adaptive: closest hit per unit of the chunk (null: hits[pixel slot])
    float4* ucol;                // adaptive: colour per unit of the pass
    float4* adapt_res;           // adaptive: running mean per pixel slot
    uint32_t* next_units;        // adaptive combine: the pixels that refine further
    uint32_t* next_cnt;
    const uint32_t* sh_count;    // shadow_kernel: pixel / entry count on the device (nullable)
    // ray binning (mrt_bin.h): the trace kernels take their rays in this order
    // (nullable: slot order).  sh_perm lists the valid shadow-ray slots (sh_perm_n
    // of them, on the device); tr_perm the chain level's closest-hit entries.
    const uint32_t* sh_perm;
    const uint32_t* sh_perm_n;
    const uint32_t* tr_perm;
    int32_t ch_bands;            // chain_trace: XCD-banded chunk queue (P.queue + (level + 1) * 256 words)
    // dome-light replay (kernels 2a / 2c of the direct shading): 2a records, per
    // shadow-ray slot, the sample's E and dot(rVec, dir) (ray_e), and per dome
    // call (lcalls per pixel slot) its sample count | RNG draws << 8 (lrec); 2c
    // then sums the recorded samples with the answers instead of sampling again
    float4* ray_e;
    uint32_t* lrec;
    int32_t lcalls;
    // motion blur (MBObject, src/MBObject.cpp): per world prim bit 0 = MBObject
    // lane; time-1 vertices parallel to verts (nullptr: no motion blur)
    const uint8_t* pflags;
    const float4* verts2;
    int32_t has_mb;
    int32_t mat_env;             // some material has its own environment map (Material::m_envMap)
    // chain chunks on estimated level capacities: ch_ovf = the chunk outgrew one (its later
    // launches do nothing, chain_fallback_kernel renders its units); the chunk's statistics
    // go to ctr and are added to ctr_out unless it did; ch_est = per level, the largest
    // entries per path seen (x 65536, + 1; atomicMax) for this pass index on this stream
    uint32_t* ch_ovf;
    unsigned long long* ctr_out;
    uint32_t* ch_est;
};

// pow(spec, specExp) of Blinn::shade (src/Blinn.cpp:219-220): glibc's powf, which the
// reference's float call resolves to, restated bit for bit (gl_powf, mrt_libm.h; round 6 --
// round 5 evaluated it in double and rounded once, within 1 ulp of glibc's)
__device__ __forceinline__ float spec_pow(float x, float e) { return gl_powf(x, e); }

// operator*(Matrix4x4, Vector3) (src/Matrix4x4.h:693-704) on rows 0-2 of T (stride 4)
__device__ __forceinline__ v3 xform_dir3(const float* T, v3 u) {
    return mk(T[0] * u.x + T[1] * u.y + T[2] * u.z, T[4] * u.x + T[5] * u.y + T[6] * u.z,
              T[8] * u.x + T[9] * u.y + T[10] * u.z);
}

// REC: the scene has reflective / refractive materials (Blinn secondary rays,
// shade_path); compiled only into the kernels that run such scenes, so the
// direct-lighting kernels keep their register budget.
// RNG keys of the counter RNG (mrt_math.h): sub-stream skey = eye-ray sample *
// 1024 + path, draw key dim = (chain level + 1) << 24 | branch << 16 | k
// (camera: dims 0-2).  branch: the dispersion branch code of the ray (0 outside
// dispersive splits; each split appends child index + 1 in two bits), so
// sibling rays of one level draw from their own keys.
__device__ __forceinline__ uint32_t level_key(int level, int branch = 0) {
    return (uint32_t)(level + 1) << 24 | (uint32_t)(branch & 0xFF) << 16;
}

// Working IOR history of the rays below the camera ray (Ray::IORList,
// src/Ray.h:43-50): a per-lane LDS column in the REC kernels.
static constexpr int kIorCap = 8;

// the alpha-test tables of a traversal (special-leaf kernels only read them)
__device__ __forceinline__ void trav_alpha(Trav& T, const RenderParams& P) {
    T.aprims = P.prims;
    T.apuv = P.puv;
    T.auv = P.uvs;
    T.amats = P.mats;
    T.atex = P.texs;
    T.pflags = P.pflags;
    T.verts = P.verts;
    T.verts2 = P.verts2;
    T.near_first = P.near_first != 0;
}

// Chain state of one path at its current level (Shader::level).
enum { kRefl = 1, kRefr = 2, kGI = 3, kDisp = 4 };
struct ChainState {
    int idx = 0, depth = 0, gi = 0, bounces = 0;  // IOR history index, level, GI / reflect-refract levels so far
    bool secondary = false;                       // isSecondary of this level's shade()
    bool refr = false;                            // the ray is a refraction ray (IS_REFRACT_RAY, src/Ray.h:18)
    int br = 0;                                   // dispersion branch code (level_key)
};
// A chain level's record (the terms of the level that spawned a child): word w at p[w * stride]
struct ChainRec {
    float* p;
    size_t stride;
    __device__ float& operator()(int w) const { return p[(size_t)w * stride]; }
};
struct LevelOut {
    DRay r2;         // the spawned child ray
    v3 val, dir;     // the level's final value / the child's direction
    bool spawn;      // a child ray was spawned (its terms are in the level record)
    bool env_miss;   // a missed child takes the environment colour (false: GI with no environment sampling)
    bool split = false;   // dispersion: three refraction children (Shader::disp_child), not r2
};

// Material::getEnvironmentColor (src/Material.cpp:44-64) without a material map:
// the scene's map or the background
__device__ __forceinline__ v3 env_or_bg(const RenderParams& P, v3 d) {
    if (P.env) return scale(tex_lookup_dir(P.env, P.env_w, P.env_h, d.x, d.y, d.z), P.env_exposure);
    return mk(P.bg[0], P.bg[1], P.bg[2]);
}
// Material::getEnvironmentColor of material M: its own map x m_envExposure first
__device__ __forceinline__ v3 mat_env(const RenderParams& P, const DevMaterial& M, v3 d) {
    if (M.env >= 0) {
        const DevTexture& t = P.texs[M.env];
        return scale(tex_lookup_dir(t.data, t.W, t.H, d.x, d.y, d.z), M.env_exposure);
    }
    return env_or_bg(P, d);
}

// Fold a child's value into its parent level (Blinn::shade, src/Blinn.cpp:
// 238-335, and calculatePathTracing's Ld, :39-89), with the reference's adds.
// `none`: the child was a GI ray that missed with no environment sampling
// (calculatePathTracing adds nothing).
__device__ __forceinline__ v3 chain_combine(const RenderParams& P, const ChainRec& rec, v3 val, bool none) {
    const v3 z = mk(0, 0, 0);
    const int info = __float_as_int(rec(0));
    const DevMaterial& M = P.mats[info & 0xFFFF];
    const int kind = info >> 16;
    const float rrRecip = rec(1), rrSpec = rec(2);
    const v3 le = mk(M.le[0], M.le[1], M.le[2]), ka = mk(M.ka[0], M.ka[1], M.ka[2]);
    if (kind == kGI) {   // Ld = 0 + (0 + diffuseColor * child) + each light's E * diffuseColor + ka
        v3 Ld = add(z, none ? z : add(z, mul(mk(rec(9), rec(10), rec(11)), val)));
        for (int i = 0; i < P.n_lights; i++) Ld = add(Ld, mk(rec(12 + 3 * i), rec(13 + 3 * i), rec(14 + 3 * i)));
        Ld = add(Ld, ka);
        const v3 Ls = mk(rec(3), rec(4), rec(5)), tr = mk(rec(6), rec(7), rec(8));
        return add(add(scale(add(add(Ld, Ls), tr), rrRecip), scale(add(z, z), rrSpec)), le);
    }
    // Lr / Lt += m_ks * shade(child) (or * the environment when the child missed)
    const v3 L = add(z, mul(mk(M.ks[0], M.ks[1], M.ks[2]), val));
    const v3 base = scale(add(add(add(z, ka), z), z), rrRecip);
    return add(add(base, scale(kind == kRefr ? add(z, L) : add(L, z), rrSpec)), le);
}

// REC: 0 direct lighting only; 1 Blinn reflection / refraction chains; 2 also
// path tracing (GI rays).  Compiled into the kernels that run such scenes only.
template <bool POINT_ONLY, bool FAST, bool INST = false, int MODE = kFused, int REC = 0>
struct Shader {
    const RenderParams& P;
    const Trav& T;
    const uint16_t* rcpT;
    const uint16_t* rsqT;
    TravStats& st;
    uint32_t pixel;
    uint32_t shadow_rays;
    uint32_t seed;
    size_t slot0;            // wavefront modes: this pixel's first ray slot
    uint32_t nslot;          //   rays so far
    uint32_t sample = 0;     // eye-ray sample of the pixel (adaptive supersampling)
    uint32_t skey = 0, dim = 0;  // RNG sub-stream / draw key
    float* iorS = nullptr;   // REC: LDS IOR column (stride kWG)
    float* lvl = nullptr;    // REC: this thread's level records (stride P.gstride)
    float time = 0.f;        // the camera ray's time (getTimeSample), inherited by the rays below it
    float shadow_time = 0.f; // sampleLight's shadow-ray time: time, or .001 for translucency (src/Blinn.cpp:229)
    size_t lrec0 = 0;        // dome-light replay: this pixel's first call record (P.lrec)
    uint32_t lcall = 0;      //   dome calls so far

    __device__ float next_rand() { return rng(pixel, skey, dim++, seed); }

    template <bool COUNT>
    __device__ bool occluded(v3 from, v3 L, float tMax) {
        shadow_rays++;
        if constexpr (MODE == kGen) {  // no shading result depends on the answer but the final sums
            const size_t s = slot0 + nslot++;
            P.ray_o[s] = make_float4(from.x, from.y, from.z, tMax);
            P.ray_d[s] = make_float4(L.x, L.y, L.z, shadow_time);
            return false;
        } else if constexpr (MODE == kResolve) {
            return P.occl[slot0 + nslot++] != 0;
        } else {
            DRay r = make_ray(from, L, shadow_time);
            DHit h{tMax, 0.f, 0.f, -1};
            return traverse<true, COUNT, FAST, INST, true, false, !INST>(T, r, 0.001f, h, st);
        }
    }

    // The shadow walk of Light::m_fastShadows = false for rectangle / dome lights
    // (src/RectangleLight.cpp:93-116, src/DomeLight.cpp:123-145), fused chain kernels
    // only (the dispatcher runs such scenes there, off the wavefront passes, whose
    // shadow answers are one bit): closest-hit rays along L, each from the previous hit
    // point and bounded by the previous hit's t (the reference's sampleHit lives
    // across the loop; the first bound is t0).  A hit whose interpolated normal
    // (HitInfo::getInterpolatedNormal, src/Ray.cpp:51-65: mesh normals, object
    // space for a proxy hit) faces the ray scales the attenuation by its
    // material's refractAmt (0 for Lambert, which the reference leaves
    // uninitialised).  Ends at a miss, when the summed t reaches `limit`, or at an
    // attenuation <= epsilon.  Every trace counts as a shadow ray.
    template <bool COUNT>
    __device__ float transmit(v3 from, v3 L, float t0, float limit) {
        float att = 1.0f, done = 0.0f, tb = t0;
        v3 o = from;
        while (done < limit && att > 0.001f) {
            shadow_rays++;
            const DRay r = make_ray(o, L, shadow_time);
            DHit h{tb, 0.f, 0.f, -1};
            if (!traverse<false, COUNT, FAST, INST>(T, r, 0.001f, h, st)) break;
            int32_t ps_i = h.prim;
            if (INST && h.prim >= P.n_world) ps_i = inst_shade_index(h.prim, nullptr);
            const PrimShade ps = P.prims[ps_i];
            const float c = 1.0f - h.a - h.b;
            const float4 n0 = P.normals[ps.n[0]], n1 = P.normals[ps.n[1]], n2 = P.normals[ps.n[2]];
            const v3 hitN = normalized(add(add(scale(mk(n0.x, n0.y, n0.z), c), scale(mk(n1.x, n1.y, n1.z), h.a)),
                                           scale(mk(n2.x, n2.y, n2.z), h.b)), rsqT);
            if (dot(hitN, neg(L)) > 0.0f) {
                const DevMaterial& M = P.mats[ps.mat];
                att *= M.type == MRT_BLINN ? M.refract : 0.0f;
            }
            o = add(o, scale(L, h.t));
            tb = h.t;
            done += h.t;
        }
        return att;
    }
    // shadow answer of a rect / dome light sample: 0 / 1, or the transparency walk
    template <bool COUNT>
    __device__ float light_vis(const DevLight& l, v3 from, v3 L, float tMax, float limit) {
        if constexpr (MODE == kFused && !POINT_ONLY && REC != 0) {
            if (l.transparent) return transmit<COUNT>(from, L, tMax, limit);
        }
        return occluded<COUNT>(from, L, tMax) ? 0.0f : 1.0f;
    }

    // PointLight::sampleLight, src/PointLight.cpp:8-81
    template <bool COUNT>
    __device__ float point_light(const DevLight& l, v3 from, v3 normal, v3 rVec, float& outSpec) {
        v3 L = sub(mk(l.pos[0], l.pos[1], l.pos[2]), from);
        float nDotL = dot(normal, L);
        if (!(nDotL > 0.0f)) { outSpec = 0.f; return 0.0f; }
        float falloff = dot(L, L);
        float distanceRecip = rsqrt_nr(falloff, rsqT);
        falloff = rcp_nr(falloff, rcpT);
        float distance = rcp_nr(distanceRecip, rcpT);
        L = scale(L, distanceRecip);
        nDotL *= distanceRecip;
        // Everything the light returns except the shadow bit is formed before the
        // shadow ray, so only three scalars stay live across its traversal.
        const float A = (l.power * falloff) * (0.25f / 3.1415926f);
        const float rdl = std_max(0.f, dot(rVec, L));
        float attenuate = 1.0f;
        if (l.cast_shadows && occluded<COUNT>(from, L, distance)) attenuate = 0.0f;
        attenuate *= nDotL;
        outSpec = rdl * attenuate;
        return A * attenuate;
    }

    // RectangleLight::sampleLight, src/RectangleLight.cpp:42-136 (fast or transparent shadows)
    template <bool COUNT>
    __device__ v3 rect_light(const DevLight& l, v3 from, v3 normal, v3 rVec, float& outSpec) {
        v3 v1 = mk(l.v1[0], l.v1[1], l.v1[2]), v2 = mk(l.v2[0], l.v2[1], l.v2[2]), w3 = mk(l.v3[0], l.v3[1], l.v3[2]);
        v3 acc = mk(0, 0, 0);
        float tmpSpec = 0.f, recip = 1.0f, falloff = 1.0f;
        int done = 0;
        bool cut = false;
        do {
            float e1 = next_rand();
            float e2 = next_rand();
            e2 = ((double)e2 > 0.99) ? (float)0.99 : e2;
            v3 rd = sub(add(add(v1, scale(sub(v2, v1), e1)), scale(sub(w3, v1), e2)), from);
            float nDotL = dot(normal, rd);
            float att = 1.0f;
            if (nDotL > 0.001f) {
                falloff = dot(rd, rd);
                float dr = rsqrt_nr(falloff, rsqT);
                falloff = rcp_nr(falloff, rcpT);
                float dist = rcp_nr(dr, rcpT);
                rd = scale(rd, dr);
                if (l.cast_shadows) att = light_vis<COUNT>(l, from, rd, dist - 0.001f, dist);
            } else {
                att = 0.0f;
            }
            float E = (l.power * falloff) * (0.25f / 3.1415926f);
            done++;
            recip = 1.0f / (float)done;
            float Es = E * recip;
            cut = ((Es + Es + Es) * 0.333333f) < l.noise;
            float Ea = E * att;
            acc = add(acc, mk(Ea, Ea, Ea));
            tmpSpec += std_max(0.f, dot(rVec, rd)) * att;
        } while (done < l.samples && !cut);
        outSpec = tmpSpec * recip;
        return scale(acc, recip);
    }

    // DomeLight::sampleLight, src/DomeLight.cpp:80-160 (fast shadows; m_numSamples
    // draws, one for secondary shading, :89).  A draw below the shading horizon is
    // redrawn without counting it (`continue` at :106 skips samplesDone++); after
    // kDomeMaxRejects such redraws in one call the loop stops (the reference would
    // not terminate when the whole map lies below the horizon).
    static constexpr int kDomeMaxRejects = 256;
    template <bool COUNT>
    __device__ v3 dome_light(const DevLight& l, v3 from, v3 normal, v3 rVec, float& outSpec, bool secondary) {
        const DevDome& D = P.domes[l.dome];
        const int numSamples = secondary ? 1 : l.samples;
        v3 acc = mk(0, 0, 0);
        float tmpSpec = 0.f, recip = 1.0f;
        if constexpr (MODE == kResolve) {
            if (P.lrec) {   // replay 2a's samples: which samples were taken, their E and the RNG
                            // draws do not depend on the answers; the sums are the loop's below
                const uint32_t rc = P.lrec[lrec0 + lcall++];
                dim += rc >> 8;
                const int ns = (int)(rc & 0xFFu);
                for (int j = 0; j < ns; j++) {
                    const size_t s = slot0 + nslot++;
                    const float4 e = P.ray_e[s];
                    const float att = P.occl[s] != 0 ? 0.0f : 1.0f;
                    shadow_rays++;
                    recip = 1.0f / (float)(j + 1);
                    acc = add(acc, scale(mk(e.x, e.y, e.z), att));
                    tmpSpec += e.w * att;
                }
                outSpec = tmpSpec * recip;
                return scale(acc, recip);
            }
        }
        const uint32_t dim0 = dim;
        int done = 0, rejects = 0;
        bool cut = false;
        do {
            const float e1 = next_rand();
            const float e2 = next_rand();
            float pdf0, pdf1;
            const float fu = dist_sample_guided(D.cdf_u, D.func_u, D.guide_u, D.nu, D.inv_int_u, e1, pdf0);
            const int iu = (int)fu;
            const int u = iu == D.nu ? iu - 1 : iu;
            const size_t cv = (size_t)u * (D.nv + 1);
            const float fv = dist_sample_guided(D.cdf_v + cv, D.func_v + (size_t)u * D.nv, D.guide_v + cv, D.nv,
                                                D.inv_int_v[u], e2, pdf1);
            const int iv = (int)fv;
            const float cosT = D.cos_v[iv], sinT = D.sin_v[iv], sinP = D.sin_u[iu], cosP = D.cos_u[iu];
            const v3 dir = mk(-sinT * cosP, -cosT, -sinT * sinP);
            if (dot(normal, dir) < 0.0f) {
                if (++rejects >= kDomeMaxRejects) break;
                continue;
            }
            const float pdf = (pdf0 * pdf1) / (kTwoPI2 * sinT);
            const float4 rc = reinterpret_cast<const float4*>(D.rad)[(size_t)iv * (D.nu + 1) + iu];   // tex_lookup_dir of dir (host table)
            const v3 img = mk(rc.x, rc.y, rc.z);
            const float inv = 1.0f / pdf;  // E = m_Gain * imageSample / pdf (Vector3::operator/)
            const v3 E = scale(scale(img, l.power), inv);
            float att = 1.0f;
            if (MODE == kGen && P.lrec) P.ray_e[slot0 + nslot] = make_float4(E.x, E.y, E.z, dot(rVec, dir));
            att = light_vis<COUNT>(l, from, dir, 1e12f, 1e12f);   // sampleHit.t = MIRO_TMAX
            done++;
            recip = 1.0f / (float)done;
            const v3 Es = scale(E, recip);
            cut = (((Es.x + Es.y) + Es.z) * 0.333333f) < l.noise;
            acc = add(acc, scale(E, att));
            tmpSpec += dot(rVec, dir) * att;
        } while (done < numSamples && !cut);
        if (MODE == kGen && P.lrec) P.lrec[lrec0 + lcall++] = (uint32_t)done | ((dim - dim0) << 8);
        outSpec = tmpSpec * recip;
        return scale(acc, recip);
    }

    // Light::sampleLight dispatch; `secondary` = the isSecondary argument
    template <bool COUNT>
    __device__ v3 sample_light(int li, v3 from, v3 normal, v3 rVec, float& spec, bool secondary = false) {
        const DevLight& l = P.lights[li];
        if (POINT_ONLY || l.type == MRT_POINT_LIGHT) {
            float e = point_light<COUNT>(l, from, normal, rVec, spec);
            return mk(e, e, e);
        }
        if constexpr (!POINT_ONLY) {
            if (l.type == MRT_DOME_LIGHT) return dome_light<COUNT>(l, from, normal, rVec, spec, secondary);
            return rect_light<COUNT>(l, from, normal, rVec, spec);
        }
        return mk(0, 0, 0);
    }

    // HitInfo::getAllInfos (normals), src/Ray.cpp:5-49
    // an instance hit (id >= n_world) names instance i's BLAS object id - hit_base
    // PrimShade index of instance hit id `prim` (and the instance)
    __device__ int32_t inst_shade_index(int32_t prim, int* inst) const {
        int lo = 0, hi = P.n_insts - 1;  // the last instance with hit_base <= id
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (P.insts[mid].hit_base <= prim) lo = mid;
            else hi = mid - 1;
        }
        if (inst) *inst = lo;
        return P.insts[lo].shade_base + (prim - P.insts[lo].hit_base);
    }
    __device__ void normals(const DHit& h, v3& N, v3& geoN, uint32_t& mat) {
        int32_t ps_i = h.prim;
        int inst = -1;
        if (INST && h.prim >= P.n_world) ps_i = inst_shade_index(h.prim, &inst);
        PrimShade ps = P.prims[ps_i];
        float4 A = P.verts[ps.v[0]], B = P.verts[ps.v[1]], C = P.verts[ps.v[2]];
        geoN = normalized(cross(mk(B.x - A.x, B.y - A.y, B.z - A.z), mk(C.x - A.x, C.y - A.y, C.z - A.z)), rsqT);
        float c = 1.0f - h.a - h.b;
        float4 n0 = P.normals[ps.n[0]], n1 = P.normals[ps.n[1]], n2 = P.normals[ps.n[2]];
        v3 s = add(add(scale(mk(n0.x, n0.y, n0.z), c), scale(mk(n1.x, n1.y, n1.z), h.a)), scale(mk(n2.x, n2.y, n2.z), h.b));
        N = normalized(s, rsqT);
        if (INST && inst >= 0) {  // HitInfo::getAllInfos with m_proxy (src/Ray.cpp:27-31)
            const float* T = P.insts[inst].inv_t;
            geoN = normalized(xform_dir3(T, geoN), rsqT);
            N = normalized(xform_dir3(T, N), rsqT);
        }
        mat = ps.mat;
        psi = ps_i;
    }

    // HitInfo::getAllInfos' texture part (src/Ray.cpp:33-47) and the maps of
    // Lambert::shade (colour, src/Lambert.cpp:32-36) / Blinn::shade (colour,
    // normal, specular, reflect, refract, src/Blinn.cpp:114-142) at the hit of the
    // last normals() call.  (u, v) interpolate the texture coordinates, or are
    // (a, b) without them; the tangent frame interpolates over the normal indices.
    int32_t psi = 0;   // PrimShade index of the last normals() call
    __device__ void maps(const DHit& h, const DevMaterial& M, bool blinn, v3& N, v3& kd, float& spec_amt, float& refl,
                         float& refr) {
        float u = h.a, v = h.b;
        v3 T = mk(0, 0, 0), BT = mk(0, 0, 0);
        const bool nmap = blinn && M.maps[kMapNormal] >= 0;
        if (P.puv) {
            const uint4 t = P.puv[psi];
            if (t.w) {
                const float c = 1.0f - h.a - h.b;
                if (nmap) {
                    const PrimShade ps = P.prims[psi];
                    const float4 t0 = P.tans[ps.n[0]], t1 = P.tans[ps.n[1]], t2 = P.tans[ps.n[2]];
                    const float4 b0 = P.btans[ps.n[0]], b1 = P.btans[ps.n[1]], b2 = P.btans[ps.n[2]];
                    T = normalized(add(add(scale(mk(t0.x, t0.y, t0.z), c), scale(mk(t1.x, t1.y, t1.z), h.a)),
                                       scale(mk(t2.x, t2.y, t2.z), h.b)), rsqT);
                    BT = normalized(add(add(scale(mk(b0.x, b0.y, b0.z), c), scale(mk(b1.x, b1.y, b1.z), h.a)),
                                        scale(mk(b2.x, b2.y, b2.z), h.b)), rsqT);
                }
                const float2 a0 = P.uvs[t.x], a1 = P.uvs[t.y], a2 = P.uvs[t.z];
                u = a0.x * c + a1.x * h.a + a2.x * h.b;
                v = a0.y * c + a1.y * h.a + a2.y * h.b;
            }
        }
        auto look = [&](int tex) {
            const DevTexture& X = P.texs[tex];
            return tex_lookup4(X.data, X.W, X.H, X.type, u, v);
        };
        if (M.maps[kMapColor] >= 0) {
            const float4 x = look(M.maps[kMapColor]);
            kd = mk(x.x, x.y, x.z);
        }
        if (!blinn) return;
        if (nmap) {   // N = texN.x*T + texN.y*BT + texN.z*N, not renormalised
            const float4 x = look(M.maps[kMapNormal]);
            N = add(add(scale(T, x.x), scale(BT, x.y)), scale(N, x.z));
        }
        if (M.maps[kMapSpecular] >= 0) {
            const float4 x = look(M.maps[kMapSpecular]);
            spec_amt = ((x.x + x.y) + x.z) * 0.3333333f * spec_amt;
        }
        if (M.maps[kMapReflect] >= 0) {
            const float4 x = look(M.maps[kMapReflect]);
            refl = ((x.x + x.y) + x.z) * 0.3333333f * refl;
        }
        if (M.maps[kMapRefract] >= 0) {
            const float4 x = look(M.maps[kMapRefract]);
            refr = ((x.x + x.y) + x.z) * 0.3333333f * refr;
        }
    }

    // Scene::sampleScene hit branch (src/Scene.cpp:224-233): m_numPaths shade()
    // calls on the camera ray, each path its own RNG sub-stream.
    template <bool COUNT>
    __device__ v3 shade(const DRay& r, const DHit& h) {
        v3 N, geoN;
        uint32_t mi;
        normals(h, N, geoN, mi);
        const DevMaterial& M = P.mats[mi];
        v3 P_ = mk(r.o[0] + h.t * r.d[0], r.o[1] + h.t * r.d[1], r.o[2] + h.t * r.d[2]);  // Ray::getPoint
        v3 kd = mk(M.kd[0], M.kd[1], M.kd[2]), ka = mk(M.ka[0], M.ka[1], M.ka[2]);
        float spec_amt = M.spec_amt, refl_unused = M.reflect, refr_unused = M.refract;
        if (P.has_maps) maps(h, M, M.type != MRT_LAMBERT, N, kd, spec_amt, refl_unused, refr_unused);
        v3 result = mk(0, 0, 0);
        // the camera ray's IOR history [1, 1.001]: Blinn::shade pops it on a
        // back-face hit and the pop persists into the next path (src/Blinn.cpp:176-179)
        IorCam cam;
        for (int path = 0; path < P.num_paths; path++) {
            skey = sample * 1024u + (uint32_t)path;
            dim = level_key(0);
            v3 sh;
            if constexpr (MODE == kFused && REC) {   // secondary rays / path tracing in the scene
                result = add(result, shade_path<COUNT>(r, h, cam));
                continue;
            }
            if (M.type == MRT_LAMBERT) {  // Lambert::shade
                v3 L = mk(0, 0, 0);
                for (int i = 0; i < P.n_lights; i++) {
                    float discard;
                    v3 E = sample_light<COUNT>(i, P_, N, mk(0, 0, 0), discard);
                    L = add(L, mul(E, kd));
                }
                sh = add(L, ka);
            } else {  // Blinn::shade, direct branch
                v3 rayD = mk(r.d[0], r.d[1], r.d[2]);
                v3 viewDir = neg(rayD);
                float vDotN = dot(viewDir, N), vDotGeoN = dot(viewDir, geoN);
                bool same = (vDotN * vDotGeoN) >= 0.0f;
                v3 n = same ? N : geoN;
                vDotN = same ? vDotN : vDotGeoN;
                if (vDotN < 0.0f) { vDotN = -vDotN; n = neg(n); }
                v3 rVec = add(rayD, scale(n, 2.0f * vDotN));
                (void)next_rand();  // Russian-roulette draw (src/Blinn.cpp:195); weight 1
                v3 ks = mk(M.ks[0], M.ks[1], M.ks[2]);
                v3 Ld = mk(0, 0, 0), Ls = mk(0, 0, 0);
                for (int i = 0; i < P.n_lights; i++) {
                    float spec = 0.f;
                    v3 E = sample_light<COUNT>(i, P_, n, rVec, spec);
                    float pw = (M.spec_exp == 1.0f) ? spec : spec_pow(spec, M.spec_exp);
                    Ls = add(Ls, scale(scale(mul(E, ks), spec_amt), pw));
                    Ld = add(Ld, mul(E, kd));
                }
                Ld = add(Ld, ka);
                v3 z = mk(0, 0, 0);
                sh = add(add(scale(add(add(Ld, Ls), z), 1.0f), scale(add(z, z), 1.0f)), mk(M.le[0], M.le[1], M.le[2]));
            }
            result = add(result, sh);
        }
        return scale(result, 1.0f / (float)P.num_paths);
    }

    // Material::fresnel, full form (src/Material.h:47-55): n1*sin(acosf(c))/n2, glibc's
    // acosf and sinf restated bit for bit (fd_acosf, gl_sinf: mrt_libm.h)
    __device__ static float fresnel(float n1, float n2, float c) {
        const float n1CosTh = n1 * c;
        const float th = fd_acosf(c);
        const float n1_n2SinTh = (n1 * gl_sinf(th)) / n2;
        const float n2CosTh = n2 * std_max(0.0f, sqrtf(1.0f - n1_n2SinTh * n1_n2SinTh));
        const float Rs = (n1CosTh - n2CosTh) / (n1CosTh + n2CosTh);
        return Rs * Rs;
    }

    // Material::getCosineDistributedSamples (src/Material.cpp:14-41): two draws,
    // RSQRTSS/RCPSS square roots, glibc's cosf / sinf of the float 2 pi e1 (gl_cosf /
    // gl_sinf, bit for bit)
    __device__ v3 cosine_sample(v3 N) {
        const float e1 = next_rand();
        float e2 = next_rand();
        e2 = ((double)e2 > 0.99) ? (float)0.99 : e2;
        const v3 a = ((double)fabsf(N.x) > 0.1) ? mk(0, 1, 0) : mk(1, 0, 0);
        const v3 u = normalized(cross(a, N), rsqT);
        const v3 v = cross(N, u);
        const float t = (2.0f * 3.1415926f) * e1;
        const float sqrte2 = rcp_nr(rsqrt_nr(e2, rsqT), rcpT);
        const float sqrt1_e2 = rcp_nr(rsqrt_nr(fabsf(1.0f - e2), rsqT), rcpT);
        const float c = gl_cosf(t), s = gl_sinf(t);
        return normalized(add(add(scale(u, c * sqrte2), scale(v, s * sqrte2)), scale(N, sqrt1_e2)), rsqT);
    }

    // (forced inline: as a call it takes the Shader's reference to the kernel's RenderParams
    // out of the kernarg segment -- a 2288-B private copy per lane, R3's REC kernels 2x slower)
    __device__ __forceinline__ v3 env_color(const DevMaterial& M, v3 d) { return mat_env(P, M, d); }

    // the camera ray's history: [1, 1.001, (a level-0 refraction push)] and its index
    struct IorCam {
        float v1 = 1.001f, v2 = 0.f;
        int idx = 1;
        __device__ float at(int i) const { return i == 0 ? 1.0f : (i == 1 ? v1 : v2); }
    };
    __device__ float& ior_at(int i) { return iorS[i * kWG]; }
    // level record word w of chain level k of the fused kernels (global memory,
    // one column per thread)
    __device__ ChainRec rec_fused(int k) const { return ChainRec{lvl + (size_t)k * P.lvl_words * P.gstride, P.gstride}; }

    // One level of Material::shade with Blinn's secondary rays and path tracing
    // (src/Blinn.cpp:39-335): Fresnel-weighted Russian roulette between direct
    // lighting (+ Blinn::calculatePathTracing's GI ray) and one reflection or
    // refraction ray (bounces < 5), with each ray's IOR history (Ray::IORList,
    // src/Ray.h:43-50; LDS column ior_at below the camera ray, `cam` for it).
    // Either the level's value is final (o.spawn = false, o.val), or it spawns
    // one child ray (o.r2): its terms go to the level record `rec` -- reflect /
    // refract: rrWeightRecip, rrWeightRecipSpec; GI: also Ls, the translucency
    // and each light's E * kd, all sampled before the child is traced (each
    // level draws from its own RNG key) -- `cs` and the IOR column become the
    // child's, and chain_combine() folds the child's value (or, if it misses,
    // the environment / nothing, o.env_miss) into the level's in the reference's
    // operation order.  The fused kernels trace the child inline (shade_path);
    // the wavefront chain kernels queue it.
    static constexpr int kMaxBounce = 5;
    uint32_t secondary = 0;
    template <bool COUNT>
    __device__ void level(const DRay& r, const DHit& h, ChainState& cs, IorCam& cam, const ChainRec& rec, LevelOut& o) {
        const v3 z = mk(0, 0, 0);
        o.spawn = false;
        o.split = false;
        dim = level_key(cs.depth, cs.br);
        v3 N, geoN;
        uint32_t mi;
        normals(h, N, geoN, mi);
        const DevMaterial& M = P.mats[mi];
        const v3 Pt = mk(r.o[0] + h.t * r.d[0], r.o[1] + h.t * r.d[1], r.o[2] + h.t * r.d[2]);
        v3 kd = mk(M.kd[0], M.kd[1], M.kd[2]);
        const v3 ka = mk(M.ka[0], M.ka[1], M.ka[2]);
        float spec_amt = M.spec_amt, reflect = M.reflect, refract = M.refract;   // localSpecAmt / ReflectAmt / RefractAmt
        if (P.has_maps) maps(h, M, M.type != MRT_LAMBERT, N, kd, spec_amt, reflect, refract);
        if (M.type == MRT_LAMBERT) {   // Lambert::shade: no secondary rays (isSecondary not passed on)
            v3 L = z;
            for (int i = 0; i < P.n_lights; i++) {
                float discard;
                L = add(L, mul(sample_light<COUNT>(i, Pt, N, z, discard), kd));
            }
            o.val = add(L, ka);
            return;
        }
        const v3 le = mk(M.le[0], M.le[1], M.le[2]);
        const v3 rayD = mk(r.d[0], r.d[1], r.d[2]);
        const v3 viewDir = neg(rayD);
        float vDotN = dot(viewDir, N);
        const float vDotGeoN = dot(viewDir, geoN);
        const bool same = (vDotN * vDotGeoN) >= 0.0f;
        v3 n = same ? N : geoN;
        vDotN = same ? vDotN : vDotGeoN;
        bool flip = false;
        if (vDotN < 0.0f) { flip = true; vDotN = -vDotN; n = neg(n); }
        v3 rVec = add(rayD, scale(n, 2.0f * vDotN));
        if (M.gloss < 1.0f) {   // glossy reflection vector (src/Blinn.cpp:166-171)
            const v3 rd = cosine_sample(n);
            rVec = normalized(add(scale(rVec, M.gloss), scale(rd, 1.0f - M.gloss)), rsqT);
        }
        // inIOR, then a back-face hit pops the (mutable) history (src/Blinn.cpp:167-185);
        // a dispersive material hit by a ray that is not a refraction ray takes
        // outIOR = m_ior[0..2] and does not pop
        const bool disp = M.disperse && !cs.refr;
        float inIOR, outIOR = M.ior;
        if (disp) {
            inIOR = cs.depth == 0 ? cam.at(cam.idx) : ior_at(cs.idx);
            outIOR = M.ior3[0];
        } else if (cs.depth == 0) {
            inIOR = cam.at(cam.idx);
            if (flip) { if (cam.idx > 0) cam.idx--; outIOR = cam.at(cam.idx); }
        } else {
            inIOR = ior_at(cs.idx);
            if (flip) { if (cs.idx > 0) cs.idx--; outIOR = ior_at(cs.idx); }
        }
        const float curIOR = cs.depth == 0 ? cam.at(cam.idx) : ior_at(cs.idx);   // r_IOR() after the pop
        float Rs = 0.f, Ts = 0.f;
        if (M.reflect > 0.0f || M.refract > 0.0f) {
            Rs = fresnel(inIOR, outIOR, vDotN);
            Ts = 1.0f - Rs;
        }
        float rr = next_rand();
        const float rrW = (1.0f - Rs * reflect) - Ts * refract;
        const float rrRecip = (rrW > 0.f) ? 1.f / rrW : 1.f;
        const float rrSpec = (1.f - rrW > 0.f) ? 1.f / (1.f - rrW) : 1.f;
        const v3 ks = mk(M.ks[0], M.ks[1], M.ks[2]);
        if (rr <= rrW) {   // direct lighting
            bool child = false;
            v3 randD = z;
            v3 Ld = z;
            if constexpr (REC == 2) {   // Blinn::calculatePathTracing (src/Blinn.cpp:39-89)
                v3 pt = z;
                if (M.emitter) {
                    pt = add(z, scale(le, M.emitted));
                } else if (cs.gi < P.max_bounces - 1) {
                    randD = cosine_sample(n);
                    child = true;
                } else {   // last bounce: the lights directly, isSecondary, rVec = 0
                    for (int i = 0; i < P.n_lights; i++) {
                        float spec = 0.f;
                        pt = add(pt, mul(sample_light<COUNT>(i, Pt, n, z, spec, true), kd));
                    }
                }
                if (!child) Ld = add(Ld, pt);
            }
            v3 Ls = z;
            for (int i = 0; i < P.n_lights; i++) {
                float spec = 0.f;
                v3 E = sample_light<COUNT>(i, Pt, n, rVec, spec, cs.secondary);
                float pw = (M.spec_exp == 1.0f) ? spec : spec_pow(spec, M.spec_exp);
                Ls = add(Ls, scale(scale(mul(E, ks), spec_amt), pw));
                const v3 term = mul(E, kd);
                if (child) { rec(12 + 3 * i) = term.x; rec(13 + 3 * i) = term.y; rec(14 + 3 * i) = term.z; }
                else Ld = add(Ld, term);
            }
            v3 tr = z;
            if (M.translucency > 0.01f) {   // lights seen through the surface (src/Blinn.cpp:224-236)
                v3 total = z;
                shadow_time = .001f;
                for (int i = 0; i < P.n_lights; i++) {
                    float spec = 0.f;
                    total = add(total, sample_light<COUNT>(i, Pt, neg(n), rVec, spec, cs.secondary));
                }
                shadow_time = time;
                tr = add(z, mul(scale(total, M.translucency), kd));
            }
            if (child) {   // descend into the GI ray: IOR history [1, current]
                rec(0) = __int_as_float((int)mi | (kGI << 16));
                rec(1) = rrRecip; rec(2) = rrSpec;
                rec(3) = Ls.x; rec(4) = Ls.y; rec(5) = Ls.z;
                rec(6) = tr.x; rec(7) = tr.y; rec(8) = tr.z;
                rec(9) = kd.x; rec(10) = kd.y; rec(11) = kd.z;   // diffuseColor (colour map) for the combine
                ior_at(0) = 1.0f; ior_at(1) = curIOR; cs.idx = 1;
                cs.depth++; cs.gi++;
                cs.secondary = true;
                cs.refr = false;   // IS_PRIMARY_RAY
                o.spawn = true;
                o.r2 = make_ray(Pt, randD, time);
                o.dir = randD;
                o.env_miss = M.sample_env && P.sample_env;
                secondary++;
                return;
            }
            Ld = add(Ld, ka);
            o.val = add(add(scale(add(add(Ld, Ls), tr), rrRecip), scale(add(z, z), rrSpec)), le);
            return;
        }
        const v3 base = scale(add(add(add(z, ka), z), z), rrRecip);   // (Ld + Ls + translucency) * rrWeightRecip
        rr = next_rand();
        bool refr, spawn;
        v3 dir;
        if (rr < reflect * Rs) {
            refr = false;
            dir = rVec;
            spawn = reflect * Rs > 0.0f && cs.bounces < kMaxBounce;
            if (spawn && cs.depth == 0) {   // the child copies the camera ray's history
                ior_at(0) = 1.0f; ior_at(1) = cam.v1; ior_at(2) = cam.v2; cs.idx = cam.idx;
            }
        } else if (disp && refract * Ts > 0.0f) {
            // dispersion (src/Blinn.cpp:275-301): three refraction children, one per
            // colour channel, traced by the caller in channel order (disp_child)
            if (cs.bounces >= kMaxBounce) {   // none traced: Lt = ks * environment along channel 2's direction
                const v3 L = add(z, mul(ks, env_color(M, disp_dir(rayD, n, vDotN, inIOR / M.ior3[2]))));
                o.val = add(add(base, scale(add(z, L), rrSpec)), le);
                return;
            }
            rec(0) = __int_as_float((int)mi | (kDisp << 16));
            rec(1) = rrRecip; rec(2) = rrSpec;
            rec(3) = 0.f; rec(4) = 0.f; rec(5) = 0.f;   // Lt
            rec(6) = __int_as_float(0); rec(7) = __int_as_float(0);   // next child, some child hit
            rec(8) = Pt.x; rec(9) = Pt.y; rec(10) = Pt.z;
            rec(11) = rayD.x; rec(12) = rayD.y; rec(13) = rayD.z;
            rec(14) = n.x; rec(15) = n.y; rec(16) = n.z;
            rec(17) = vDotN; rec(18) = inIOR;
            rec(19) = M.ior3[0]; rec(20) = M.ior3[1]; rec(21) = M.ior3[2];
            rec(22) = __int_as_float(cs.depth == 0 ? cam.idx : cs.idx);
            rec(23) = __int_as_float(cs.gi); rec(24) = __int_as_float(cs.bounces); rec(25) = __int_as_float(cs.br);
            if (cs.depth > 0)
                for (int j = 0; j < kIorCap; j++) rec(26 + j) = ior_at(j);
            o.spawn = true;
            o.split = true;
            return;
        } else if (refract * Ts > 0.0f) {
            refr = true;
            const float q = inIOR / outIOR;
            const float sq = std_max(0.0f, sqrtf(1.0f - (q * q) * (1.0f - vDotN * vDotN)));
            dir = normalized(add(scale(rayD, q), scale(n, q * vDotN - sq)), rsqT);
            spawn = cs.bounces < kMaxBounce;
            if (spawn) {   // r_IOR.push(outIOR) on the mutable history, the child copies it
                if (cs.depth == 0) {
                    if (cam.idx == 0) cam.v1 = outIOR; else cam.v2 = outIOR;
                    ior_at(0) = 1.0f; ior_at(1) = cam.v1; ior_at(2) = cam.v2; cs.idx = cam.idx + 1;
                } else {
                    ior_at(cs.idx + 1) = outIOR; cs.idx++;
                }
            }
        } else {   // refraction branch with nothing to refract: Lr = Lt = 0
            o.val = add(add(base, scale(add(z, z), rrSpec)), le);
            return;
        }
        if (spawn) {
            rec(0) = __int_as_float((int)mi | ((refr ? kRefr : kRefl) << 16));
            rec(1) = rrRecip; rec(2) = rrSpec;
            cs.depth++; cs.bounces++;
            cs.secondary = false;   // shade(..) with the default isSecondary
            cs.refr = refr;         // IS_REFRACT_RAY / IS_REFLECT_RAY
            o.spawn = true;
            o.r2 = make_ray(Pt, dir, time);
            o.dir = dir;
            o.env_miss = true;
            secondary++;
            return;
        }
        const v3 L = add(z, mul(ks, env_color(M, dir)));   // Lr / Lt += m_ks * environment
        o.val = add(add(base, scale(refr ? add(z, L) : add(L, z), rrSpec)), le);
    }

    // the refraction direction of Blinn::shade (src/Blinn.cpp:281-283,307-309)
    __device__ v3 disp_dir(v3 rayD, v3 n, float vDotN, float q) const {
        const float sq = std_max(0.0f, sqrtf(1.0f - (q * q) * (1.0f - vDotN * vDotN)));
        return normalized(add(scale(rayD, q), scale(n, q * vDotN - sq)), rsqT);
    }
    // Child i of the dispersive split recorded at level k: its ray, its chain state
    // and its IOR history (the parent's with outIOR[i] pushed, src/Blinn.cpp:285-286;
    // on the camera ray the push persists into its later paths, as at level 0 above).
    __device__ DRay disp_child(const ChainRec& rec, int k, int i, ChainState& cs, IorCam& cam) {
        const float outI = rec(19 + i);
        const v3 dir = disp_dir(mk(rec(11), rec(12), rec(13)), mk(rec(14), rec(15), rec(16)), rec(17), rec(18) / outI);
        const int pidx = __float_as_int(rec(22));
        if (k == 0) {
            if (cam.idx == 0) cam.v1 = outI; else cam.v2 = outI;
            ior_at(0) = 1.0f; ior_at(1) = cam.v1; ior_at(2) = cam.v2;
        } else {
            for (int j = 0; j < kIorCap; j++) ior_at(j) = rec(26 + j);
            ior_at(pidx + 1) = outI;
        }
        cs.idx = pidx + 1;
        cs.depth = k + 1;
        cs.gi = __float_as_int(rec(23));
        cs.bounces = __float_as_int(rec(24)) + 1;
        cs.secondary = false;
        cs.refr = true;
        cs.br = ((__float_as_int(rec(25)) << 2) | (i + 1)) & 0xFF;
        secondary++;
        return make_ray(mk(rec(8), rec(9), rec(10)), dir, time);
    }

    // Blinn::shade's recursion for one path, fused: each level's child ray is
    // traced inline, depth first, and a finished level's value is folded into
    // its parent's.  A chain level (one child) folds with chain_combine; a
    // dispersive level (three children, src/Blinn.cpp:275-301) adds each hit
    // child's colour masked to its channel, then traces the next child; a missed
    // dispersive child adds nothing, and with no child hit Lt takes the
    // environment along channel 2's direction.
    template <bool COUNT>
    __device__ v3 shade_path(DRay r, DHit h, IorCam& cam) {
        const v3 z = mk(0, 0, 0);
        ChainState cs;
        for (;;) {
            LevelOut o;
            const int d = cs.depth;
            level<COUNT>(r, h, cs, cam, rec_fused(d), o);
            v3 val = z;
            bool none = false, start = false;
            int k;
            if (!o.spawn) {
                val = o.val;
                k = d - 1;
            } else if (o.split) {
                start = true;   // level d starts its dispersive children
                k = d;
            } else {
                DHit h2{1e12f, 0.f, 0.f, -1};
                if (traverse<false, COUNT, FAST, INST>(T, o.r2, 0.001f, h2, st)) {
                    r = o.r2;
                    h = h2;
                    continue;
                }
                none = !o.env_miss;   // the missed child's value: environment, or nothing (GI, no env)
                val = none ? z : env_color(P.mats[__float_as_int(rec_fused(d)(0)) & 0xFFFF], o.dir);
                k = d;
            }
            bool descend = false;
            for (; k >= 0; k--) {   // fold up until a level has a child left to trace
                const ChainRec rec = rec_fused(k);
                const int info = __float_as_int(rec(0));
                if ((info >> 16) != kDisp) {
                    val = chain_combine(P, rec, val, none);
                    none = false;
                    continue;
                }
                const DevMaterial& M = P.mats[info & 0xFFFF];
                const v3 ks = mk(M.ks[0], M.ks[1], M.ks[2]);
                int i = __float_as_int(rec(6));
                if (!start) {   // child i - 1 hit and has its value: Lt += m_ks * (refraction * mask)
                    const v3 mask = mk(i == 1 ? 1.0f : 0.0f, i == 2 ? 1.0f : 0.0f, i == 3 ? 1.0f : 0.0f);
                    const v3 Lt = add(mk(rec(3), rec(4), rec(5)), mul(ks, mul(val, mask)));
                    rec(3) = Lt.x; rec(4) = Lt.y; rec(5) = Lt.z;
                    rec(7) = __int_as_float(1);
                }
                start = false;
                while (i < 3) {
                    const DRay c = disp_child(rec, k, i, cs, cam);
                    rec(6) = __int_as_float(++i);
                    DHit h2{1e12f, 0.f, 0.f, -1};
                    if (traverse<false, COUNT, FAST, INST>(T, c, 0.001f, h2, st)) {
                        r = c;
                        h = h2;
                        descend = true;
                        break;
                    }
                }
                if (descend) break;
                v3 Lt = mk(rec(3), rec(4), rec(5));
                if (__float_as_int(rec(7)) == 0) {   // doEnv: no child hit
                    const v3 dir2 = disp_dir(mk(rec(11), rec(12), rec(13)), mk(rec(14), rec(15), rec(16)), rec(17),
                                             rec(18) / rec(21));
                    Lt = add(Lt, mul(ks, env_color(M, dir2)));
                }
                const v3 ka = mk(M.ka[0], M.ka[1], M.ka[2]), le = mk(M.le[0], M.le[1], M.le[2]);
                const v3 base = scale(add(add(add(z, ka), z), z), rec(1));
                val = add(add(base, scale(add(z, Lt), rec(2))), le);
                none = false;
            }
            if (!descend) return val;
        }
    }
};

__device__ __forceinline__ uint8_t map8(const uint8_t* lut, float v) { return lut[map_index(v)]; }

// Tile schedule of a persistent wave (one 8x8 tile = one wave step).
//   sched 0: static grid-stride over all tiles.
//   sched 1: static XCD bands -- workgroups b, b+8, ... (observed to share one XCD
//            and its L2; placement is a speed hint only) walk one eighth.
//   sched 2: dynamic -- 8 tile counters (one 128-B line each), counter c hands
//            out tiles c, c+8, ...; a wave starts at counter blockIdx & 7 and moves
//            to the next counter when one runs dry, so every wave stays busy until
//            the frame is done.
//   sched 3: dynamic, counter c hands out the contiguous band c (L2 locality per
//            XCD) with the same stealing.
// Counters are zeroed per launch; every wave sees -1 after at most 8 empty probes.
// The kernel-argument block, re-read from the kernarg segment at this point: the
// compiler can no longer keep its fields in SGPRs across the traversals (where it
// ran out of SGPRs and spilled them to VGPR lanes); a few scalar-cache loads per
// tile instead.
// (The block is the kernel's only explicit argument: offset 0 of the kernarg segment.)
__device__ __forceinline__ const RenderParams& reload_params() {
    typedef const __attribute__((address_space(4))) RenderParams cparams;
    cparams* p = (cparams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const RenderParams*)p;
}

// This lane's index in its wave (v_mbcnt): recomputed where it is used instead of
// being held in a register across the traversals.
__device__ __forceinline__ int lane_id() { return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

struct TileSched {
    const RenderParams& P;
    int mode, cur, step, end, home, probe, band;
    uint32_t deq_ticks = 0;  // count mode: wall-clock ticks of the last dequeue
    __device__ __forceinline__ TileSched(const RenderParams& P_, int wave, int) : P(P_) {
        mode = P.sched;
        home = blockIdx.x & 7;
        probe = 0;
        band = (P.n_tiles + 7) >> 3;
        if (mode == 1 && (gridDim.x & 7) == 0) {
            int local = blockIdx.x >> 3, per = gridDim.x >> 3;
            int beg = home * band;
            end = min(P.n_tiles, beg + band);
            cur = beg + local * 4 + wave;
            step = per * 4;
        } else {
            if (mode == 1) mode = 0;
            cur = blockIdx.x * 4 + wave;
            step = gridDim.x * 4;
            end = P.n_tiles;
        }
    }
    __device__ __forceinline__ int dequeue() {
        int item = -1;
        const uint64_t q0 = P.wave_log ? wall_clock64() : 0;
        if (lane_id() == 0) {
            while (probe < 8) {
                const int c = (home + probe) & 7;
                const unsigned v = atomicAdd(P.queue + c * 32, 1u);
                const long idx = (mode == 3) ? (v < (unsigned)band ? (long)c * band + v : (long)P.n_tiles)
                                             : (long)c + 8l * v;
                if (idx < P.n_tiles) { item = (int)idx; break; }
                probe++;
            }
        }
        item = __builtin_amdgcn_readlane(item, 0);   // lane 0's atomic, as a scalar
        if (P.wave_log) deq_ticks = (uint32_t)(wall_clock64() - q0);
        return item;
    }
    // items are wave-uniform: readfirstlane puts them (and the frame / camera
    // lookups derived from them) in SGPRs
    __device__ __forceinline__ int first() {
        if (mode >= 2) return __builtin_amdgcn_readfirstlane(dequeue());
        return __builtin_amdgcn_readfirstlane(cur < end ? cur : -1);
    }
    __device__ __forceinline__ int next(int item) {
        if (mode >= 2) return __builtin_amdgcn_readfirstlane(dequeue());
        item += step;
        return __builtin_amdgcn_readfirstlane(item < end ? item : -1);
    }
};

// work item (8x8 tile, wave-uniform) -> frame of the item (frame mode: 0)
__device__ __forceinline__ int item_frame(const RenderParams& P, int item) {
    // clamped: an out-of-range id renders with the last camera instead of reading
    // past the kernel argument block
    return P.mode == 0 ? 0 : (int)min((uint32_t)P.buckets[item >> 4] / (uint32_t)P.buckets_per_frame, (uint32_t)(P.n_cams - 1));
}

// work item + lane -> pixel (x, y) and output slot
__device__ __forceinline__ bool item_pixel(const RenderParams& P, int item, int lane, int& x, int& y, size_t& slot) {
    if (P.mode == 0) {
        int tx = item % P.tiles_x, ty = item / P.tiles_x;
        x = tx * 8 + (lane & 7);
        y = ty * 8 + (lane >> 3);
        slot = (size_t)y * P.cam[0].W + x;
    } else {
        int bslot = item >> 4, sub = item & 15;
        int b = (int)((uint32_t)P.buckets[bslot] % (uint32_t)P.buckets_per_frame);
        int bx = b % P.buckets_x, by = b / P.buckets_x;
        int lx = (sub & 3) * 8 + (lane & 7), ly = (sub >> 2) * 8 + (lane >> 3);
        x = bx * 32 + lx;
        y = by * 32 + ly;
        slot = (size_t)bslot * 1024 + ly * 32 + lx;
    }
    return x < P.cam[0].W && y < P.cam[0].H;
}

// Store a pixel's linear RGB (before Image::Map) and its 8-bit Map (src/Image.cpp:19-35,
// 71-87) at its slot.  Frame mode and bucket tiles: the slot is the output index.  With
// frame_out (mrt_render_batch_frames_async) a bucket slot's pixel goes straight to its
// place in frame f of n_cams consecutive W*H frames -- e.g. rank 0's frame mapped into
// this process (mrt_ipc_open), so a rank of the multi-GPU split writes its buckets
// where they belong and no gather / unpack follows; pixels outside the frame and
// items of frames >= n_cams write nothing.
__device__ __forceinline__ void store_rgb(const RenderParams& P, size_t slot, v3 col) {
    if (P.frame_out) {
        const uint32_t id = (uint32_t)P.buckets[slot >> 10];
        const uint32_t bpf = (uint32_t)P.buckets_per_frame, f = id / bpf, b = id % bpf;
        const int x = (int)(b % (uint32_t)P.buckets_x) * 32 + (int)(slot & 31);
        const int y = (int)(b / (uint32_t)P.buckets_x) * 32 + (int)((slot >> 5) & 31);
        const int W = P.cam[0].W, H = P.cam[0].H;
        if (f >= (uint32_t)P.n_cams || x >= W || y >= H) return;
        slot = ((size_t)f * H + y) * W + x;
    }
    if (P.out_rgb) {
        float* o = P.out_rgb + 3 * slot;
        o[0] = col.x; o[1] = col.y; o[2] = col.z;
    }
    if (P.out_rgb8) {
        uint8_t* o8 = P.out_rgb8 + 3 * slot;
        o8[0] = map8(P.gamma, col.x); o8[1] = map8(P.gamma, col.y); o8[2] = map8(P.gamma, col.z);
    }
}

__device__ __forceinline__ void load_tables(const uint16_t* g, uint16_t* s, int words32) {
    for (int i = threadIdx.x; i < words32; i += kWG) reinterpret_cast<uint32_t*>(s)[i] = reinterpret_cast<const uint32_t*>(g)[i];
    __syncthreads();
}

// TIMES: write this wave's wall-clock record (wave log, span counters).  A fused
// kernel flushing two ray kinds writes it once, with log_nodes -- the other kind's
// node visits -- added to the wave log's node count.
template <bool COUNT, bool PRIMARY = false, bool TIMES = true>
__device__ __forceinline__ void flush_stats(const RenderParams& P, const TravStats& st, uint32_t shadow, int lane,
                                            uint64_t t0, uint32_t tiles, uint32_t log_nodes = 0, int wave = -1) {
    if (TIMES && (COUNT || P.wave_log) && lane == 0) {   // ramp / tail of the persistent waves
        const uint64_t t1 = wall_clock64();
        if (P.wave_log) {
            const int w = wave >= 0 ? wave : (int)(threadIdx.x >> 6);   // (wave: the caller's scalar index)
            unsigned long long* r = P.wave_log + kLogWords * ((size_t)blockIdx.x * (kWG / 64) + w);
            r[0] = t0; r[1] = t1; r[2] = tiles;
        }
        unsigned long long* c = P.ctr + (PRIMARY ? CTR_TP : CTR_TS);
        atomicMax(c + 0, (unsigned long long)~t0);
        atomicMax(c + 1, (unsigned long long)t0);
        atomicMax(c + 2, (unsigned long long)~t1);
        atomicMax(c + 3, (unsigned long long)t1);
    }
    // shadow rays (shade kernel) or primary hits (primary kernel), always counted
    unsigned long long sh = shadow;
    for (int off = 32; off > 0; off >>= 1) sh += __shfl_down(sh, off);
    if (lane == 0 && sh) atomicAdd(&P.ctr[PRIMARY ? CTR_HITS : CTR_SHADOW], sh);
    if (COUNT) {
        unsigned long long nv = st.nodes, lv = st.leaves, uv = st.uniform, xv = log_nodes;
        int msp = st.max_sp;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_down(nv, off);
            lv += __shfl_down(lv, off);
            uv += __shfl_down(uv, off);
            xv += __shfl_down(xv, off);
            msp = max(msp, __shfl_down(msp, off));
        }
        if (lane == 0) {
            if (TIMES && P.wave_log)
                P.wave_log[kLogWords * ((size_t)blockIdx.x * (kWG / 64) + (wave >= 0 ? wave : (int)(threadIdx.x >> 6))) + 3] = nv + xv;
            atomicAdd(&P.ctr[CTR_NODES], nv);
            atomicAdd(&P.ctr[CTR_LEAVES], lv);
            if (PRIMARY) {
                atomicAdd(&P.ctr[CTR_NODES_P], nv);
                atomicAdd(&P.ctr[CTR_LEAVES_P], lv);
                atomicAdd(&P.ctr[CTR_UNIFORM_P], uv);
            }
            atomicMax(&P.ctr[CTR_MAXSP], (unsigned long long)msp);
        }
    }
    if (st.overflow) atomicOr(&P.ctr[CTR_OVERFLOW], 1ull);
}

// reflection / refraction rays of a wave (Shader::shade_path), always counted
__device__ __forceinline__ void flush_secondary(const RenderParams& P, uint32_t n, int lane) {
    unsigned long long v = n;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if (lane == 0 && v) atomicAdd(&P.ctr[CTR_SECONDARY], v);
}

// Camera::eyeRayAdaptive (src/Camera.cpp:116-174) of eye-ray sample `skey`: two
// jitter draws (dims 0, 1) over [x0, x1] x [y0, y1] of the pixel, the time draw
// (dim 2, getTimeSample), then with an aperture >= epsilon the lens point,
// rejection-sampled from the unit disc (dims 3, 4, 5, ...), and the ray from it
// through the focal point.  Deterministic per (pixel, sample), so the shading
// kernels recompute the camera ray instead of storing it.
struct EyeRay {
    v3 o, d;
    float time;
};
__device__ __forceinline__ EyeRay eye_ray(const CamParams& cam, uint32_t seed, int x, int y, uint32_t skey, float x0,
                                          float x1, float y0, float y1, const uint16_t* rsqT) {
    const uint32_t pixel = (uint32_t)(y * cam.W + x);
    const float ur = rng(pixel, skey, 0, seed), vr = rng(pixel, skey, 1, seed);
    const float xo = (x1 - x0) * ur + x0, yo = (y1 - y0) * vr + y0;
    const float Up = cam.left + (cam.right - cam.left) * (((float)x + xo) / (float)cam.W);
    const float Vp = cam.bottom + (cam.top - cam.bottom) * (((float)y + yo) / (float)cam.H);
    const v3 U = mk(cam.u[0], cam.u[1], cam.u[2]), Vv = mk(cam.v[0], cam.v[1], cam.v[2]), W = mk(cam.w[0], cam.w[1], cam.w[2]);
    const v3 eye = mk(cam.eye[0], cam.eye[1], cam.eye[2]);
    const v3 d = normalized(sub(add(scale(U, Up), scale(Vv, Vp)), W), rsqT);
    const float tr = rng(pixel, skey, 2, seed);
    const float time = 1.f - ((tr * tr) * tr) * cam.shutter;   // getTimeSample, src/Camera.h:46
    if (!(cam.aperture >= 0.001f)) return EyeRay{eye, d, time};   // m_aperture < epsilon: pinhole
    const v3 focal = add(scale(d, cam.focus), eye);
    float lu, lv;
    uint32_t k = 3;
    do {   // 1.0 - 2 * getRand: exact in float (1 - 2r is representable or rounds once either way)
        lu = 1.0f - 2.0f * rng(pixel, skey, k, seed);
        lv = 1.0f - 2.0f * rng(pixel, skey, k + 1, seed);
        k += 2;
    } while (lu * lu + lv * lv > 1.0f && k < 3 + 2 * 64);
    const v3 o = add(scale(add(scale(U, lu), scale(Vv, lv)), cam.aperture), eye);
    return EyeRay{o, normalized(sub(focal, o), rsqT), time};
}
// the 1-spp camera ray (eyeRayAdaptive(x, y, .5, .5, .5, .5), sample 0)
__device__ __forceinline__ EyeRay camera_ray(const CamParams& cam, uint32_t seed, int x, int y, const uint16_t* rsqT) {
    return eye_ray(cam, seed, x, y, 0u, 0.5f, 0.5f, 0.5f, 0.5f, rsqT);
}

// Kernel 1: Camera::eyeRayAdaptive + closest-hit BVH::intersect per pixel.
// Writes the HitInfo record (t, a, b, prim) to P.hits[slot].
// CHECK: the special-leaf scene has alpha-mapped or motion-blurred lanes (false: instances only)
// XONE: the walk loop's exit form (traverse_impl; same bits), picked per scene by the host
template <bool COUNT, int MINW, bool FAST, bool INST = false, bool CHECK = true, bool XONE = false>
__global__ void __launch_bounds__(kWG, MINW) primary_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    load_tables(P.tables, s_tab, 1024);
    const uint64_t t0 = (COUNT || P.wave_log) ? wall_clock64() : 0;
    const uint16_t* rcpT = s_tab;           // per triangle test: LDS
    const uint16_t* rsqT = P.tables + 2048; // a few per pixel: global (L1-resident)
    // (lane / wave indices and the tile's parameters are recomputed / re-read where
    // used, so they hold no registers across the traversal: see frame1_kernel)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, rcpT, s_stack + tid, P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    uint32_t nhits = 0;
    unsigned long long wave_steps = 0;  // count mode: sum over tiles of max lane node visits
    TileSched ts(P, wave, lane);
    uint32_t ntiles = 0;
    for (int item = ts.first(); item >= 0; item = ts.next(item)) {
        const RenderParams& PA = reload_params();
        if (PA.wave_log && lane_id() == 0 && ntiles < kLogTiles) {
            unsigned long long* r = PA.wave_log + kLogWords * ((size_t)blockIdx.x * (kWG / 64) + wave);
            r[4 + ntiles] = ((unsigned long long)item << 40) | (wall_clock64() & ((1ull << 40) - 1));
            r[4 + kLogTiles + ntiles] = ts.deq_ticks;
        }
        ntiles++;
        int x, y;
        size_t slot;
        const uint32_t n0 = st.nodes;
        if (item_pixel(PA, item, lane_id(), x, y, slot)) {
            const int f = item_frame(PA, item);
            const CamParams& cam = PA.cam[f];
            const EyeRay er = camera_ray(cam, PA.seed + (uint32_t)f, x, y, rsqT);
            DRay r = make_ray(er.o, er.d, er.time);
            DHit h{1e12f, 0.f, 0.f, -1};
            if (!traverse<false, COUNT, FAST, INST, CHECK, false, XONE, XONE && !INST>(T, r, 0.001f, h, st)) h.prim = -1;
            const RenderParams& PC = reload_params();
            item_pixel(PC, item, lane_id(), x, y, slot);  // recompute: keeps it out of the traversal's live set
            PC.hits[slot] = make_float4(h.t, h.a, h.b, __int_as_float(h.prim));
            nhits += h.prim >= 0 ? 1u : 0u;  // wave-reduced in flush_stats
        }
        if (COUNT) {
            uint32_t dmax = st.nodes - n0;
            for (int off = 32; off > 0; off >>= 1) dmax = max(dmax, (uint32_t)__shfl_xor(dmax, off));
            wave_steps += dmax;
        }
    }
    if (COUNT && lane == 0) atomicAdd(&P.ctr[CTR_WAVE_STEPS_P], wave_steps);
    flush_stats<COUNT, true>(P, st, nhits, lane, t0, ntiles);
}

// Kernel 2: Scene::sampleScene shading of the primary hit with shadow rays.
template <bool COUNT, bool POINT_ONLY, bool FAST, bool INST = false, int MODE = kFused, int REC = 0, int MINW = 1>
__global__ void __launch_bounds__(kWG, MINW) shade_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    __shared__ float s_ior[REC ? kIorCap * kWG : 1];
    load_tables(P.tables, s_tab, 1024);
    const uint64_t t0 = (COUNT || P.wave_log) ? wall_clock64() : 0;
    const uint16_t* rcpT = s_tab;           // per triangle test: LDS
    const uint16_t* rsqT = P.tables + 2048; // a few per pixel: global (L1-resident)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, rcpT, s_stack + tid, P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    uint32_t shadow_total = 0, secondary_total = 0;
    TileSched ts(P, wave, lane);
    uint32_t ntiles = 0;
    for (int item = ts.first(); item >= 0; item = ts.next(item)) {
        if (P.wave_log && lane == 0 && ntiles < kLogTiles)
        {
            unsigned long long* r = P.wave_log + kLogWords * ((size_t)blockIdx.x * (kWG / 64) + wave);
            r[4 + ntiles] = ((unsigned long long)item << 40) | (wall_clock64() & ((1ull << 40) - 1));
            r[4 + kLogTiles + ntiles] = ts.deq_ticks;
        }
        ntiles++;
        int x, y;
        size_t slot;
        if (!item_pixel(P, item, lane, x, y, slot)) {
            if (MODE == kGen && P.mode != 0) P.nrays[slot] = 0;  // bucket slot outside the frame
            continue;
        }
        float4 hv = P.hits[slot];
        DHit h{hv.x, hv.y, hv.z, __float_as_int(hv.w)};
        v3 col;
        if (h.prim >= 0) {
            const int f = item_frame(P, item);
            const CamParams& cam = P.cam[f];
            const uint32_t seed = P.seed + (uint32_t)f;
            const EyeRay er = camera_ray(cam, seed, x, y, rsqT);
            DRay r = make_ray(er.o, er.d, er.time);
            Shader<POINT_ONLY, FAST, INST, MODE, REC> S{P, T, rcpT, rsqT, st, (uint32_t)(y * cam.W + x), 0u, seed,
                                                   slot * (size_t)P.max_shadow, 0u};
            S.time = S.shadow_time = er.time;
            S.lrec0 = slot * (size_t)P.lcalls;
            if constexpr (REC) { S.iorS = s_ior + tid; S.lvl = P.lvl + (blockIdx.x * kWG + tid); }
            col = S.template shade<COUNT>(r, h);
            shadow_total += S.shadow_rays;
            secondary_total += S.secondary;
            if (MODE == kGen) P.nrays[slot] = (uint8_t)S.nslot;
        } else if (MODE == kGen) {
            P.nrays[slot] = 0;
            continue;
        } else if (P.env) {  // environment map lookup of the missed ray (src/Scene.cpp:236-239)
            const int f = item_frame(P, item);
            const v3 d = camera_ray(P.cam[f], P.seed + (uint32_t)f, x, y, rsqT).d;
            col = scale(tex_lookup_dir(P.env, P.env_w, P.env_h, d.x, d.y, d.z), P.env_exposure);
        } else {
            col = mk(P.bg[0], P.bg[1], P.bg[2]);
        }
        if (MODE == kGen) continue;
        store_rgb(P, slot, col);
    }
    flush_secondary(P, secondary_total, lane);
    flush_stats<COUNT>(P, st, MODE == kResolve ? 0u : shadow_total, lane, t0, ntiles);
}

// getSum (src/Scene.cpp:245-248): 1^2 + ... + n^2 through the float 1/6
__device__ __forceinline__ int sum_squares(int n) { return (int)((float)(n * (n + 1) * (2 * n + 1)) * 0.16666667f); }

// Image::linear_to_gammaF[int(min(v, 1) * 32767)] (src/Scene.cpp:278-283).
// Deviation: a negative / NaN channel (an out-of-bounds read there) uses entry 0.
__device__ __forceinline__ float gamma_f(const float* lut, float v) {
    const float c = (v > 1.f) ? 1.f : v;
    const float f = c * 32767.f;
    return lut[(f >= 0.f) ? (int)f : 0];
}

// Kernel 3: Scene::adaptiveSampleScene (src/Scene.cpp:252-293), fused.  One
// persistent launch; a lane loops over its pixel's eye rays -- the centre
// sample, then levels 2.. of n x n jittered sub-samples (eyeRayAdaptive with
// offsets [i/n, (i+1)/n] x [j/n, (j+1)/n], src/Camera.cpp:144-150) -- each
// through Scene::sampleScene (closest hit, shading with inline shadow rays,
// environment / background on a miss), with the reference's running mean and
// gamma-space stop test after every level.  Eye ray k of a pixel draws from
// RNG stream (pixel, k): ray 0 is the 1-spp frame path's ray.
// Schedules: P.refill_min == 0: a wave takes an 8x8 tile and runs until its
// last lane's pixel stops.  P.refill_min > 0 (lane refill): a lane whose pixel
// has stopped takes the next pixel as soon as refill_min lanes of its wave are
// idle (pixels dealt in tile order from 8 per-XCD bands), so a wave runs one
// eye ray per busy lane per step instead of waiting for its slowest pixel.
// Every pixel's eye rays, draws and sums are the same under both schedules.
template <bool COUNT, bool POINT_ONLY, bool FAST, bool INST, int REC = 0, int MINW = 1>
__global__ void __launch_bounds__(kWG, MINW) adaptive_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    __shared__ float s_ior[REC ? kIorCap * kWG : 1];
    load_tables(P.tables, s_tab, 1024);
    const uint64_t t0 = (COUNT || P.wave_log) ? wall_clock64() : 0;
    const uint16_t* rcpT = s_tab;
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, rcpT, s_stack + tid, P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    uint32_t shadow_total = 0, eye_rays = 0, eye_hits = 0, secondary_total = 0;
    uint32_t ntiles = 0;
    // the lane's pixel and its running state
    int x = 0, y = 0, f = 0;
    size_t slot = 0;
    uint32_t pixel = 0, seed = 0, sample = 0;
    v3 result = mk(0, 0, 0), cur = mk(0, 0, 0);
    int level = 1, i = 0, j = 0;
    // start pixel `lane_` of work item `item` (false: outside the frame)
    auto start = [&](int item, int lane_) __attribute__((always_inline)) {
        if (!item_pixel(P, item, lane_, x, y, slot)) return false;
        f = item_frame(P, item);
        seed = P.seed + (uint32_t)f;
        pixel = (uint32_t)(y * P.cam[f].W + x);
        sample = 0;
        result = mk(0, 0, 0);
        cur = mk(0, 0, 0);
        level = 1; i = 0; j = 0;
        return true;
    };
    // one eye ray of the lane's pixel; true when the pixel is done (written)
    // (always inlined: called from both schedules below, it became a call, and a call takes
    // the RenderParams out of the kernarg segment -- 2288 B of scratch per lane, A3 2x slower)
    auto step = [&]() __attribute__((always_inline)) {
        const CamParams& cam = P.cam[f];
        float x0 = 0.5f, x1 = 0.5f, y0 = 0.5f, y1 = 0.5f;
        if (level > 1) {
            const float off = 1.0f / (float)level;
            x0 = (float)i * off; x1 = (float)(i + 1) * off;
            y0 = (float)j * off; y1 = (float)(j + 1) * off;
        }
        const EyeRay er = eye_ray(cam, seed, x, y, sample * 1024u, x0, x1, y0, y1, rsqT);
        const v3 d = er.d;
        const DRay r = make_ray(er.o, d, er.time);
        DHit h{1e12f, 0.f, 0.f, -1};
        v3 col;
        eye_rays++;
        const bool hit = traverse<false, COUNT, FAST, INST, true, false, !INST, !INST>(T, r, 0.001f, h, st);
        if (sample == 0) P.hits[slot] = make_float4(h.t, h.a, h.b, __int_as_float(hit ? h.prim : -1));
        if (hit) {
            eye_hits++;
            Shader<POINT_ONLY, FAST, INST, kFused, REC> S{P, T, rcpT, rsqT, st, pixel, 0u, seed, 0, 0u};
            S.sample = sample;
            S.time = S.shadow_time = er.time;
            if constexpr (REC) { S.iorS = s_ior + tid; S.lvl = P.lvl + (blockIdx.x * kWG + tid); }
            col = S.template shade<COUNT>(r, h);
            shadow_total += S.shadow_rays;
            secondary_total += S.secondary;
        } else if (P.env) {
            col = scale(tex_lookup_dir(P.env, P.env_w, P.env_h, d.x, d.y, d.z), P.env_exposure);
        } else {
            col = mk(P.bg[0], P.bg[1], P.bg[2]);
        }
        sample++;
        bool cut = false;
        if (level == 1) {
            result = col;
            level = 2;
        } else {
            cur = add(cur, col);
            if (++j < level) return false;
            j = 0;
            if (++i < level) return false;
            i = 0;
            const float pre = (float)sum_squares(level - 1), now = (float)(level * level);
            const v3 nr = scale(add(scale(result, pre), cur), 1.0f / (pre + now));
            const float tx = gamma_f(P.gammaF, result.x) - gamma_f(P.gammaF, nr.x);
            const float ty = gamma_f(P.gammaF, result.y) - gamma_f(P.gammaF, nr.y);
            const float tz = gamma_f(P.gammaF, result.z) - gamma_f(P.gammaF, nr.z);
            cut = fmaxf(fabsf(tx), fmaxf(fabsf(ty), fabsf(tz))) < P.noise;
            result = nr;
            cur = mk(0, 0, 0);
            level++;
        }
        if ((level <= P.max_subdivs && !cut) || level <= P.min_subdivs) return false;
        store_rgb(P, slot, result);
        return true;
    };
    if (P.refill_min <= 0) {
        TileSched ts(P, wave, lane);
        for (int item = ts.first(); item >= 0; item = ts.next(item)) {
            ntiles++;
            if (!start(item, lane)) continue;
            while (!step()) {}
        }
    } else {
        // pixels p = item * 64 + lane of the work items, dealt from 8 bands (one
        // counter each, 128 B apart); a wave dequeues as many as it has idle lanes
        const size_t n_px = (size_t)P.n_tiles * 64;
        auto band_lo = [&](int k) { return n_px * (size_t)k / 8; };
        int band = blockIdx.x & 7, probes = 0;
        bool exhausted = false, active = false;
        for (;;) {
            const unsigned long long idle = __ballot(!active);
            const int nidle = __popcll(idle);
            if (!exhausted && (nidle >= P.refill_min || nidle == 64)) {
                unsigned long long got = ~0ull, hi = 0;
                if (lane == 0) {
                    while (probes < 8) {
                        const size_t lo = band_lo(band), bend = band_lo(band + 1);
                        const unsigned long long v =
                            atomicAdd(reinterpret_cast<unsigned long long*>(P.queue + band * 32), (unsigned long long)nidle);
                        if (lo + v < bend) { got = lo + v; hi = bend; break; }
                        band = (band + 1) & 7;
                        probes++;
                    }
                }
                got = __shfl(got, 0);
                hi = __shfl(hi, 0);
                if (got == ~0ull) {
                    exhausted = true;
                } else if (!active) {
                    const size_t p = (size_t)got + (size_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    if (p < (size_t)hi) {
                        ntiles++;
                        active = start((int)(p >> 6), (int)(p & 63));
                    }
                }
            }
            if (__ballot(active) == 0) {
                if (exhausted) break;
                continue;
            }
            if (active && step()) active = false;
        }
    }
    unsigned long long er = eye_rays, eh = eye_hits;
    for (int off = 32; off > 0; off >>= 1) {
        er += __shfl_down(er, off);
        eh += __shfl_down(eh, off);
    }
    if (lane == 0) {
        atomicAdd(&P.ctr[CTR_RAYS_P], er);
        atomicAdd(&P.ctr[CTR_HITS], eh);
    }
    flush_secondary(P, secondary_total, lane);
    flush_stats<COUNT, false>(P, st, shadow_total, lane, t0, ntiles);
}

using KernelFn = void (*)(RenderParams);

template <template <bool, bool, bool, bool, int> class K, int REC>
static KernelFn pick4(bool c, bool po, bool f, bool inst) {
    if (inst) return c ? (f ? K<true, false, true, true, REC>::fn : K<true, false, false, true, REC>::fn)
                       : (f ? K<false, false, true, true, REC>::fn : K<false, false, false, true, REC>::fn);
    if (po) return c ? (f ? K<true, true, true, false, REC>::fn : K<true, true, false, false, REC>::fn)
                     : (f ? K<false, true, true, false, REC>::fn : K<false, true, false, false, REC>::fn);
    return c ? (f ? K<true, false, true, false, REC>::fn : K<true, false, false, false, REC>::fn)
             : (f ? K<false, false, true, false, REC>::fn : K<false, false, false, false, REC>::fn);
}
template <bool C, bool PO, bool F, bool I, int REC>
struct ShadeK { static constexpr KernelFn fn = shade_kernel<C, PO, F, I, kFused, REC>; };

// defined in mrt_frame.hip: the one-point-light frame / shade kernels at an
// occupancy target w; pow: a Blinn material with specExp != 1
KernelFn pick_frame1(int w, bool c, bool f, bool pow, int walk);
KernelFn pick_shade1(bool c, bool f, bool pow);
// defined in mrt_rec.hip: the fused chain kernels (rec 1: reflection / refraction,
// 2: + path tracing) and the adaptive supersampling kernels (any rec)
KernelFn pick_shade_rec(bool c, bool po, bool f, bool inst, int rec);
KernelFn pick_adaptive(bool c, bool po, bool f, bool inst, int rec);
// defined in mrt_chain.hip: the wavefront chain engine
KernelFn pick_chain0(bool resolve, bool po, bool inst, int rec);
KernelFn pick_chain_shade(bool resolve, bool po, bool inst, int rec);
KernelFn pick_chain_trace(bool c, bool f, bool inst, int step);
KernelFn pick_chain_compact();
KernelFn pick_chain_merge();
KernelFn pick_chain_fallback(bool po, bool inst, int rec, bool count);
KernelFn pick_chain_finish();
KernelFn pick_chain_fold();
KernelFn pick_unit_eye(bool c, bool f, bool inst);
KernelFn pick_adapt_combine();

}  // namespace mrt
