// mrt_chain.hip -- the wavefront chain engine: Blinn reflection / refraction
// rays, dispersive three-way splits, path tracing (Shader REC 1 / 2) and
// adaptive supersampling, level by level instead of one lane walking its
// whole recursion.
//
// The fused kernels (shade_kernel<REC>, adaptive_kernel<REC>) keep every
// level's shading state live across each secondary and shadow traversal: 256
// VGPRs plus scratch, one wave per SIMD.  Here the recursion of Shader::level
// calls of one path (src/Blinn.cpp:39-335) is cut at each child ray and run as
// a tree of entries, one level at a time over all paths of a chunk:
//
//   chain0   (per work unit: one eye ray of a pixel) level 0 of every path of
//            the unit (the camera ray's IOR history persists across its paths)
//            in two passes around the shadow rays: kGen writes the shadow rays,
//            kResolve shades with the answers.  A level either ends (its value
//            -> ch_val) or spawns children into the sparse spawn slots of its
//            entry (entry * ch_split + i): one reflection / refraction / GI
//            ray, or, at a dispersive material, three refraction rays (one per
//            colour channel, Shader::disp_child), with its level record written
//            for the fold;
//   compact  spawn slots of level k -> dense entries of level k + 1
//            (block-aggregated: one atomic per 1024 slots), each keeping its
//            parent entry; ch_map[slot] = the dense child, for the fold;
//   trace    closest hit of every level-k + 1 entry, and the any-hit answers of
//            level k's shadow rays (traversal only: few registers, full
//            occupancy);
//   shade    level k + 1 of every entry (kGen): shadow rays and children;
//   resolve  (after the last level) every level shaded again with its shadow
//            answers: ch_val of the entries that end, level records;
//   fold     per level, deepest first: every spawning entry gathers its
//            children's values through ch_map -- chain_combine for one child,
//            the masked channel sums of src/Blinn.cpp:275-301 for a split;
//   finish   per unit: the paths averaged (Scene::sampleScene); the pixel
//            written, or, under adaptive supersampling, the unit's colour.
//
// Adaptive supersampling (Scene::adaptiveSampleScene, src/Scene.cpp:252-293)
// runs as passes n = 1, 2, .. over the pixels still refining: pass n renders
// n^2 jittered eye rays per such pixel through the engine above (unit_eye
// traces them), then adapt_combine forms the running mean, applies the stop
// test and lists the pixels of pass n + 1.
//
// Every ray, every RNG draw (keyed by pixel, eye sample, path, level and
// dispersion branch) and every add is the fused kernel's, so the two engines
// give bit-identical frames (tests/test_chain.py, test_secondary.py,
// test_path_trace.py, test_dispersion.py, test_adaptive.py).  A pass whose
// entries do not fit the scratch budget runs in chunks of units.
#include "mrt_shader.h"

namespace mrt {

// per-entry chain state word: IOR index, GI levels, reflect / refract levels,
// isSecondary, env_miss (the entry's own miss rule), refraction ray, branch code
__device__ __forceinline__ uint32_t pack_state(const ChainState& cs, bool env_miss) {
    return (uint32_t)cs.idx | (uint32_t)cs.gi << 4 | (uint32_t)cs.bounces << 12 | (cs.secondary ? 1u << 16 : 0u) |
           (env_miss ? 1u << 17 : 0u) | (cs.refr ? 1u << 18 : 0u) | (uint32_t)(cs.br & 0xFF) << 19;
}
__device__ __forceinline__ void unpack_state(uint32_t w, ChainState& cs, bool& env_miss) {
    cs.idx = (int)(w & 15u);
    cs.gi = (int)((w >> 4) & 255u);
    cs.bounces = (int)((w >> 12) & 15u);
    cs.secondary = (w >> 16) & 1u;
    env_miss = (w >> 17) & 1u;
    cs.refr = (w >> 18) & 1u;
    cs.br = (int)((w >> 19) & 255u);
}

// ch_val flags (.w bits): the entry's ray missed (a split parent skips it); its
// value is "nothing" (a GI ray missed without environment sampling); its value
// is still to be folded from its children (pending), which are a split
// value is the missed ray's direction, the parent's environment still to be looked up
// (a material with its own environment map, Material::getEnvironmentColor)
enum { kValMissed = 1, kValNone = 2, kValPending = 4, kValSplit = 8, kValEnvDir = 16 };

__device__ __forceinline__ uint32_t lofs(const RenderParams& P, int k) { return P.ch_lofs[k]; }
// The chunk outgrew a level's estimated capacity: its remaining launches return at
// once and chain_fallback_kernel renders its units instead.
__device__ __forceinline__ bool chunk_dead(const RenderParams& P) { return P.ch_ovf != nullptr && *P.ch_ovf != 0u; }
__device__ __forceinline__ uint32_t lcap(const RenderParams& P, int k) { return P.ch_lofs[k + 1] - P.ch_lofs[k]; }
// level record of entry e of level k: lvl_words consecutive floats
__device__ __forceinline__ ChainRec chain_rec(const RenderParams& P, int k, uint32_t e) {
    return ChainRec{P.ch_rec + ((size_t)lofs(P, k) + e) * (size_t)P.lvl_words, 1};
}
__device__ __forceinline__ void write_val(const RenderParams& P, int k, uint32_t e, v3 v, uint32_t flags) {
    P.ch_val[(size_t)lofs(P, k) + e] = make_float4(v.x, v.y, v.z, __uint_as_float(flags));
}
// shadow-ray slots of chain level k (each level keeps its own until the resolve pass)
__device__ __forceinline__ size_t shadow_base(const RenderParams& P, int k) {
    return (size_t)lofs(P, k) * (size_t)P.max_shadow;
}

// ------------------------------------------------------------------ units
// units of this chunk (the pass's count is on the device under adaptive passes)
__device__ __forceinline__ uint32_t chunk_units(const RenderParams& P) {
    const uint32_t nn = P.adapt_n > 1 ? (uint32_t)(P.adapt_n * P.adapt_n) : 1u;
    const uint32_t total = P.unit_cnt ? *P.unit_cnt * nn : P.units_total;
    return total > P.unit_base ? min(P.n_units, total - P.unit_base) : 0u;
}
struct UnitPix {
    int x, y, f;
    size_t slot;
    uint32_t sample;   // eye-ray sample of the pixel (RNG sub-stream sample * 1024 + path)
    int i, j;          // sub-cell of an adaptive pass n >= 2
    bool valid;
};
// unit ug of the pass (global index)
__device__ __forceinline__ UnitPix unit_pixel(const RenderParams& P, uint32_t ug) {
    UnitPix U;
    int item, lane;
    U.sample = 0;
    U.i = U.j = 0;
    if (P.units && P.adapt_n > 1) {
        const uint32_t nn = (uint32_t)(P.adapt_n * P.adapt_n), r = ug % nn;
        const uint32_t id = P.units[ug / nn];
        item = (int)(id >> 6);
        lane = (int)(id & 63u);
        U.i = (int)(r / (uint32_t)P.adapt_n);
        U.j = (int)(r % (uint32_t)P.adapt_n);
        U.sample = (uint32_t)sum_squares(P.adapt_n - 1) + r;   // rays 0 .. of the pixel, level by level
    } else {
        item = (int)(ug >> 6);
        lane = (int)(ug & 63u);
    }
    U.valid = item_pixel(P, item, lane, U.x, U.y, U.slot);
    U.f = item_frame(P, item);
    return U;
}
// the unit's eye ray: Camera::eyeRayAdaptive over the unit's cell (the centre
// at pass 1 and without supersampling)
__device__ __forceinline__ EyeRay unit_eye(const RenderParams& P, const UnitPix& U, const uint16_t* rsqT) {
    const CamParams& cam = P.cam[U.f];
    const uint32_t seed = P.seed + (uint32_t)U.f;
    if (P.adapt_n <= 1) return camera_ray(cam, seed, U.x, U.y, rsqT);
    const float off = 1.0f / (float)P.adapt_n;
    return eye_ray(cam, seed, U.x, U.y, U.sample * 1024u, (float)U.i * off, (float)(U.i + 1) * off, (float)U.j * off,
                   (float)(U.j + 1) * off, rsqT);
}
__device__ __forceinline__ float4 unit_hit(const RenderParams& P, uint32_t u, const UnitPix& U) {
    return P.uhits ? P.uhits[u] : P.hits[U.slot];
}
// The camera ray's time of chunk path p (every ray below the camera ray carries
// it): the getTimeSample draw of the unit's eye ray (shared by all its paths).
__device__ __forceinline__ float unit_time(const RenderParams& P, const UnitPix& U) {
    const CamParams& cam = P.cam[U.f];
    const float tr = rng((uint32_t)(U.y * cam.W + U.x), U.sample * 1024u, 2, P.seed + (uint32_t)U.f);
    return 1.f - ((tr * tr) * tr) * cam.shutter;
}

// A spawned child at sparse slot s: its ray, state word and the IOR column
// (the child's history, written by Shader::level / disp_child).
__device__ __forceinline__ void write_spawn(const RenderParams& P, uint32_t s, const DRay& r2, uint32_t path_id,
                                            const ChainState& cs, bool env_miss, const float* iorS) {
    const size_t cap = P.ch_spcap;
    P.ch_sp[s] = make_float4(r2.o[0], r2.o[1], r2.o[2], __uint_as_float(path_id));
    P.ch_sp[cap + s] = make_float4(r2.d[0], r2.d[1], r2.d[2], __uint_as_float(pack_state(cs, env_miss)));
    P.ch_sp[2 * cap + s] = make_float4(iorS[1 * kWG], iorS[2 * kWG], iorS[3 * kWG], iorS[4 * kWG]);
    P.ch_sp[3 * cap + s] = make_float4(iorS[5 * kWG], iorS[6 * kWG], iorS[7 * kWG], 0.f);
}

// After Shader::level of entry e (level k) spawned: kGen writes the children
// (a split: the three channel rays, in channel order) and their flags; kResolve
// marks the entry pending.  A split child's history / state come from the
// recorded level (disp_child), whose camera-ray push (k == 0) also carries on
// into the unit's next path -- so it runs in both modes.
template <class SH>
__device__ __forceinline__ void spawn_children(const RenderParams& P, SH& S, int k, uint32_t e, uint32_t path_id,
                                               ChainState& cs, typename SH::IorCam& cam, const LevelOut& o, bool gen) {
    const uint32_t s0 = e * (uint32_t)P.ch_split;
    if (o.split) {
        const ChainRec rec = chain_rec(P, k, e);
        for (int i = 0; i < 3; i++) {
            ChainState c2 = cs;
            const DRay r2 = S.disp_child(rec, k, i, c2, cam);
            if (gen) {
                write_spawn(P, s0 + (uint32_t)i, r2, path_id, c2, true, S.iorS);
                P.ch_flag[s0 + (uint32_t)i] = 1;
            }
        }
        if (!gen) write_val(P, k, e, mk(0, 0, 0), kValPending | kValSplit);
        return;
    }
    if (gen) {
        write_spawn(P, s0, o.r2, path_id, cs, o.env_miss, S.iorS);
        P.ch_flag[s0] = 1;
        for (int i = 1; i < P.ch_split; i++) P.ch_flag[s0 + (uint32_t)i] = 0;
    } else {
        write_val(P, k, e, mk(0, 0, 0), kValPending);
    }
}
__device__ __forceinline__ void no_children(const RenderParams& P, uint32_t e) {
    const uint32_t s0 = e * (uint32_t)P.ch_split;
    for (int i = 0; i < P.ch_split; i++) P.ch_flag[s0 + (uint32_t)i] = 0;
}

// Level 0 of every path of the chunk's units, one lane per unit.  Path id =
// chunk unit * num_paths + path.  MODE kGen writes each path's shadow rays
// (level-0 slots p * max_shadow + j, count in nrays[p]) and its spawned
// children (the spawn decision, the child rays and their IOR histories do not
// depend on the shadow answers); kResolve runs the same shading with the
// answers and writes the path's value or marks it pending.  No traversal runs
// in either, so the shading state never has to live across one.
template <bool POINT_ONLY, bool INST, int REC, int MODE>
__global__ void __launch_bounds__(kWG) chain0_kernel(RenderParams P) {
    __shared__ float s_ior[kIorCap * kWG];
    if (chunk_dead(P)) return;
    const uint16_t* rcpT = P.tables;          // no triangle tests here: both tables from global (L1)
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, false, false, P.leaves, rcpT, nullptr, nullptr, P.gstride};   // unused: no traversal
    TravStats st;
    uint32_t shadow_total = 0, secondary_total = 0;
    const uint32_t n = chunk_units(P), np = (uint32_t)P.num_paths;
    for (uint32_t u0 = (uint32_t)blockIdx.x * kWG + (uint32_t)(tid & ~63); u0 < n; u0 += gridDim.x * (uint32_t)kWG) {
        const uint32_t u = u0 + (uint32_t)lane;
        if (u >= n) continue;
        const UnitPix U = unit_pixel(P, P.unit_base + u);
        DHit h{1e12f, 0.f, 0.f, -1};
        if (U.valid) {
            const float4 hv = unit_hit(P, u, U);
            h = DHit{hv.x, hv.y, hv.z, __float_as_int(hv.w)};
        }
        const uint32_t pbase = u * np;
        if (!U.valid || h.prim < 0) {   // nothing to shade: no shadow rays, no spawns (finish writes env / background)
            for (uint32_t path = 0; path < np; path++) {
                if (MODE == kGen) {
                    P.nrays[pbase + path] = 0;
                    no_children(P, pbase + path);
                } else {
                    write_val(P, 0, pbase + path, mk(0, 0, 0), kValMissed);   // never pending (the fold skips it)
                }
            }
            continue;
        }
        const CamParams& cam = P.cam[U.f];
        const uint32_t seed = P.seed + (uint32_t)U.f;
        const EyeRay er = unit_eye(P, U, rsqT);
        const DRay r = make_ray(er.o, er.d, er.time);
        Shader<POINT_ONLY, false, INST, MODE, REC> S{P, T, rcpT, rsqT, st, (uint32_t)(U.y * cam.W + U.x), 0u, seed, 0,
                                                     0u};
        S.iorS = s_ior + tid;
        S.time = S.shadow_time = er.time;
        typename Shader<POINT_ONLY, false, INST, MODE, REC>::IorCam icam;
        for (uint32_t path = 0; path < np; path++) {
            const uint32_t p = pbase + path;
            S.skey = U.sample * 1024u + path;
            S.slot0 = (size_t)p * (size_t)P.max_shadow;
            S.nslot = 0;
            ChainState cs;
            LevelOut o;
            S.template level<false>(r, h, cs, icam, chain_rec(P, 0, p), o);
            if (MODE == kGen) P.nrays[p] = (uint8_t)S.nslot;
            if (o.spawn) spawn_children(P, S, 0, p, p, cs, icam, o, MODE == kGen);
            else if (MODE == kGen) no_children(P, p);
            else write_val(P, 0, p, o.val, 0u);
        }
        shadow_total += S.shadow_rays;
        secondary_total += S.secondary;
    }
    if (MODE == kGen) {
        flush_stats<false>(P, st, shadow_total, lane, 0, 0);
        flush_secondary(P, secondary_total, lane);
    }
}

// Spawn slots of level k (P.ch_level) -> dense entries of level k + 1.  A
// block takes 1024 slots (4 per thread), orders its spawns by (round, wave,
// lane) and reserves their entries with one atomic; ch_map[slot] = the entry.
static constexpr int kCompactGroup = 4 * kWG;
__global__ void __launch_bounds__(kWG) chain_compact_kernel(RenderParams P) {
    __shared__ uint32_t s_cnt[4 * (kWG / 64)];
    __shared__ uint32_t s_base;
    if (chunk_dead(P)) return;
    const int k = P.ch_level;
    const uint32_t ne = k == 0 ? chunk_units(P) * (uint32_t)P.num_paths : P.ch_cnt[k];
    const uint32_t n = ne * (uint32_t)P.ch_split;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t cap = P.ch_spcap, dst0 = lofs(P, k + 1), dcap = lcap(P, k + 1);
    uint32_t* map = P.ch_map + (size_t)P.ch_split * lofs(P, k);
    for (uint32_t g = blockIdx.x * (uint32_t)kCompactGroup; g < n; g += gridDim.x * (uint32_t)kCompactGroup) {
        bool f[4];
        uint32_t rank[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t e = g + (uint32_t)(j * kWG + tid);
            f[j] = e < n && P.ch_flag[e] != 0;
            const unsigned long long m = __ballot(f[j]);
            rank[j] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (lane == 0) s_cnt[j * (kWG / 64) + wave] = (uint32_t)__popcll(m);
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t tot = 0;
            for (int i = 0; i < 4 * (kWG / 64); i++) {
                const uint32_t c = s_cnt[i];
                s_cnt[i] = tot;
                tot += c;
            }
            s_base = tot ? atomicAdd(&P.ch_cnt[k + 1], tot) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (!f[j]) continue;
            const uint32_t e = g + (uint32_t)(j * kWG + tid);
            const uint32_t d = s_base + s_cnt[j * (kWG / 64) + wave] + rank[j];
            if (d >= dcap) {   // past the level's (estimated) capacity: the chunk goes to the fallback
                if (P.ch_ovf) *P.ch_ovf = 1u;
                else atomicOr(&P.ctr[CTR_OVERFLOW], 2ull);
                map[e] = 0xFFFFFFFFu;
                continue;
            }
            map[e] = d;
            const float4 o = P.ch_sp[e], dd = P.ch_sp[cap + e], i0 = P.ch_sp[2 * cap + e], i1 = P.ch_sp[3 * cap + e];
            P.ch_ray[2 * dst0 + d] = o;
            P.ch_ray[2 * dst0 + dcap + d] = dd;
            P.ch_ior[2 * dst0 + d] = i0;
            P.ch_ior[2 * dst0 + dcap + d] = make_float4(i1.x, i1.y, i1.z, __uint_as_float(e / (uint32_t)P.ch_split));
        }
        __syncthreads();   // s_cnt / s_base reused by the next group
    }
}

// One launch per chain level k = P.ch_level: the closest hits of level k's
// entries (nA of them; the children spawned by level k - 1) and the any-hit
// answers of level k - 1's shadow rays (nB slots), which no longer wait for
// each other -- a level's resolve needs its shadow answers only at the end of
// the chunk.  Wave-uniform 64-slot chunks, the closest-hit chunks first.
//
// STEP (instanced scenes): 0 -- a shadow ray walks with traverse(), whose ProxyObject
// lanes run their BLAS walks nested inside the world walk; 1 / 2 -- it walks with
// anyhit_step_inst (2: alpha-mapped / motion-blurred lanes), one node per step for world
// and BLAS nodes alike, the proxy walks deferred onto the stack (an any-hit answer does
// not depend on the visit order), so lanes in and out of instances share every step.
template <bool COUNT, bool FAST, bool INST, int MINW = 1, int STEP = 0>
__global__ void __launch_bounds__(kWG, MINW) chain_trace_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    if (chunk_dead(P)) return;
    const int k = P.ch_level;
    const uint32_t nA = k < P.ch_levels ? P.ch_cnt[k] : 0u;
    const uint32_t m = (uint32_t)P.max_shadow;
    const uint32_t nprev = k == 1 ? chunk_units(P) * (uint32_t)P.num_paths : P.ch_cnt[k - 1];
    // binned orders (mrt_bin.h): sh_perm lists level k - 1's valid shadow-ray slots, tr_perm
    // level k's entries; a ray's answer does not depend on which lane traces it
    const uint32_t nB = P.ch_skip_shadow ? 0u : (P.sh_perm ? *P.sh_perm_n : nprev * m);   // skip: their own launch
    const uint32_t chA = (nA + 63u) >> 6, chunks = chA + ((nB + 63u) >> 6);
    const uint32_t wave_id = (uint32_t)blockIdx.x * (kWG / 64) + (uint32_t)(threadIdx.x >> 6);
    if ((uint32_t)blockIdx.x * (kWG / 64) >= chunks) return;   // the block has no chunks (before any barrier)
    load_tables(P.tables, s_tab, 1024);
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, s_tab, s_stack + tid,
           P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    const size_t base = lofs(P, k), cap = k < P.ch_levels ? lcap(P, k) : 0, sb = shadow_base(P, k - 1);
    const uint8_t* nrays = P.nrays + lofs(P, k - 1);
    const uint32_t np = (uint32_t)P.num_paths;
    unsigned long long wave_steps = 0;
    // (always inlined: as a call from the two schedules below it takes the RenderParams out
    // of the kernarg segment, a 2288-B private copy per lane)
    auto chunk = [&](uint32_t c) __attribute__((always_inline)) {   // one 64-slot chunk, one ray per lane
        const uint32_t n0 = st.nodes;
        if (c < chA) {   // closest hit of entry e
            uint32_t e = (c << 6) + (uint32_t)lane;
            if (e < nA) {
                if (P.tr_perm) e = P.tr_perm[e];
                const float4 o = P.ch_ray[2 * base + e], d = P.ch_ray[2 * base + cap + e];
                float time = 0.f;
                if (INST && P.has_mb) time = unit_time(P, unit_pixel(P, P.unit_base + __float_as_uint(o.w) / np));
                const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), time);
                DHit h{1e12f, 0.f, 0.f, -1};
                const bool hit = traverse<false, COUNT, FAST, INST>(T, r, 0.001f, h, st);
                P.ch_hit[base + e] = make_float4(h.t, h.a, h.b, __int_as_float(hit ? h.prim : -1));
            }
        } else {         // shadow ray j of level k - 1's entry (or path) s, any hit
            uint32_t i = ((c - chA) << 6) + (uint32_t)lane;
            bool ok = i < nB;
            if (ok && P.sh_perm) {
                i = P.sh_perm[i];
            } else if (ok) {
                const uint32_t s = i / m;
                ok = i - s * m < (uint32_t)nrays[s];
            }
            if (ok) {
                const float4 o = P.ray_o[sb + i], d = P.ray_d[sb + i];
                const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), d.w);
                if constexpr (INST && STEP > 0) {
                    AnyState as;
                    as.q = r;
                    as.cur = 0;
                    as.sp = 0;
                    as.aoff = -1;
                    bool hit = false;
                    while (!anyhit_step_inst<COUNT, FAST, STEP == 2>(T, 0.001f, o.w, as, P.ray_o + sb, P.ray_d + sb, i,
                                                                    hit, st)) {
                    }
                    P.occl[sb + i] = hit ? 1 : 0;
                } else {
                    DHit h{o.w, 0.f, 0.f, -1};
                    P.occl[sb + i] = traverse<true, COUNT, FAST, INST>(T, r, 0.001f, h, st) ? 1 : 0;
                }
            }
        }
        if (COUNT) {   // the chunk's wave steps: its longest ray's node visits
            uint32_t v = st.nodes - n0;
            for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor(v, off));
            wave_steps += v;
        }
    };
    if (P.ch_bands) {
        // XCD bands: the chunk range is cut into 8 contiguous bands and a workgroup
        // on XCD b mod 8 takes chunks of band b mod 8 from that band's counter,
        // then steals from the others -- with binned rays (mrt_bin.h) a band holds
        // neighbouring direction / origin cells, so one XCD's 4 MB L2 holds the
        // nodes of its share of the rays instead of the whole hierarchy's
        unsigned int* q = P.queue + (size_t)(k + 1) * 256;   // this level's 8 counters, 32 words apart
        int band = blockIdx.x & 7, probes = 0;
        for (;;) {
            uint32_t c = 0xFFFFFFFFu;
            if (lane == 0) {
                while (probes < 8) {
                    const uint32_t lo = (uint32_t)((uint64_t)chunks * (uint32_t)band / 8u);
                    const uint32_t hi = (uint32_t)((uint64_t)chunks * (uint32_t)(band + 1) / 8u);
                    const uint32_t v = lo < hi ? atomicAdd(q + band * 32, 1u) : 0u;
                    if (lo + v < hi) { c = lo + v; break; }
                    band = (band + 1) & 7;
                    probes++;
                }
            }
            c = __shfl(c, 0);
            if (c == 0xFFFFFFFFu) break;
            chunk(c);
        }
    } else {
        for (uint32_t c = wave_id; c < chunks; c += gridDim.x * (kWG / 64)) chunk(c);
    }
    if (COUNT) {
        unsigned long long nv = st.nodes, lv = st.leaves;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_down(nv, off);
            lv += __shfl_down(lv, off);
        }
        if (lane == 0) {
            atomicAdd(&P.ctr[CTR_NODES], nv);
            atomicAdd(&P.ctr[CTR_LEAVES], lv);
            atomicAdd(&P.ctr[CTR_NODES_S], nv);          // chain engine: the trace launches' visits
            atomicAdd(&P.ctr[CTR_WAVE_STEPS_S], wave_steps);   //   and wave steps (lane utilisation)
        }
    }
    if (st.overflow) atomicOr(&P.ctr[CTR_OVERFLOW], 1ull);
}

// Shading of chain level k >= 1.  kGen (one launch per level, k =
// P.ch_level): every entry that hit writes its shadow rays (level-k slots
// e * max_shadow + j) and its spawned children.  kResolve (one launch per
// chunk, all levels 1 .. ch_levels - 1): a missed ray ends its path with the
// environment (or nothing: a GI ray without environment sampling; a split
// child: nothing, flagged missed), a hit is shaded again with its shadow
// answers and writes its value or marks itself pending.
template <bool POINT_ONLY, bool INST, int REC, int MODE>
__global__ void __launch_bounds__(kWG) chain_shade_kernel(RenderParams P) {
    __shared__ float s_ior[kIorCap * kWG];
    if (chunk_dead(P)) return;
    const uint16_t* rcpT = P.tables;
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, false, false, P.leaves, rcpT, nullptr, nullptr, P.gstride};   // unused: no traversal
    TravStats st;
    uint32_t shadow_total = 0, secondary_total = 0;
    const uint32_t np = (uint32_t)P.num_paths;
    float* iorS = s_ior + tid;
    const int k0 = MODE == kGen ? P.ch_level : 1, k1 = MODE == kGen ? P.ch_level + 1 : P.ch_levels;
    for (int k = k0; k < k1; k++) {
        const uint32_t n = P.ch_cnt[k];
        const size_t base = lofs(P, k), cap = lcap(P, k);
        for (uint32_t e0 = (uint32_t)blockIdx.x * kWG + (uint32_t)(tid & ~63); e0 < n; e0 += gridDim.x * (uint32_t)kWG) {
            const uint32_t e = e0 + (uint32_t)lane;
            if (e >= n) continue;
            const float4 o = P.ch_ray[2 * base + e], d = P.ch_ray[2 * base + cap + e];
            const uint32_t p = __float_as_uint(o.w);
            ChainState cs;
            bool env_miss;
            unpack_state(__float_as_uint(d.w), cs, env_miss);
            cs.depth = k;
            const float4 hv = P.ch_hit[base + e];
            const DHit h{hv.x, hv.y, hv.z, __float_as_int(hv.w)};
            if (h.prim < 0) {   // the child missed: environment (Lr / Lt, or GI with sampleEnv) or nothing
                if (MODE == kGen) {
                    P.nrays[base + e] = 0;
                    if (k + 1 < P.ch_levels) no_children(P, e);
                } else if (env_miss && P.mat_env) {   // the fold looks up the parent material's map
                    write_val(P, k, e, mk(d.x, d.y, d.z), kValMissed | kValEnvDir);
                } else {
                    write_val(P, k, e, env_miss ? env_or_bg(P, mk(d.x, d.y, d.z)) : mk(0, 0, 0),
                              kValMissed | (env_miss ? 0u : kValNone));
                }
                continue;
            }
            // the unit of path p (pixel, eye sample: the RNG keys; frame of a batched launch)
            const uint32_t u = p / np, path = p - u * np;
            const UnitPix U = unit_pixel(P, P.unit_base + u);
            const float4 i0 = P.ch_ior[2 * base + e], i1 = P.ch_ior[2 * base + cap + e];
            iorS[0] = 1.0f;
            iorS[1 * kWG] = i0.x; iorS[2 * kWG] = i0.y; iorS[3 * kWG] = i0.z; iorS[4 * kWG] = i0.w;
            iorS[5 * kWG] = i1.x; iorS[6 * kWG] = i1.y; iorS[7 * kWG] = i1.z;
            const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z));
            Shader<POINT_ONLY, false, INST, MODE, REC> S{P, T, rcpT, rsqT, st, (uint32_t)(U.y * P.cam[U.f].W + U.x), 0u,
                                                        P.seed + (uint32_t)U.f,
                                                        shadow_base(P, k) + (size_t)e * (size_t)P.max_shadow, 0u};
            S.iorS = iorS;
            S.skey = U.sample * 1024u + path;
            if (INST && P.has_mb) S.time = S.shadow_time = unit_time(P, U);
            typename Shader<POINT_ONLY, false, INST, MODE, REC>::IorCam icam;   // unused below the camera ray
            LevelOut lo;
            S.template level<false>(r, h, cs, icam, chain_rec(P, k, e), lo);
            if (MODE == kGen) P.nrays[base + e] = (uint8_t)S.nslot;
            if (lo.spawn && k + 1 >= P.ch_levels) {   // deeper than the chain bound (cannot happen)
                if (MODE != kGen) {
                    atomicOr(&P.ctr[CTR_OVERFLOW], 2ull);
                    write_val(P, k, e, mk(0, 0, 0), 0u);
                }
            } else if (lo.spawn) {
                spawn_children(P, S, k, e, p, cs, icam, lo, MODE == kGen);
            } else if (MODE == kGen) {
                if (k + 1 < P.ch_levels) no_children(P, e);
            } else {
                write_val(P, k, e, lo.val, 0u);
            }
            shadow_total += S.shadow_rays;
            secondary_total += S.secondary;   // after spawn_children: a split's children count there
        }
    }
    if (MODE == kGen) {
        flush_stats<false>(P, st, shadow_total, lane, 0, 0);
        flush_secondary(P, secondary_total, lane);
    }
}

// Fold of level k (deepest first): every pending entry takes its value from its
// children at level k + 1 (Blinn::shade's returns): one child through
// chain_combine; a dispersive split adds each child that hit, masked to its
// channel, Lt += m_ks * (refraction * mask) in channel order, and with no child
// hit Lt takes m_ks * the environment along channel 2's direction
// (src/Blinn.cpp:275-301, Shader::shade_path's fold).
__global__ void __launch_bounds__(kWG) chain_fold_kernel(RenderParams P) {
    if (chunk_dead(P)) return;
    const int k = P.ch_level;
    const uint32_t n = k == 0 ? chunk_units(P) * (uint32_t)P.num_paths : P.ch_cnt[k];
    const uint16_t* rsqT = P.tables + 2048;
    const uint32_t* map = P.ch_map + (size_t)P.ch_split * lofs(P, k);
    const size_t cb = lofs(P, k + 1);
    const v3 z = mk(0, 0, 0);
    for (uint32_t e = blockIdx.x * kWG + threadIdx.x; e < n; e += gridDim.x * kWG) {
        const size_t g = (size_t)lofs(P, k) + e;
        const float4 v = P.ch_val[g];
        const uint32_t fl = __float_as_uint(v.w);
        if (!(fl & kValPending)) continue;
        const ChainRec rec = chain_rec(P, k, e);
        v3 val;
        if (!(fl & kValSplit)) {
            const float4 c = P.ch_val[cb + map[(size_t)e * P.ch_split]];
            v3 cv = mk(c.x, c.y, c.z);
            if (__float_as_uint(c.w) & kValEnvDir) cv = mat_env(P, P.mats[__float_as_int(rec(0)) & 0xFFFF], cv);
            val = chain_combine(P, rec, cv, (__float_as_uint(c.w) & kValNone) != 0);
        } else {
            const DevMaterial& M = P.mats[__float_as_int(rec(0)) & 0xFFFF];
            const v3 ks = mk(M.ks[0], M.ks[1], M.ks[2]);
            v3 Lt = mk(rec(3), rec(4), rec(5));
            bool any = false;
            for (int i = 0; i < 3; i++) {
                const float4 c = P.ch_val[cb + map[(size_t)e * P.ch_split + i]];
                if (__float_as_uint(c.w) & kValMissed) continue;   // a missed child adds nothing
                const v3 mask = mk(i == 0 ? 1.0f : 0.0f, i == 1 ? 1.0f : 0.0f, i == 2 ? 1.0f : 0.0f);
                Lt = add(Lt, mul(ks, mul(mk(c.x, c.y, c.z), mask)));
                any = true;
            }
            if (!any) {   // doEnv: no child hit
                const v3 rayD = mk(rec(11), rec(12), rec(13)), nn = mk(rec(14), rec(15), rec(16));
                const float vDotN = rec(17), q = rec(18) / rec(21);
                const float sq = std_max(0.0f, sqrtf(1.0f - (q * q) * (1.0f - vDotN * vDotN)));
                const v3 dir2 = normalized(add(scale(rayD, q), scale(nn, q * vDotN - sq)), rsqT);
                Lt = add(Lt, mul(ks, mat_env(P, M, dir2)));
            }
            const v3 ka = mk(M.ka[0], M.ka[1], M.ka[2]), le = mk(M.le[0], M.le[1], M.le[2]);
            const v3 base = scale(add(add(add(z, ka), z), z), rec(1));
            val = add(add(base, scale(add(z, Lt), rec(2))), le);
        }
        P.ch_val[g] = make_float4(val.x, val.y, val.z, __uint_as_float(0u));
    }
}

// Per unit of the chunk: the paths' values summed in path order and averaged
// as Scene::sampleScene does (src/Scene.cpp:224-233); a missed eye ray takes
// the environment / background.  Frame / bucket mode: float RGB + Image::Map
// 8-bit of the pixel; adaptive passes: the unit's colour (ucol).
__global__ void __launch_bounds__(kWG) chain_finish_kernel(RenderParams P) {
    if (chunk_dead(P)) return;
    const uint16_t* rsqT = P.tables + 2048;
    const uint32_t np = (uint32_t)P.num_paths, n = chunk_units(P);
    for (uint32_t u = blockIdx.x * kWG + threadIdx.x; u < n; u += gridDim.x * kWG) {
        const UnitPix U = unit_pixel(P, P.unit_base + u);
        if (!U.valid) continue;
        const float4 hv = unit_hit(P, u, U);
        v3 col;
        if (__float_as_int(hv.w) >= 0) {
            v3 result = mk(0, 0, 0);
            for (uint32_t path = 0; path < np; path++) {
                const float4 v = P.ch_val[u * np + path];
                result = add(result, mk(v.x, v.y, v.z));
            }
            col = scale(result, 1.0f / (float)P.num_paths);
        } else {
            col = P.env ? env_or_bg(P, unit_eye(P, U, rsqT).d) : mk(P.bg[0], P.bg[1], P.bg[2]);
        }
        if (P.ucol) {
            P.ucol[P.unit_base + u] = make_float4(col.x, col.y, col.z, 0.f);
            continue;
        }
        store_rgb(P, U.slot, col);
    }
}

// Adaptive pass n: the eye rays of the chunk's units, closest hits into uhits
// (the centre ray of pass 1 is also the pixel's hit record, as the fused
// adaptive kernel writes it).  Counts eye rays and eye-ray hits.
template <bool COUNT, bool FAST, bool INST, int MINW = 1>
__global__ void __launch_bounds__(kWG, MINW) unit_eye_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    const uint32_t n = chunk_units(P);
    if ((uint32_t)blockIdx.x * kWG >= n) return;   // before any barrier
    load_tables(P.tables, s_tab, 1024);
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, s_tab, s_stack + tid,
           P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    uint32_t rays = 0, hits = 0;
    for (uint32_t u0 = (uint32_t)blockIdx.x * kWG + (uint32_t)(tid & ~63); u0 < n; u0 += gridDim.x * (uint32_t)kWG) {
        const uint32_t u = u0 + (uint32_t)lane;
        if (u >= n) continue;
        const UnitPix U = unit_pixel(P, P.unit_base + u);
        DHit h{1e12f, 0.f, 0.f, -1};
        bool hit = false;
        if (U.valid) {
            const EyeRay er = unit_eye(P, U, rsqT);
            hit = traverse<false, COUNT, FAST, INST>(T, make_ray(er.o, er.d, er.time), 0.001f, h, st);
            rays++;
            hits += hit ? 1u : 0u;
        }
        const float4 rec = make_float4(h.t, h.a, h.b, __int_as_float(hit ? h.prim : -1));
        P.uhits[u] = rec;
        if (U.valid && U.sample == 0) P.hits[U.slot] = rec;
    }
    unsigned long long er = rays, eh = hits;
    for (int off = 32; off > 0; off >>= 1) {
        er += __shfl_down(er, off);
        eh += __shfl_down(eh, off);
    }
    if (lane == 0) {
        if (er) atomicAdd(&P.ctr[CTR_RAYS_P], er);
        if (eh) atomicAdd(&P.ctr[CTR_HITS], eh);
    }
    if (COUNT) {
        unsigned long long nv = st.nodes, lv = st.leaves;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_down(nv, off);
            lv += __shfl_down(lv, off);
        }
        if (lane == 0) {
            atomicAdd(&P.ctr[CTR_NODES], nv);
            atomicAdd(&P.ctr[CTR_LEAVES], lv);
        }
    }
    if (st.overflow) atomicOr(&P.ctr[CTR_OVERFLOW], 1ull);
}

// End of a chunk (one block): its statistics into the frame's unless it outgrew a
// level (the fallback counts its units then), and per level the entries per path
// it needed (x 65536, + 1) into the stream's capacity estimates for this pass --
// exact up to the level that overflowed, unknown (all ones) past it.
__global__ void __launch_bounds__(64) chain_merge_kernel(RenderParams P) {
    const int i = threadIdx.x;
    const bool dead = chunk_dead(P);
    if (dead && i == 0) atomicAdd(P.ctr_out + CTR_FALLBACK, 1ull);
    if (!dead && i < CTR_N) {
        const unsigned long long v = P.ctr[i];
        if (i == CTR_MAXSP || (i >= CTR_TP && i < CTR_TS + 4)) atomicMax(P.ctr_out + i, v);
        else if (i == CTR_OVERFLOW) { if (v) atomicOr(P.ctr_out + i, v); }
        else if (v) atomicAdd(P.ctr_out + i, v);
    }
    if (!P.ch_est || i == 0 || i >= P.ch_levels) return;
    const uint32_t paths = chunk_units(P) * (uint32_t)P.num_paths;
    if (!paths) return;
    // a level below one that overflowed was not measured: it leaves the estimate as it
    // is (unseen levels keep the worst-case size until a chunk measures them), so one
    // fallback chunk never pins a level to the worst case for the scene's lifetime
    for (int k = 1; k < i; k++)
        if (P.ch_cnt[k] > lcap(P, k)) return;
    const uint64_t r = ((uint64_t)P.ch_cnt[i] * 65536u + paths - 1) / paths + 1;
    atomicMax(P.ch_est + i, (uint32_t)min<uint64_t>(r, 0xFFFFFFFEull));
}

// The units of a chunk that outgrew a level's estimated capacity, rendered by the
// fused chain shading (Shader::shade: every path's tree depth first, the same rays,
// draws and adds as the engine -- tests/test_chain.py) from the units' eye-ray hits,
// written as chain_finish writes them.  Nothing to do (one uniform load) otherwise.
// COUNT: a count-mode frame, whose node / leaf visit statistics then include these units.
template <bool POINT_ONLY, bool INST, int REC, bool COUNT>
__global__ void __launch_bounds__(kWG) chain_fallback_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    __shared__ float s_ior[kIorCap * kWG];
    if (!chunk_dead(P)) return;
    load_tables(P.tables, s_tab, 1024);
    const uint16_t* rcpT = s_tab;
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, false, P.scalar_nodes, P.leaves, rcpT, s_stack + tid, P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    uint32_t shadow_total = 0, secondary_total = 0;
    const uint32_t n = chunk_units(P);
    for (uint32_t u = blockIdx.x * kWG + (uint32_t)tid; u < n; u += gridDim.x * kWG) {
        const UnitPix U = unit_pixel(P, P.unit_base + u);
        if (!U.valid) continue;
        const float4 hv = unit_hit(P, u, U);
        const DHit h{hv.x, hv.y, hv.z, __float_as_int(hv.w)};
        const EyeRay er = unit_eye(P, U, rsqT);
        v3 col;
        if (h.prim >= 0) {
            const CamParams& cam = P.cam[U.f];
            Shader<POINT_ONLY, false, INST, kFused, REC> S{P, T, rcpT, rsqT, st, (uint32_t)(U.y * cam.W + U.x), 0u,
                                                        P.seed + (uint32_t)U.f, 0, 0u};
            S.sample = U.sample;
            S.time = S.shadow_time = er.time;
            S.iorS = s_ior + tid;
            S.lvl = P.lvl + (blockIdx.x * kWG + tid);
            col = S.template shade<COUNT>(make_ray(er.o, er.d, er.time), h);
            shadow_total += S.shadow_rays;
            secondary_total += S.secondary;
        } else {
            col = P.env ? env_or_bg(P, er.d) : mk(P.bg[0], P.bg[1], P.bg[2]);
        }
        if (P.ucol) {
            P.ucol[P.unit_base + u] = make_float4(col.x, col.y, col.z, 0.f);
            continue;
        }
        store_rgb(P, U.slot, col);
    }
    flush_secondary(P, secondary_total, lane);
    flush_stats<COUNT>(P, st, shadow_total, lane, 0, 0);
}

// After adaptive pass n: per pixel of the pass, Scene::adaptiveSampleScene's
// bookkeeping in the fused adaptive kernel's order -- pass 1 sets the result;
// pass n >= 2 adds its n^2 colours in (i, j) order, forms the running mean with
// getSum's float 1/6 and the gamma-space change; then the pixel either refines
// (listed for pass n + 1) or is written (float RGB + Image::Map 8-bit).
__global__ void __launch_bounds__(kWG) adapt_combine_kernel(RenderParams P) {
    const int n = P.adapt_n;
    const uint32_t nn = (uint32_t)(n * n);
    const uint32_t npx = P.unit_cnt ? *P.unit_cnt : P.units_total;
    for (uint32_t r = blockIdx.x * kWG + threadIdx.x; r < npx; r += gridDim.x * kWG) {
        const uint32_t id = P.units ? P.units[r] : r;   // item << 6 | lane
        int x, y;
        size_t slot;
        if (!item_pixel(P, (int)(id >> 6), (int)(id & 63u), x, y, slot)) continue;
        v3 result;
        bool cut = false;
        if (n == 1) {
            const float4 c = P.ucol[r];
            result = mk(c.x, c.y, c.z);
        } else {
            const float4 rv = P.adapt_res[slot];
            result = mk(rv.x, rv.y, rv.z);
            v3 cur = mk(0, 0, 0);
            for (uint32_t q = 0; q < nn; q++) {
                const float4 c = P.ucol[(size_t)r * nn + q];
                cur = add(cur, mk(c.x, c.y, c.z));
            }
            const float pre = (float)sum_squares(n - 1), now = (float)(n * n);
            const v3 nr = scale(add(scale(result, pre), cur), 1.0f / (pre + now));
            const float tx = gamma_f(P.gammaF, result.x) - gamma_f(P.gammaF, nr.x);
            const float ty = gamma_f(P.gammaF, result.y) - gamma_f(P.gammaF, nr.y);
            const float tz = gamma_f(P.gammaF, result.z) - gamma_f(P.gammaF, nr.z);
            cut = fmaxf(fabsf(tx), fmaxf(fabsf(ty), fabsf(tz))) < P.noise;
            result = nr;
        }
        const int level = n + 1;
        if ((level <= P.max_subdivs && !cut) || level <= P.min_subdivs) {
            P.adapt_res[slot] = make_float4(result.x, result.y, result.z, 0.f);
            P.next_units[atomicAdd(P.next_cnt, 1u)] = id;
            continue;
        }
        store_rgb(P, slot, result);
    }
}

// kernel variants: point lights only x instanced scene x REC (1, 2) x MODE (gen, resolve)
template <int MODE, int REC>
static KernelFn chain0_fn(bool po, bool inst) {
    return po ? (inst ? chain0_kernel<true, true, REC, MODE> : chain0_kernel<true, false, REC, MODE>)
              : (inst ? chain0_kernel<false, true, REC, MODE> : chain0_kernel<false, false, REC, MODE>);
}
template <int MODE, int REC>
static KernelFn chain_shade_fn(bool po, bool inst) {
    return po ? (inst ? chain_shade_kernel<true, true, REC, MODE> : chain_shade_kernel<true, false, REC, MODE>)
              : (inst ? chain_shade_kernel<false, true, REC, MODE> : chain_shade_kernel<false, false, REC, MODE>);
}
KernelFn pick_chain0(bool resolve, bool po, bool inst, int rec) {
    if (rec == 2) return resolve ? chain0_fn<kResolve, 2>(po, inst) : chain0_fn<kGen, 2>(po, inst);
    return resolve ? chain0_fn<kResolve, 1>(po, inst) : chain0_fn<kGen, 1>(po, inst);
}
KernelFn pick_chain_shade(bool resolve, bool po, bool inst, int rec) {
    if (rec == 2) return resolve ? chain_shade_fn<kResolve, 2>(po, inst) : chain_shade_fn<kGen, 2>(po, inst);
    return resolve ? chain_shade_fn<kResolve, 1>(po, inst) : chain_shade_fn<kGen, 1>(po, inst);
}
KernelFn pick_chain_trace(bool c, bool f, bool inst, int step) {
    if (!c && !inst)   // occupancy target of the plain-scene trace (timed variants)
        return f ? chain_trace_kernel<false, true, false, 8> : chain_trace_kernel<false, false, false, 8>;
    if (inst && step == 1)
        return c ? (f ? chain_trace_kernel<true, true, true, 1, 1> : chain_trace_kernel<true, false, true, 1, 1>)
                 : (f ? chain_trace_kernel<false, true, true, 1, 1> : chain_trace_kernel<false, false, true, 1, 1>);
    if (inst && step == 2)
        return c ? (f ? chain_trace_kernel<true, true, true, 1, 2> : chain_trace_kernel<true, false, true, 1, 2>)
                 : (f ? chain_trace_kernel<false, true, true, 1, 2> : chain_trace_kernel<false, false, true, 1, 2>);
    if (inst) return c ? (f ? chain_trace_kernel<true, true, true> : chain_trace_kernel<true, false, true>)
                       : (f ? chain_trace_kernel<false, true, true> : chain_trace_kernel<false, false, true>);
    return c ? (f ? chain_trace_kernel<true, true, false> : chain_trace_kernel<true, false, false>)
             : (f ? chain_trace_kernel<false, true, false> : chain_trace_kernel<false, false, false>);
}
KernelFn pick_unit_eye(bool c, bool f, bool inst) {
    if (inst) return c ? (f ? unit_eye_kernel<true, true, true> : unit_eye_kernel<true, false, true>)
                       : (f ? unit_eye_kernel<false, true, true> : unit_eye_kernel<false, false, true>);
    if (!c) return f ? unit_eye_kernel<false, true, false, 7> : unit_eye_kernel<false, false, false, 7>;
    return f ? unit_eye_kernel<true, true, false> : unit_eye_kernel<true, false, false>;
}
KernelFn pick_chain_compact() { return chain_compact_kernel; }
KernelFn pick_chain_merge() { return chain_merge_kernel; }
template <bool C>
static KernelFn chain_fallback_fn(bool po, bool inst, int rec) {
    if (rec == 2) return po ? (inst ? chain_fallback_kernel<true, true, 2, C> : chain_fallback_kernel<true, false, 2, C>)
                            : (inst ? chain_fallback_kernel<false, true, 2, C> : chain_fallback_kernel<false, false, 2, C>);
    return po ? (inst ? chain_fallback_kernel<true, true, 1, C> : chain_fallback_kernel<true, false, 1, C>)
              : (inst ? chain_fallback_kernel<false, true, 1, C> : chain_fallback_kernel<false, false, 1, C>);
}
KernelFn pick_chain_fallback(bool po, bool inst, int rec, bool count) {
    return count ? chain_fallback_fn<true>(po, inst, rec) : chain_fallback_fn<false>(po, inst, rec);
}
KernelFn pick_chain_finish() { return chain_finish_kernel; }
KernelFn pick_chain_fold() { return chain_fold_kernel; }
KernelFn pick_adapt_combine() { return adapt_combine_kernel; }

}  // namespace mrt
