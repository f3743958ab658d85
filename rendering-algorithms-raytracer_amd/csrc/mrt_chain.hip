// mrt_chain.hip -- the wavefront chain engine: Blinn reflection / refraction
// rays and path tracing (Shader REC 1 / 2) level by level instead of one lane
// walking its whole chain.
//
// The fused kernels (shade_kernel<REC>) keep every level's shading state live
// across each secondary and shadow traversal: 256 VGPRs plus scratch, one
// wave per SIMD.  Here the chain of Shader::level calls
// of one path (src/Blinn.cpp:39-335) is cut at each child ray:
//
//   chain0   (per pixel, tile schedule)  level 0 of every path of the pixel
//            (the camera ray's IOR history persists across its paths) in two
//            passes around shadow_kernel, as the direct path's 2a / 2b / 2c:
//            kGen writes the shadow rays, kResolve shades with the answers.
//            A path either ends (final value -> ch_tv / ch_te) or spawns a
//            child into the sparse spawn slots at its own index, with its
//            level record (ch_rec) written for the combine;
//   compact  spawn slots of level k -> dense level k+1 (block-aggregated:
//            one atomic per 1024 slots), each entry keeping its parent index;
//   trace    closest hit of every level-k+1 entry (traversal only: few
//            registers, full occupancy);
//   shade    level k+1 of every entry (kGen, shadow_kernel, kResolve): a miss
//            ends the path with the environment (or nothing, a GI ray without
//            environment sampling), a hit runs Shader::level, which ends it or
//            spawns again;
//   resolve  (after the last level) every level shaded again with its shadow
//            answers: level records and final values;
//   path     per path: the final value folded up its chain with
//            chain_combine (deepest first, the parent indices);
//   finish   per pixel: the paths averaged and the pixel written (float RGB +
//            Image::Map 8-bit).
//
// Every ray, every RNG draw (keyed by pixel, path and level) and every add is
// the fused kernel's, so the two engines give bit-identical frames
// (tests/test_secondary.py, tests/test_path_trace.py).  A frame whose slots do
// not fit the scratch budget runs in chunks of work items.
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

__device__ __forceinline__ size_t lvl_off(const RenderParams& P, int k) { return (size_t)k * P.ch_cap; }
// level record of entry e of level k: lvl_words consecutive floats (the combine
// walks one path's chain, so a record is read as a unit)
__device__ __forceinline__ ChainRec chain_rec(const RenderParams& P, int k, uint32_t e) {
    return ChainRec{P.ch_rec + ((size_t)k * P.ch_cap + e) * (size_t)P.lvl_words, 1};
}
static constexpr uint32_t kDeadPath = 0xFFFFFFFFu;   // ch_te of a path whose camera ray missed

// A spawned child at sparse slot s: its ray, state word and the IOR column
// (the child's history, written by Shader::level).
__device__ __forceinline__ void write_spawn(const RenderParams& P, uint32_t s, const LevelOut& o, uint32_t path_id,
                                            const ChainState& cs, const float* iorS) {
    const size_t cap = P.ch_cap;
    P.ch_sp[s] = make_float4(o.r2.o[0], o.r2.o[1], o.r2.o[2], __uint_as_float(path_id));
    P.ch_sp[cap + s] = make_float4(o.r2.d[0], o.r2.d[1], o.r2.d[2], __uint_as_float(pack_state(cs, o.env_miss)));
    P.ch_sp[2 * cap + s] = make_float4(iorS[1 * kWG], iorS[2 * kWG], iorS[3 * kWG], iorS[4 * kWG]);
    P.ch_sp[3 * cap + s] = make_float4(iorS[5 * kWG], iorS[6 * kWG], iorS[7 * kWG], 0.f);
}

// a path's final value: level k's value (or a missed child's) and where it ended
__device__ __forceinline__ void write_final(const RenderParams& P, uint32_t path_id, v3 v, int level, bool none,
                                            uint32_t entry) {
    P.ch_tv[path_id] = make_float4(v.x, v.y, v.z, __uint_as_float((uint32_t)level | (none ? 1u << 8 : 0u)));
    P.ch_te[path_id] = entry;
}

// shadow-ray slots of chain level k (each level keeps its own until the resolve pass)
__device__ __forceinline__ size_t shadow_base(const RenderParams& P, int k) {
    return (size_t)k * P.ch_cap * (size_t)P.max_shadow;
}

// The camera ray's time of path p of the chunk (every ray below the camera ray
// carries it): the getTimeSample draw of the pixel's eye ray (sample 0, shared
// by all its paths).
__device__ __forceinline__ float path_time(const RenderParams& P, uint32_t p) {
    const uint32_t pl = p / (uint32_t)P.num_paths;
    int x, y;
    size_t slot;
    item_pixel(P, P.item_base + (int)(pl >> 6), (int)(pl & 63u), x, y, slot);
    const int f = item_frame(P, P.item_base + (int)(pl >> 6));
    const CamParams& cam = P.cam[f];
    const float tr = rng((uint32_t)(y * cam.W + x), 0u, 2, P.seed + (uint32_t)f);
    return 1.f - ((tr * tr) * tr) * cam.shutter;
}

// Level 0 of every path of a chunk's pixels (tile schedule over the chunk's
// work items).  Path id = (work item of the chunk * 64 + lane) * num_paths + path.
// MODE kGen writes each path's shadow rays (level-0 slots p * max_shadow + j,
// count in nrays[p]) and its spawned child (the spawn decision, the child ray
// and its IOR history do not depend on the shadow answers); kResolve runs the
// same shading with the answers and writes the level record or the path's
// final value.  No traversal runs in either, so the shading state never has to
// live across one.
template <bool POINT_ONLY, bool INST, int REC, int MODE>
__global__ void __launch_bounds__(kWG) chain0_kernel(RenderParams P) {
    __shared__ float s_ior[kIorCap * kWG];
    const uint16_t* rcpT = P.tables;          // no triangle tests here: both tables from global (L1)
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    Trav T{P.nodes, false, false, P.leaves, rcpT, nullptr, nullptr, P.gstride};   // unused: no traversal
    TravStats st;
    uint32_t shadow_total = 0, secondary_total = 0;
    TileSched ts(P, wave, lane);
    for (int item = ts.first(); item >= 0; item = ts.next(item)) {
        int x, y;
        size_t slot;
        const bool valid = item_pixel(P, P.item_base + item, lane, x, y, slot);
        DHit h{1e12f, 0.f, 0.f, -1};
        if (valid) {
            const float4 hv = P.hits[slot];
            h = DHit{hv.x, hv.y, hv.z, __float_as_int(hv.w)};
        }
        const uint32_t pbase = ((uint32_t)item * 64u + (uint32_t)lane) * (uint32_t)P.num_paths;
        if (!valid || h.prim < 0) {   // nothing to shade: no shadow rays, no spawns (finish writes env / background)
            if (MODE == kGen)
                for (int path = 0; path < P.num_paths; path++) {
                    P.nrays[pbase + path] = 0;
                    P.ch_flag[pbase + path] = 0;
                    P.ch_te[pbase + path] = kDeadPath;
                }
            continue;
        }
        const int f = item_frame(P, P.item_base + item);
        const CamParams& cam = P.cam[f];
        const uint32_t seed = P.seed + (uint32_t)f;
        const EyeRay er = camera_ray(cam, seed, x, y, rsqT);
        const DRay r = make_ray(er.o, er.d, er.time);
        Shader<POINT_ONLY, false, INST, MODE, REC> S{P, T, rcpT, rsqT, st, (uint32_t)(y * cam.W + x), 0u, seed, 0, 0u};
        S.iorS = s_ior + tid;
        S.time = S.shadow_time = er.time;
        typename Shader<POINT_ONLY, false, INST, MODE, REC>::IorCam icam;
        for (int path = 0; path < P.num_paths; path++) {
            const uint32_t p = pbase + (uint32_t)path;
            S.skey = (uint32_t)path;   // eye-ray sample 0
            S.slot0 = (size_t)p * (size_t)P.max_shadow;
            S.nslot = 0;
            ChainState cs;
            LevelOut o;
            S.template level<false>(r, h, cs, icam, chain_rec(P, 0, p), o);
            if (MODE == kGen) {
                P.nrays[p] = (uint8_t)S.nslot;
                if (o.spawn) write_spawn(P, p, o, p, cs, S.iorS);
                P.ch_flag[p] = o.spawn ? 1 : 0;
            } else if (!o.spawn) {
                write_final(P, p, o.val, 0, false, p);
            }
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
// lane) and reserves their entries with one atomic.
static constexpr int kCompactGroup = 4 * kWG;
__global__ void __launch_bounds__(kWG) chain_compact_kernel(RenderParams P) {
    __shared__ uint32_t s_cnt[4 * (kWG / 64)];
    __shared__ uint32_t s_base;
    const int k = P.ch_level;
    const uint32_t n = k == 0 ? (uint32_t)P.n_tiles * 64u * (uint32_t)P.num_paths : P.ch_cnt[k];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t cap = P.ch_cap, dst0 = lvl_off(P, k + 1);
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
            if (d >= P.ch_cap) { atomicOr(&P.ctr[CTR_OVERFLOW], 2ull); continue; }   // cannot happen: <= one child per slot
            const float4 o = P.ch_sp[e], dd = P.ch_sp[cap + e], i0 = P.ch_sp[2 * cap + e], i1 = P.ch_sp[3 * cap + e];
            P.ch_ray[2 * dst0 + d] = o;
            P.ch_ray[2 * dst0 + cap + d] = dd;
            P.ch_ior[2 * dst0 + d] = i0;
            P.ch_ior[2 * dst0 + cap + d] = make_float4(i1.x, i1.y, i1.z, __uint_as_float(e));
        }
        __syncthreads();   // s_cnt / s_base reused by the next group
    }
}

// One launch per chain level k = P.ch_level: the closest hits of level k's
// entries (nA of them; the children spawned by level k - 1) and the any-hit
// answers of level k - 1's shadow rays (nB slots), which no longer wait for
// each other -- a level's resolve needs its shadow answers only at the end of
// the chunk.  Wave-uniform 64-slot chunks, the closest-hit chunks first.
template <bool COUNT, bool FAST, bool INST, int MINW = 1>
__global__ void __launch_bounds__(kWG, MINW) chain_trace_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    const int k = P.ch_level;
    const uint32_t nA = k < P.ch_levels ? P.ch_cnt[k] : 0u;
    const uint32_t m = (uint32_t)P.max_shadow;
    const uint32_t nprev = k == 1 ? (uint32_t)P.n_tiles * 64u * (uint32_t)P.num_paths : P.ch_cnt[k - 1];
    const uint32_t nB = nprev * m;
    const uint32_t chA = (nA + 63u) >> 6, chunks = chA + ((nB + 63u) >> 6);
    const uint32_t wave_id = (uint32_t)blockIdx.x * (kWG / 64) + (uint32_t)(threadIdx.x >> 6);
    if ((uint32_t)blockIdx.x * (kWG / 64) >= chunks) return;   // the block has no chunks (before any barrier)
    load_tables(P.tables, s_tab, 1024);
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes != 0, P.leaves, s_tab, s_stack + tid,
           P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    const size_t base = lvl_off(P, k), cap = P.ch_cap, sb = shadow_base(P, k - 1);
    const uint8_t* nrays = P.nrays + (size_t)(k - 1) * cap;
    for (uint32_t c = wave_id; c < chunks; c += gridDim.x * (kWG / 64)) {
        if (c < chA) {   // closest hit of entry e
            const uint32_t e = (c << 6) + (uint32_t)lane;
            if (e >= nA) continue;
            const float4 o = P.ch_ray[2 * base + e], d = P.ch_ray[2 * base + cap + e];
            const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z),
                                    INST && P.has_mb ? path_time(P, __float_as_uint(o.w)) : 0.f);
            DHit h{1e12f, 0.f, 0.f, -1};
            const bool hit = traverse<false, COUNT, FAST, INST>(T, r, 0.001f, h, st);
            P.ch_hit[base + e] = make_float4(h.t, h.a, h.b, __int_as_float(hit ? h.prim : -1));
        } else {         // shadow ray j of level k - 1's entry (or path) s, any hit
            const uint32_t i = ((c - chA) << 6) + (uint32_t)lane, s = i / m;
            if (i >= nB || i - s * m >= (uint32_t)nrays[s]) continue;
            const float4 o = P.ray_o[sb + i], d = P.ray_d[sb + i];
            const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), d.w);
            DHit h{o.w, 0.f, 0.f, -1};
            P.occl[sb + i] = traverse<true, COUNT, FAST, INST>(T, r, 0.001f, h, st) ? 1 : 0;
        }
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

// Shading of chain level k >= 1.  kGen (one launch per level, k =
// P.ch_level): every entry that hit writes its shadow rays (level-k slots
// e * max_shadow + j) and its spawned child.  kResolve (one launch per chunk,
// all levels 1 .. ch_levels - 1): a missed child ends its path with the
// environment (or nothing: a GI ray without environment sampling), a hit is
// shaded again with its shadow answers and writes its level record or the
// path's final value.
template <bool POINT_ONLY, bool INST, int REC, int MODE>
__global__ void __launch_bounds__(kWG) chain_shade_kernel(RenderParams P) {
    __shared__ float s_ior[kIorCap * kWG];
    const uint16_t* rcpT = P.tables;
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, false, false, P.leaves, rcpT, nullptr, nullptr, P.gstride};   // unused: no traversal
    TravStats st;
    uint32_t shadow_total = 0, secondary_total = 0;
    const size_t cap = P.ch_cap;
    const uint32_t np = (uint32_t)P.num_paths;
    float* iorS = s_ior + tid;
    const int k0 = MODE == kGen ? P.ch_level : 1, k1 = MODE == kGen ? P.ch_level + 1 : P.ch_levels;
    for (int k = k0; k < k1; k++) {
        const uint32_t n = P.ch_cnt[k];
        const size_t base = lvl_off(P, k);
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
                    P.nrays[(size_t)k * cap + e] = 0;
                    P.ch_flag[e] = 0;
                } else {
                    write_final(P, p, env_miss ? env_or_bg(P, mk(d.x, d.y, d.z)) : mk(0, 0, 0), k, !env_miss, e);
                }
                continue;
            }
            // the pixel of path p (RNG key, frame of a batched launch)
            const uint32_t pl = p / np, path = p - pl * np;
            int x, y;
            size_t slot;
            item_pixel(P, P.item_base + (int)(pl >> 6), (int)(pl & 63u), x, y, slot);
            const int f = item_frame(P, P.item_base + (int)(pl >> 6));
            const float4 i0 = P.ch_ior[2 * base + e], i1 = P.ch_ior[2 * base + cap + e];
            iorS[0] = 1.0f;
            iorS[1 * kWG] = i0.x; iorS[2 * kWG] = i0.y; iorS[3 * kWG] = i0.z; iorS[4 * kWG] = i0.w;
            iorS[5 * kWG] = i1.x; iorS[6 * kWG] = i1.y; iorS[7 * kWG] = i1.z;
            const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z));
            Shader<POINT_ONLY, false, INST, MODE, REC> S{P, T, rcpT, rsqT, st, (uint32_t)(y * P.cam[f].W + x), 0u,
                                                        P.seed + (uint32_t)f,
                                                        shadow_base(P, k) + (size_t)e * (size_t)P.max_shadow, 0u};
            S.iorS = iorS;
            S.skey = path;
            if (INST && P.has_mb) S.time = S.shadow_time = path_time(P, p);
            typename Shader<POINT_ONLY, false, INST, MODE, REC>::IorCam icam;   // unused below the camera ray
            LevelOut lo;
            S.template level<false>(r, h, cs, icam, chain_rec(P, k, e), lo);
            shadow_total += S.shadow_rays;
            secondary_total += S.secondary;
            if (MODE == kGen) {
                P.nrays[(size_t)k * cap + e] = (uint8_t)S.nslot;
                const bool spawn = lo.spawn && k + 1 < P.ch_levels;
                if (spawn) write_spawn(P, e, lo, p, cs, iorS);
                P.ch_flag[e] = spawn ? 1 : 0;
            } else if (lo.spawn && k + 1 >= P.ch_levels) {   // deeper than the chain bound (cannot happen)
                atomicOr(&P.ctr[CTR_OVERFLOW], 2ull);
                write_final(P, p, mk(0, 0, 0), k, false, e);
            } else if (!lo.spawn) {
                write_final(P, p, lo.val, k, false, e);
            }
        }
    }
    if (MODE == kGen) {
        flush_stats<false>(P, st, shadow_total, lane, 0, 0);
        flush_secondary(P, secondary_total, lane);
    }
}

// One lane per path of the chunk: the path's final value folded up its chain
// with chain_combine, deepest level first (Blinn::shade's returns), into ch_tv.
__global__ void __launch_bounds__(kWG) chain_path_kernel(RenderParams P) {
    const size_t cap = P.ch_cap;
    const uint32_t n = (uint32_t)P.n_tiles * 64u * (uint32_t)P.num_paths;
    for (uint32_t p = blockIdx.x * kWG + threadIdx.x; p < n; p += gridDim.x * kWG) {
        uint32_t e = P.ch_te[p];
        if (e == kDeadPath) continue;
        const float4 tv = P.ch_tv[p];
        const uint32_t bits = __float_as_uint(tv.w);
        v3 val = mk(tv.x, tv.y, tv.z);
        bool none = (bits >> 8) & 1u;
        for (int kk = (int)(bits & 255u) - 1; kk >= 0; kk--) {
            const uint32_t pe = __float_as_uint(P.ch_ior[2 * lvl_off(P, kk + 1) + cap + e].w);   // parent entry
            val = chain_combine(P, chain_rec(P, kk, pe), val, none);
            none = false;
            e = pe;
        }
        P.ch_tv[p] = make_float4(val.x, val.y, val.z, 0.f);
    }
}

// Per pixel of the chunk: the paths' values summed in path order and averaged
// as Scene::sampleScene does (src/Scene.cpp:224-233); a missed camera ray takes
// the environment / background.  Float RGB + Image::Map 8-bit.
__global__ void __launch_bounds__(kWG) chain_finish_kernel(RenderParams P) {
    const int tid = threadIdx.x, lane = tid & 63;
    const uint16_t* rsqT = P.tables + 2048;
    const uint32_t np = (uint32_t)P.num_paths;
    for (int item = (int)(blockIdx.x * (kWG / 64) + (tid >> 6)); item < P.n_tiles; item += (int)(gridDim.x * (kWG / 64))) {
        int x, y;
        size_t slot;
        if (!item_pixel(P, P.item_base + item, lane, x, y, slot)) continue;
        const float4 hv = P.hits[slot];
        v3 col;
        if (__float_as_int(hv.w) >= 0) {
            v3 result = mk(0, 0, 0);
            const uint32_t pbase = ((uint32_t)item * 64u + (uint32_t)lane) * np;
            for (uint32_t path = 0; path < np; path++) {
                const float4 v = P.ch_tv[pbase + path];
                result = add(result, mk(v.x, v.y, v.z));
            }
            col = scale(result, 1.0f / (float)P.num_paths);
        } else {
            const int f = item_frame(P, P.item_base + item);
            col = P.env ? env_or_bg(P, camera_ray(P.cam[f], P.seed + (uint32_t)f, x, y, rsqT).d) : mk(P.bg[0], P.bg[1], P.bg[2]);
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
KernelFn pick_chain_trace(bool c, bool f, bool inst, int waves) {
    if (waves == 8 && !c && !inst)   // occupancy target of the plain-scene trace (timed variants)
        return f ? chain_trace_kernel<false, true, false, 8> : chain_trace_kernel<false, false, false, 8>;
    if (inst) return c ? (f ? chain_trace_kernel<true, true, true> : chain_trace_kernel<true, false, true>)
                       : (f ? chain_trace_kernel<false, true, true> : chain_trace_kernel<false, false, true>);
    return c ? (f ? chain_trace_kernel<true, true, false> : chain_trace_kernel<true, false, false>)
             : (f ? chain_trace_kernel<false, true, false> : chain_trace_kernel<false, false, false>);
}
KernelFn pick_chain_compact() { return chain_compact_kernel; }
KernelFn pick_chain_finish() { return chain_finish_kernel; }
KernelFn pick_chain_path() { return chain_path_kernel; }

}  // namespace mrt
