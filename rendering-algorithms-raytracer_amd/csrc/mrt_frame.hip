// mrt_frame.hip -- the single-point-light frame kernels (BASELINE configs C1-C3):
// frame1_kernel (camera ray, closest hit, shading and the shadow ray in one
// launch per frame) and shade1_kernel (the same shading from hit records).  A
// translation unit of its own: the headline kernel recompiles in seconds and the
// library's kernels compile in parallel.
#include "mrt_kernels.h"
#include "mrt_shader.h"

namespace mrt {

// Shading of one primary hit for one point light and num_paths == 1 (the
// BASELINE configs C1-C3): HitInfo::getAllInfos + Ray::getPoint, the
// Lambert/Blinn set-up, straight-line PointLight::sampleLight with only the
// light's three pre-shadow scalars live across the any-hit traversal, then the
// material sums.  Same operations in the same order as Shader::shade.  r is the
// camera ray, (ht, ha, hb, prim) its closest hit.
// POW: some Blinn material has specExp != 1 (Blinn::shade's pow, src/Blinn.cpp:220).  Scenes
// without one run the POW = false kernels, which carry no double-precision pow: its
// polynomial constants, hoisted out of the tile loop, took VGPRs and scratch.
template <bool COUNT, bool FAST, bool POW, int WALK = 1>
__device__ __forceinline__ v3 shade1_hit(const RenderParams& P, const Trav& T, TravStats& st, const DRay& r, float ht,
                                         float ha, float hb, int prim, const uint16_t* rcpT, const uint16_t* rsqT,
                                         uint32_t& shadow_total) {
    const v3 rayD = mk(r.d[0], r.d[1], r.d[2]);
    const PrimShade ps = P.prims[prim];
    const uint32_t mi = ps.mat;
    const bool lambert = P.mats[mi].type == MRT_LAMBERT;
    const float4 A = P.verts[ps.v[0]], B = P.verts[ps.v[1]], C = P.verts[ps.v[2]];
    const v3 geoN = normalized(cross(mk(B.x - A.x, B.y - A.y, B.z - A.z), mk(C.x - A.x, C.y - A.y, C.z - A.z)), rsqT);
    const float c = 1.0f - ha - hb;
    const float4 n0 = P.normals[ps.n[0]], n1 = P.normals[ps.n[1]], n2 = P.normals[ps.n[2]];
    const v3 N = normalized(add(add(scale(mk(n0.x, n0.y, n0.z), c), scale(mk(n1.x, n1.y, n1.z), ha)),
                                scale(mk(n2.x, n2.y, n2.z), hb)), rsqT);
    const v3 from = mk(r.o[0] + ht * r.d[0], r.o[1] + ht * r.d[1], r.o[2] + ht * r.d[2]);
    // Lambert::shade uses the shading normal and no reflection vector;
    // Blinn::shade flips to the viewer's side (src/Blinn.cpp:150-170).
    v3 n = N, rVec = mk(0, 0, 0);
    if (!lambert) {
        const v3 viewDir = neg(rayD);
        float vDotN = dot(viewDir, N);
        const float vDotGeoN = dot(viewDir, geoN);
        const bool same = (vDotN * vDotGeoN) >= 0.0f;
        n = same ? N : geoN;
        vDotN = same ? vDotN : vDotGeoN;
        if (vDotN < 0.0f) { vDotN = -vDotN; n = neg(n); }
        rVec = add(rayD, scale(n, 2.0f * vDotN));
    }
    // PointLight::sampleLight (src/PointLight.cpp:8-81), as Shader::point_light
    const DevLight& l = P.lights[0];
    v3 L = sub(mk(l.pos[0], l.pos[1], l.pos[2]), from);
    float nDotL = dot(n, L);
    float e = 0.f, spec = 0.f;
    if (nDotL > 0.0f) {
        float falloff = dot(L, L);
        const float distanceRecip = rsqrt_nr(falloff, rsqT);
        falloff = rcp_nr(falloff, rcpT);
        const float distance = rcp_nr(distanceRecip, rcpT);
        L = scale(L, distanceRecip);
        nDotL *= distanceRecip;
        float Aterm = (l.power * falloff) * (0.25f / 3.1415926f);
        float rdl = std_max(0.f, dot(rVec, L));
        // Only these three scalars stay live across the shadow traversal: without the
        // pin the compiler sinks both products below it, keeping rVec, L, falloff and
        // the light's power live instead (4 spilled values per pixel)
        asm volatile("" : "+v"(Aterm), "+v"(rdl), "+v"(nDotL));
        float attenuate = 1.0f;
        if (l.cast_shadows) {
            const DRay sr = make_ray(from, L);
            DHit sh{distance, 0.f, 0.f, -1};
            shadow_total++;
            if (traverse<true, COUNT, FAST, false, true, WALK == 2, WALK != 0>(T, sr, 0.001f, sh, st)) attenuate = 0.0f;
        }
        attenuate *= nDotL;
        spec = rdl * attenuate;
        e = Aterm * attenuate;
    }
    const DevMaterial& M = P.mats[mi];
    const v3 E = mk(e, e, e);
    const v3 kd = mk(M.kd[0], M.kd[1], M.kd[2]), ka = mk(M.ka[0], M.ka[1], M.ka[2]);
    v3 sh;
    if (lambert) {
        sh = add(add(mk(0, 0, 0), mul(E, kd)), ka);
    } else {
        const v3 ks = mk(M.ks[0], M.ks[1], M.ks[2]);
        const float pw = (!POW || M.spec_exp == 1.0f) ? spec : spec_pow(spec, M.spec_exp);
        const v3 Ls = add(mk(0, 0, 0), scale(scale(mul(E, ks), M.spec_amt), pw));
        const v3 Ld = add(add(mk(0, 0, 0), mul(E, kd)), ka);
        const v3 z = mk(0, 0, 0);
        sh = add(add(scale(add(add(Ld, Ls), z), 1.0f), scale(add(z, z), 1.0f)), mk(M.le[0], M.le[1], M.le[2]));
    }
    // the path average of Scene::sampleScene with num_paths == 1 (the only case
    // these kernels run): x * (1 / 1) == x, so the scale is left out
    return add(mk(0, 0, 0), sh);
}

// Kernel 2, specialised for one point light and num_paths == 1: shade1_hit of
// every pixel's hit record (the two-launch path; frame1_kernel fuses both).
template <bool COUNT, bool FAST, int MINW, bool POW>
__global__ void __launch_bounds__(kWG, MINW) shade1_kernel(RenderParams P) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    load_tables(P.tables, s_tab, 1024);
    const uint64_t t0 = (COUNT || P.wave_log) ? wall_clock64() : 0;
    const uint16_t* rcpT = s_tab;           // per triangle test: LDS
    const uint16_t* rsqT = P.tables + 2048; // a few per pixel: global (L1-resident)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, rcpT, s_stack + tid, P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    uint32_t shadow_total = 0;
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
        if (!item_pixel(P, item, lane, x, y, slot)) continue;
        const float4 hv = P.hits[slot];
        const int prim = __float_as_int(hv.w);
        v3 col = mk(P.bg[0], P.bg[1], P.bg[2]);
        if (prim >= 0) {
            const int f = item_frame(P, item);
            const EyeRay er = camera_ray(P.cam[f], P.seed + (uint32_t)f, x, y, rsqT);
            col = shade1_hit<COUNT, FAST, POW>(P, T, st, make_ray(er.o, er.d), hv.x, hv.y, hv.z, prim, rcpT, rsqT, shadow_total);
        }
        item_pixel(P, item, lane, x, y, slot);
        store_rgb(P, slot, col);
    }
    flush_stats<COUNT, false>(P, st, shadow_total, lane, t0, ntiles);
}

// Kernel 1+2 fused for one point light and num_paths == 1 (C1-C3): per pixel
// the camera ray, its closest hit, then shade1_hit (the shadow ray any-hit) in
// the same lane -- one persistent launch per frame, no hit-record hand-off
// (the record is written only when the caller asks for hits, P.hits != null),
// one launch tail instead of two.  Every ray's visits and every operation are
// those of primary_kernel + shade1_kernel, so the frame is bit-identical.
// LN: the hierarchy's top kLdsNodes nodes are staged in LDS (+8 KB per workgroup)
// and both walks read their wave-uniform visits from there (traverse_impl); the
// host runs it when asked (tuning "lds_nodes").
// WALK (traverse_impl): 0 the walk loop with a second exit (stack overflow returns), 1 one
// exit (XONE), 2 one exit + LN, 3 one exit and one latch (OL) for the camera rays' walk.
// Same bits either way; the host runs 3 unless tuned (walk_exit, walk_latch, lds_nodes).
template <bool COUNT, bool FAST, int MINW, bool POW, int WALK = 1>
__global__ void __launch_bounds__(kWG, MINW) frame1_kernel(RenderParams P) {
    constexpr bool LN = WALK == 2;
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    __shared__ QNode s_top[LN ? kLdsNodes : 1];
    if (LN)   // (the host runs LN only on hierarchies of at least kLdsNodes nodes)
        for (int i = threadIdx.x; i < kLdsNodes * 32; i += kWG)
            reinterpret_cast<uint32_t*>(s_top)[i] = reinterpret_cast<const uint32_t*>(P.nodes)[i];
    load_tables(P.tables, s_tab, 1024);   // (its barrier also covers s_top)
    const uint64_t t0 = (COUNT || P.wave_log) ? wall_clock64() : 0;
    const uint16_t* rcpT = s_tab;
    const uint16_t* rsqT = P.tables + 2048;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave: an SGPR
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, rcpT, s_stack + tid, P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    if (LN) T.lnodes = s_top;
    TravStats st, ss;   // primary / shadow rays (count mode)
    uint32_t nhits = 0, shadow_total = 0;
    unsigned long long wave_steps = 0, wave_steps_s = 0;   // count mode: per tile, the max node steps over lanes
    TileSched ts(P, wave, lane);
    uint32_t ntiles = 0;
    for (int item = ts.first(); item >= 0; item = ts.next(item)) {
        const RenderParams& PA = reload_params();   // camera, tile and diagnostics parameters
        if (PA.wave_log && lane_id() == 0 && ntiles < kLogTiles) {
            unsigned long long* r = PA.wave_log + kLogWords * ((size_t)blockIdx.x * (kWG / 64) + wave);
            r[4 + ntiles] = ((unsigned long long)item << 40) | (wall_clock64() & ((1ull << 40) - 1));
            r[4 + kLogTiles + ntiles] = ts.deq_ticks;
        }
        ntiles++;
        int x, y;
        size_t slot;
        const uint32_t n0 = st.nodes, s0 = ss.nodes;
        if (item_pixel(PA, item, lane_id(), x, y, slot)) {
            const int f = item_frame(PA, item);
            const EyeRay er = camera_ray(PA.cam[f], PA.seed + (uint32_t)f, x, y, rsqT);
            const DRay r = make_ray(er.o, er.d);
            DHit h{1e12f, 0.f, 0.f, -1};
            const bool hit = traverse<false, COUNT, FAST, false, true, LN, WALK != 0, WALK == 3>(T, r, 0.001f, h, st);
            const RenderParams& PB = reload_params();   // shading parameters
            v3 col = mk(PB.bg[0], PB.bg[1], PB.bg[2]);
            if (hit) {
                nhits++;
                col = shade1_hit<COUNT, FAST, POW, WALK>(PB, T, ss, r, h.t, h.a, h.b, h.prim, rcpT, rsqT, shadow_total);
            }
            const RenderParams& PC = reload_params();   // outputs
            item_pixel(PC, item, lane_id(), x, y, slot);   // recompute: keeps it out of the traversals' live set
            if (PC.hits) PC.hits[slot] = make_float4(h.t, h.a, h.b, __int_as_float(hit ? h.prim : -1));
            store_rgb(PC, slot, col);
        }
        if (COUNT) {
            uint32_t dmax = st.nodes - n0, smax = ss.nodes - s0;
            for (int off = 32; off > 0; off >>= 1) {
                dmax = max(dmax, (uint32_t)__shfl_xor(dmax, off));
                smax = max(smax, (uint32_t)__shfl_xor(smax, off));
            }
            wave_steps += dmax;
            wave_steps_s += smax;
        }
    }
    if (COUNT) {   // the shadow rays' node visits and wave steps (the latency model of bench.py)
        unsigned long long sv = ss.nodes;
        for (int off = 32; off > 0; off >>= 1) sv += __shfl_down(sv, off);
        if (lane_id() == 0) {
            atomicAdd(&P.ctr[CTR_WAVE_STEPS_P], wave_steps);
            atomicAdd(&P.ctr[CTR_WAVE_STEPS_S], wave_steps_s);
            atomicAdd(&P.ctr[CTR_NODES_S], sv);
        }
    }
    // one wall-clock record per wave (the primary span counters; the wave log counts both kinds' nodes)
    flush_stats<COUNT, true>(P, st, nhits, lane_id(), t0, ntiles, ss.nodes, wave);
    flush_stats<COUNT, false, false>(P, ss, shadow_total, lane_id(), t0, ntiles, 0, wave);
}

template <int W, bool POW>
static KernelFn shade1_fn(bool c, bool f) {
    return c ? (f ? shade1_kernel<true, true, W, POW> : shade1_kernel<true, false, W, POW>)
             : (f ? shade1_kernel<false, true, W, POW> : shade1_kernel<false, false, W, POW>);
}
template <int W, bool POW, int WALK>
static KernelFn frame1_fn(bool c, bool f) {
    return c ? (f ? frame1_kernel<true, true, W, POW, WALK> : frame1_kernel<true, false, W, POW, WALK>)
             : (f ? frame1_kernel<false, true, W, POW, WALK> : frame1_kernel<false, false, W, POW, WALK>);
}
template <int WALK>
static KernelFn pick_frame1_walk(int w, bool c, bool f, bool pow) {
    if (pow) return w == 1 ? frame1_fn<1, true, WALK>(c, f) : frame1_fn<6, true, WALK>(c, f);
    switch (w) {
        case 1: return frame1_fn<1, false, WALK>(c, f);
        case 5: return frame1_fn<5, false, WALK>(c, f);
        case 7: return frame1_fn<7, false, WALK>(c, f);
        case 8: return frame1_fn<8, false, WALK>(c, f);
        default: return frame1_fn<6, false, WALK>(c, f);
    }
}
// pow: a Blinn material with specExp != 1 (those scenes run at 6 waves, or unbounded);
// walk: 0 two-exit walk loop, 1 one exit, 2 one exit + the LDS top-node walk, 3 one exit + one latch
KernelFn pick_frame1(int w, bool c, bool f, bool pow, int walk) {
    switch (walk) {
        case 0: return pick_frame1_walk<0>(w, c, f, pow);
        case 2: return pick_frame1_walk<2>(w, c, f, pow);
        case 3: return pick_frame1_walk<3>(w, c, f, pow);
        default: return pick_frame1_walk<1>(w, c, f, pow);
    }
}
// (the two-launch path: fused = 0, or a caller that wants hit records) at 5 waves
KernelFn pick_shade1(bool c, bool f, bool pow) { return pow ? shade1_fn<5, true>(c, f) : shade1_fn<5, false>(c, f); }
}  // namespace mrt
