// mrt_kernels.h -- device-side hot path (included by mrt_device.hip only).
//
// One lane = one pixel (or one query ray).  The traversal reproduces the
// reference's QBVH stack order exactly (src/BVH.cpp:1128-1178): the node's
// four boxes are tested once when it is popped (QBVH_Node::intersect,
// src/BVH.cpp:391-414), leaf slots are intersected immediately in slot order
// (intersect4, src/BVH.cpp:1298-1459), hit inner slots are pushed in slot order
// so the highest slot is visited next.  The highest hit child is kept in a
// register instead of a push+pop.  Stack: per-lane column in LDS (kLdsStack
// entries, conflict-free [entry][lane] layout) spilling to a per-thread global
// column beyond that.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/mrt.h"
#include "mrt_math.h"
#include "mrt_texture.h"
#include "mrt_types.h"

namespace mrt {

static constexpr int kWG = 256;          // threads per workgroup (4 waves)
static constexpr int kLdsStack = 16;     // stack entries per lane kept in LDS (max seen: 11)
static constexpr int kGlobalStack = 240; // spill entries per thread in HBM: 256 in all, the reference's stack (src/BVH.cpp:1133)
static constexpr int kTableWords = 4096; // rcp[2048] + rsqrt[2048] (u16)
static constexpr int kLdsNodes = 64;     // LN walks: the world hierarchy's first 64 nodes (breadth first) staged in LDS

struct DRay {
    float o[3], d[3], id[3];
    bool finite;  // o and id finite: no box-test value can be NaN (see box_test_fast)
    float time;   // Ray::time (src/Ray.h): where an MBObject lane's triangle is (motion blur)
};

// Ray(threadID, o, d, ...), src/Ray.h:71-101: id = 1/d, +-1e12 for d == 0.
__device__ __forceinline__ DRay make_ray(v3 o, v3 d) {
    DRay r;
    r.o[0] = o.x; r.o[1] = o.y; r.o[2] = o.z;
    r.d[0] = d.x; r.d[1] = d.y; r.d[2] = d.z;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float v = 1.0f / r.d[k];
        if (r.d[k] == 0.f) v = (v < -0.f) ? -1e12f : 1e12f;
        r.id[k] = v;
    }
    r.finite = __builtin_isfinite(r.o[0]) & __builtin_isfinite(r.o[1]) & __builtin_isfinite(r.o[2]) &
               __builtin_isfinite(r.id[0]) & __builtin_isfinite(r.id[1]) & __builtin_isfinite(r.id[2]);
    r.time = 0.f;
    return r;
}
__device__ __forceinline__ DRay make_ray(v3 o, v3 d, float time) {
    DRay r = make_ray(o, d);
    r.time = time;
    return r;
}

struct DHit {
    float t, a, b;
    int32_t prim;
    int32_t inst = -1;  // ProxyObject of the hit (-1: world triangle)
};

struct Trav {
    const QNode* __restrict__ nodes;
    bool fast_box;            // all node boxes finite and fast box test enabled
    int scalar_nodes;         // bit 0: scalar fetch of wave-uniform nodes, bit 1: of wave-uniform triangles,
                              // bit 2: octant-ordered box test for waves whose rays share an octant (tuning)
    const DLeaf* __restrict__ leaves;
    const uint16_t* rcpT;     // LDS
    int32_t* lds;             // this lane's LDS stack column (stride kWG)
    int32_t* gstk;            // this thread's global spill column (stride gstride)
    uint32_t gstride;
    const DevInstance* inst = nullptr;  // ProxyObjects (instanced scenes)
    // alpha-mapped triangles (Material::m_alphaMap, src/BVH.cpp:1397-1445): the
    // shading records, texture coordinates, materials and map textures
    const PrimShade* aprims = nullptr;
    const uint4* apuv = nullptr;        // per prim: texture-coordinate indices, w = has texcoords
    const float2* auv = nullptr;
    const DevMaterial* amats = nullptr;
    const DevTexture* atex = nullptr;
    // motion-blurred triangles (MBObject, src/MBObject.cpp): per world prim bit 0
    // = MBObject lane (nullptr: no motion blur); vertices at time 0 / time 1
    // (PrimShade vertex indices)
    const uint8_t* pflags = nullptr;
    const float4* verts = nullptr;
    const float4* verts2 = nullptr;
    bool near_first = false;   // any-hit walks descend into the nearest hit child first (order-free answer)
    const QNode* lnodes = nullptr;   // LN walks: nodes 0 .. kLdsNodes - 1 (the hierarchy's top levels) in LDS
};

struct TravStats {
    uint32_t nodes = 0, leaves = 0, uniform = 0;  // uniform: visits in wave-uniform node steps
    int max_sp = 0;
    bool overflow = false;
};

__device__ __forceinline__ bool stk_push(const Trav& c, int& sp, int32_t v) {
    if (sp < kLdsStack) c.lds[sp * kWG] = v;
    else if (sp < kLdsStack + kGlobalStack) c.gstk[(size_t)(sp - kLdsStack) * c.gstride] = v;
    else return false;
    sp++;
    return true;
}
__device__ __forceinline__ int32_t stk_pop(const Trav& c, int& sp) {
    --sp;
    return sp < kLdsStack ? c.lds[sp * kWG] : c.gstk[(size_t)(sp - kLdsStack) * c.gstride];
}

// v[i] for a lane-varying i as three selects (no divergent branch tree).
__device__ __forceinline__ int32_t sel4(const int4& v, int i) {
    const int32_t lo = (i & 1) ? v.y : v.x, hi = (i & 1) ? v.w : v.z;
    return (i & 2) ? hi : lo;
}

// One triangle of intersect4 (src/BVH.cpp:1298-1459), same operations and
// rounding as the reference's SSE lane.  The reference tests all four lanes of
// a packet against result.t at packet entry and keeps the lowest accepted t
// (first lane on ties); walking the triangles in order and accepting only
// t < current best selects the same winner.  Empty lanes are zero triangles:
// det = 0 -> rcp_nr = NaN rejects them exactly as in the reference.
__device__ __forceinline__ bool tri_test(const float* __restrict__ T, const DRay& r, float tMin, float tBest,
                                         float& ot, float& oa, float& ob, const uint16_t* rcpT) {
    const float ax = T[0], ay = T[1], az = T[2], e0x = T[3], e0y = T[4], e0z = T[5], e1x = T[6], e1y = T[7], e1z = T[8];
    const float px = r.d[1] * e1z - r.d[2] * e1y;
    const float py = -1.0f * (r.d[0] * e1z - r.d[2] * e1x);
    const float pz = r.d[0] * e1y - r.d[1] * e1x;
    const float det = e0x * px + (e0y * py + e0z * pz);
    const float inv = rcp_nr(det, rcpT);
    const float tx = r.o[0] - ax, ty = r.o[1] - ay, tz = r.o[2] - az;
    const float a = inv * (tx * px + (ty * py + tz * pz));
    // no active lane has a in [0, 1] (most tests of a packet the wave's rays miss):
    // the wave skips b and t -- every lane's answer is "no hit" either way
    if (__ballot((a >= 0.0f) & (a <= 1.0f)) == 0) {
        ot = a; oa = a; ob = a;
        return false;
    }
    const float qx = ty * e0z - tz * e0y;
    const float qy = -1.0f * (tx * e0z - tz * e0x);
    const float qz = tx * e0y - ty * e0x;
    const float b = inv * (r.d[0] * qx + (r.d[1] * qy + r.d[2] * qz));
    const float t = inv * (e1x * qx + (e1y * qy + e1z * qz));
    ot = t; oa = a; ob = b;
    // the reference's a <= 1 and b <= 1 lanes are implied: with a, b >= 0 (so neither is
    // NaN), a + b rounds to at least max(a, b), so (a + b) <= 1 bounds both
    return (a >= 0.0f) & (b >= 0.0f) & ((a + b) <= 1.0f) & (t >= tMin) & (t < tBest);
}

// QBVH_Node::intersect (src/BVH.cpp:391-414) -> 4-bit hit mask.
__device__ __forceinline__ int box_test(const float4* bx, const DRay& r, float tMin, float tMax) {
    float4 mnx = bx[0], mny = bx[1], mnz = bx[2], mxx = bx[3], mxy = bx[4], mxz = bx[5];
    float lx[4] = {mnx.x, mnx.y, mnx.z, mnx.w}, ly[4] = {mny.x, mny.y, mny.z, mny.w}, lz[4] = {mnz.x, mnz.y, mnz.z, mnz.w};
    float hx[4] = {mxx.x, mxx.y, mxx.z, mxx.w}, hy[4] = {mxy.x, mxy.y, mxy.z, mxy.w}, hz[4] = {mxz.x, mxz.y, mxz.z, mxz.w};
    int m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float t0x = (lx[i] - r.o[0]) * r.id[0], t1x = (hx[i] - r.o[0]) * r.id[0];
        float t0y = (ly[i] - r.o[1]) * r.id[1], t1y = (hy[i] - r.o[1]) * r.id[1];
        float t0z = (lz[i] - r.o[2]) * r.id[2], t1z = (hz[i] - r.o[2]) * r.id[2];
        float t0 = sse_max(sse_min(t0x, t1x), sse_max(sse_min(t0y, t1y), sse_min(t0z, t1z)));
        float t1 = sse_min(sse_max(t0x, t1x), sse_min(sse_max(t0y, t1y), sse_max(t0z, t1z)));
        m |= (int)(sse_max(t0, tMin) <= sse_min(t1, tMax)) << i;
    }
    return m;
}

// Same mask as box_test on the hardware min/max.  Precondition: ray origin,
// 1/d and the node boxes are finite, so every slab value is finite or +-inf,
// never NaN.  Then v_min/v_max (IEEE minnum/maxnum) return the same number as
// the MINPS/MAXPS selects except possibly the sign of a zero, and the only
// consumer of these values is `imin <= imax`, for which -0 == +0.
// present (wave-uniform; 15 = all): slots 2 and 3 are tested only when their bit is set.
// A built hierarchy's empty slots are its nodes' last ones (25% of all slots in the
// BASELINE scenes); an empty slot's bit is masked by the node's kinds either way, so
// skipping its test changes no bit.
__device__ __forceinline__ int box_test_fast(const float4* bx, const DRay& r, float tMin, float tMax, int present = 15) {
    float4 mnx = bx[0], mny = bx[1], mnz = bx[2], mxx = bx[3], mxy = bx[4], mxz = bx[5];
    float lx[4] = {mnx.x, mnx.y, mnx.z, mnx.w}, ly[4] = {mny.x, mny.y, mny.z, mny.w}, lz[4] = {mnz.x, mnz.y, mnz.z, mnz.w};
    float hx[4] = {mxx.x, mxx.y, mxx.z, mxx.w}, hy[4] = {mxy.x, mxy.y, mxy.z, mxy.w}, hz[4] = {mxz.x, mxz.y, mxz.z, mxz.w};
    int m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (i >= 2 && !((present >> i) & 1)) continue;
        float t0x = (lx[i] - r.o[0]) * r.id[0], t1x = (hx[i] - r.o[0]) * r.id[0];
        float t0y = (ly[i] - r.o[1]) * r.id[1], t1y = (hy[i] - r.o[1]) * r.id[1];
        float t0z = (lz[i] - r.o[2]) * r.id[2], t1z = (hz[i] - r.o[2]) * r.id[2];
        float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                   __builtin_fmaxf(__builtin_fminf(t0z, t1z), tMin));
        float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                   __builtin_fminf(__builtin_fmaxf(t0z, t1z), tMax));
        m |= (int)(t0 <= t1) << i;
    }
    return m;
}

// box_test_fast for a ray whose direction signs are known at compile time (S bit k:
// 1/d[k] < 0).  For 1/d >= 0 the rounded (lo - o) * (1/d) <= (hi - o) * (1/d) whenever
// lo <= hi (rounding is monotone), so the slab minimum is the lo distance and the
// maximum the hi one; for 1/d < 0 the other way round.  Every slot box of a built
// hierarchy has lo <= hi on each axis (checked at upload: DeviceState::boxes_ordered),
// and empty slots are masked by the caller, so the mask equals box_test_fast's with
// half of its min / max work (the near / far planes are picked by register, not by
// an instruction).
template <int S>
__device__ __forceinline__ int box_test_oct(const float4* bx, const DRay& r, float tMin, float tMax, int present = 15) {
    const float4 nx = bx[(S & 1) ? 3 : 0], fx = bx[(S & 1) ? 0 : 3];
    const float4 ny = bx[(S & 2) ? 4 : 1], fy = bx[(S & 2) ? 1 : 4];
    const float4 nz = bx[(S & 4) ? 5 : 2], fz = bx[(S & 4) ? 2 : 5];
    const float lx[4] = {nx.x, nx.y, nx.z, nx.w}, ly[4] = {ny.x, ny.y, ny.z, ny.w}, lz[4] = {nz.x, nz.y, nz.z, nz.w};
    const float hx[4] = {fx.x, fx.y, fx.z, fx.w}, hy[4] = {fy.x, fy.y, fy.z, fy.w}, hz[4] = {fz.x, fz.y, fz.z, fz.w};
    int m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        if (i >= 2 && !((present >> i) & 1)) continue;
        const float t0 = __builtin_fmaxf(__builtin_fmaxf((lx[i] - r.o[0]) * r.id[0], (ly[i] - r.o[1]) * r.id[1]),
                                         __builtin_fmaxf((lz[i] - r.o[2]) * r.id[2], tMin));
        const float t1 = __builtin_fminf(__builtin_fminf((hx[i] - r.o[0]) * r.id[0], (hy[i] - r.o[1]) * r.id[1]),
                                         __builtin_fminf((hz[i] - r.o[2]) * r.id[2], tMax));
        m |= (int)(t0 <= t1) << i;
    }
    return m;
}
// box_test_fast, or box_test_oct when the wave's rays share one octant (s < 8, wave-uniform)
__device__ __forceinline__ int box_test_sel(const float4* bx, const DRay& r, float tMin, float tMax, int s,
                                            int present = 15) {
    switch (s) {
        case 0: return box_test_oct<0>(bx, r, tMin, tMax, present);
        case 1: return box_test_oct<1>(bx, r, tMin, tMax, present);
        case 2: return box_test_oct<2>(bx, r, tMin, tMax, present);
        case 3: return box_test_oct<3>(bx, r, tMin, tMax, present);
        case 4: return box_test_oct<4>(bx, r, tMin, tMax, present);
        case 5: return box_test_oct<5>(bx, r, tMin, tMax, present);
        case 6: return box_test_oct<6>(bx, r, tMin, tMax, present);
        case 7: return box_test_oct<7>(bx, r, tMin, tMax, present);
        default: return box_test_fast(bx, r, tMin, tMax, present);
    }
}
// the wave-uniform octant of the active lanes' rays (1/d sign bits), or 8 when they differ
__device__ __forceinline__ int wave_octant(const DRay& r) {
    const int oct = (int)(r.id[0] < 0.f) | (int)(r.id[1] < 0.f) << 1 | (int)(r.id[2] < 0.f) << 2;
    const int o0 = __builtin_amdgcn_readfirstlane(oct);
    return __ballot(oct != o0) == 0 ? o0 : 8;
}

// box_test_fast that also returns each slot's entry distance (the slab max of
// the mins, clamped by tMin): any-hit walks may visit the nearest child first.
__device__ __forceinline__ int box_test_fast_t(const float4* bx, const DRay& r, float tMin, float tMax, float (&tn)[4]) {
    float4 mnx = bx[0], mny = bx[1], mnz = bx[2], mxx = bx[3], mxy = bx[4], mxz = bx[5];
    float lx[4] = {mnx.x, mnx.y, mnx.z, mnx.w}, ly[4] = {mny.x, mny.y, mny.z, mny.w}, lz[4] = {mnz.x, mnz.y, mnz.z, mnz.w};
    float hx[4] = {mxx.x, mxx.y, mxx.z, mxx.w}, hy[4] = {mxy.x, mxy.y, mxy.z, mxy.w}, hz[4] = {mxz.x, mxz.y, mxz.z, mxz.w};
    int m = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        float t0x = (lx[i] - r.o[0]) * r.id[0], t1x = (hx[i] - r.o[0]) * r.id[0];
        float t0y = (ly[i] - r.o[1]) * r.id[1], t1y = (hy[i] - r.o[1]) * r.id[1];
        float t0z = (lz[i] - r.o[2]) * r.id[2], t1z = (hz[i] - r.o[2]) * r.id[2];
        float t0 = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(t0x, t1x), __builtin_fminf(t0y, t1y)),
                                   __builtin_fmaxf(__builtin_fminf(t0z, t1z), tMin));
        float t1 = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(t0x, t1x), __builtin_fmaxf(t0y, t1y)),
                                   __builtin_fminf(__builtin_fmaxf(t0z, t1z), tMax));
        tn[i] = t0;
        m |= (int)(t0 <= t1) << i;
    }
    return m;
}
// the slot of `bits` (non-empty) with the smallest entry distance
__device__ __forceinline__ int nearest_slot(int bits, const float (&tn)[4]) {
    int best = 31 - __builtin_clz((unsigned)bits);
    float bt = tn[best];
#pragma unroll
    for (int i = 0; i < 4; i++)
        if (((bits >> i) & 1) && tn[i] < bt) { bt = tn[i]; best = i; }
    return best;
}

// Device child word of a QNode slot: >= 0 inner node; kEmptySlot; otherwise
// ~(leaf << 4 | check << 3 | proxy << 2 | (count - 1)) with count = objects in
// the packet, proxy = the packet has ProxyObject (checkOut) lanes and check = it
// has alpha-mapped or motion-blurred triangles (the host re-encodes the
// canonical ~leaf on upload).
__host__ __device__ __forceinline__ int32_t leaf_child(uint32_t leaf, int count, bool proxy = false, bool check = false) {
    return ~(int32_t)((leaf << 4) | (check ? 8u : 0u) | (proxy ? 4u : 0u) | (uint32_t)(count - 1));
}

// QNode::pad[0] of a device node: its slot kinds, set on upload from the child
// words (mrt_device.hip, upload_scene): bits 0-3 inner child, 4-7 leaf packet,
// 8-11 leaf packet with ProxyObject lanes.  One dword of the node's own line, read
// instead of decoding the four child words in every step.
__host__ __device__ __forceinline__ uint32_t slot_kinds(const int32_t child[4]) {
    uint32_t k = 0;
    for (int i = 0; i < 4; i++) {
        const int32_t ch = child[i];
        if (ch >= 0) k |= 1u << i;
        else if (ch != kEmptySlot) k |= (1u << (4 + i)) | ((~(uint32_t)ch & 4u) ? 1u << (8 + i) : 0u);
    }
    return k;
}
__device__ __forceinline__ int node_kinds(const float4* q) { return reinterpret_cast<const int32_t*>(q)[28]; }
__device__ __forceinline__ int kinds_inner(int k) { return k & 15; }
__device__ __forceinline__ int kinds_leaf(int k) { return (k >> 4) & 15; }
__device__ __forceinline__ int kinds_proxy(int k) { return (k >> 8) & 15; }

// An MBObject lane of intersect4 (src/BVH.cpp:1316-1334): the triangle at the
// ray's time, A = time * A2 + (1 - time) * A1 and the edges from the
// interpolated B and C, then the lane's usual test.
__device__ __noinline__ bool mb_tri_test(const Trav& c, int32_t prim, const DRay& r, float tMin, float tBest, float& ot,
                                         float& oa, float& ob) {
    const PrimShade& ps = c.aprims[prim];
    const float time = r.time, _1_time = 1.f - time;
    const float4 a1 = c.verts[ps.v[0]], b1 = c.verts[ps.v[1]], c1 = c.verts[ps.v[2]];
    const float4 a2 = c.verts2[ps.v[0]], b2 = c.verts2[ps.v[1]], c2 = c.verts2[ps.v[2]];
    float T[9];
    T[0] = time * a2.x + _1_time * a1.x; T[1] = time * a2.y + _1_time * a1.y; T[2] = time * a2.z + _1_time * a1.z;
    T[3] = (time * b2.x + _1_time * b1.x) - T[0]; T[4] = (time * b2.y + _1_time * b1.y) - T[1];
    T[5] = (time * b2.z + _1_time * b1.z) - T[2];
    T[6] = (time * c2.x + _1_time * c1.x) - T[0]; T[7] = (time * c2.y + _1_time * c1.y) - T[1];
    T[8] = (time * c2.z + _1_time * c1.z) - T[2];
    return tri_test(T, r, tMin, tBest, ot, oa, ob, c.rcpT);
}

// intersect4's alpha test (src/BVH.cpp:1401-1423) for lane k of leaf packet
// `leaf`: the triangle's material has an alpha map and getLookupAlpha at the
// hit's (u, v) -- interpolated texture coordinates, or (a, b) without them --
// is below 0.5.  Such a triangle is skipped; with the lanes walked in slot order
// and only t < best accepted, the first surviving lane of lowest t wins, as in
// the reference's t-ordered retry loop.  aoff: PrimShade index of the leaf's
// prim 0 (0 in the world; an instance's shade_base inside its BLAS, whose
// alpha-mapped triangles -- the reference's tree proxies -- are tested too).
__device__ __noinline__
bool alpha_rejects(const Trav& c, uint32_t leaf, int k, float a, float b, int32_t aoff) {
    const int32_t prim = c.leaves[leaf].prim[k] + aoff;
    const int am = c.amats[c.aprims[prim].mat].maps[kMapAlpha];
    if (am < 0) return false;
    float u = a, v = b;
    if (c.apuv) {
        const uint4 t = c.apuv[prim];
        if (t.w) {
            const float cc = 1.0f - a - b;
            const float2 t0 = c.auv[t.x], t1 = c.auv[t.y], t2 = c.auv[t.z];
            u = t0.x * cc + t1.x * a + t2.x * b;
            v = t0.y * cc + t1.y * a + t2.y * b;
        }
    }
    const DevTexture& T = c.atex[am];
    return tex_lookup4(T.data, T.W, T.H, T.type, u, v).w < 0.5f;
}

__device__ __forceinline__ float dp4(const float* row, float x, float y, float z, float w) {
    const float p0 = row[0] * x, p1 = row[1] * y, p2 = row[2] * z, p3 = row[3] * w;
    return (p0 + p1) + (p2 + p3);  // DPPS 0xFF
}

// ProxyObject::intersect (src/ProxyObject.cpp:78-82): the origin through
// multiplyAndDivideByW (DPPS 0xFF dots, RCPSS w; o.w = 1), the direction through
// the 4-wide dots with d.w = 0 (src/Matrix4x4.h:706-748, src/Ray.h:140-141).
__device__ __forceinline__ DRay object_ray(const DevInstance& I, const DRay& r, const uint16_t* rcpT) {
    const float ox = r.o[0], oy = r.o[1], oz = r.o[2], dx = r.d[0], dy = r.d[1], dz = r.d[2];
    const float w = rcp_nr(dp4(I.inv + 12, ox, oy, oz, 1.0f), rcpT);
    const v3 o = mk(w * dp4(I.inv, ox, oy, oz, 1.0f), w * dp4(I.inv + 4, ox, oy, oz, 1.0f),
                    w * dp4(I.inv + 8, ox, oy, oz, 1.0f));
    const v3 d = mk(dp4(I.inv, dx, dy, dz, 0.0f), dp4(I.inv + 4, dx, dy, dz, 0.0f), dp4(I.inv + 8, dx, dy, dz, 0.0f));
    return make_ray(o, d, r.time);
}

// Triangle k of leaf packet `leaf` (intersect4's lane), for the active lanes of a
// traversal's flattened leaf loop.  When every active lane tests the same
// triangle (coherent rays on one leaf: most primary and point-light shadow steps)
// its 36 bytes come once through the scalar cache into SGPRs, not 64 times
// through the vector path; tri_test then reads them as SGPR operands.  Distinct
// markers end the two branches so the compiler cannot merge them (see
// traverse_impl's node fetch).  The same test either way.
__device__ __forceinline__ bool tri_test_lane(const Trav& c, uint32_t leaf, int k, const DRay& r, float tMin,
                                              float tBest, float& t, float& a, float& b) {
    int ok;
    const uint32_t key = (leaf << 2) | (uint32_t)k;
    const uint32_t k0 = __builtin_amdgcn_readfirstlane(key);
    if ((c.scalar_nodes & 2) && __ballot(key != k0) == 0) {
        typedef const __attribute__((address_space(4))) float cfloat;
        cfloat* q = (cfloat*)(const void*)(c.leaves[k0 >> 2].tri[k0 & 3]);
        float T[9];
#pragma unroll
        for (int i = 0; i < 9; i++) T[i] = q[i];
        ok = tri_test(T, r, tMin, tBest, t, a, b, c.rcpT) ? 1 : 0;
        asm volatile("; mrt: scalar triangle" : "+v"(ok));
    } else {
        ok = tri_test(c.leaves[leaf].tri[k], r, tMin, tBest, t, a, b, c.rcpT) ? 1 : 0;
        asm volatile("; mrt: vector triangle" : "+v"(ok));
    }
    return ok != 0;
}

template <bool ANY, bool COUNT, bool FAST, bool INST = false, bool BL = false, bool CHECK = true, bool LN = false,
          bool XONE = true, bool OL = false>
__device__ bool traverse_impl(const Trav& c, const DRay& r, float tMin, DHit& h, TravStats& st, int32_t root = 0,
                              int sp0 = 0, int32_t aoff = 0);

// One ProxyObject lane: its BLAS traversed with the object-space ray, the
// current t as tMax, on the same stack above the caller's entries.
template <bool ANY, bool COUNT, bool FAST, bool CHECK = true>
__device__ __forceinline__ bool proxy_hit(const Trav& c, int inst, const DRay& r, float tMin, DHit& h,
                                          TravStats& st, int sp) {
    const DevInstance& I = c.inst[inst];
    const DRay ro = object_ray(I, r, c.rcpT);
    // BLAS packets with alpha-mapped triangles (check bit): PrimShade = shade_base + BLAS object
    // (the nested walk keeps the two-exit loop: C5's primary launch measured 37% slower with
    // one exit, traverse_impl XONE)
    if (FAST && ro.finite)
        return traverse_impl<ANY, COUNT, true, false, true, CHECK, false, false>(c, ro, tMin, h, st, I.root, sp, I.shade_base);
    return traverse_impl<ANY, COUNT, false, false, true, CHECK, false, false>(c, ro, tMin, h, st, I.root, sp, I.shade_base);
}

// BVH::intersect, QBVH branch (src/BVH.cpp:1128-1178).  Returns hit; h.prim is
// then the packed triangle slot (leaf << 2 | k), resolved by traverse().  On a
// stack overflow st.overflow is set and the query is abandoned.
//
// Per popped node: the 4-slot box mask (branch-free); hit inner slots other
// than the highest are pushed in slot order (branch-free LDS writes, so the
// highest is visited next and kept in a register); then the hit leaf slots
// are intersected in slot order in ONE flattened per-lane loop, one triangle
// per iteration, so a wave runs max-over-lanes(triangles) iterations instead
// of one packet loop per slot.  Same visit order and same t at every box test
// as the reference.
//
// INST: leaf packets with ProxyObject lanes (child-word bit 2) intersect those
// lanes first, in lane order (intersect4, src/BVH.cpp:1305-1315), each through
// a nested BLAS traversal (proxy_hit); root / sp0 start such a nested walk.
// INST / BL (a BLAS walk): packets with the check bit (3) test alpha-mapped
// lanes -- and, in the world, motion-blurred ones.
// CHECK = false: the scene has no alpha-mapped or motion-blurred lanes (no check bit
// is set), so their tests -- calls of the noinline mb_tri_test / alpha_rejects, whose
// call ABI costs the walk registers and scratch -- are compiled out.
// LN: wave-uniform visits of the hierarchy's top nodes (index < kLdsNodes, renumbered
// breadth first on upload) read them from LDS (c.lnodes, one broadcast address)
// instead of the scalar cache -- faster where the top levels end most rays (tuning
// lds_nodes, off by default: mrt_device.hip).
template <bool ANY, bool COUNT, bool FAST, bool INST, bool BL, bool CHECK, bool LN, bool XONE, bool OL>
__device__ bool traverse_impl(const Trav& c, const DRay& r, float tMin, DHit& h, TravStats& st, int32_t root,
                              int sp0, int32_t aoff) {
    int sp = sp0;
    int32_t cur = root;
    bool hit = false;
    // octant-ordered box tests (box_test_oct) when every active lane's ray has the same
    // direction signs: most primary tiles and point-light shadow rays
    const int soct = (FAST && !(ANY && c.near_first) && (c.scalar_nodes & 4)) ? wave_octant(r) : 8;
    while (true) {
        // stack top read at the start of the step: the LDS latency overlaps the
        // node fetch and box test (used only if this step pops)
        // (entry min(sp - 1, kLdsStack - 1) as unsigned: an in-column address for every sp)
        const int32_t peek = c.lds[__builtin_elementwise_min((uint32_t)(sp - 1), (uint32_t)(kLdsStack - 1)) * kWG];
        int m, kinds;
        int4 ch;
        // Wave-uniform node (all active lanes on one node, ~70% of primary
        // steps): fetch it once through the scalar cache into SGPRs instead of
        // 64 copies through the vector memory path.
        const int32_t c0 = __builtin_amdgcn_readfirstlane(cur);
        float tn[4] = {0.f, 0.f, 0.f, 0.f};   // slot entry distances (any-hit near-first order)
        if (LN && FAST && c0 < kLdsNodes && __ballot(cur != c0) == 0) {
            const QNode& nd = c.lnodes[c0];   // one wave-uniform LDS address: broadcast reads
            ch = make_int4(nd.child[0], nd.child[1], nd.child[2], nd.child[3]);
            kinds = (int)nd.pad[0];
            float4 bx[6];
#pragma unroll
            for (int k = 0; k < 6; k++) bx[k] = make_float4(nd.box[4 * k], nd.box[4 * k + 1], nd.box[4 * k + 2], nd.box[4 * k + 3]);
            m = (ANY && c.near_first) ? box_test_fast_t(bx, r, tMin, h.t, tn) : box_test_sel(bx, r, tMin, h.t, soct);
            asm volatile("; mrt: lds node" : "+v"(m));
        } else if (FAST && (c.scalar_nodes & 1) && __ballot(cur != c0) == 0) {
            // constant address space + uniform address -> s_load_dwordx16 (node
            // data is read-only for the whole launch)
            typedef const __attribute__((address_space(4))) float cfloat;
            typedef const __attribute__((address_space(4))) int32_t cint;
            cfloat* q = (cfloat*)(const void*)(c.nodes + c0);
            cint* qc = (cint*)(q + 24);
            ch = make_int4(qc[0], qc[1], qc[2], qc[3]);
            kinds = qc[4];
            float4 bx[6];
#pragma unroll
            for (int k = 0; k < 6; k++) bx[k] = make_float4(q[4 * k], q[4 * k + 1], q[4 * k + 2], q[4 * k + 3]);
            // the node's occupied slots (SGPR): its empty trailing slots are not tested
            const int present = __builtin_amdgcn_readfirstlane((kinds | (kinds >> 4)) & 15);
            // (the near-first test keeps all four: skipping measured 3% slower on D1's dome shadows)
            m = (ANY && c.near_first) ? box_test_fast_t(bx, r, tMin, h.t, tn)
                                      : box_test_sel(bx, r, tMin, h.t, soct, present);
            // distinct markers end the two branches, so the compiler cannot sink their
            // identical box tests into one block fed by 24 v_mov copies of the SGPR node:
            // this branch reads the boxes straight from SGPRs
            asm volatile("; mrt: scalar node" : "+v"(m));
        } else {
            const float4* q = reinterpret_cast<const float4*>(c.nodes + cur);
            ch = reinterpret_cast<const int4*>(q)[6];
            kinds = node_kinds(q);
            m = FAST ? ((ANY && c.near_first) ? box_test_fast_t(q, r, tMin, h.t, tn) : box_test_sel(q, r, tMin, h.t, soct))
                     : box_test(q, r, tMin, h.t);
            asm volatile("; mrt: vector node" : "+v"(m));
        }
        if (COUNT) {
            st.nodes++;
            if (__ballot(cur != c0) == 0) st.uniform++;  // all active lanes of the wave on one node
        }
        const int inner = m & kinds_inner(kinds);
        int lm = m & kinds_leaf(kinds);
        bool have_next = false;
        int32_t nxt = 0;
        if (inner) {
            // next: the highest hit slot (the reference's order); an any-hit walk in
            // near-first mode takes the nearest instead (its answer is order-free)
            const int top = (FAST && ANY && c.near_first) ? nearest_slot(inner, tn) : 31 - __builtin_clz((unsigned)inner);
            const int rest = inner ^ (1 << top);
            bool ovf = false;
            if (rest) {
                if (sp + 4 <= kLdsStack) {
                    c.lds[sp * kWG] = ch.x; sp += rest & 1;
                    c.lds[sp * kWG] = ch.y; sp += (rest >> 1) & 1;
                    c.lds[sp * kWG] = ch.z; sp += (rest >> 2) & 1;
                    c.lds[sp * kWG] = ch.w; sp += (rest >> 3) & 1;
                } else {
                    bool pushed = true;
#pragma unroll
                    for (int i = 0; i < 4; i++)
                        if ((rest >> i) & 1) pushed = pushed && stk_push(c, sp, sel4(ch, i));
                    // overflow (flagged).  XONE: the walk ends at the loop's one exit (the pop
                    // test below, with the stack emptied) instead of returning from here --
                    // an extra exit of the divergent loop costs exec-mask bookkeeping in every
                    // step (SALU -19% per step, C3 -7%, C4 -6%); the two-exit form stays as
                    // tuning walk_exit 0 (round 6: the bunny scenes' tail effect)
                    if (!pushed) {
                        st.overflow = true;
                        if (!XONE) return hit;
                        sp = sp0;
                        ovf = true;
                    }
                }
                if (COUNT && sp > st.max_sp) st.max_sp = sp;
            }
            nxt = sel4(ch, top);
            have_next = !ovf;
        }
        if (lm) {
            uint32_t leaf = 0;
            int k = 0, cnt = 0;
            bool check = false;
            while (true) {
                if (k == cnt) {
                    if (!lm) break;
                    const int s = __builtin_ctz((unsigned)lm);
                    lm &= lm - 1;
                    const uint32_t v = ~(uint32_t)sel4(ch, s);
                    leaf = v >> 4;
                    cnt = (int)(v & 3u) + 1;
                    k = 0;
                    check = CHECK && (INST || BL) && (v & 8u);
                    if (COUNT) st.leaves++;
                    if (INST && (v & 4u)) {
                        for (int j = 0; j < cnt; j++) {
                            const int32_t pm = c.leaves[leaf].prim[j];
                            if (pm > -2) continue;  // a triangle lane
                            DHit hi{h.t, 0.f, 0.f, -1};
                            const bool ph = proxy_hit<ANY, COUNT, FAST, CHECK>(c, -2 - pm, r, tMin, hi, st, sp);
                            if (st.overflow) return hit;
                            if (ph) {
                                if (ANY) return true;
                                h.t = hi.t; h.a = hi.a; h.b = hi.b; h.prim = hi.prim; h.inst = -2 - pm;
                                hit = true;
                            }
                        }
                    }
                }
                float t, a, b;
                bool ok;
                if (CHECK && (INST || BL) && check) {   // alpha-mapped / motion-blurred lanes
                    const int32_t pm = c.leaves[leaf].prim[k];
                    ok = (!BL && pm >= 0 && c.pflags && (c.pflags[pm] & 1u))
                             ? mb_tri_test(c, pm, r, tMin, h.t, t, a, b)
                             : tri_test(c.leaves[leaf].tri[k], r, tMin, h.t, t, a, b, c.rcpT);
                    ok = ok && !alpha_rejects(c, leaf, k, a, b, aoff);
                } else {
                    ok = tri_test_lane(c, leaf, k, r, tMin, h.t, t, a, b);
                }
                if (ok) {
                    if (ANY) return true;   // (an any-hit walk: returning here measured faster than a flag)
                    h.t = t; h.a = a; h.b = b; h.prim = (int32_t)((leaf << 2) | (uint32_t)k);
                    if (INST) h.inst = -1;
                    hit = true;
                }
                k++;
            }
        }
        if (OL) {
            // One back edge (OL): the next node is nxt or the popped entry, chosen by select
            // (the LDS top was read at the step's start; a pop from the global column, like the
            // walk's end, sits behind one compare).  With a branch per case the loop has two
            // latches, which the compiler's structurisation nests: lanes that pop wait until
            // every lane of the wave has ended its descent (§4, "walk loop latches").
            int32_t g = peek;
            // one compare for both rare cases: sp == sp0 (the walk is done) or sp > kLdsStack
            // (sp >= sp0 always; a walk entered above kLdsStack pops from the global column only)
            const uint32_t lds_left = sp0 < kLdsStack ? (uint32_t)(kLdsStack - sp0) : 0u;
            if (!have_next && (uint32_t)(sp - 1 - sp0) >= lds_left) {
                if (sp == sp0) break;
                g = c.gstk[(size_t)(sp - 1 - kLdsStack) * c.gstride];
            }
            cur = have_next ? nxt : g;
            sp -= have_next ? 0 : 1;
        } else if (have_next) {
            cur = nxt;
        } else {
            if (sp == sp0) break;
            if (sp <= kLdsStack) { cur = peek; sp--; }
            else cur = stk_pop(c, sp);
        }
    }
    return hit;
}

// One node visit of an any-hit traversal, resumable (traverse_impl's loop body
// for ANY, no instancing): the caller keeps cur / sp between calls, so a lane
// can drop a finished ray and start another while its wave keeps going (lane
// refill in shadow_kernel).  The visit order and every test are traverse_impl's.
// Returns true when the ray is done: `hit` = a triangle was accepted; otherwise
// the stack ran empty (miss) or overflowed (st.overflow).
template <bool COUNT, bool FAST>
__device__ __forceinline__ bool anyhit_step(const Trav& c, const DRay& r, float tMin, float tMax, int32_t& cur,
                                            int& sp, bool& hit, TravStats& st) {
    int m, kinds;
    int4 ch;
    const int32_t c0 = __builtin_amdgcn_readfirstlane(cur);
    float tn[4] = {0.f, 0.f, 0.f, 0.f};
    if (FAST && (c.scalar_nodes & 1) && __ballot(cur != c0) == 0) {   // wave-uniform node: scalar fetch
        typedef const __attribute__((address_space(4))) float cfloat;
        typedef const __attribute__((address_space(4))) int32_t cint;
        cfloat* q = (cfloat*)(const void*)(c.nodes + c0);
        cint* qc = (cint*)(q + 24);
        ch = make_int4(qc[0], qc[1], qc[2], qc[3]);
        kinds = qc[4];
        float4 bx[6];
#pragma unroll
        for (int k = 0; k < 6; k++) bx[k] = make_float4(q[4 * k], q[4 * k + 1], q[4 * k + 2], q[4 * k + 3]);
        m = c.near_first ? box_test_fast_t(bx, r, tMin, tMax, tn) : box_test_fast(bx, r, tMin, tMax);
        asm volatile("; mrt: scalar node" : "+v"(m));   // see traverse_impl
    } else {
        const float4* q = reinterpret_cast<const float4*>(c.nodes + cur);
        ch = reinterpret_cast<const int4*>(q)[6];
        kinds = node_kinds(q);
        m = FAST ? (c.near_first ? box_test_fast_t(q, r, tMin, tMax, tn) : box_test_fast(q, r, tMin, tMax))
                 : box_test(q, r, tMin, tMax);
        asm volatile("; mrt: vector node" : "+v"(m));
    }
    if (COUNT) st.nodes++;
    const int inner = m & kinds_inner(kinds);
    int lm = m & kinds_leaf(kinds);
    bool have_next = false;
    int32_t nxt = 0;
    if (inner) {
        const int top = (FAST && c.near_first) ? nearest_slot(inner, tn) : 31 - __builtin_clz((unsigned)inner);
        const int rest = inner ^ (1 << top);
        if (rest) {
            if (sp + 4 <= kLdsStack) {
                c.lds[sp * kWG] = ch.x; sp += rest & 1;
                c.lds[sp * kWG] = ch.y; sp += (rest >> 1) & 1;
                c.lds[sp * kWG] = ch.z; sp += (rest >> 2) & 1;
                c.lds[sp * kWG] = ch.w; sp += (rest >> 3) & 1;
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if ((rest >> i) & 1)
                        if (!stk_push(c, sp, sel4(ch, i))) { st.overflow = true; return true; }
            }
            if (COUNT && sp > st.max_sp) st.max_sp = sp;
        }
        nxt = sel4(ch, top);
        have_next = true;
    }
    if (lm) {
        uint32_t leaf = 0;
        int k = 0, cnt = 0;
        while (true) {
            if (k == cnt) {
                if (!lm) break;
                const int s = __builtin_ctz((unsigned)lm);
                lm &= lm - 1;
                const uint32_t v = ~(uint32_t)sel4(ch, s);
                leaf = v >> 4;
                cnt = (int)(v & 3u) + 1;
                k = 0;
                if (COUNT) st.leaves++;
            }
            float t, a, b;
            if (tri_test(c.leaves[leaf].tri[k], r, tMin, tMax, t, a, b, c.rcpT)) { hit = true; return true; }
            k++;
        }
    }
    if (have_next) { cur = nxt; return false; }
    if (sp == 0) return true;
    cur = stk_pop(c, sp);
    return false;
}

// Resumable any-hit step over the world hierarchy AND the instance BLASes
// (special-leaf scenes: ProxyObject, alpha-mapped and motion-blurred lanes),
// for the lane-refill schedule of shadow_kernel.  An any-hit answer does not
// depend on the visit order -- it is "some triangle of the leaves whose boxes
// all pass with tMax is accepted", a set fixed by the ray -- so the proxy lanes
// of a world leaf are deferred: pushed as stack entries (-2 - instance).
// Proxy entries are pushed, and so popped, in the world context; popping one
// enters the instance: the lane's ray becomes its object-space ray
// (object_ray) and a -1 entry below the BLAS root marks the return, where the
// world ray is rebuilt from its slot (one ray in registers, not two).  Every
// box and triangle test is traverse_impl's.  CHECK: the scene has alpha-mapped
// or motion-blurred lanes (child-word bit 3).
struct AnyState {
    DRay q;        // the current ray: the world ray, or the object-space ray inside an instance
    int32_t cur;   // node to visit; -1: leave the instance; <= -2: enter instance -2 - cur
    int sp;
    int32_t aoff;  // -1 in the world, else the instance's shade_base (alpha lanes of its BLAS)
};
template <bool COUNT, bool FAST, bool CHECK>
__device__ __forceinline__ bool anyhit_step_inst(const Trav& c, float tMin, float tMax, AnyState& s,
                                                 const float4* ray_o, const float4* ray_d, uint32_t e, bool& hit,
                                                 TravStats& st) {
    // Leaving and entering an instance share the step with the node visit that
    // follows, so every lane runs the same box test in every step (no step in
    // which some lanes only transform a ray while the others visit nodes).
    if (s.cur == -1) {   // back to the world ray, then the next stack entry
        const float4 o = ray_o[e], d = ray_d[e];
        s.q = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), d.w);
        s.aoff = -1;
        if (s.sp == 0) return true;
        s.cur = stk_pop(c, s.sp);
    }
    if (s.cur <= -2) {   // enter instance -2 - cur: object-space ray, its BLAS root
        const int i = -2 - s.cur;
        if (!stk_push(c, s.sp, -1)) { st.overflow = true; return true; }
        s.q = object_ray(c.inst[i], s.q, c.rcpT);
        s.cur = c.inst[i].root;
        s.aoff = c.inst[i].shade_base;
    }
    const DRay& q = s.q;
    const float4* qn = reinterpret_cast<const float4*>(c.nodes + s.cur);
    const int4 ch = reinterpret_cast<const int4*>(qn)[6];
    const int kinds = node_kinds(qn);
    float tn[4] = {0.f, 0.f, 0.f, 0.f};
    const bool fast = FAST && q.finite;
    const int m = fast ? (c.near_first ? box_test_fast_t(qn, q, tMin, tMax, tn) : box_test_fast(qn, q, tMin, tMax))
                       : box_test(qn, q, tMin, tMax);
    if (COUNT) st.nodes++;
    const int inner = m & kinds_inner(kinds);
    int lm = m & kinds_leaf(kinds);
    // a hit leaf packet with proxy lanes: its instance walks run before the
    // descent (all hit inner children go onto the stack below them), so deferred
    // proxies never pile up along the path -- the stack stays near 4 per level
    const bool proxies = (lm & kinds_proxy(kinds)) != 0;
    bool have_next = false;
    int32_t nxt = 0;
    if (inner) {
        const int top = (fast && c.near_first) ? nearest_slot(inner, tn) : 31 - __builtin_clz((unsigned)inner);
        const int rest = proxies ? inner : inner ^ (1 << top);
        if (rest) {
            if (s.sp + 4 <= kLdsStack) {
                c.lds[s.sp * kWG] = ch.x; s.sp += rest & 1;
                c.lds[s.sp * kWG] = ch.y; s.sp += (rest >> 1) & 1;
                c.lds[s.sp * kWG] = ch.z; s.sp += (rest >> 2) & 1;
                c.lds[s.sp * kWG] = ch.w; s.sp += (rest >> 3) & 1;
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if ((rest >> i) & 1)
                        if (!stk_push(c, s.sp, sel4(ch, i))) { st.overflow = true; return true; }
            }
            if (COUNT && s.sp > st.max_sp) st.max_sp = s.sp;
        }
        nxt = sel4(ch, top);
        have_next = !proxies;
    }
    while (lm) {
        const int sl = __builtin_ctz((unsigned)lm);
        lm &= lm - 1;
        const uint32_t v = ~(uint32_t)sel4(ch, sl);
        const uint32_t leaf = v >> 4;
        const int cnt = (int)(v & 3u) + 1;
        if (COUNT) st.leaves++;
        for (int k = 0; k < cnt; k++) {
            if (v & 4u) {   // proxy lanes (world packets only): deferred instance walks
                const int32_t pm = c.leaves[leaf].prim[k];
                if (pm <= -2) {
                    if (!stk_push(c, s.sp, pm)) { st.overflow = true; return true; }
                    continue;
                }
            }
            float t, a, b;
            bool ok;
            if (CHECK && (v & 8u)) {   // world: alpha / motion blur; BLAS: alpha
                const int32_t pm = c.leaves[leaf].prim[k];
                ok = (s.aoff < 0 && pm >= 0 && c.pflags && (c.pflags[pm] & 1u))
                         ? mb_tri_test(c, pm, q, tMin, tMax, t, a, b)
                         : tri_test(c.leaves[leaf].tri[k], q, tMin, tMax, t, a, b, c.rcpT);
                ok = ok && !alpha_rejects(c, leaf, k, a, b, s.aoff < 0 ? 0 : s.aoff);
            } else {
                ok = tri_test(c.leaves[leaf].tri[k], q, tMin, tMax, t, a, b, c.rcpT);
            }
            if (ok) { hit = true; return true; }
        }
    }
    if (have_next) { s.cur = nxt; return false; }
    if (s.sp == 0) return true;
    s.cur = stk_pop(c, s.sp);
    return false;
}

// FAST (node boxes known finite) uses the hardware min/max slab test for rays
// whose origin and 1/d are finite; any other ray takes the exact loop.  A
// closest hit's packed slot is resolved to the global prim id here.
// An instance hit's id is the instance's hit_base + its BLAS object index.
// XONE: the one-exit walk loop (traverse_impl) -- frame1_kernel, primary_kernel and the
// shadow and adaptive kernels of plain scenes (C4 -6%, A3 -4%); off in the chain engine
// (P4 +21%, R3 +4% with it) and nested BLAS walks.
// OL: the one-latch loop end (traverse_impl) -- the closest-hit walks of primary_kernel and
// the adaptive kernel of plain scenes, and frame1_kernel's unless the host picks the nested
// form (tuning walk_latch 0); any-hit walks and the chain engine keep the nested form
// (round 6 A/B).
template <bool ANY, bool COUNT, bool FAST = false, bool INST = false, bool CHECK = true, bool LN = false,
          bool XONE = false, bool OL = false>
__device__ __forceinline__ bool traverse(const Trav& c, const DRay& r, float tMin, DHit& h, TravStats& st) {
    const bool hit = (FAST && r.finite) ? traverse_impl<ANY, COUNT, true, INST, false, CHECK, LN, XONE, OL>(c, r, tMin, h, st)
                                        : traverse_impl<ANY, COUNT, false, INST, false, CHECK, false, XONE, OL>(c, r, tMin, h, st);
    if (!ANY && hit) {
        h.prim = c.leaves[(uint32_t)h.prim >> 2].prim[h.prim & 3];
        if (INST && h.inst >= 0) h.prim += c.inst[h.inst].hit_base;
    }
    return hit;
}

}  // namespace mrt
