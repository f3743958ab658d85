// mrt_math.h -- the reference's numeric contract, shared by host and device.
//
// The reference computes in IEEE single precision with x86 SSE approximate
// reciprocals: rcp_nr = 2r - x*r*r (r = RCPSS), rsqrt_nr = (0.5a)(3 - x*a*a)
// (a = RSQRTSS) -- reference src/SSE.h:67-101; dot products use DPPS
// (src/Vector3.h:279-288), SoA dots add as x + (y + z) (src/SSE.h:111-114).
// RCPSS/RSQRTSS are reproduced bit-exactly from 2 x 2048-entry tables captured
// on an Intel host (tools/gen_x86_tables.c, verified over all 2^32 inputs).
// Every entry has exponent 126 and <= 12 significant mantissa bits, so the
// device keeps them as 2 x 4 KB of u16 in LDS: bits = 0x3F000000 | (e << 11).
//
// Build with -ffp-contract=off: every expression below is a sequence of
// individually rounded IEEE ops in the reference's order (no FMA contraction).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MRT_HD __host__ __device__ __forceinline__
#else
#define MRT_HD static inline
#endif

namespace mrt {

MRT_HD uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }
MRT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }

// Device: an empty asm on a value keeps the load that produced it on the
// straight-line path (otherwise the compiler sinks the table load into a
// divergent branch around the rare NaN/inf inputs).
#ifdef __HIP_DEVICE_COMPILE__
#define MRT_OPAQUE(v) asm volatile("" : "+v"(v))
#else
#define MRT_OPAQUE(v) (void)0
#endif

// 12-bit packed table entry -> float bits in [0.5, 1)
MRT_HD uint32_t tbl_bits(uint16_t e) { return 0x3F000000u | ((uint32_t)e << 11); }

// RCPSS emulation; T = 2048-entry packed rcp table; the table index is in range for
// every input.  On |x| bits a = u & 0x7FFFFFFF: a normal x (exponent e in 1..252)
// gives exponent 253 - e and the entry's 12 mantissa bits; e >= 253 (and inf) ->
// +-0; zero / denormal -> +-inf; NaN -> quiet NaN.  (Equal to the table emulation on
// all 2^32 float bit patterns on the CPU, tests/native/rcp_sweep.c at stride 1, every
// 61st in the CPU suite and every 257th on the GPU, tests/test_numerics.py; the tables
// themselves are checked against the live instructions on all 2^32 inputs,
// tools/gen_x86_tables.c.)
// The exponent classes outside 1..252 (zero / denormal, e >= 253, inf, NaN): the
// select chain over the normal-path value r, which it leaves as is for a normal x.
MRT_HD uint32_t x86_rcp_special(uint32_t u, uint32_t r) {
    const uint32_t a = u & 0x7FFFFFFFu, s = u & 0x80000000u;
    r = a >= 0x7E800000u ? s : r;                                  // e >= 253: below FLT_MIN -> +-0; inf -> +-0
    r = a < 0x00800000u ? (s | 0x7F800000u) : r;                  // zero / denormal -> +-inf
    r = a > 0x7F800000u ? (u | 0x00400000u) : r;                  // NaN -> quiet
    return r;
}
// Normal x: ((253 << 23 | entry << 11) - (e << 23)) | sign (no borrow reaches the sign).
// The device takes the select chain only when some lane of the wave needs it (one
// compare per test; a triangle test's det is almost never outside the normal range),
// instead of three compare + select pairs, each select waiting on its compare, per
// triangle test (round 6: -8 VALU instructions and -3 wait states per test).
MRT_HD float x86_rcp(float x, const uint16_t* T) {
    const uint32_t u = f2u(x), ex = u & 0x7F800000u;
    uint32_t t = T[(u >> 12) & 0x7FFu];
    MRT_OPAQUE(t);
    uint32_t r = ((0x7E800000u | (t << 11)) - ex) | (u & 0x80000000u);
    const bool special = ex - 0x00800000u >= 0x7E000000u;        // e == 0 or e >= 253
#ifdef __HIP_DEVICE_COMPILE__
    if (__ballot(special) != 0) {
        r = x86_rcp_special(u, r);
        asm volatile("; mrt: rcp special" : "+v"(r));   // keeps the chain in its branch
    }
#else
    if (special) r = x86_rcp_special(u, r);
#endif
    return u2f(r);
}

// RSQRTSS emulation; T = 2048-entry packed rsqrt table ([odd exponent][10 bits]).
MRT_HD float x86_rsqrt(float x, const uint16_t* T) {
    const uint32_t u = f2u(x), s = u & 0x80000000u, e = (u >> 23) & 0xFFu, m = u & 0x7FFFFFu;
    const int E = (int)e - 127, odd = E & 1, k = (E - odd) >> 1;    // E - odd is even: exact halving
    uint32_t t = tbl_bits(T[(odd << 10) | (m >> 13)]);
    MRT_OPAQUE(t);
    uint32_t r = ((uint32_t)(126 - k) << 23) | (t & 0x7FFFFFu);
    r = s ? 0xFFC00000u : r;                                       // negative -> NaN
    r = e == 0u ? (s | 0x7F800000u) : r;                          // +-0 / denormal -> +-inf
    MRT_OPAQUE(r);
    r = e == 0xFFu ? (m ? (u | 0x00400000u) : (s ? 0xFFC00000u : 0u)) : r;
    return u2f(r);
}

// recipss / recipps (src/SSE.h:67-86)
MRT_HD float rcp_nr(float x, const uint16_t* T) {
    float r = x86_rcp(x, T);
    return (2.0f * r) - (x * (r * r));
}
// fastrsqrtss / fastrsqrtps (src/SSE.h:88-101)
MRT_HD float rsqrt_nr(float x, const uint16_t* T) {
    float a = x86_rsqrt(x, T);
    float muls = (x * a) * a;
    return (0.5f * a) * (3.0f - muls);
}

MRT_HD float sse_min(float a, float b) { return a < b ? a : b; }  // MINPS
MRT_HD float sse_max(float a, float b) { return a > b ? a : b; }  // MAXPS
MRT_HD float std_min(float a, float b) { return b < a ? b : a; }  // std::min
MRT_HD float std_max(float a, float b) { return a < b ? b : a; }  // std::max

struct v3 { float x, y, z; };
MRT_HD v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
MRT_HD v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
MRT_HD v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
MRT_HD v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
MRT_HD v3 scale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
MRT_HD v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
// DPPS imm 0x71: (x*x' + y*y') + (z*z' + 0)
MRT_HD float dot(v3 a, v3 b) {
    float p0 = a.x * b.x, p1 = a.y * b.y, p2 = a.z * b.z;
    return (p0 + p1) + (p2 + 0.0f);
}
MRT_HD v3 cross(v3 a, v3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
MRT_HD v3 normalized(v3 a, const uint16_t* T_rsqrt) { return scale(a, rsqrt_nr(dot(a, a), T_rsqrt)); }

// 32768-entry gamma LUT lookup index (Image::Map, src/Image.cpp:71-76); negative /
// NaN (UB in the reference's unsigned-short cast) -> 0.
MRT_HD uint32_t map_index(float r) {
    float rMap = 32768.0f * r;
    if (rMap > 32768.0f) return 32768u;
    if (!(rMap >= 0.0f)) return 0u;
    return (uint32_t)(uint16_t)(int)rMap;
}

// Counter-based RNG standing in for Scene::getRand's global MT pool
// (src/Scene.cpp:30-47); same float mapping ((float)u + 0.5) * 2^-32 in double.
MRT_HD uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
MRT_HD float rng(uint32_t pixel, uint32_t sample, uint32_t dim, uint32_t seed) {
    uint32_t h = mix32(seed ^ 0x9E3779B9u);
    h = mix32(h ^ pixel);
    h = mix32(h ^ (sample * 0x85EBCA6Bu));
    h = mix32(h ^ (dim * 0xC2B2AE35u));
    return (float)(((double)(float)h + 0.5) * (1.0 / 4294967296.0));
}

}  // namespace mrt
