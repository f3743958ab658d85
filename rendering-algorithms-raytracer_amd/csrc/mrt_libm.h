// mrt_libm.h -- the float libm calls of the reference's lat-long lookups and
// Fresnel term, restated for host and device.
//
// The reference calls atan2 / acos on floats (src/Texture.cpp:82-83,92-93) and
// acosf (src/Material.h:51).  With `using namespace std` (src/Material.h:8) these
// resolve to the float overloads: atan2f / acosf of the C library.  Third-party
// dependency: glibc 2.35 (Ubuntu 2.35-0ubuntu3, the image's libm), whose
// sysdeps/ieee754/flt-32 e_acosf.c, e_atan2f.c and s_atanf.c are Sun's fdlibm
// single-precision algorithms (plain float arithmetic; no FMA variant on x86-64).
// Below is that published algorithm, op for op, so the device returns the bits the
// reference's own calls return on this platform.  Pinned by tests/test_libm.py:
// acosf over all 2^32 inputs and atan2f over the special cases and 2^26 seeded
// pairs, bit-identical to the host's libm.
//
// Requires -ffp-contract=off (each a*b+c is two roundings, as in the C source),
// correctly rounded division and sqrtf, and IEEE denormals (the device build's
// defaults; see mrt_math.h).
#pragma once
#include "mrt_math.h"

namespace mrt {

// __ieee754_acosf (fdlibm e_acosf.c)
MRT_HD float fd_acosf(float x) {
    const float one = 1.0f, pi = u2f(0x40490fdau), pio2_hi = u2f(0x3fc90fdau), pio2_lo = u2f(0x33a22168u);
    const float pS0 = u2f(0x3e2aaaabu), pS1 = u2f(0xbea6b090u), pS2 = u2f(0x3e4e0aa8u), pS3 = u2f(0xbd241146u),
                pS4 = u2f(0x3a4f7f04u), pS5 = u2f(0x3811ef08u);
    const float qS1 = u2f(0xc019d139u), qS2 = u2f(0x4001572du), qS3 = u2f(0xbf303361u), qS4 = u2f(0x3d9dc62eu);
    const int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) {   // |x| == 1
        if (hx > 0) return 0.0f;
        return pi + 2.0f * pio2_lo;
    }
    if (ix > 0x3f800000) return (x - x) / (x - x);   // |x| > 1 (or NaN): NaN
    if (ix < 0x3f000000) {   // |x| < 0.5
        if (ix <= 0x32800000) return pio2_hi + pio2_lo;   // |x| < 2^-26
        const float z = x * x;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float r = p / q;
        return pio2_hi - (x - (pio2_lo - x * r));
    }
    if (hx < 0) {   // x < -0.5
        const float z = (one + x) * 0.5f;
        const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
        const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
        const float s = __builtin_sqrtf(z);
        const float r = p / q;
        const float w = r * s - pio2_lo;
        return pi - 2.0f * (s + w);
    }
    // x > 0.5
    const float z = (one - x) * 0.5f;
    const float s = __builtin_sqrtf(z);
    const float df = u2f(f2u(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const float q = one + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    const float r = p / q;
    const float w = r * s + c;
    return 2.0f * (df + w);
}

// __atanf (fdlibm s_atanf.c)
MRT_HD float fd_atanf(float x) {
    const float atanhi[4] = {u2f(0x3eed6338u), u2f(0x3f490fdau), u2f(0x3f7b985eu), u2f(0x3fc90fdau)};
    const float atanlo[4] = {u2f(0x31ac3769u), u2f(0x33222168u), u2f(0x33140fb4u), u2f(0x33a22168u)};
    const float aT0 = u2f(0x3eaaaaabu), aT1 = u2f(0xbe4ccccdu), aT2 = u2f(0x3e124925u), aT3 = u2f(0xbde38e38u),
                aT4 = u2f(0x3dba2e6eu), aT5 = u2f(0xbd9d8795u), aT6 = u2f(0x3d886b35u), aT7 = u2f(0xbd6ef16bu),
                aT8 = u2f(0x3d4bda59u), aT9 = u2f(0xbd15a221u), aT10 = u2f(0x3c8569d7u);
    const float one = 1.0f;
    const int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {   // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;   // NaN
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {   // |x| < 0.4375
        if (ix < 0x31000000) return x;   // |x| < 2^-29
        id = -1;
    } else {
        x = __builtin_fabsf(x);
        if (ix < 0x3f980000) {   // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); }   // 7/16 <= |x| < 11/16
            else { id = 1; x = (x - one) / (x + one); }                              // 11/16 <= |x| < 19/16
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); }   // |x| < 2.4375
            else { id = 3; x = -1.0f / x; }                                        // 2.4375 <= |x| < 2^25
        }
    }
    const float z = x * x, w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

// __ieee754_atan2f (fdlibm e_atan2f.c)
MRT_HD float fd_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = u2f(0x3f490fdbu), pi_o_2 = u2f(0x3fc90fdbu), pi = u2f(0x40490fdbu),
                pi_lo = u2f(0xb3bbbd2eu);
    const int32_t hx = (int32_t)f2u(x), ix = hx & 0x7fffffff;
    const int32_t hy = (int32_t)f2u(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;   // NaN
    if (hx == 0x3f800000) return fd_atanf(y);               // x == 1
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      // 2 * sign(x) + sign(y)
    if (iy == 0) {   // y == 0
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;   // x == 0
    if (ix == 0x7f800000) {   // x infinite
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;   // y infinite
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 26) z = pi_o_2 + 0.5f * pi_lo;         // |y / x| > 2^26
    else if (hx < 0 && k < -26) z = 0.0f;          // |y| / x < -2^26
    else z = fd_atanf(__builtin_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// ---- sinf / cosf: glibc 2.35 sysdeps/ieee754/flt-32 s_sinf.c, s_cosf.c, sincosf.h and
// sincosf_data.c (the Arm optimized-routines algorithm: double-precision evaluation, one
// rounding to float at the end).  The reference calls them in Fresnel's sin(acosf)
// (src/Material.h:51) and the cosine sampler's cos / sin (src/Material.cpp:41).  On
// x86-64 glibc runs the variant built with -mfma (__sinf_fma / __cosf_fma, selected at
// run time on every FMA-capable CPU), where GCC contracts each a + b * c of the C
// source into one fused multiply-add; so does this restatement, with fma() (host libm,
// correctly rounded; device v_fma_f64).  The constants are sincosf_data.c's
// (__sincosf_table, __inv_pio4), checked against the image's libm.so.6 bytes.
// Pinned by tests/test_libm.py: every one of the 2^32 inputs of each, bit-identical to
// the host's sinf / cosf.
MRT_HD uint32_t gl_abstop12(float x) { return (f2u(x) >> 20) & 0x7ffu; }

// sinf_poly: the sine (n even) or cosine (n odd) polynomial of x (x2 = x * x); `neg`
// selects __sincosf_table[1], whose cosine coefficients are negated
MRT_HD float gl_sinf_poly(double x, double x2, bool neg, int n) {
    const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7, s3c = -0x1.994eb3774cf24p-13;
    const double sg = neg ? -1.0 : 1.0;
    if ((n & 1) == 0) {
        const double x3 = x * x2;
        const double s1 = fma(x2, s3c, s2c);
        const double x7 = x3 * x2;
        const double s = fma(x3, s1c, x);
        return (float)fma(x7, s1, s);
    }
    const double c0 = sg * 0x1p0, c1c = sg * -0x1.ffffffd0c621cp-2, c2c = sg * 0x1.55553e1068f19p-5,
                 c3c = sg * -0x1.6c087e89a359dp-10, c4c = sg * 0x1.99343027bf8c3p-16;
    const double x4 = x2 * x2;
    const double c2 = fma(x2, c4c, c3c);
    const double c1 = fma(x2, c1c, c0);
    const double x6 = x4 * x2;
    const double c = fma(x4, c2c, c1);
    return (float)fma(x6, c2, c);
}

// reduce_fast (no TOINT_INTRINSICS on x86-64): hpi_inv prescaled by 2^24, the quadrant
// in bits 24..31 of the truncated product; |x| < 120
MRT_HD double gl_reduce_fast(double x, int& n) {
    const double r = x * 0x1.45f306dc9c883p+23;
    n = ((int32_t)r + 0x800000) >> 24;
    return fma(-(double)n, 0x1.921fb54442d18p+0, x);   // x - n * hpi, contracted
}

// __inv_pio4[i]: bytes i - 3 .. i of 4 / pi's fraction (0xA2F9836E4E441529FC2757D1...),
// big-endian, zeros before the first
MRT_HD uint32_t gl_inv_pio4(int i) {
    const uint64_t w[3] = {0xA2F9836E4E441529ull, 0xFC2757D1F534DDC0ull, 0xDB6295993C439041ull};
    uint32_t v = 0;
    for (int k = i - 3; k <= i; k++) v = (v << 8) | (k < 0 ? 0u : (uint32_t)(w[k >> 3] >> (56 - 8 * (k & 7))) & 0xffu);
    return v;
}

// reduce_large: |x| >= 120 by a 32 x 96-bit product with 4 / pi (integer arithmetic)
MRT_HD double gl_reduce_large(uint32_t xi, int& np) {
    const int a = (int)((xi >> 26) & 15u);
    const int shift = (int)((xi >> 23) & 7u);
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * gl_inv_pio4(a));   // a 32-bit product, as in the C source
    const uint64_t res1 = (uint64_t)xi * gl_inv_pio4(a + 4);
    const uint64_t res2 = (uint64_t)xi * gl_inv_pio4(a + 8);
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    np = (int)n;
    return x * 0x1.921fb54442d18p-62;   // pi63
}

MRT_HD double gl_quadrant_sign(int q) { return ((q & 3) == 1 || (q & 3) == 2) ? -1.0 : 1.0; }

// sinf (s_sinf.c); cos = true: cosf (s_cosf.c)
MRT_HD float gl_sincosf(float y, bool cos) {
    double x = y;
    const uint32_t top = gl_abstop12(y);
    if (top < gl_abstop12(0x1.921fb6p-1f)) {   // |y| < pi / 4
        const double x2 = x * x;
        if (top < gl_abstop12(0x1p-12f)) return cos ? 1.0f : y;
        return gl_sinf_poly(x, x2, false, cos ? 1 : 0);
    }
    if (top < gl_abstop12(120.0f)) {
        int n;
        x = gl_reduce_fast(x, n);
        const double s = gl_quadrant_sign(n);
        return gl_sinf_poly(x * s, x * x, (n & 2) != 0, cos ? n ^ 1 : n);
    }
    if (top < gl_abstop12(__builtin_inff())) {
        const uint32_t xi = f2u(y);
        const int sign = (int)(xi >> 31);
        int n;
        x = gl_reduce_large(xi, n);
        const double s = gl_quadrant_sign(n + sign);
        return gl_sinf_poly(x * s, x * x, ((n + sign) & 2) != 0, cos ? n ^ 1 : n);
    }
    return (y - y) / (y - y);   // __math_invalidf: inf or NaN -> NaN
}
MRT_HD float gl_sinf(float y) { return gl_sincosf(y, false); }
MRT_HD float gl_cosf(float y) { return gl_sincosf(y, true); }

// ---- powf: glibc 2.35 sysdeps/ieee754/flt-32 e_powf.c, powf_log2_data.c and exp2f_data.c
// (Arm optimized-routines: log2 of x from a 16-entry table and a degree-5 polynomial,
// y * log2(x), then exp2 from a 32-entry table and a cubic), the x86-64 FMA build
// (__powf_fma): each a * b + c contracted into one fma.  The reference calls it in
// Blinn::shade's pow(lightSpec, localSpecExp) (src/Blinn.cpp:219).  Constants from the
// image's libm.so.6 (__powf_log2_data, __exp2f_data; no TOINT_INTRINSICS on x86-64, so
// POWF_SCALE = 1).  Pinned by tests/test_libm.py against the host's powf.
static constexpr double kPowfInvc[16] = {0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010b0p+0, 0x1.3c995b0b80385p+0, 0x1.30d190c8864a5p+0, 0x1.25e227b0b8ea0p+0, 0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0, 0x1.0953f419900a7p+0, 0x1.0000000000000p+0, 0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aa0p-1, 0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
static constexpr double kPowfLogc[16] = {-0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2, -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7af0p-3, -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4, -0x1.a6f9db6475fcep-5, 0x0.0p+0, 0x1.338ca9f24f53dp-4, 0x1.476a9543891bap-3, 0x1.e840b4ac4e4d2p-3, 0x1.40645f0c6651cp-2, 0x1.88e9c2c1b9ff8p-2, 0x1.ce0a44eb17bccp-2};
static constexpr double kPowfPoly[5] = {0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1, 0x1.71547652ab82bp+0};
static constexpr uint64_t kExp2fTab[32] = {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull, 0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull, 0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull, 0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull, 0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull, 0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull, 0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull, 0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

MRT_HD bool gl_zeroinfnan(uint32_t i) { return 2 * i - 1 >= 2u * 0x7f800000u - 1; }
MRT_HD bool gl_issignaling(uint32_t i) { return 2 * (i ^ 0x00400000u) > 2u * 0x7fc00000u; }
// 0: y is not an integer, 1: an odd integer, 2: an even integer
MRT_HD int gl_checkint(uint32_t iy) {
    const int e = (int)(iy >> 23 & 0xffu);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
MRT_HD double gl_log2_inline(uint32_t ix) {
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;
    const double invc = kPowfInvc[i], logc = kPowfLogc[i];
    const double z = (double)u2f(iz);
    const double r = fma(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double y = fma(kPowfPoly[0], r, kPowfPoly[1]);
    const double p = fma(kPowfPoly[2], r, kPowfPoly[3]);
    const double r4 = r2 * r2;
    double q = fma(kPowfPoly[4], r, y0);
    q = fma(p, r2, q);
    y = fma(y, r4, q);
    return y;
}
MRT_HD double gl_exp2_inline(double xd, uint32_t sign_bias) {
    const double shift = 0x1.8p+47;   // shift_scaled = 0x1.8p52 / 32
    double kd = xd + shift;
    const uint64_t ki = __builtin_bit_cast(uint64_t, kd);
    kd -= shift;
    const double r = xd - kd;
    uint64_t t = kExp2fTab[ki % 32];
    const uint64_t ski = ki + sign_bias;
    t += ski << (52 - 5);
    const double s = __builtin_bit_cast(double, t);
    const double z = fma(0x1.c6af84b912394p-5, r, 0x1.ebfce50fac4f3p-3);
    const double r2 = r * r;
    double y = fma(0x1.62e42ff0c52d6p-1, r, 1.0);
    y = fma(z, r2, y);
    return y * s;
}
MRT_HD float gl_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = f2u(x);
    const uint32_t iy = f2u(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || gl_zeroinfnan(iy)) {
        // x < 0x1p-126, inf or NaN, or y zero, inf or NaN
        if (gl_zeroinfnan(iy)) {
            if (2 * iy == 0) return gl_issignaling(ix) ? x + y : 1.0f;
            if (ix == 0x3f800000u) return gl_issignaling(iy) ? x + y : 1.0f;
            if (2 * ix > 2u * 0x7f800000u || 2 * iy > 2u * 0x7f800000u) return x + y;
            if (2 * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2 * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;   // |x| < 1 && y == inf, or |x| > 1 && y == -inf
            return y * y;
        }
        if (gl_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && gl_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1 / x2 : x2;
        }
        if (ix & 0x80000000u) {   // finite x < 0
            const int yint = gl_checkint(iy);
            if (yint == 0) return (x - x) / (x - x);   // __math_invalidf
            if (yint == 1) sign_bias = 1u << (5 + 11);
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {   // subnormal x: normalised, its exponent negative
            ix = f2u(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = gl_log2_inline(ix);
    const double ylogx = (double)y * logx;
    if (((__builtin_bit_cast(uint64_t, ylogx) >> 47) & 0xffffu) >= (__builtin_bit_cast(uint64_t, 126.0) >> 47)) {
        // |y * log(x)| >= 126: __math_oflowf / __math_uflowf (0x1p97f squared, 0x1p-95f squared)
        if (ylogx > 0x1.fffffffd1d571p+6) { const float v = sign_bias ? -0x1p97f : 0x1p97f; return v * 0x1p97f; }
        if (ylogx <= -150.0) { const float v = sign_bias ? -0x1p-95f : 0x1p-95f; return v * 0x1p-95f; }
    }
    return (float)gl_exp2_inline(ylogx, sign_bias);
}

}  // namespace mrt
