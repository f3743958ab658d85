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

}  // namespace mrt
