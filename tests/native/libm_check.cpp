// csrc/mrt_libm.h (the device's restatement of glibc's fdlibm atan2f / acosf)
// against the host libm the reference's float overloads call (tests/test_libm.py).
//   libm_check acos LO HI        -- acosf over float bit patterns [LO, HI)
//   libm_check atan2 N SEED      -- atan2f over N seeded pairs (a quarter with
//                                   exponents near each other) plus the specials
//   libm_check sin LO HI / cos LO HI -- sinf / cosf (glibc's FMA build restated)
//   libm_check powx LO HI Y...   -- powf(x, Y) over x bit patterns [LO, HI) for each Y
//   libm_check pow N SEED        -- powf over N seeded pairs plus the specials
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mrt_libm.h"

using namespace mrt;
static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static bool same(float a, float b) { return bits(a) == bits(b) || (isnan(a) && isnan(b)); }

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    uint64_t bad = 0, n = 0;
    if (!strcmp(argv[1], "sin") || !strcmp(argv[1], "cos")) {
        const bool c = argv[1][0] == 'c';
        const uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0);
        for (uint64_t u = lo; u < hi; u++, n++) {
            const float x = u2f((uint32_t)u);
            const float ref = c ? cosf(x) : sinf(x), got = c ? gl_cosf(x) : gl_sinf(x);
            if (!same(ref, got) && bad++ < 5) printf("%s %08x ref %08x got %08x\n", argv[1], (unsigned)u, bits(ref), bits(got));
        }
    } else if (!strcmp(argv[1], "powx")) {
        const uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0);
        for (int a = 4; a < argc; a++) {
            const float y = strtof(argv[a], 0);
            for (uint64_t u = lo; u < hi; u++, n++) {
                const float x = u2f((uint32_t)u);
                if (!same(powf(x, y), gl_powf(x, y)) && bad++ < 5) printf("powf %08x %08x\n", (unsigned)u, bits(y));
            }
        }
    } else if (!strcmp(argv[1], "pow")) {
        const uint64_t N = strtoull(argv[2], 0, 0);
        uint64_t s = strtoull(argv[3], 0, 0) | 1;
        const float sp[] = {0.f, -0.f, 1.f, -1.f, 2.f, -2.f, 0.5f, -3.f, INFINITY, -INFINITY, NAN, 1e-30f, -1e-30f, 1e30f,
                            1.4e-45f, -1.4e-45f, 3.4e38f, 8.f, 32.f, 100.f, -0.5f, 1.0000001f, 0.99999994f};
        for (float y : sp)
            for (float x : sp) {
                n++;
                if (!same(powf(x, y), gl_powf(x, y)) && bad++ < 5) printf("powf %08x %08x\n", bits(x), bits(y));
            }
        for (uint64_t i = 0; i < N; i++, n++) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            uint32_t ux = (uint32_t)s, uy = (uint32_t)(s >> 32);
            if (i % 2 == 1) {   // x in (0, 2), y of moderate size: the non-special path
                ux = (ux & 0x007fffffu) | ((((ux >> 23) & 31u) + 100u) << 23);
                uy = (uy & 0x807fffffu) | ((((uy >> 23) & 15u) + 120u) << 23);
            }
            const float x = u2f(ux), y = u2f(uy);
            if (!same(powf(x, y), gl_powf(x, y)) && bad++ < 5) printf("powf %08x %08x\n", ux, uy);
        }
    } else if (!strcmp(argv[1], "acos")) {
        const uint64_t lo = strtoull(argv[2], 0, 0), hi = strtoull(argv[3], 0, 0);
        for (uint64_t u = lo; u < hi; u++, n++) {
            const float x = u2f((uint32_t)u);
            if (!same(acosf(x), fd_acosf(x)) && bad++ < 5) printf("acosf %08x\n", (unsigned)u);
        }
    } else {
        const uint64_t N = strtoull(argv[2], 0, 0);
        uint64_t s = strtoull(argv[3], 0, 0) | 1;
        const float sp[] = {0.f, -0.f, 1.f, -1.f, INFINITY, -INFINITY, NAN, 1e-30f, -1e-30f, 1e30f, 1.4e-45f, 3.4e38f};
        for (float y : sp)
            for (float x : sp) {
                n++;
                if (!same(atan2f(y, x), fd_atan2f(y, x)) && bad++ < 5) printf("atan2f %08x %08x\n", bits(y), bits(x));
            }
        for (uint64_t i = 0; i < N; i++, n++) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            uint32_t uy = (uint32_t)s, ux = (uint32_t)(s >> 32);
            if (i % 4 == 1) {   // |y / x| within 2^+-16: the polynomial branches
                ux = (ux & 0x807fffffu) | ((((ux >> 23) & 15u) + 120u) << 23);
                uy = (uy & 0x807fffffu) | ((((uy >> 23) & 15u) + 120u) << 23);
            }
            const float y = u2f(uy), x = u2f(ux);
            if (!same(atan2f(y, x), fd_atan2f(y, x)) && bad++ < 5) printf("atan2f %08x %08x\n", uy, ux);
        }
    }
    printf("checked %llu mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad ? 1 : 0;
}
