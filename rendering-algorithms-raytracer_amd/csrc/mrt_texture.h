// mrt_texture.h -- lat-long texture lookup and Distribution1D sampling (host and
// device: the dome tables are built on the host with the same lookup the
// device uses for shading).
//
// Texture::getLookup / getLookup3 / getLookupXYZ3 / getPixel (reference
// src/Texture.cpp:43-125) for RGB / HDR float images (RawImage m_rawData, row 0 =
// top scanline of the file, 3 floats per texel), and Distribution1D::sample
// (src/DomeLight.h:31-38).  Same single-precision operations in the same order as
// the reference; atan2 / acos of floats are the float overloads the reference
// calls (atan2f / acosf), restated bit-exactly from glibc's fdlibm code in
// mrt_libm.h.
#pragma once
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "mrt_libm.h"
#include "mrt_math.h"

namespace mrt {

static constexpr float kPI = 3.1415926f;                // src/Miro.h:57
static constexpr float kInvPI = 1.0f / kPI;             // _1_PI, src/Miro.h:59
static constexpr float kTwoPI2 = 2.f * (kPI * kPI);     // _2_PI2, src/Miro.h:58-61

// float -> int as the x86 truncating conversion does for in-range values; NaN
// and out-of-range inputs (reference UB) map to 0 so every read stays in bounds.
MRT_HD int trunc_i32(float f) { return (f > -2147483648.0f && f < 2147483648.0f) ? (int)f : 0; }

// Texture::getPixel (src/Texture.cpp:100-125), "tile" addressing.
MRT_HD v3 tex_pixel(const float* rgb, int W, int H, int x, int y) {
    x = x % W;
    if (x < 0) x += W;
    y = y % H;
    if (y < 0) y += H;
    const float* p = rgb + 3 * ((size_t)y * W + x);
    return mk(p[0], p[1], p[2]);
}

// Texture::getLookup3 (src/Texture.cpp:43-78): wrap to [0,1), flip v, bilinear.
MRT_HD v3 tex_lookup3(const float* rgb, int W, int H, float u, float v) {
    u = u - (float)trunc_i32(u);
    v = v - (float)trunc_i32(v);
    if (u < 0.0f) u = u + 1.0f;
    if (v < 0.0f) v = v + 1.0f;
    v = 1.0f - v;
    const float px = u * (float)W, py = v * (float)H;
    const float x1 = floorf(px), x2 = x1 + 1.0f, dx = px - x1;
    const float y1 = floorf(py), y2 = y1 + 1.0f, dy = py - y1;
    const int ix1 = trunc_i32(x1), ix2 = trunc_i32(x2), iy1 = trunc_i32(y1), iy2 = trunc_i32(y2);
    const v3 p11 = tex_pixel(rgb, W, H, ix1, iy1), p21 = tex_pixel(rgb, W, H, ix2, iy1);
    const v3 p12 = tex_pixel(rgb, W, H, ix1, iy2), p22 = tex_pixel(rgb, W, H, ix2, iy2);
    const float wx = 1.0f - dx, wy = 1.0f - dy;
    const v3 q1 = add(scale(p11, wx), scale(p21, dx));
    const v3 q2 = add(scale(p12, wx), scale(p22, dx));
    return add(scale(q1, wy), scale(q2, dy));
}

#if defined(__HIPCC__)   // float4 (device code; the host builds no material maps)
// Texture::getPixel for every RawImage type (src/Texture.cpp:100-125): GRAYSCALE
// (g, g, g, 1), RGB (r, g, b, 1), RGBA, HDR (r, g, b, the next texel's red -- 0
// past the last texel, where the reference reads beyond the array).
MRT_HD float4 tex_pixel4(const float* d, int W, int H, int type, int x, int y) {
    x = x % W;
    if (x < 0) x += W;
    y = y % H;
    if (y < 0) y += H;
    const size_t i = (size_t)y * W + x;
    if (type == 1) return make_float4(d[i], d[i], d[i], 1.0f);
    if (type == 4) return make_float4(d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]);
    if (type == 3) return make_float4(d[3 * i], d[3 * i + 1], d[3 * i + 2], 1.0f);
    return make_float4(d[3 * i], d[3 * i + 1], d[3 * i + 2], i + 1 < (size_t)W * H ? d[3 * i + 3] : 0.0f);
}

// Texture::getLookup (src/Texture.cpp:43-72) of a material map: wrap to [0,1),
// flip v, bilinear over four channels (getLookupAlpha = its w, :12-41).
MRT_HD float4 tex_lookup4(const float* d, int W, int H, int type, float u, float v) {
    u = u - (float)trunc_i32(u);
    v = v - (float)trunc_i32(v);
    if (u < 0.0f) u = u + 1.0f;
    if (v < 0.0f) v = v + 1.0f;
    v = 1.0f - v;
    const float px = u * (float)W, py = v * (float)H;
    const float x1 = floorf(px), x2 = x1 + 1.0f, dx = px - x1;
    const float y1 = floorf(py), y2 = y1 + 1.0f, dy = py - y1;
    const int ix1 = trunc_i32(x1), ix2 = trunc_i32(x2), iy1 = trunc_i32(y1), iy2 = trunc_i32(y2);
    const float4 p11 = tex_pixel4(d, W, H, type, ix1, iy1), p21 = tex_pixel4(d, W, H, type, ix2, iy1);
    const float4 p12 = tex_pixel4(d, W, H, type, ix1, iy2), p22 = tex_pixel4(d, W, H, type, ix2, iy2);
    const float wx = 1.0f - dx, wy = 1.0f - dy;
    const float4 q1 = make_float4(p11.x * wx + p21.x * dx, p11.y * wx + p21.y * dx, p11.z * wx + p21.z * dx,
                                  p11.w * wx + p21.w * dx);
    const float4 q2 = make_float4(p12.x * wx + p22.x * dx, p12.y * wx + p22.y * dx, p12.z * wx + p22.z * dx,
                                  p12.w * wx + p22.w * dx);
    return make_float4(q1.x * wy + q2.x * dy, q1.y * wy + q2.y * dy, q1.z * wy + q2.z * dy, q1.w * wy + q2.w * dy);
}
#endif

// Texture::getLookupXYZ3 (src/Texture.cpp:80-98): direction -> (u, v).
//   theta = atan2(z, x) + PI; phi = acos(y);   (atan2f / acosf: fd_atan2f / fd_acosf)
//   u = theta * 0.5 * _1_PI   (double arithmetic, rounded to float)
//   v = 1.0 - phi * _1_PI     (float product, double subtraction)
MRT_HD v3 tex_lookup_dir(const float* rgb, int W, int H, float x, float y, float z) {
    const float theta = fd_atan2f(z, x) + kPI;
    const float phi = fd_acosf(y);
    const float u = (float)((double)theta * 0.5 * (double)kInvPI);
    const float v = (float)(1.0 - (double)(phi * kInvPI));
    return tex_lookup3(rgb, W, H, u, v);
}

// Distribution1D::sample (src/DomeLight.h:31-38): std::lower_bound over the n+1
// CDF entries, offset = position - 1.  The offset is clamped to [0, n-1]; it is
// outside only for u <= cdf[0] = 0, which the RNG never produces (reference UB).
MRT_HD float dist_sample(const float* cdf, const float* func, int n, float inv_func_int, float u, float& pdf) {
    int first = 0, len = n + 1;
    while (len > 0) {
        const int half = len >> 1;
        if (cdf[first + half] < u) {
            first += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    int o = first - 1;
    o = o < 0 ? 0 : (o > n - 1 ? n - 1 : o);
    const float c0 = cdf[o], c1 = cdf[o + 1];
    const float du = (u - c0) / (c1 - c0);
    pdf = func[o] * inv_func_int;
    return (float)o + du;
}

// CDF guide table of a Distribution1D with n entries (cdf[0..n]): bucket b(x) =
// clamp((int)(x * n), 0, n - 1); g[b] = the first index i with b(cdf[i]) >= b,
// b = 0..n.  b() is monotone and the CDF non-decreasing, so for any u the
// lower_bound of u lies in [g[b(u)], g[b(u) + 1]] (entries before g[b(u)] have
// a smaller bucket, so are < u; entry g[b(u) + 1] has a larger one, so is > u;
// with no such entry cdf[n] = 1 >= u).  A derived table of the device sampler.
MRT_HD int guide_bucket(float x, int n) {
    const int b = trunc_i32(x * (float)n);
    return b < 0 ? 0 : (b > n - 1 ? n - 1 : b);
}
inline void guide_table(const float* cdf, int n, int32_t* g) {
    int i = 0;
    for (int b = 0; b <= n; b++) {
        while (i <= n && guide_bucket(cdf[i], n) < b) i++;
        g[b] = i;
    }
}

// Distribution1D::sample with the search narrowed by the guide table: the same
// lower_bound position, so the same sample and pdf as dist_sample.
MRT_HD float dist_sample_guided(const float* cdf, const float* func, const int32_t* guide, int n, float inv_func_int,
                                float u, float& pdf) {
    const int b = guide_bucket(u, n);
    const int lo = guide[b], hi = guide[b + 1] < n ? guide[b + 1] : n;
    int first = lo, len = hi - lo + 1;
    while (len > 0) {
        const int half = len >> 1;
        if (cdf[first + half] < u) {
            first += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    int o = first - 1;
    o = o < 0 ? 0 : (o > n - 1 ? n - 1 : o);
    const float c0 = cdf[o], c1 = cdf[o + 1];
    const float du = (u - c0) / (c1 - c0);
    pdf = func[o] * inv_func_int;
    return (float)o + du;
}

}  // namespace mrt
