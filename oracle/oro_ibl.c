/*
 * oro_ibl.c -- TEST INFRASTRUCTURE ONLY (see mrt_oracle.h for the contract).
 *
 * CPU restatement of the image-based-lighting inputs of the reference hot path:
 *   HDRLoader::load / decrunch / oldDecrunch / workOnRGBE  src/hdrloader.cpp:29-190
 *   Texture::getLookup3 / getLookupXYZ3 / getPixel           src/Texture.cpp:43-125
 *   Distribution1D                                            src/DomeLight.h:10-42
 *   DomeLight::setTexture                                     src/DomeLight.cpp:8-78
 *
 * Deviations, all where the reference has undefined behaviour: a header or
 * resolution line longer than its 200-byte buffers, EOF inside the header, a
 * resolution line without both sizes, an RLE run past the end of a scanline and
 * an old-style run with no previous pixel fail the load (negative return)
 * instead of corrupting memory; rows after a short read are zero (uninitialised
 * in the reference); float -> int conversions of NaN / out-of-range values give
 * 0.  libm: the dome tables call sinf / cosf as the reference does (the
 * product's host code calls the same glibc functions); atan2 / acos of the
 * lookups are evaluated in double and rounded once (the reference calls the
 * float overloads of the MSVC CRT: parity with those is unpinned).
 */
#include "oro_ibl.h"

int oro_libm_float = 1;

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const float PI_F = 3.1415926f;            /* src/Miro.h:57 */
static const float INV_PI = 1.0f / 3.1415926f;   /* _1_PI, src/Miro.h:59 */

/* ---------------------------------------------------------------- HDR */
typedef unsigned char rgbe_t[4];

/* oldDecrunch, src/hdrloader.cpp:161-190, filling row[pos ..].
 * 1 = ok, 0 = EOF (the reference's false), -1 = rejected (reference UB). */
static int old_decrunch(rgbe_t* row, int pos, int len, FILE* f) {
    int rshift = 0;
    while (len > 0) {
        row[pos][0] = (unsigned char)fgetc(f);
        row[pos][1] = (unsigned char)fgetc(f);
        row[pos][2] = (unsigned char)fgetc(f);
        row[pos][3] = (unsigned char)fgetc(f);
        if (feof(f)) return 0;
        if (row[pos][0] == 1 && row[pos][1] == 1 && row[pos][2] == 1) {
            if (pos == 0 || rshift >= 32) return -1;          /* reads row[-1] / shift UB */
            long long n = (long long)row[pos][3] << rshift;
            if (n > len) return -1;                            /* run past the scanline */
            for (long long i = n; i > 0; i--) {
                memcpy(row[pos], row[pos - 1], 4);
                pos++;
                len--;
            }
            rshift += 8;
        } else {
            pos++;
            len--;
            rshift = 0;
        }
    }
    return 1;
}

/* decrunch, src/hdrloader.cpp:118-159 (same return convention) */
static int decrunch(rgbe_t* row, int len, FILE* f) {
    if (len < 8 || len > 0x7fff) return old_decrunch(row, 0, len, f);
    int i = fgetc(f);
    if (i != 2) {
        fseek(f, -1, SEEK_CUR);
        return old_decrunch(row, 0, len, f);
    }
    row[0][1] = (unsigned char)fgetc(f);
    row[0][2] = (unsigned char)fgetc(f);
    i = fgetc(f);
    if (row[0][1] != 2 || (row[0][2] & 128)) {
        row[0][0] = 2;
        row[0][3] = (unsigned char)i;
        return old_decrunch(row, 1, len - 1, f);
    }
    for (i = 0; i < 4; i++) {
        int j = 0;
        while (j < len) {
            unsigned char code = (unsigned char)fgetc(f);
            if (code > 128) {
                code &= 127;
                unsigned char val = (unsigned char)fgetc(f);
                if (j + code > len) return -1;
                while (code--) row[j++][i] = val;
            } else {
                if (j + code > len) return -1;
                while (code--) row[j++][i] = (unsigned char)fgetc(f);
            }
        }
    }
    return feof(f) ? 0 : 1;
}

/* convertComponent, src/hdrloader.cpp:99-104 */
static float convert_component(int expo, int val) {
    float v = val / 256.0f;
    float d = (float)pow(2.0, (double)expo);
    return v * d;
}

/* HDRLoader::load, src/hdrloader.cpp:29-97.  rgb == NULL: header only. */
int ibl_hdr_read(const char* path, float* rgb, int cap_w, int cap_h, int* w_out, int* h_out) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    char str[10];
    if (fread(str, 10, 1, f) != 1 || memcmp(str, "#?RADIANCE", 10)) { fclose(f); return -2; }
    fseek(f, 1, SEEK_CUR);
    int n = 0, ch;
    char c = 0, oldc;
    for (;;) {                                   /* header up to "\n\n", cmd[200] */
        oldc = c;
        ch = fgetc(f);
        if (ch == EOF) { fclose(f); return -2; }
        c = (char)ch;
        if (c == 0xa && oldc == 0xa) break;
        if (n >= 200) { fclose(f); return -2; }
        n++;
    }
    char reso[201];
    n = 0;
    for (;;) {                                   /* resolution line, reso[200] */
        ch = fgetc(f);
        if (ch == EOF || n >= 200) { fclose(f); return -2; }
        reso[n++] = (char)ch;
        if (ch == 0xa) break;
    }
    reso[n] = 0;
    int w = 0, h = 0;
    if (sscanf(reso, "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0 || (long long)w * h > (1LL << 28)) {
        fclose(f);
        return -2;
    }
    *w_out = w;
    *h_out = h;
    if (!rgb) { fclose(f); return 0; }
    if (cap_w != w || cap_h != h) { fclose(f); return -3; }
    memset(rgb, 0, sizeof(float) * 3 * (size_t)w * h);
    rgbe_t* row = (rgbe_t*)malloc(sizeof(rgbe_t) * (size_t)w);
    float* cols = rgb;
    int rc = 0;
    for (int y = h - 1; y >= 0; y--) {           /* scanlines in file order, top first */
        int r = decrunch(row, w, f);
        if (r < 0) { rc = -4; break; }
        if (r == 0) break;
        for (int x = 0; x < w; x++) {            /* workOnRGBE */
            int expo = row[x][3] - 128;
            cols[0] = convert_component(expo, row[x][0]);
            cols[1] = convert_component(expo, row[x][1]);
            cols[2] = convert_component(expo, row[x][2]);
            cols += 3;
        }
    }
    free(row);
    fclose(f);
    return rc;
}

/* ---------------------------------------------------------------- texture */
static int trunc_i32(float v) { return (v > -2147483648.0f && v < 2147483648.0f) ? (int)v : 0; }

/* Texture::getPixel, src/Texture.cpp:100-125 (tiled addressing) */
static const float* texel(const ibl_image* t, int x, int y) {
    x = x % t->W;
    if (x < 0) x += t->W;
    y = y % t->H;
    if (y < 0) y += t->H;
    return t->rgb + 3 * ((size_t)y * t->W + x);
}

/* Texture::getLookup + getLookup3, src/Texture.cpp:43-78 */
void ibl_lookup3(const ibl_image* t, float u, float v, float out[3]) {
    u = u - (float)trunc_i32(u);
    v = v - (float)trunc_i32(v);
    if (u < 0.0f) u = u + 1.0f;
    if (v < 0.0f) v = v + 1.0f;
    v = 1.0f - v;                                /* textures start with v = 0 at the top */
    float px = u * (float)t->W, py = v * (float)t->H;
    float x1 = floorf(px), x2 = x1 + 1.0f, dx = px - x1;
    float y1 = floorf(py), y2 = y1 + 1.0f, dy = py - y1;
    const float* p11 = texel(t, trunc_i32(x1), trunc_i32(y1));
    const float* p21 = texel(t, trunc_i32(x2), trunc_i32(y1));
    const float* p12 = texel(t, trunc_i32(x1), trunc_i32(y2));
    const float* p22 = texel(t, trunc_i32(x2), trunc_i32(y2));
    for (int k = 0; k < 3; k++) {
        float q1 = p11[k] * (1.0f - dx) + p21[k] * dx;
        float q2 = p12[k] * (1.0f - dx) + p22[k] * dx;
        out[k] = q1 * (1.0f - dy) + q2 * dy;
    }
}

/* Texture::getLookupXYZ3, src/Texture.cpp:80-98: atan2(z, x) and acos(y) of
 * floats (atan2f / acosf, oro_libm_float); u = theta * 0.5 * _1_PI and
 * v = 1.0 - phi * _1_PI are evaluated in double (double literals) and rounded. */
void ibl_lookup_dir(const ibl_image* t, float x, float y, float z, float out[3]) {
    float theta = oro_atan2(z, x) + PI_F;
    float phi = oro_acos(y);
    float u = (float)((double)theta * 0.5 * (double)INV_PI);
    float v = (float)(1.0 - (double)(phi * INV_PI));
    ibl_lookup3(t, u, v, out);
}

/* ---------------------------------------------------------------- Distribution1D */
/* Distribution1D(f, n) + computeStep1dCDF, src/DomeLight.h:11-30 */
static void dist_init(ibl_dist* d, const float* f, int n) {
    d->func = (float*)malloc(sizeof(float) * n);
    d->cdf = (float*)malloc(sizeof(float) * (n + 1));
    d->count = n;
    memcpy(d->func, f, sizeof(float) * n);
    d->cdf[0] = 0.f;
    for (int i = 1; i < n + 1; ++i) d->cdf[i] = d->cdf[i - 1] + d->func[i - 1] / (float)n;
    d->funcInt = d->cdf[n];
    for (int i = 1; i < n + 1; ++i) d->cdf[i] /= d->funcInt;
    d->invFuncInt = 1.f / d->funcInt;
    d->invCount = 1.f / (float)n;
}

/* Distribution1D::sample, src/DomeLight.h:31-38: std::lower_bound over the
 * n + 1 CDF values; the offset is clamped to [0, n-1] (outside only for
 * u <= 0, reference UB). */
float ibl_dist_sample(const ibl_dist* d, float u, float* pdf) {
    int first = 0, len = d->count + 1;
    while (len > 0) {
        int half = len >> 1;
        if (d->cdf[first + half] < u) {
            first += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    int o = first - 1;
    if (o < 0) o = 0;
    if (o > d->count - 1) o = d->count - 1;
    u = (u - d->cdf[o]) / (d->cdf[o + 1] - d->cdf[o]);
    *pdf = d->func[o] * d->invFuncInt;
    return (float)o + u;
}

/* DomeLight::setTexture, src/DomeLight.cpp:8-78.  Returns -1 when the map has
 * no positive radiance (the reference would then divide by a zero integral
 * and index its tables with NaN). */
int ibl_dome_init(ibl_dome* d, const ibl_image* t) {
    memset(d, 0, sizeof *d);
    int nu = t->W, nv = t->H;
    d->nu = nu;
    d->nv = nv;
    float* img = (float*)malloc(sizeof(float) * (size_t)nu * nv);
    for (int u = 0; u < nu; ++u) {
        float up = (float)u / (float)nu;
        for (int v = 0; v < nv; ++v) {
            float vp = (float)v / (float)nv, L[3];
            ibl_lookup3(t, up, vp, L);
            img[v + (size_t)u * nv] = ((L[0] + L[1]) + L[2]) * 0.333333f;   /* Vector3::average */
        }
    }
    int mx = nu > nv ? nu : nv;
    float* func = (float*)malloc(sizeof(float) * mx);
    float* sinVals = (float*)malloc(sizeof(float) * nv);
    for (int i = 0; i < nv; ++i) sinVals[i] = sinf(PI_F * (float)(i + .5) / (float)nv);
    d->v = (ibl_dist*)calloc((size_t)nu, sizeof(ibl_dist));
    for (int u = 0; u < nu; ++u) {
        for (int v = 0; v < nv; ++v) func[v] = img[(size_t)u * nv + v] * sinVals[v];
        dist_init(&d->v[u], func, nv);
    }
    for (int u = 0; u < nu; ++u) func[u] = d->v[u].funcInt;
    dist_init(&d->u, func, nu);
    d->cosU = (float*)malloc(sizeof(float) * (nu + 1));
    d->sinU = (float*)malloc(sizeof(float) * (nu + 1));
    d->cosV = (float*)malloc(sizeof(float) * (nv + 1));
    d->sinV = (float*)malloc(sizeof(float) * (nv + 1));
    float invCount = 1.f / (float)nu;
    for (int i = 0; i < nu + 1; ++i) d->cosU[i] = cosf((float)i * invCount * 2.f * PI_F);
    for (int i = 0; i < nu + 1; ++i) d->sinU[i] = sinf((float)i * invCount * 2.f * PI_F);
    invCount = 1.f / (float)nv;
    for (int i = 0; i < nv + 1; ++i) d->cosV[i] = cosf((float)i * invCount * PI_F);
    for (int i = 0; i < nv + 1; ++i) d->sinV[i] = sinf((float)i * invCount * PI_F);
    free(img);
    free(func);
    free(sinVals);
    return (d->u.funcInt > 0.0f && isfinite(d->u.funcInt)) ? 0 : -1;
}

void ibl_dome_free(ibl_dome* d) {
    if (d->v)
        for (int u = 0; u < d->nu; ++u) { free(d->v[u].func); free(d->v[u].cdf); }
    free(d->v);
    free(d->u.func);
    free(d->u.cdf);
    free(d->cosU); free(d->sinU); free(d->cosV); free(d->sinV);
    memset(d, 0, sizeof *d);
}
