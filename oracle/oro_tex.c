/*
 * oro_tex.c -- TEST INFRASTRUCTURE ONLY (see mrt_oracle.h for the contract).
 *
 * CPU restatement of the texture inputs of Blinn / Lambert's maps and the
 * alpha-mapped any-hit test:
 *   RawImage::loadImage / loadTGA / loadPPM      src/RawImage.cpp:16-188
 *   Image::generateGammaTables (gamma_to_linear)  src/Image.cpp:19-27
 *   Texture::getLookup / getLookupAlpha / getPixel src/Texture.cpp:12-72,100-125
 *
 * Deviations, all where the reference has undefined behaviour: a short TGA /
 * PPM body and an unsupported TGA type fail the load (negative return; the
 * reference keeps uninitialised or NULL data); getPixel wraps negative texel
 * coordinates into range (the reference indexes before the array); the HDR
 * type's fourth component (the next texel's red, src/Texture.cpp:120-123) is 0
 * for the last texel (read past the array there).
 */
#include "oro_tex.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int tex_channels(int type) { return type == ORO_TEX_GRAY ? 1 : type == ORO_TEX_RGBA ? 4 : 3; }

/* float -> int as the x86 truncating conversion for in-range values; NaN and
 * out-of-range (reference UB) give 0 */
static int trunc_i(float f) { return (f > -2147483648.0f && f < 2147483648.0f) ? (int)f : 0; }

/* Image::gamma_to_linear[i] = (unsigned short)(int)(pow(i / 255.0f, GAMMA) * 32768.0 + 0.5),
 * GAMMA = 2.2f, std::pow(float, float) (src/Image.cpp:14,24-27) */
static unsigned short g_g2l[256];
static int g_g2l_ready = 0;
static void gamma_to_linear_table(void) {
    if (g_g2l_ready) return;
    for (int i = 0; i < 256; i++) g_g2l[i] = (unsigned short)(int)((double)powf((float)i / 255.0f, 2.2f) * 32768.0 + 0.5);
    g_g2l_ready = 1;
}

static int rd_u8(FILE* f, unsigned char* v) { return fread(v, 1, 1, f) == 1 ? 0 : -1; }
static int rd_i16(FILE* f, short* v) { return fread(v, 2, 1, f) == 1 ? 0 : -1; }   /* little-endian host */

/* RawImage::loadTGA, src/RawImage.cpp:89-188: 18-byte header (the ID field is
 * not skipped), uncompressed type 2 / 3 only, rows flipped, colour bytes through
 * gamma_to_linear / 32768, an alpha byte / 255, B and R swapped. */
static int load_tga(const char* path, float* out, int cap_w, int cap_h, int* w, int* h, int* type) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    unsigned char c, tp, depth;
    short i16, width, height;
    int bad = 0;   /* the header fields in file order (operands of | are unsequenced) */
    bad |= rd_u8(f, &c);
    bad |= rd_u8(f, &c);
    bad |= rd_u8(f, &tp);
    bad |= rd_i16(f, &i16);
    bad |= rd_i16(f, &i16);
    bad |= rd_u8(f, &c);
    bad |= rd_i16(f, &i16);
    bad |= rd_i16(f, &i16);
    bad |= rd_i16(f, &width);
    bad |= rd_i16(f, &height);
    bad |= rd_u8(f, &depth);
    bad |= rd_u8(f, &c);
    const int mode = depth / 8;
    if (bad || (tp != 2 && tp != 3) || width <= 0 || height <= 0 || (mode != 1 && mode != 3 && mode != 4)) {
        fclose(f);
        return -2;
    }
    *w = width;
    *h = height;
    *type = mode == 1 ? ORO_TEX_GRAY : mode == 3 ? ORO_TEX_RGB : ORO_TEX_RGBA;
    if (!out) { fclose(f); return 0; }
    if (cap_w != width || cap_h != height) { fclose(f); return -3; }
    const size_t total = (size_t)width * height * mode;
    unsigned char* img = (unsigned char*)malloc(total);
    unsigned char* flip = (unsigned char*)malloc(total);
    const size_t got = fread(img, 1, total, f);
    fclose(f);
    if (got != total) { free(img); free(flip); return -4; }
    for (int i = 0; i < height; i++)
        memcpy(flip + (size_t)(height - i - 1) * width * mode, img + (size_t)i * width * mode, (size_t)width * mode);
    gamma_to_linear_table();
    for (size_t i = 0; i < total; i++) out[i] = (float)g_g2l[flip[i]] / 32768.f;
    if (mode == 4)
        for (size_t i = 3; i < total; i += 4) out[i] = (float)flip[i] / 255.f;
    if (mode >= 3)
        for (size_t i = 0; i < total; i += (size_t)mode) {
            const float a = out[i];
            out[i] = out[i + 2];
            out[i + 2] = a;
        }
    free(img);
    free(flip);
    return 0;
}

/* RawImage::loadPPM, src/RawImage.cpp:33-88: binary P6, '#' comment lines
 * skipped before the size and the maxval lines, bytes / 255 (no gamma). */
static int load_ppm(const char* path, float* out, int cap_w, int cap_h, int* w, int* h, int* type) {
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    char buf[3][128];
    if (!fgets(buf[0], 128, f)) { fclose(f); return -2; }
    do {
        if (!fgets(buf[0], 128, f)) { fclose(f); return -2; }
    } while (buf[0][0] == '#');
    buf[1][0] = buf[2][0] = 0;
    if (sscanf(buf[0], "%127s %127s", buf[1], buf[2]) != 2) { fclose(f); return -2; }
    const int W = atoi(buf[1]), H = atoi(buf[2]);
    do {
        if (!fgets(buf[0], 128, f)) { fclose(f); return -2; }
    } while (buf[0][0] == '#');
    if (W <= 0 || H <= 0) { fclose(f); return -2; }
    *w = W;
    *h = H;
    *type = ORO_TEX_RGB;
    if (!out) { fclose(f); return 0; }
    if (cap_w != W || cap_h != H) { fclose(f); return -3; }
    const size_t total = (size_t)W * H * 3;
    unsigned char* raw = (unsigned char*)malloc(total);
    const size_t got = fread(raw, total, 1, f);
    fclose(f);
    if (got != 1) { free(raw); return -4; }
    for (size_t i = 0; i < total; i++) out[i] = (float)raw[i] / 255;
    free(raw);
    return 0;
}

int tex_image_read(const char* path, float* out, int cap_w, int cap_h, int* w, int* h, int* type) {
    const char* dot = strrchr(path, '.');
    const char* ext = dot ? dot + 1 : "";
    if (!strcmp(ext, "tga") || !strcmp(ext, "TGA")) return load_tga(path, out, cap_w, cap_h, w, h, type);
    if (!strcmp(ext, "ppm") || !strcmp(ext, "PPM")) return load_ppm(path, out, cap_w, cap_h, w, h, type);
    if (!strcmp(ext, "hdr") || !strcmp(ext, "HDR")) {
        *type = ORO_TEX_HDR;
        return ibl_hdr_read(path, out, cap_w, cap_h, w, h);
    }
    return -5;   /* RawImage::loadImage ignores other extensions */
}

/* Texture::getPixel, src/Texture.cpp:100-125 ("tile"): x % W, y % H */
static void pixel4(const ibl_image* t, int x, int y, float p[4]) {
    x %= t->W;
    if (x < 0) x += t->W;
    y %= t->H;
    if (y < 0) y += t->H;
    const size_t i = (size_t)y * t->W + x;
    const float* d = t->rgb;
    switch (t->type) {
        case ORO_TEX_GRAY: p[0] = p[1] = p[2] = d[i]; p[3] = 1.0f; break;
        case ORO_TEX_RGB: p[0] = d[3 * i]; p[1] = d[3 * i + 1]; p[2] = d[3 * i + 2]; p[3] = 1.0f; break;
        case ORO_TEX_RGBA: p[0] = d[4 * i]; p[1] = d[4 * i + 1]; p[2] = d[4 * i + 2]; p[3] = d[4 * i + 3]; break;
        default:   /* HDR: m_rawData[base + 3], the next texel's red */
            p[0] = d[3 * i]; p[1] = d[3 * i + 1]; p[2] = d[3 * i + 2];
            p[3] = (i + 1 < (size_t)t->W * t->H) ? d[3 * i + 3] : 0.0f;
    }
}

void tex_lookup4(const ibl_image* t, float u, float v, float out[4]) {
    u = u - (float)trunc_i(u);
    v = v - (float)trunc_i(v);
    if (u < 0.0f) u = u + 1.0f;
    if (v < 0.0f) v = v + 1.0f;
    v = 1.0f - v;                                /* textures start with v = 0 at the top */
    float px = u * (float)t->W, py = v * (float)t->H;
    float x1 = floorf(px), x2 = x1 + 1.0f, dx = px - x1;
    float y1 = floorf(py), y2 = y1 + 1.0f, dy = py - y1;
    float p11[4], p21[4], p12[4], p22[4];
    pixel4(t, trunc_i(x1), trunc_i(y1), p11);
    pixel4(t, trunc_i(x2), trunc_i(y1), p21);
    pixel4(t, trunc_i(x1), trunc_i(y2), p12);
    pixel4(t, trunc_i(x2), trunc_i(y2), p22);
    for (int k = 0; k < 4; k++) {
        float q1 = p11[k] * (1.0f - dx) + p21[k] * dx;
        float q2 = p12[k] * (1.0f - dx) + p22[k] * dx;
        out[k] = q1 * (1.0f - dy) + q2 * dy;
    }
}
