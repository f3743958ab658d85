/*
 * oro_ibl.h -- TEST INFRASTRUCTURE ONLY (see mrt_oracle.h for the contract).
 * Internal interface of oro_ibl.c: the image-based-lighting inputs of the CPU
 * restatement (HDR loading, lat-long lookups, Distribution1D, dome tables).
 */
#ifndef ORO_IBL_H
#define ORO_IBL_H

#include <math.h>

typedef struct {            /* RawImage (src/RawImage.h): W*H*channels floats, row 0 = top */
    float* rgb;
    int W, H;
    int type;               /* ORO_TEX_HDR (0, 3 floats, the IBL maps), _GRAY (1), _RGB (3), _RGBA (4) */
} ibl_image;

typedef struct {            /* Distribution1D, src/DomeLight.h:10-42 */
    float* func;
    float* cdf;
    float funcInt, invFuncInt, invCount;
    int count;
} ibl_dist;

typedef struct {            /* DomeLight::setTexture products, src/DomeLight.cpp:8-78 */
    int nu, nv;
    ibl_dist u;             /* over the column integrals                        */
    ibl_dist* v;            /* nu distributions over v                          */
    float *cosU, *sinU;     /* nu + 1 */
    float *cosV, *sinV;     /* nv + 1 */
} ibl_dome;

/* HDRLoader::load; rgb == NULL reads the header only.  0 = ok, < 0 error. */
int ibl_hdr_read(const char* path, float* rgb, int cap_w, int cap_h, int* w, int* h);
/* Texture::getLookup3 / getLookupXYZ3 */
void ibl_lookup3(const ibl_image* t, float u, float v, float out[3]);
void ibl_lookup_dir(const ibl_image* t, float x, float y, float z, float out[3]);
/* 0 = ok; -1 = the map has no positive radiance */
int ibl_dome_init(ibl_dome* d, const ibl_image* tex);
void ibl_dome_free(ibl_dome* d);
float ibl_dist_sample(const ibl_dist* d, float u, float* pdf);

/* The reference's libm calls on floats resolve to the float overloads under g++
 * (`using namespace std` + <math.h>): sin(acosf(x)) -> sinf / acosf (src/Material.h:51),
 * pow(float, float) -> powf (src/Blinn.cpp:219), atan2 / acos -> atan2f / acosf
 * (src/Texture.cpp:82-83,92-93), cos / sin -> cosf / sinf (src/Material.cpp:41).
 * atan2f / acosf are always glibc's (the device restates them bit-exactly).  For
 * sinf / cosf / powf the convention is selectable (oro_set_libm): 1 (default) = glibc's
 * float functions, the reference's own calls; 0 = the function in double, rounded once
 * (the HIP device's convention, within 1 ulp of glibc's). */
extern int oro_libm_float;
static inline float oro_acos(float x) { return acosf(x); }
static inline float oro_atan2(float y, float x) { return atan2f(y, x); }
static inline float oro_sin(float x) { return oro_libm_float ? sinf(x) : (float)sin((double)x); }
static inline float oro_cos(float x) { return oro_libm_float ? cosf(x) : (float)cos((double)x); }
static inline float oro_pow(float x, float y) { return oro_libm_float ? powf(x, y) : (float)pow((double)x, (double)y); }

#endif
