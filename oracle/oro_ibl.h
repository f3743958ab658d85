/*
 * oro_ibl.h -- TEST INFRASTRUCTURE ONLY (see mrt_oracle.h for the contract).
 * Internal interface of oro_ibl.c: the image-based-lighting inputs of the CPU
 * restatement (HDR loading, lat-long lookups, Distribution1D, dome tables).
 */
#ifndef ORO_IBL_H
#define ORO_IBL_H

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

#endif
