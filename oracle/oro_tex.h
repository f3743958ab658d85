/*
 * oro_tex.h -- TEST INFRASTRUCTURE ONLY (see mrt_oracle.h for the contract).
 * Internal interface of oro_tex.c: RawImage loading (TGA / PPM / HDR) and the
 * four-channel Texture::getLookup of the material maps.
 */
#ifndef ORO_TEX_H
#define ORO_TEX_H
#include "oro_ibl.h"

enum { ORO_TEX_HDR = 0, ORO_TEX_GRAY = 1, ORO_TEX_RGB = 3, ORO_TEX_RGBA = 4 };

/* floats per texel of a texture type */
int tex_channels(int type);
/* RawImage::loadImage by extension (src/RawImage.cpp:16-27).  out == NULL reads
 * the size and type only.  0 = ok, < 0 = error. */
int tex_image_read(const char* path, float* out, int cap_w, int cap_h, int* w, int* h, int* type);
/* Texture::getLookup (src/Texture.cpp:43-72): wrap, flip v, bilinear, 4 channels */
void tex_lookup4(const ibl_image* t, float u, float v, float out[4]);

#endif
