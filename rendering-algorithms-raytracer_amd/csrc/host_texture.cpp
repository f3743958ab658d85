// host_texture.cpp -- images and dome-light tables, host side of libmrt.
//
// HDRLoader::load (reference src/hdrloader.cpp:29-190): Radiance RGBE with
// new-style per-channel run-length scanlines and old-style (flat, or (1,1,1,n)
// repeat) scanlines, decoded to W*H*3 floats with the top scanline first, as
// RawImage::loadHDR keeps them (src/RawImage.cpp:29-32).
// DomeLight::setTexture (src/DomeLight.cpp:8-78): a Distribution1D over v of
// each column's texel averages x sin(theta), a Distribution1D over u of the
// column integrals, and the sin / cos tables of the sampled angles -- built with
// the same Texture::getLookup3 the device uses (mrt_texture.h).
//
// Inputs on which the reference would overrun memory fail with MRT_ERR_IO
// instead: header / resolution lines beyond its 200-byte buffers, a run past
// the end of a scanline, an old-style run with no previous pixel.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <array>
#include <cmath>
#include <string>
#include <vector>

#include "mrt_scene.h"
#include "mrt_texture.h"

namespace mrt {
namespace {

using Rgbe = std::array<uint8_t, 4>;

struct InFile {
    FILE* f;
    explicit InFile(const char* path) : f(fopen(path, "rb")) {}
    ~InFile() {
        if (f) fclose(f);
    }
};

inline uint8_t next_byte(FILE* f) { return (uint8_t)fgetc(f); }

enum class Line { kOk, kEnd, kBad };  // scanline read; kEnd = the reference's `false`

// oldDecrunch (src/hdrloader.cpp:161-190): pixels from `at` to the end of the
// row; (1,1,1,n) repeats the previous pixel n << shift times, each consecutive
// run marker shifting n by 8 more bits.
Line read_flat(FILE* f, std::vector<Rgbe>& row, size_t at) {
    int shift = 0;
    while (at < row.size()) {
        Rgbe p;
        for (uint8_t& c : p) c = next_byte(f);
        if (feof(f)) return Line::kEnd;
        row[at] = p;
        if (p[0] == 1 && p[1] == 1 && p[2] == 1) {
            if (at == 0 || shift >= 32) return Line::kBad;
            const uint64_t n = (uint64_t)p[3] << shift;
            if (n > row.size() - at) return Line::kBad;
            for (uint64_t k = 0; k < n; k++, at++) row[at] = row[at - 1];
            shift += 8;
        } else {
            at++;
            shift = 0;
        }
    }
    return Line::kOk;
}

// decrunch (src/hdrloader.cpp:118-159)
Line read_scanline(FILE* f, std::vector<Rgbe>& row) {
    const size_t len = row.size();
    if (len < 8 || len > 0x7fff) return read_flat(f, row, 0);
    if (fgetc(f) != 2) {
        fseek(f, -1, SEEK_CUR);
        return read_flat(f, row, 0);
    }
    const uint8_t g = next_byte(f), b = next_byte(f);
    const uint8_t e = next_byte(f);
    if (g != 2 || (b & 128)) {
        row[0] = Rgbe{2, g, b, e};
        return read_flat(f, row, 1);
    }
    for (int ch = 0; ch < 4; ch++) {
        for (size_t j = 0; j < len;) {
            uint8_t code = next_byte(f);
            if (code > 128) {
                code &= 127;
                const uint8_t val = next_byte(f);
                if (j + code > len) return Line::kBad;
                for (; code > 0; code--) row[j++][ch] = val;
            } else {
                if (j + code > len) return Line::kBad;
                for (; code > 0; code--) row[j++][ch] = next_byte(f);
            }
        }
    }
    return feof(f) ? Line::kEnd : Line::kOk;
}

// convertComponent (src/hdrloader.cpp:99-104): (v / 256) * 2^expo, exact in float
inline float rgbe_component(int expo, int v) { return ((float)v / 256.0f) * (float)ldexp(1.0, expo); }

// Distribution1D(f, n) + computeStep1dCDF (src/DomeLight.h:11-30); returns the
// integral the CDF was normalised by.
float step_cdf(const float* f, int n, float* func, float* cdf) {
    cdf[0] = 0.f;
    for (int i = 1; i <= n; i++) {
        func[i - 1] = f[i - 1];
        cdf[i] = cdf[i - 1] + f[i - 1] / (float)n;
    }
    const float c = cdf[n];
    for (int i = 1; i <= n; i++) cdf[i] /= c;
    return c;
}

}  // namespace

// HDRLoader::load (src/hdrloader.cpp:29-97); rgb == nullptr reads the header only.
int load_hdr(const char* path, int& W, int& H, std::vector<float>* rgb, std::string& err) {
    InFile in(path);
    FILE* f = in.f;
    const std::string p(path);
    if (!f) { err = "cannot open " + p; return MRT_ERR_IO; }
    char magic[10];
    if (fread(magic, 10, 1, f) != 1 || memcmp(magic, "#?RADIANCE", 10) != 0) {
        err = p + ": not a Radiance HDR file";
        return MRT_ERR_IO;
    }
    fseek(f, 1, SEEK_CUR);
    // header lines up to the first empty line (two consecutive '\n')
    int prev = 0, stored = 0;
    for (;;) {
        const int c = fgetc(f);
        if (c == EOF) { err = p + ": truncated HDR header"; return MRT_ERR_IO; }
        if (c == '\n' && prev == '\n') break;
        if (++stored > 200) { err = p + ": HDR header longer than 200 bytes"; return MRT_ERR_IO; }
        prev = c;
    }
    std::string reso;
    for (;;) {
        const int c = fgetc(f);
        if (c == EOF || reso.size() >= 200) { err = p + ": bad HDR resolution line"; return MRT_ERR_IO; }
        reso.push_back((char)c);
        if (c == '\n') break;
    }
    int w = 0, h = 0;
    if (sscanf(reso.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0 || (int64_t)w * h > (int64_t(1) << 28)) {
        err = p + ": unsupported HDR resolution line (only \"-Y H +X W\")";
        return MRT_ERR_IO;
    }
    W = w;
    H = h;
    if (!rgb) return MRT_OK;
    rgb->assign((size_t)w * h * 3, 0.f);
    std::vector<Rgbe> row((size_t)w);
    float* out = rgb->data();
    for (int y = h - 1; y >= 0; y--) {  // scanlines in file order, top first
        const Line r = read_scanline(f, row);
        if (r == Line::kBad) { err = p + ": RLE run past the end of a scanline"; return MRT_ERR_IO; }
        if (r == Line::kEnd) break;     // the reference stops at a short scanline too
        for (const Rgbe& px : row) {    // workOnRGBE
            const int e = (int)px[3] - 128;
            *out++ = rgbe_component(e, px[0]);
            *out++ = rgbe_component(e, px[1]);
            *out++ = rgbe_component(e, px[2]);
        }
    }
    return MRT_OK;
}

// DomeLight::setTexture (src/DomeLight.cpp:8-78)
int build_dome(const Texture& t, DomeTables& d, std::string& err) {
    const int nu = t.W, nv = t.H;
    d.nu = nu;
    d.nv = nv;
    std::vector<float> img((size_t)nu * nv);
    for (int u = 0; u < nu; u++) {
        const float up = (float)u / (float)nu;
        for (int v = 0; v < nv; v++) {
            const float vp = (float)v / (float)nv;
            const v3 L = tex_lookup3(t.rgb.data(), t.W, t.H, up, vp);
            img[(size_t)u * nv + v] = ((L.x + L.y) + L.z) * 0.333333f;  // Vector3::average
        }
    }
    std::vector<float> sin_theta(nv);
    for (int i = 0; i < nv; i++) sin_theta[i] = sinf(kPI * (float)(i + .5) / (float)nv);
    d.func_v.resize((size_t)nu * nv);
    d.cdf_v.resize((size_t)nu * (nv + 1));
    d.int_v.resize(nu);
    d.inv_int_v.resize(nu);
    std::vector<float> col(nv);
    for (int u = 0; u < nu; u++) {
        for (int v = 0; v < nv; v++) col[v] = img[(size_t)u * nv + v] * sin_theta[v];
        d.int_v[u] = step_cdf(col.data(), nv, &d.func_v[(size_t)u * nv], &d.cdf_v[(size_t)u * (nv + 1)]);
        d.inv_int_v[u] = 1.f / d.int_v[u];
    }
    d.func_u.resize(nu);
    d.cdf_u.resize((size_t)nu + 1);
    d.int_u = step_cdf(d.int_v.data(), nu, d.func_u.data(), d.cdf_u.data());
    if (!(d.int_u > 0.f) || !std::isfinite(d.int_u)) {
        err = "dome texture has no positive radiance (zero Distribution1D integral)";
        return MRT_ERR_INVALID;
    }
    d.inv_int_u = 1.f / d.int_u;
    d.cos_u.resize((size_t)nu + 1);
    d.sin_u.resize((size_t)nu + 1);
    d.cos_v.resize((size_t)nv + 1);
    d.sin_v.resize((size_t)nv + 1);
    float inv = 1.f / (float)nu;
    for (int i = 0; i <= nu; i++) d.cos_u[i] = cosf((float)i * inv * 2.f * kPI);
    for (int i = 0; i <= nu; i++) d.sin_u[i] = sinf((float)i * inv * 2.f * kPI);
    inv = 1.f / (float)nv;
    for (int i = 0; i <= nv; i++) d.cos_v[i] = cosf((float)i * inv * kPI);
    for (int i = 0; i <= nv; i++) d.sin_v[i] = sinf((float)i * inv * kPI);
    return MRT_OK;
}

}  // namespace mrt
