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
#include <stdlib.h>
#include <string.h>

#include <algorithm>
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
    // derived tables of the device sampler: the lat-long lookup of every table
    // direction (Shader::dome_light reads it instead of evaluating atan2 / acos
    // per sample; the same tex_lookup_dir code, evaluated here once per cell) and
    // the CDF guide tables
    d.rad.assign((size_t)4 * (nu + 1) * (nv + 1), 0.f);
    for (int iv = 0; iv <= nv; iv++)
        for (int iu = 0; iu <= nu; iu++) {
            const float cosT = d.cos_v[iv], sinT = d.sin_v[iv], sinP = d.sin_u[iu], cosP = d.cos_u[iu];
            const v3 L = tex_lookup_dir(t.rgb.data(), t.W, t.H, -sinT * cosP, -cosT, -sinT * sinP);
            float* q = &d.rad[4 * ((size_t)iv * (nu + 1) + iu)];
            q[0] = L.x; q[1] = L.y; q[2] = L.z;
        }
    d.guide_u.resize((size_t)nu + 1);
    guide_table(d.cdf_u.data(), nu, d.guide_u.data());
    d.guide_v.resize((size_t)nu * (nv + 1));
    for (int u = 0; u < nu; u++) guide_table(&d.cdf_v[(size_t)u * (nv + 1)], nv, &d.guide_v[(size_t)u * (nv + 1)]);
    return MRT_OK;
}


// ------------------------------------------------------------------ TGA / PPM
// Image::gamma_to_linear (src/Image.cpp:19-27): (int)(powf(i / 255.0f, 2.2f) * 32768.0 + 0.5)
static const unsigned short* gamma_to_linear() {
    static unsigned short t[256];
    static bool ready = false;
    if (!ready) {
        for (int i = 0; i < 256; i++) t[i] = (unsigned short)(int)((double)powf((float)i / 255.0f, 2.2f) * 32768.0 + 0.5);
        ready = true;
    }
    return t;
}

// RawImage::loadTGA (src/RawImage.cpp:89-188): the 18-byte header read field by
// field (the image-ID field is not skipped, as in the reference), uncompressed
// types 2 / 3 only, rows flipped, colour bytes through gamma_to_linear / 32768,
// the alpha byte / 255, B and R swapped.  A short body fails (reference: UB).
static int load_tga(const char* path, int& W, int& H, int& type, std::vector<float>* data, std::string& err) {
    FILE* f = fopen(path, "rb");
    if (!f) { err = std::string("cannot open ") + path; return MRT_ERR_IO; }
    unsigned char hdr[18];
    if (fread(hdr, 1, 18, f) != 18) { fclose(f); err = "short TGA header"; return MRT_ERR_IO; }
    const unsigned char tp = hdr[2], depth = hdr[16];
    const int w = (int16_t)(hdr[12] | hdr[13] << 8), h = (int16_t)(hdr[14] | hdr[15] << 8);
    const int mode = depth / 8;
    if ((tp != 2 && tp != 3) || w <= 0 || h <= 0 || (mode != 1 && mode != 3 && mode != 4)) {
        fclose(f);
        err = "unsupported TGA (uncompressed 8/24/32-bit true colour or grey only)";
        return MRT_ERR_IO;
    }
    W = w;
    H = h;
    type = mode == 1 ? kTexGray : mode == 3 ? kTexRGB : kTexRGBA;
    if (!data) { fclose(f); return MRT_OK; }
    const size_t row = (size_t)w * mode, total = row * h;
    std::vector<unsigned char> img(total);
    const size_t got = fread(img.data(), 1, total, f);
    fclose(f);
    if (got != total) { err = "short TGA body"; return MRT_ERR_IO; }
    const unsigned short* g2l = gamma_to_linear();
    data->assign(total, 0.f);
    float* out = data->data();
    for (int y = 0; y < h; y++) {   // file row y -> row h - 1 - y
        const unsigned char* src = img.data() + (size_t)y * row;
        float* dst = out + (size_t)(h - 1 - y) * row;
        for (size_t j = 0; j < row; j++) dst[j] = (float)g2l[src[j]] / 32768.f;
        if (mode == 4)
            for (size_t j = 3; j < row; j += 4) dst[j] = (float)src[j] / 255.f;
    }
    if (mode >= 3)
        for (size_t i = 0; i < total; i += (size_t)mode) std::swap(out[i], out[i + 2]);
    return MRT_OK;
}

// RawImage::loadPPM (src/RawImage.cpp:33-88): binary P6; '#' lines skipped before
// the size and the maxval lines; bytes / 255.
static int load_ppm(const char* path, int& W, int& H, int& type, std::vector<float>* data, std::string& err) {
    FILE* f = fopen(path, "rb");
    if (!f) { err = std::string("cannot open ") + path; return MRT_ERR_IO; }
    char buf[128], a[128], b[128];
    bool ok = fgets(buf, 128, f) != nullptr;
    do ok = ok && fgets(buf, 128, f) != nullptr;
    while (ok && buf[0] == '#');
    ok = ok && sscanf(buf, "%127s %127s", a, b) == 2;
    const int w = ok ? atoi(a) : 0, h = ok ? atoi(b) : 0;
    do ok = ok && fgets(buf, 128, f) != nullptr;
    while (ok && buf[0] == '#');
    if (!ok || w <= 0 || h <= 0) { fclose(f); err = "bad PPM header"; return MRT_ERR_IO; }
    W = w;
    H = h;
    type = kTexRGB;
    if (!data) { fclose(f); return MRT_OK; }
    const size_t total = (size_t)w * h * 3;
    std::vector<unsigned char> raw(total);
    const size_t got = fread(raw.data(), total, 1, f);
    fclose(f);
    if (got != 1) { err = "short PPM body"; return MRT_ERR_IO; }
    data->resize(total);
    for (size_t i = 0; i < total; i++) (*data)[i] = (float)raw[i] / 255;
    return MRT_OK;
}

int load_image(const char* path, int& W, int& H, int& type, std::vector<float>* data, std::string& err) {
    const char* dot = strrchr(path, '.');
    const std::string ext = dot ? dot + 1 : "";
    if (ext == "tga" || ext == "TGA") return load_tga(path, W, H, type, data, err);
    if (ext == "ppm" || ext == "PPM") return load_ppm(path, W, H, type, data, err);
    if (ext == "hdr" || ext == "HDR") {
        type = kTexHDR;
        return load_hdr(path, W, H, data, err);
    }
    err = "RawImage::loadImage reads .tga, .ppm and .hdr only";
    return MRT_ERR_IO;
}

// TriangleMesh::preCalc, USE_TRI_PACKETS branch (src/TriangleMesh.cpp:105-148):
// every triangle with a non-zero uv edge cross product writes the tangent frame
// of its three normal slots (later triangles overwrite).  Deviation: slots no
// triangle writes are zero (uninitialised memory in the reference).
void mesh_tangents(Mesh& m) {
    m.tan.clear();
    m.btan.clear();
    if (m.tidx.empty()) return;
    const uint16_t* RS = host_rsqrt_table();
    m.tan.assign(m.normals.size(), v3{0, 0, 0});
    m.btan.assign(m.normals.size(), v3{0, 0, 0});
    for (int32_t i = 0; i < m.nt(); i++) {
        const uint32_t* vi = &m.vidx[3 * (size_t)i];
        const v3 A = m.verts[vi[0]], B = m.verts[vi[1]], C = m.verts[vi[2]];
        const v3 AC = sub(C, A), AB = sub(B, A);
        const uint32_t* ti = &m.tidx[3 * (size_t)i];
        const float e1x = m.uv[2 * ti[1]] - m.uv[2 * ti[0]], e1y = m.uv[2 * ti[1] + 1] - m.uv[2 * ti[0] + 1];
        const float e2x = m.uv[2 * ti[2]] - m.uv[2 * ti[0]], e2y = m.uv[2 * ti[2] + 1] - m.uv[2 * ti[0] + 1];
        const float cp = e1y * e2x - e1x * e2y;
        if (cp == 0.0f) continue;
        const float mul = 1.f / cp;
        const v3 tangent = normalized(scale(add(scale(AB, -e2x), scale(AC, e1y)), mul), RS);
        const uint32_t* ni = &m.nidx[3 * (size_t)i];
        for (int k = 0; k < 3; k++) {
            const v3 normal = m.normals[ni[k]];
            m.tan[ni[k]] = normalized(sub(tangent, scale(normal, dot(normal, tangent))), RS);
            m.btan[ni[k]] = cross(m.tan[ni[k]], normal);
        }
    }
}

}  // namespace mrt
