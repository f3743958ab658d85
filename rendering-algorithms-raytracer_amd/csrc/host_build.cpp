// host_build.cpp -- OBJ loading and QBVH construction (host side of libmrt).
//
// Restates the reference's scene-build semantics so that the device traverses
// the same hierarchy the reference would build for the same input:
//   TriangleMesh::loadObj           src/TriangleMeshLoad.cpp:99-214
//   BVH::build (USE_BINS, USE_QBVH) src/BVH.cpp:457-575
//   BVH_Node::buildBin              src/BVH.cpp:625-689
//   BVH_Node::partitionSweepBin     src/BVH.cpp:691-901
//   BVH_Node::calcSAHCost           src/BVH.cpp:1076-1106
//   QBVH_Node::build / buildTriBundle src/BVH.cpp:64-389
// The binary tree is built into a flat arena and collapsed in one pass into the
// HBM layout (mrt_types.h).  Quirks of the reference that shape the tree are
// kept on purpose (they are pinned by SURVEY.md's explosion01 node/leaf counts):
//   * the loose partition does not swap bin ids with the objects it moves;
//   * the <128-object sweep's left/right areas skip the first/last object;
//   * qsort is glibc's stable merge sort (so std::stable_sort).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <climits>
#include <mutex>
#include <thread>
#include <cmath>
#include <string>

#include "mrt_scene.h"

#define MRT_TABLE_QUAL static const
#include "x86_approx_tables.inc"

namespace mrt {

namespace {
struct Tables {
    uint16_t rcp[2048], rsq[2048];
    uint8_t gamma[32769];
    float gammaF[32769];
    Tables() {
        for (int i = 0; i < 2048; i++) {
            rcp[i] = (uint16_t)((MRT_RCP_TABLE[i] >> 11) & 0xFFFu);
            rsq[i] = (uint16_t)((MRT_RSQRT_TABLE[i] >> 11) & 0xFFFu);
        }
        // Image::generateGammaTables (src/Image.cpp:19-35): float pow, double tail.
        const float GAMMA = 2.2f;
        for (int i = 0; i < 32769; i++) {
            float r2 = (float)((double)powf(i / 32768.0f, 1 / GAMMA) * 255.0 + 0.5);
            gammaF[i] = r2;
            gamma[i] = (uint8_t)(int)r2;
        }
    }
};
const Tables& tables() {
    static Tables t;
    return t;
}
}  // namespace

const uint16_t* host_rcp_table() { return tables().rcp; }
const uint16_t* host_rsqrt_table() { return tables().rsq; }
const uint8_t* host_gamma_lut() { return tables().gamma; }
const float* host_gamma_float_lut() { return tables().gammaF; }

// ------------------------------------------------------------------ Matrix4x4
namespace {
struct Mat4 {
    float m[4][4];
};
Mat4 identity() {
    Mat4 M{};
    M.m[0][0] = M.m[1][1] = M.m[2][2] = M.m[3][3] = 1.0f;
    return M;
}
// Matrix4x4::invert (src/Matrix4x4.h:353-412): cofactors, 1/det in double.
Mat4 inverse(const Mat4& A) {
    const float(*a)[4] = A.m;
    auto t2 = [](float p, float q, float r, float s) { return p * q - r * s; };
    float T34_12 = t2(a[2][0], a[3][1], a[2][1], a[3][0]), T34_13 = t2(a[2][0], a[3][2], a[2][2], a[3][0]);
    float T34_14 = t2(a[2][0], a[3][3], a[2][3], a[3][0]), T34_23 = t2(a[2][1], a[3][2], a[2][2], a[3][1]);
    float T34_24 = t2(a[2][1], a[3][3], a[2][3], a[3][1]), T34_34 = t2(a[2][2], a[3][3], a[2][3], a[3][2]);
    float T24_12 = t2(a[1][0], a[3][1], a[1][1], a[3][0]), T24_13 = t2(a[1][0], a[3][2], a[1][2], a[3][0]);
    float T24_14 = t2(a[1][0], a[3][3], a[1][3], a[3][0]), T24_23 = t2(a[1][1], a[3][2], a[1][2], a[3][1]);
    float T24_24 = t2(a[1][1], a[3][3], a[1][3], a[3][1]), T24_34 = t2(a[1][2], a[3][3], a[1][3], a[3][2]);
    float T23_12 = t2(a[1][0], a[2][1], a[1][1], a[2][0]), T23_13 = t2(a[1][0], a[2][2], a[1][2], a[2][0]);
    float T23_14 = t2(a[1][0], a[2][3], a[1][3], a[2][0]), T23_23 = t2(a[1][1], a[2][2], a[1][2], a[2][1]);
    float T23_24 = t2(a[1][1], a[2][3], a[1][3], a[2][1]), T23_34 = t2(a[1][2], a[2][3], a[1][3], a[2][2]);
    auto s3 = [](float p, float q, float r, float s, float u, float v) { return p * q - r * s + u * v; };
    float sd11 = s3(a[1][1], T34_34, a[1][2], T34_24, a[1][3], T34_23);
    float sd12 = s3(a[1][0], T34_34, a[1][2], T34_14, a[1][3], T34_13);
    float sd13 = s3(a[1][0], T34_24, a[1][1], T34_14, a[1][3], T34_12);
    float sd14 = s3(a[1][0], T34_23, a[1][1], T34_13, a[1][2], T34_12);
    float sd21 = s3(a[0][1], T34_34, a[0][2], T34_24, a[0][3], T34_23);
    float sd22 = s3(a[0][0], T34_34, a[0][2], T34_14, a[0][3], T34_13);
    float sd23 = s3(a[0][0], T34_24, a[0][1], T34_14, a[0][3], T34_12);
    float sd24 = s3(a[0][0], T34_23, a[0][1], T34_13, a[0][2], T34_12);
    float sd31 = s3(a[0][1], T24_34, a[0][2], T24_24, a[0][3], T24_23);
    float sd32 = s3(a[0][0], T24_34, a[0][2], T24_14, a[0][3], T24_13);
    float sd33 = s3(a[0][0], T24_24, a[0][1], T24_14, a[0][3], T24_12);
    float sd34 = s3(a[0][0], T24_23, a[0][1], T24_13, a[0][2], T24_12);
    float sd41 = s3(a[0][1], T23_34, a[0][2], T23_24, a[0][3], T23_23);
    float sd42 = s3(a[0][0], T23_34, a[0][2], T23_14, a[0][3], T23_13);
    float sd43 = s3(a[0][0], T23_24, a[0][1], T23_14, a[0][3], T23_12);
    float sd44 = s3(a[0][0], T23_23, a[0][1], T23_13, a[0][2], T23_12);
    float det = a[0][0] * sd11 - a[0][1] * sd12 + a[0][2] * sd13 - a[0][3] * sd14;
    float di = (float)(1.0 / (double)det);
    Mat4 R;
    const float sd[4][4] = {{sd11, sd12, sd13, sd14}, {sd21, sd22, sd23, sd24},
                            {sd31, sd32, sd33, sd34}, {sd41, sd42, sd43, sd44}};
    // R(r,c) = (-1)^(r+c) * sd[c][r] * di
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) R.m[r][c] = (((r + c) & 1) ? -sd[c][r] : sd[c][r]) * di;
    return R;
}
Mat4 transpose(const Mat4& A) {
    Mat4 R;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) R.m[r][c] = A.m[c][r];
    return R;
}
// DPPS 0xFF: (p0 + p1) + (p2 + p3)
inline float dp4(const float* row, const float* u) {
    float p0 = row[0] * u[0], p1 = row[1] * u[1], p2 = row[2] * u[2], p3 = row[3] * u[3];
    return (p0 + p1) + (p2 + p3);
}
// multiplyAndDivideByW(__m128 (x,y,z,1)), src/Matrix4x4.h:744-748
v3 xform_point(const Mat4& M, v3 p) {
    const float u[4] = {p.x, p.y, p.z, 1.0f};
    float w = rcp_nr(dp4(M.m[3], u), host_rcp_table());
    return mk(w * dp4(M.m[0], u), w * dp4(M.m[1], u), w * dp4(M.m[2], u));
}
// operator*(Matrix4x4, Vector3), src/Matrix4x4.h:693-704 (non-SSE path)
v3 xform_dir(const Mat4& M, v3 u) {
    return mk(M.m[0][0] * u.x + M.m[0][1] * u.y + M.m[0][2] * u.z,
              M.m[1][0] * u.x + M.m[1][1] * u.y + M.m[1][2] * u.z,
              M.m[2][0] * u.x + M.m[2][1] * u.y + M.m[2][2] * u.z);
}

// atoi(s) = (int)strtol(s, NULL, 10) (glibc): leading white space, a sign,
// decimal digits; out of long range -> LONG_MAX / LONG_MIN; then the long is
// truncated to int
int atoi_exact(const char* s) {
    while (*s == ' ' || (*s >= '\t' && *s <= '\r')) s++;
    bool neg = false;
    if (*s == '+' || *s == '-') neg = *s++ == '-';
    uint64_t v = 0;
    bool sat = false;
    for (; *s >= '0' && *s <= '9'; s++) {
        if (!sat) {
            v = v * 10 + (uint64_t)(*s - '0');
            if (v > (uint64_t)LONG_MAX + (neg ? 1u : 0u)) sat = true;
        }
    }
    long r;
    if (sat) r = neg ? LONG_MIN : LONG_MAX;
    else r = neg ? (long)(0 - v) : (long)v;
    return (int)r;
}

// getIndices, src/TriangleMeshLoad.cpp:67-97
void split_indices(char* word, int& vi, int& ti, int& ni) {
    static char blank[] = " ";
    char* tp = blank;
    char* np = blank;
    for (char* p = word; *p; ++p) {
        if (*p != '/') continue;
        if (tp == blank) tp = p + 1;
        else np = p + 1;
        *p = '\0';
    }
    vi = atoi_exact(word);
    ti = atoi_exact(tp);
    ni = atoi_exact(np);
}
}  // namespace

namespace {
int build_threads();
}  // namespace

namespace {
inline bool is_space(char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }   // isspace, C locale

// sscanf(s, "%f %f ... %f", out...) for n floats, exact: a plain decimal token
// ([+-] digits [. digits] [(e|E) [+-] digits], at most 19 significant digits,
// ended by white space or the end) is converted as m * 10^e in double -- one
// correctly rounded operation while m < 2^53 and |e| <= 22 -- and rounded to
// float, which equals strtof's correctly rounded result unless the double lands
// exactly on a float rounding midpoint.  Anything else (that midpoint, hex, inf,
// nan, subnormal or out-of-range values, fewer than n tokens, malformed
// tokens) returns false and the caller runs sscanf itself.
bool fast_floats(const char* s, int n, float* out) {
    static const double p10[23] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9, 1e10, 1e11,
                                   1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
    for (int k = 0; k < n; k++) {
        while (is_space(*s)) s++;
        bool neg = false;
        if (*s == '+' || *s == '-') neg = *s++ == '-';
        uint64_t m = 0;
        int sig = 0, digits = 0, e10 = 0;
        for (; *s >= '0' && *s <= '9'; s++, digits++) {
            if (m || *s != '0') { if (++sig > 19) return false; m = m * 10 + (uint64_t)(*s - '0'); }
        }
        if (*s == '.') {
            for (s++; *s >= '0' && *s <= '9'; s++, digits++) {
                if (m || *s != '0') { if (++sig > 19) return false; m = m * 10 + (uint64_t)(*s - '0'); }
                e10--;
            }
        }
        if (!digits) return false;
        if (*s == 'e' || *s == 'E') {
            s++;
            bool eneg = false;
            if (*s == '+' || *s == '-') eneg = *s++ == '-';
            if (!(*s >= '0' && *s <= '9')) return false;
            int x = 0;
            for (; *s >= '0' && *s <= '9'; s++) { if (x < 10000) x = x * 10 + (*s - '0'); }
            e10 += eneg ? -x : x;
        }
        if (*s && !is_space(*s)) return false;
        if (m == 0) { out[k] = neg ? -0.0f : 0.0f; continue; }
        if (m > (1ull << 53) || e10 > 22 || e10 < -22) return false;
        double d = (double)m;
        d = e10 < 0 ? d / p10[-e10] : d * p10[e10];
        if (!(d >= 1.1754943508222875e-38 && d <= 3.4028234663852886e38)) return false;   // normal floats only
        uint64_t bits;
        memcpy(&bits, &d, sizeof bits);
        if ((bits & 0x1FFFFFFFull) == 0x10000000ull) return false;   // a float midpoint: ambiguous
        const float f = (float)d;
        out[k] = neg ? -f : f;
    }
    return true;
}
// sscanf(s, "%31s %31s %31s") into tok (tokens not reached stay as they are)
void scan_tokens(const char* s, char (&tok)[3][32]) {
    for (int k = 0; k < 3; k++) {
        while (is_space(*s)) s++;
        if (!*s) return;
        int i = 0;
        while (*s && !is_space(*s) && i < 31) tok[k][i++] = *s++;
        tok[k][i] = '\0';
    }
}

// One fgets(line, 80, fp) chunk of the file at p (end = file end): up to 79
// bytes, through the first '\n'.  A line longer than 79 characters is several
// chunks, each parsed as a line of its own (the reference's behaviour); a chunk
// boundary is fixed by its line's start, so cutting the file at line starts
// keeps the chunk sequence.
inline size_t chunk_len(const char* p, const char* end) {
    const size_t lim = std::min<size_t>(79, (size_t)(end - p));
    const void* nl = memchr(p, '\n', lim);
    return nl ? (size_t)((const char*)nl - p) + 1 : lim;
}
inline void chunk_copy(char (&line)[81], const char* p, size_t n) {
    memcpy(line, p, n);
    line[n] = '\0';
}

// A byte range of the file (starting at a line start) and what it holds.
struct ObjRange {
    size_t b = 0, e = 0;
    int nv = 0, nt = 0, nn = 0, nf = 0;   // pass 1: v / vt / vn / f chunks
    // pass 2: faces without a normal on their last corner (face-normal events)
    struct FaceNormal {
        uint32_t tri, verts_loaded;        // triangle index; vertices loaded before the face
        size_t pos;                        // chunk offset (error order)
    };
    std::vector<FaceNormal> fn;
    size_t err_pos = SIZE_MAX;             // first error of the range (file offset)
    std::string err;
};

// Runs f(r) for every range on up to `threads` threads.
template <typename F>
void for_ranges(std::vector<ObjRange>& rs, int threads, F f) {
    if (threads <= 1 || rs.size() <= 1) {
        for (ObjRange& r : rs) f(r);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> ts;
    const int n = std::min<int>(threads, (int)rs.size());
    for (int i = 0; i < n; i++)
        ts.emplace_back([&] {
            for (size_t k; (k = next.fetch_add(1)) < rs.size();) f(rs[k]);
        });
    for (auto& t : ts) t.join();
}
}  // namespace

// TriangleMesh::loadObj, src/TriangleMeshLoad.cpp:99-214: vertices through
// ctm with the rcp_nr w-divide; normals through the inverse transpose and
// renormalised; a face without a normal on its last corner gets a face normal
// appended at slot `nn` (the reference also stores its index triple at
// m_normalIndices[nn]).  Reference UB (negative / out-of-range indices, slot
// overflow) -> MRT_ERR_IO.
//
// Parallel form of the reference's two sequential passes over 79-character
// fgets chunks, with the same result bit for bit at any thread count: the
// mapped file is cut into ranges at line starts; pass 1 counts each range's
// v / vt / vn / f chunks, prefix sums give every range its first vertex,
// normal, texture-coordinate and triangle index, and pass 2 parses the ranges
// concurrently into their slots (sscanf per chunk, as the reference).  The
// face normals then run as a third pass in file order of their slots:
//   * the reference reads the face's vertices as loaded at that point of the
//     file -- a vertex defined further down is still the zero vector -- so each
//     event keeps the count of vertices loaded before it;
//   * the index triple it writes at m_normalIndices[nn] is overwritten by
//     triangle nn's own corners (those with a normal index) when triangle nn
//     comes later in the file, and overwrites them when it came earlier.
// Errors are reported for the first offending chunk in file order.
int load_obj(const char* path, const float* ctm16, Mesh& out, std::string& err) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) {
        err = std::string("cannot open ") + path;
        return MRT_ERR_IO;
    }
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
        close(fd);
        err = std::string("cannot stat ") + path;
        return MRT_ERR_IO;
    }
    const size_t size = (size_t)sb.st_size;
    const char* base = nullptr;
    if (size) {
        void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) {
            close(fd);
            err = std::string("cannot map ") + path;
            return MRT_ERR_IO;
        }
        base = static_cast<const char*>(m);
    }
    close(fd);
    struct Unmap {
        const char* p;
        size_t n;
        ~Unmap() { if (p) munmap(const_cast<char*>(p), n); }
    } unmap{base, size};
    const char* end = base + size;
    const bool trace = getenv("MRT_BUILD_TRACE") != nullptr;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const auto t0 = now();

    Mat4 ctm = identity();
    if (ctm16) memcpy(ctm.m, ctm16, sizeof(float) * 16);
    const Mat4 nctm = transpose(inverse(ctm));
    const uint16_t* RS = host_rsqrt_table();

    // ranges: about MRT_OBJ_RANGE_BYTES (default 1 MiB) each, cut after a '\n'
    int threads = build_threads();
    size_t per = 1u << 20;
    if (const char* e = getenv("MRT_OBJ_RANGE_BYTES")) {
        const long v = atol(e);
        if (v >= 1) per = (size_t)v;
    }
    std::vector<ObjRange> rs;
    for (size_t b = 0; b < size;) {
        size_t e = std::min(size, b + per);
        if (e < size) {
            const void* nl = memchr(base + e, '\n', size - e);
            e = nl ? (size_t)((const char*)nl - base) + 1 : size;
        }
        ObjRange r;
        r.b = b;
        r.e = e;
        rs.push_back(std::move(r));
        b = e;
    }
    // pass 1: counts
    for_ranges(rs, threads, [&](ObjRange& r) {
        char line[81];
        for (const char* p = base + r.b; p < base + r.e;) {
            const size_t n = chunk_len(p, end);
            chunk_copy(line, p, n);
            p += n;
            if (line[0] == 'v') {
                if (line[1] == 'n') r.nn++;
                else if (line[1] == 't') r.nt++;
                else r.nv++;
            } else if (line[0] == 'f') {
                r.nf++;
            }
        }
    });
    const auto t1 = now();
    int nv = 0, nt = 0, nn = 0, nf = 0;
    std::vector<int> bv(rs.size()), bt(rs.size()), bn(rs.size()), bf(rs.size());
    for (size_t k = 0; k < rs.size(); k++) {
        bv[k] = nv; bt[k] = nt; bn[k] = nn; bf[k] = nf;
        nv += rs[k].nv; nt += rs[k].nt; nn += rs[k].nn; nf += rs[k].nf;
    }
    if (nt) {   // got texture coordinates
        out.uv.assign((size_t)2 * nt, 0.f);
        out.tidx.assign((size_t)3 * nf, 0u);
    }
    out.verts.assign((size_t)nv, v3{0, 0, 0});
    out.normals.assign((size_t)3 * nv + 1, v3{0, 0, 0});
    out.vidx.assign((size_t)3 * nf, 0u);
    out.nidx.assign((size_t)3 * nf, 0u);
    std::vector<uint8_t> own((size_t)nf, 0);   // corners whose normal index the face itself wrote
    const auto t2 = now();
    // pass 2: parse into the slots
    for_ranges(rs, threads, [&](ObjRange& r) {
        const size_t k = (size_t)(&r - rs.data());
        int nverts = bv[k], nnorm = bn[k], ntex = bt[k], ntris = bf[k];
        char line[81];
        for (const char* p = base + r.b; p < base + r.e;) {
            const size_t pos = (size_t)(p - base), len = chunk_len(p, end);
            chunk_copy(line, p, len);
            p += len;
            if (line[0] == 'v') {
                float x = 0, y = 0, z = 0;
                if (line[1] == 'n') {
                    float f3[3];
                    if (fast_floats(&line[2], 3, f3)) { x = f3[0]; y = f3[1]; z = f3[2]; }
                    else sscanf(&line[2], "%f %f %f\n", &x, &y, &z);
                    if (nnorm >= 3 * nv + 1) { r.err_pos = pos; r.err = "too many normals"; return; }
                    out.normals[nnorm++] = normalized(xform_dir(nctm, mk(x, y, z)), RS);
                } else if (line[1] == 't') {
                    float f2[2];
                    if (fast_floats(&line[2], 2, f2)) { x = f2[0]; y = f2[1]; }
                    else sscanf(&line[2], "%f %f\n", &x, &y);
                    out.uv[2 * (size_t)ntex] = x;
                    out.uv[2 * (size_t)ntex + 1] = y;
                    ntex++;
                } else {
                    float f3[3];
                    if (fast_floats(&line[1], 3, f3)) { x = f3[0]; y = f3[1]; z = f3[2]; }
                    else sscanf(&line[1], "%f %f %f\n", &x, &y, &z);
                    out.verts[nverts++] = xform_point(ctm, mk(x, y, z));
                }
            } else if (line[0] == 'f') {
                char tok[3][32];
                tok[0][0] = tok[1][0] = tok[2][0] = 0;
                scan_tokens(&line[1], tok);
                int v = 0, t = 0, n = 0;
                for (int c = 0; c < 3; c++) {
                    split_indices(tok[c], v, t, n);
                    if (v <= 0 || v > nv) { r.err_pos = pos; r.err = "face vertex index out of range"; return; }
                    out.vidx[3 * (size_t)ntris + c] = (uint32_t)(v - 1);
                    if (n) {
                        out.nidx[3 * (size_t)ntris + c] = (uint32_t)(n - 1);
                        own[(size_t)ntris] |= (uint8_t)(1u << c);
                    }
                    if (t && nt) {
                        if (t < 0 || t > nt) { r.err_pos = pos; r.err = "face texture-coordinate index out of range"; return; }
                        out.tidx[3 * (size_t)ntris + c] = (uint32_t)(t - 1);
                    }
                }
                if (!n) r.fn.push_back(ObjRange::FaceNormal{(uint32_t)ntris, (uint32_t)nverts, pos});
                ntris++;
            }
        }
    });
    const auto t3 = now();
    // pass 3: face normals, slot nn = (vn lines) + (earlier such faces)
    size_t err_pos = SIZE_MAX;
    for (const ObjRange& r : rs)
        if (r.err_pos < err_pos) { err_pos = r.err_pos; err = r.err; }
    std::vector<size_t> fbase(rs.size());
    size_t nfn = 0;
    for (size_t k = 0; k < rs.size(); k++) { fbase[k] = nfn; nfn += rs[k].fn.size(); }
    const long slot_lim = std::min<long>((long)nf, 3l * nv);   // nn >= nf || nn >= 3 nv: overflow
    for (size_t k = 0; k < rs.size(); k++) {
        for (size_t i = 0; i < rs[k].fn.size(); i++) {
            if ((long)nn + (long)(fbase[k] + i) >= slot_lim) {   // the first overflowing face (slots only grow)
                if (rs[k].fn[i].pos < err_pos) { err_pos = rs[k].fn[i].pos; err = "face-normal slot overflow"; }
                k = rs.size();
                break;
            }
        }
        if (k == rs.size()) break;
    }
    if (err_pos != SIZE_MAX) return MRT_ERR_IO;
    for_ranges(rs, threads, [&](ObjRange& r) {
        const size_t k = (size_t)(&r - rs.data());
        for (size_t i = 0; i < r.fn.size(); i++) {
            const ObjRange::FaceNormal& F = r.fn[i];
            const uint32_t slot = (uint32_t)((size_t)nn + fbase[k] + i);
            const uint32_t* f = &out.vidx[3 * (size_t)F.tri];
            auto vert = [&](uint32_t j) { return j < F.verts_loaded ? out.verts[j] : v3{0, 0, 0}; };
            const v3 a = vert(f[0]);
            const v3 e1 = sub(vert(f[1]), a);
            const v3 e2 = sub(vert(f[2]), a);
            out.normals[slot] = normalized(cross(e1, e2), RS);
            const uint8_t keep = slot > F.tri ? own[slot] : 0;   // triangle `slot` parsed later keeps its own corners
            for (int c = 0; c < 3; c++)
                if (!((keep >> c) & 1)) out.nidx[3 * (size_t)slot + c] = slot;
        }
    });
    const auto t4 = now();
    if (trace)
        fprintf(stderr, "[mrt] load_obj %s: %zu ranges, %d threads: count %.1f ms, alloc %.1f ms, parse %.1f ms, "
                "face normals %.1f ms\n", path, rs.size(), threads, ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4));
    const int nn_final = nn + (int)nfn;
    out.normals.resize((size_t)std::max(nn_final, 1));
    out.vidx.resize((size_t)3 * nf);
    out.nidx.resize((size_t)3 * nf);
    if (!out.tidx.empty()) out.tidx.resize((size_t)3 * nf);
    for (uint32_t i : out.nidx)
        if (i >= out.normals.size()) { err = "normal index out of range"; return MRT_ERR_IO; }
    return MRT_OK;
}

// ------------------------------------------------------------------ BVH
namespace {

struct Box {
    float mn[3], mx[3];
};
inline Box empty_box() {  // AABB(): bbMin(MIRO_TMAX), bbMax(-MIRO_TMAX), src/Object.h:13
    return Box{{1e12f, 1e12f, 1e12f}, {-1e12f, -1e12f, -1e12f}};
}
inline Box merge(const Box& a, const Box& b) {  // AABB(bb1, bb2), src/Object.h:16-23
    Box r;
    for (int k = 0; k < 3; k++) {
        r.mn[k] = std_min(a.mn[k], b.mn[k]);
        r.mx[k] = std_max(a.mx[k], b.mx[k]);
    }
    return r;
}
inline float area(const Box& b) {  // AABB::getArea, src/Object.h:32-34
    float dx = b.mx[0] - b.mn[0];
    float s = ((dx + b.mx[2]) - b.mn[2]) * (b.mx[1] - b.mn[1]);
    return 2.0f * (s + dx * (b.mx[2] - b.mn[2]));
}
inline float sah(int ln, float la, int rn, float ra) {  // calcSAHCost, src/BVH.cpp:1076-1106
    if (ln + rn >= 32) return ((float)ln) * la + ((float)rn) * ra;
    auto pen = [](int n) { return n % 4 == 0 ? 0.5f : n % 3 == 0 ? 10.f : n % 2 == 0 ? 100.f : 1000.f; };
    return ((float)ln) * la * pen(ln) + ((float)rn) * ra * pen(rn);
}
// cvttss2si: out-of-range / NaN -> INT_MIN
inline int trunc_x86(float f) {
    if (!(f >= -2147483648.0f && f < 2147483648.0f)) return (int)0x80000000u;
    return (int)f;
}

struct BNode {
    Box box;
    int32_t left = -1;   // children are left, left+1
    int32_t start = 0, count = 0;
    bool leaf = false;
};

// Worker threads for the host build: MRT_BUILD_THREADS, else the affinity
// mask capped by OMP_NUM_THREADS (the GPU box's CPU share), at most 64.
int build_threads() {
    if (const char* e = getenv("MRT_BUILD_THREADS")) {
        const int v = atoi(e);
        if (v >= 1) return std::min(v, 64);
    }
    int n = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (const char* e = getenv("OMP_NUM_THREADS")) {
        const int v = atoi(e);
        if (v >= 1) n = std::min(n, v);
    }
    return std::max(1, std::min(n, 64));
}

// Fork-join pool of the host build: run() queues a task under a ticket,
// wait() runs queued tasks until that ticket is done (so nested fork-join never
// blocks a thread).  Workers take the oldest (largest) tasks, a waiting thread
// the newest.
class Pool {
   public:
    struct Ticket {
        std::atomic<bool> done{false};
    };
    explicit Pool(int n) {
        for (int i = 1; i < n; i++) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& w : workers_) w.join();
    }
    int size() const { return (int)workers_.size() + 1; }
    void run(Ticket* t, std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(Item{t, std::move(f)});
        }
        cv_.notify_one();
    }
    void wait(Ticket* t) {
        while (!t->done.load(std::memory_order_acquire)) {
            Item it;
            bool got = false;
            {
                std::lock_guard<std::mutex> g(mu_);
                if (!q_.empty()) { it = std::move(q_.back()); q_.pop_back(); got = true; }
            }
            if (got) exec(it);
            else std::this_thread::yield();
        }
    }

   private:
    struct Item {
        Ticket* t = nullptr;
        std::function<void()> f;
    };
    static void exec(Item& it) {
        it.f();
        it.t->done.store(true, std::memory_order_release);
    }
    void loop() {
        for (;;) {
            Item it;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                it = std::move(q_.front());
                q_.pop_front();
            }
            exec(it);
        }
    }
    std::vector<std::thread> workers_;
    std::deque<Item> q_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
};

// The binned-SAH build, task-parallel with results independent of the thread
// count: a node's two subtrees only read and write their own object ranges, so
// they are built as concurrent tasks (binary-node slots come from an atomic
// arena; the 4-wide collapse numbers nodes and leaves by its own preorder walk,
// so arena order does not matter); the per-node passes over many objects
// (bounds, centroid bounds, bin boxes and counts, bin ids) are split across
// threads with exact reductions (min / max / integer sums); the loose in-place
// partition stays sequential, as its quirk depends on the visit order.
class Builder {
   public:
    // objects (om_[o], ot_[o]) or, where (*oi_)[o] >= 0, ProxyObject (*oi_)[o];
    // the hierarchy goes to nodes / leaves
    Builder(const Scene& s, const std::vector<int32_t>& om, const std::vector<int32_t>& ot,
            const std::vector<int32_t>* oi, std::vector<QNode>& nodes, std::vector<QLeaf>& leaves, int threads)
        : s_(s), om_(om), ot_(ot), oi_(oi), nodes_(nodes), leaves_(leaves), threads_(std::max(1, threads)) {}

    int run(std::string& err) {
        const int n = (int)om_.size();
        std::unique_ptr<Pool> pool;
        if (threads_ > 1 && n >= kTaskMin) pool.reset(new Pool(threads_));
        pool_ = pool.get();
        tri_box_.resize(n);
        cen_obj_.resize((size_t)3 * n);
        objs_.resize(n);
        pre_.resize(n);
        cen_.resize((size_t)3 * n);
        bin_ids_.resize(n);
        par_for(n, [&](int lo, int hi, int) {
            for (int i = lo; i < hi; i++) {
                tri_box_[i] = tri_aabb(i);
                for (int k = 0; k < 3; k++) cen_obj_[3 * i + k] = (tri_box_[i].mn[k] + tri_box_[i].mx[k]) * 0.5f;
                objs_[i] = i;
                pre_[i] = tri_box_[i];
                for (int k = 0; k < 3; k++) cen_[3 * i + k] = cen_obj_[3 * i + k];
            }
        }, true);
        const auto t0 = std::chrono::steady_clock::now();
        bn_.resize((size_t)2 * n + 2);
        bn_next_ = 1;
        build_bin(0, 0, n, 0);
        if (fail_) {
            err = fail_msg_;
            return MRT_ERR_BUILD;
        }
        const auto t1 = std::chrono::steady_clock::now();
        bn_.resize((size_t)bn_next_.load());
        bin_leaves = bin_leaves_.load();
        bin_depth = bin_depth_.load();
        collapse();
        if (getenv("MRT_BUILD_TRACE")) {
            const auto t2 = std::chrono::steady_clock::now();
            fprintf(stderr, "[mrt build] %d objects, %d threads: binary %.1f ms, collapse %.1f ms\n", n, threads_,
                    std::chrono::duration<double, std::milli>(t1 - t0).count(),
                    std::chrono::duration<double, std::milli>(t2 - t1).count());
        }
        return MRT_OK;
    }

    int bin_leaves = 0, bin_depth = 0, q_depth = 0;

   private:
    // objects in a node before its passes are split across threads (the
    // reference's loose partition makes very uneven splits -- 1.09 M -> 2 k + 1.09 M
    // at the buddha root -- so a long chain of large nodes is the critical path)
    static constexpr int kParMin = 1 << 14;
    static constexpr int kTaskMin = 1 << 11;   // objects in a subtree before it becomes its own task

    // fn(lo, hi, chunk) over [0, n) in contiguous chunks, in parallel when n is
    // large and threads are free; chunk c covers [c*n/T, (c+1)*n/T)
    template <typename F>
    int par_for(int n, F fn, bool force = false) {
        int T = 1;
        if (pool_ && (n >= kParMin || (force && n >= 4096))) T = std::min(std::min(threads_, 64), std::max(1, n / 2048));
        if (T <= 1) {
            fn(0, n, 0);
            return 1;
        }
        std::vector<Pool::Ticket> tk(T);
        for (int c = 1; c < T; c++)
            pool_->run(&tk[c], [&, c] { fn((int)((int64_t)n * c / T), (int)((int64_t)n * (c + 1) / T), c); });
        fn(0, (int)((int64_t)n / T), 0);
        for (int c = 1; c < T; c++) pool_->wait(&tk[c]);
        return T;
    }

    bool is_proxy(int o) const { return oi_ && (*oi_)[o] >= 0; }
    // TriangleMesh::getAABB (src/TriangleMesh.cpp:156-195) / ProxyObject::getAABB
    // an MBObject lane: a world triangle of a mesh with time-1 vertices
    bool is_mb(int o) const { return oi_ && !is_proxy(o) && !s_.meshes[om_[o]].verts2.empty(); }
    static Box box3(v3 A, v3 B, v3 C) {
        return Box{{std_min(A.x, std_min(B.x, C.x)), std_min(A.y, std_min(B.y, C.y)), std_min(A.z, std_min(B.z, C.z))},
                   {std_max(A.x, std_max(B.x, C.x)), std_max(A.y, std_max(B.y, C.y)), std_max(A.z, std_max(B.z, C.z))}};
    }
    Box tri_aabb(int o) const {
        if (is_proxy(o)) {
            const float* b = s_.instances[(*oi_)[o]].box;
            return Box{{b[0], b[1], b[2]}, {b[3], b[4], b[5]}};
        }
        const Mesh& m = s_.meshes[om_[o]];
        const uint32_t* f = &m.vidx[3 * (size_t)ot_[o]];
        const Box b = box3(m.verts[f[0]], m.verts[f[1]], m.verts[f[2]]);
        if (!is_mb(o)) return b;
        // MBObject::getAABB: AABB(m_mesh->getAABB(i), m_mesh_t2->getAABB(i)) (src/MBObject.cpp)
        return merge(b, box3(m.verts2[f[0]], m.verts2[f[1]], m.verts2[f[2]]));
    }

    // qsort(objs, n, sizeof(Object*), Object::sortBy{X,Y,Z}Component): glibc msort is
    // stable, so std::stable_sort with the same three-way comparator.
    void sort_by_axis(int start, int n, int axis) {
        const float* c = cen_obj_.data();
        std::stable_sort(objs_.begin() + start, objs_.begin() + start + n,
                         [c, axis](int a, int b) { return c[3 * a + axis] < c[3 * b + axis]; });
    }

    // BVH_Node::buildBin, src/BVH.cpp:625-689
    void build_bin(int node, int start, int n, int depth) {
        if (fail_) return;
        Box b = empty_box();
        {   // the node box: std::min / std::max merges are exact, so chunked partial boxes merge to the same box
            Box part[64];
            const int T = par_for(n, [&](int lo, int hi, int c) {
                Box q = empty_box();
                for (int i = lo; i < hi; i++) q = merge(q, tri_box_[objs_[start + i]]);
                part[c] = q;
            });
            for (int c = 0; c < T; c++) b = merge(b, part[c]);
        }
        bn_[node].box = b;
        if (n <= 4) {
            bn_[node].leaf = true;
            bn_[node].start = start;
            bn_[node].count = n;
            bin_leaves_++;
            return;
        }
        int d = bin_depth_.load();
        while (depth + 1 > d && !bin_depth_.compare_exchange_weak(d, depth + 1)) {}
        unsigned part = 0;
        partition(start, n, part);
        if (fail_) return;
        unsigned ln = part + 1u, rn = (unsigned)n - part - 1u;
        if (ln == 0u || rn == 0u || ln > (unsigned)n) {
            fail("BVH partition produced an empty side (reference would recurse forever)");
            return;
        }
        const int32_t l = bn_next_.fetch_add(2);
        bn_[node].left = l;
        // the left subtree as a task of its own while a thread is free
        if (pool_ && (int)ln >= kTaskMin) {
            Pool::Ticket t;
            pool_->run(&t, [=] { build_bin(l, start, (int)ln, depth + 1); });
            build_bin(l + 1, start + (int)ln, (int)rn, depth + 1);
            pool_->wait(&t);
        } else {
            build_bin(l, start, (int)ln, depth + 1);
            build_bin(l + 1, start + (int)ln, (int)rn, depth + 1);
        }
    }

    // BVH_Node::partitionSweepBin, src/BVH.cpp:691-901
    void partition(int start, int n, unsigned& partPt) {
        float best = INFINITY;
        unsigned bestAxis = 0;
        int binPart = 0;
        int* objs = objs_.data() + start;
        Box* pre = pre_.data() + start;
        float* cen = cen_.data() + 3 * (size_t)start;
        if (n >= 128) {
            Box bb = empty_box();
            {
                Box part[64];
                const int T = par_for(n, [&](int lo, int hi, int c) {
                    Box q = empty_box();
                    for (int i = lo; i < hi; i++)
                        for (int k = 0; k < 3; k++) {
                            q.mn[k] = std_min(q.mn[k], cen[3 * i + k]);
                            q.mx[k] = std_max(q.mx[k], cen[3 * i + k]);
                        }
                    part[c] = q;
                });
                for (int c = 0; c < T; c++)
                    for (int k = 0; k < 3; k++) {
                        bb.mn[k] = std_min(bb.mn[k], part[c].mn[k]);
                        bb.mx[k] = std_max(bb.mx[k], part[c].mx[k]);
                    }
            }
            float len[3] = {bb.mx[0] - bb.mn[0], bb.mx[1] - bb.mn[1], bb.mx[2] - bb.mn[2]};
            bool any = false;
            for (int axis = 0; axis < 3; axis++) {
                // Reference UB guard: a zero extent gives kl = inf and NaN bins.
                if (!(len[axis] > 0.0f)) continue;
                any = true;
                float kl = (float)8 * (1.0f - 0.001f) / len[axis], ko = bb.mn[axis];
                Box bins[8];
                int cnt[8] = {0};
                for (int i = 0; i < 8; i++) bins[i] = empty_box();
                {
                    Box pb[64][8];
                    int pc[64][8];
                    std::atomic<bool> bad{false};
                    const int T = par_for(n, [&](int lo, int hi, int c) {
                        Box lb[8];   // this chunk's bins, local: published once (no shared lines in the loop)
                        int lc[8] = {0};
                        for (int j = 0; j < 8; j++) lb[j] = empty_box();
                        for (int i = lo; i < hi; i++) {
                            int id = trunc_x86(kl * (cen[3 * i + axis] - ko));
                            if (id < 0 || id > 7) { bad = true; return; }
                            lb[id] = merge(lb[id], pre[i]);
                            lc[id]++;
                        }
                        for (int j = 0; j < 8; j++) { pb[c][j] = lb[j]; pc[c][j] = lc[j]; }
                    });
                    if (bad) { fail("bin id out of range"); return; }
                    for (int c = 0; c < T; c++)
                        for (int j = 0; j < 8; j++) { bins[j] = merge(bins[j], pb[c][j]); cnt[j] += pc[c][j]; }
                }
                float la[8], ra[8];
                Box acc = empty_box();
                for (int i = 0; i < 7; i++) { acc = merge(acc, bins[i]); la[i] = area(acc); }
                acc = empty_box();
                int rnum = 0;
                for (int i = 7; i > 0; i--) {
                    rnum += cnt[i];
                    acc = merge(acc, bins[i]);
                    ra[i] = area(acc);
                    float c = sah(n - rnum, la[i - 1], rnum, ra[i]);
                    if (c < best) { best = c; binPart = i; bestAxis = (unsigned)axis; }
                }
            }
            if (!any) { partPt = (unsigned)(n / 2 - 1); return; }
            float kl = (float)8 * (1.0f - 0.001f) / len[bestAxis], ko = bb.mn[bestAxis];
            int* ids = bin_ids_.data() + start;   // this node's own range of the scratch
            par_for(n, [&](int lo, int hi, int) {
                for (int i = lo; i < hi; i++) ids[i] = trunc_x86(kl * (cen[3 * i + bestAxis] - ko));
            });
            // Loose in-place partition, src/BVH.cpp:769-792 (ids are NOT swapped).
            if (pool_ && n >= kParMin) { loose_partition_par(start, n, ids, binPart, partPt); return; }
            int rev = n - 1;
            for (int i = 0; i < n; i++) {
                if (ids[i] < binPart) continue;
                while (rev >= 0 && ids[rev] >= binPart) rev--;
                if (rev <= i) { partPt = (unsigned)(i - 1); return; }
                std::swap(pre[i], pre[rev]);
                for (int k = 0; k < 3; k++) std::swap(cen[3 * i + k], cen[3 * rev + k]);
                std::swap(objs[i], objs[rev]);
                rev--;
            }
            return;
        }
        // Small nodes: full sweep per axis, src/BVH.cpp:794-899.
        float la[128], ra[128];
        for (int axis = 0; axis < 3; axis++) {
            sort_by_axis(start, n, axis);
            Box acc = empty_box();
            la[0] = INFINITY;
            for (int i = 1; i < n; i++) { acc = merge(acc, tri_box_[objs[i]]); la[i] = area(acc); }
            acc = empty_box();
            ra[n - 1] = INFINITY;
            for (int i = n - 2; i >= 0; i--) {
                acc = merge(acc, tri_box_[objs[i]]);
                ra[i] = area(acc);
                float c = sah(i + 1, la[i], n - i - 1, ra[i]);
                if (c < best) { best = c; partPt = (unsigned)i; bestAxis = (unsigned)axis; }
            }
        }
        if (bestAxis < 2) sort_by_axis(start, n, (int)bestAxis);
    }

    // The loose partition in parallel.  The ids are never swapped, so the
    // reference's sweep is fixed by the static id array: the k-th position with
    // id >= binPart from the left (B_k) swaps objects with the k-th position
    // with id < binPart from the right (S_k) while S_k > B_k; the sweep stops
    // at the first B_K without such a partner (S_K <= B_K, or none left) with
    // partPt = B_K - 1, and leaves partPt as it was when no B_K is left.  The
    // pairs are disjoint, so the swaps run in parallel.
    void loose_partition_par(int start, int n, const int* ids, int binPart, unsigned& partPt) {
        int* objs = objs_.data() + start;
        Box* pre = pre_.data() + start;
        float* cen = cen_.data() + 3 * (size_t)start;
        const int T = std::min(threads_, 64);
        std::vector<int> nb(T + 1, 0), ns(T + 1, 0);
        auto lo_of = [&](int c) { return (int)((int64_t)n * c / T); };
        std::vector<Pool::Ticket> tk(T);
        auto each = [&](auto fn) {
            for (int c = 1; c < T; c++) pool_->run(&tk[c], [&, c] { fn(c); });
            fn(0);
            for (int c = 1; c < T; c++) { pool_->wait(&tk[c]); tk[c].done = false; }
        };
        each([&](int c) {
            int b = 0;
            for (int i = lo_of(c); i < lo_of(c + 1); i++) b += ids[i] >= binPart;
            nb[c + 1] = b;
            ns[c + 1] = (lo_of(c + 1) - lo_of(c)) - b;
        });
        for (int c = 0; c < T; c++) { nb[c + 1] += nb[c]; ns[c + 1] += ns[c]; }
        const int NB = nb[T], NS = ns[T];
        std::vector<int> B(NB), S(NS);   // B ascending; S descending (k-th small from the right)
        each([&](int c) {
            int b = nb[c], sm = NS - 1 - ns[c];
            for (int i = lo_of(c); i < lo_of(c + 1); i++) {
                if (ids[i] >= binPart) B[b++] = i;
                else S[sm--] = i;
            }
        });
        int lo = 0, hi = std::min(NB, NS);   // K = first k with S_k <= B_k (monotone in k)
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (S[mid] <= B[mid]) hi = mid; else lo = mid + 1;
        }
        const int K = lo;
        each([&](int c) {
            const int k0 = (int)((int64_t)K * c / T), k1 = (int)((int64_t)K * (c + 1) / T);
            for (int k = k0; k < k1; k++) {
                const int i = B[k], r = S[k];
                std::swap(pre[i], pre[r]);
                for (int a = 0; a < 3; a++) std::swap(cen[3 * i + a], cen[3 * r + a]);
                std::swap(objs[i], objs[r]);
            }
        });
        if (K < NB) partPt = (unsigned)(B[K] - 1);
    }

    // QBVH_Node::build, src/BVH.cpp:100-389 -- preorder node numbering, leaf
    // packets numbered in creation order (nodeNum).  Two passes so subtrees can
    // be built in parallel into their own index ranges: count() gives every
    // binary node that roots a 4-wide node the size of its 4-wide subtree, then
    // qbuild() fills node qi from binary node b with the children in the
    // reference's slot order, handing each child subtree the index ranges a
    // sequential preorder walk would give it.
    void init_node(int32_t qi) {
        QNode q{};
        for (int k = 0; k < 4; k++) q.child[k] = kEmptySlot;
        nodes_[qi] = q;
    }
    void set_box(int32_t qi, int slot, int32_t b) {
        const Box& x = bn_[b].box;
        float* box = nodes_[qi].box;
        box[0 + slot] = x.mn[0]; box[4 + slot] = x.mn[1]; box[8 + slot] = x.mn[2];
        box[12 + slot] = x.mx[0]; box[16 + slot] = x.mx[1]; box[20 + slot] = x.mx[2];
    }
    // buildTriBundle, src/BVH.cpp:64-98: a ProxyObject lane keeps a zero
    // triangle (checkOut lane, rejected by det = 0)
    void make_leaf(int32_t li, int32_t b) {
        QLeaf L{};
        for (int i = 0; i < 4; i++) L.prim[i] = -1;
        for (int i = 0; i < bn_[b].count; i++) {
            int o = objs_[bn_[b].start + i];
            L.prim[i] = o;
            if (is_proxy(o) || is_mb(o)) continue;   // checkOut lanes: no triangle data
            const Mesh& m = s_.meshes[om_[o]];
            const uint32_t* f = &m.vidx[3 * (size_t)ot_[o]];
            v3 A = m.verts[f[0]], B = m.verts[f[1]], C = m.verts[f[2]];
            L.t[0 + i] = A.x; L.t[4 + i] = A.y; L.t[8 + i] = A.z;
            L.t[12 + i] = B.x - A.x; L.t[16 + i] = B.y - A.y; L.t[20 + i] = B.z - A.z;
            L.t[24 + i] = C.x - A.x; L.t[28 + i] = C.y - A.y; L.t[32 + i] = C.z - A.z;
        }
        leaves_[li] = L;
    }
    // slot assignment of a 4-wide node built from binary node b: (slot, binary
    // node) in the order the reference fills them; returns the count
    int slots(int32_t b, int32_t (&sl)[4], int32_t (&bb)[4]) const {
        const BNode& n = bn_[b];
        if (n.leaf) { sl[0] = 0; bb[0] = b; return 1; }   // only the root can be a leaf
        const int32_t c0 = n.left, c1 = n.left + 1;
        const bool l0 = bn_[c0].leaf, l1 = bn_[c1].leaf;
        if (l0 && l1) { sl[0] = 0; bb[0] = c0; sl[1] = 1; bb[1] = c1; return 2; }
        if (l0) {   // leaf, then child 1's two children in slots 1, 2
            const int32_t g0 = bn_[c1].left;
            sl[0] = 0; bb[0] = c0; sl[1] = 1; bb[1] = g0; sl[2] = 2; bb[2] = g0 + 1;
            return 3;
        }
        if (l1) {   // child 0's two children in slots 0, 1, leaf in slot 2 -- the leaf is filled first
            const int32_t g0 = bn_[c0].left;
            sl[0] = 2; bb[0] = c1; sl[1] = 0; bb[1] = g0; sl[2] = 1; bb[2] = g0 + 1;
            return 3;
        }
        const int32_t g[4] = {bn_[c0].left, bn_[c0].left + 1, bn_[c1].left, bn_[c1].left + 1};
        for (int k = 0; k < 4; k++) { sl[k] = k; bb[k] = g[k]; }
        return 4;
    }
    // pass 1: 4-wide nodes / leaf packets of the subtree of binary node b (b roots a 4-wide node)
    void count(int32_t b, int depth) {
        int32_t sl[4], bb[4];
        const int k = slots(b, sl, bb);
        Pool::Ticket tk[4];
        bool spawned[4] = {false, false, false, false};
        for (int i = 0; i < k; i++) {
            if (bn_[bb[i]].leaf) continue;
            if (pool_ && depth < 5) { spawned[i] = true; pool_->run(&tk[i], [=] { count(bb[i], depth + 1); }); }
            else count(bb[i], depth + 1);
        }
        int32_t nn = 1, nl = 0;
        for (int i = 0; i < k; i++) {
            if (bn_[bb[i]].leaf) { nl++; continue; }
            if (spawned[i]) pool_->wait(&tk[i]);
            nn += qn_[bb[i]];
            nl += ql_[bb[i]];
        }
        qn_[b] = nn;
        ql_[b] = nl;
    }
    // pass 2: node qi from binary node b; its child nodes start at index nb, leaves at lb
    void qbuild(int32_t qi, int32_t b, int depth, int32_t nb, int32_t lb) {
        int d = q_depth_.load();
        while (depth > d && !q_depth_.compare_exchange_weak(d, depth)) {}
        init_node(qi);
        int32_t sl[4], bb[4];
        const int k = slots(b, sl, bb);
        for (int i = 0; i < k; i++) set_box(qi, sl[i], bb[i]);
        Pool::Ticket tk[4];
        bool spawned[4] = {false, false, false, false};
        for (int i = 0; i < k; i++) {
            const int32_t g = bb[i];
            if (bn_[g].leaf) {
                nodes_[qi].child[sl[i]] = ~lb;
                make_leaf(lb++, g);
                continue;
            }
            const int32_t c = nb, cn = nb + 1, cl = lb;
            nodes_[qi].child[sl[i]] = c;
            nb += qn_[g];
            lb += ql_[g];
            if (pool_ && depth < 6) { spawned[i] = true; pool_->run(&tk[i], [=] { qbuild(c, g, depth + 1, cn, cl); }); }
            else qbuild(c, g, depth + 1, cn, cl);
        }
        for (int i = 0; i < k; i++)
            if (spawned[i]) pool_->wait(&tk[i]);
    }
    void collapse() {
        qn_.assign(bn_.size(), 0);
        ql_.assign(bn_.size(), 0);
        count(0, 0);
        nodes_.resize((size_t)qn_[0]);
        leaves_.resize((size_t)ql_[0]);
        qbuild(0, 0, 1, 1, 0);
        q_depth = q_depth_.load();
    }

    void fail(const char* m) {
        std::lock_guard<std::mutex> g(fail_mu_);
        if (!fail_) fail_msg_ = m;
        fail_ = true;
    }

    const Scene& s_;
    const std::vector<int32_t>& om_;
    const std::vector<int32_t>& ot_;
    const std::vector<int32_t>* oi_;
    std::vector<QNode>& nodes_;
    std::vector<QLeaf>& leaves_;
    const int threads_;
    std::vector<Box> tri_box_, pre_;
    std::vector<float> cen_obj_, cen_;
    std::vector<int> objs_, bin_ids_;
    std::vector<BNode> bn_;
    std::atomic<int32_t> bn_next_{1};
    std::atomic<int> bin_leaves_{0}, bin_depth_{0}, q_depth_{0};
    Pool* pool_ = nullptr;
    std::vector<int32_t> qn_, ql_;   // collapse: QBVH nodes / leaf packets of the 4-wide subtree rooted at a binary node
    std::atomic<bool> fail_{false};
    std::mutex fail_mu_;
    std::string fail_msg_;

   public:
    int32_t bin_nodes() const { return (int32_t)bn_.size(); }
};

}  // namespace

// Scene::preCalc -> BVH::build, src/Scene.cpp:62-79 + src/BVH.cpp:457-575.
int build_qbvh(Scene& s, std::string& err) {
    auto t0 = std::chrono::steady_clock::now();
    for (Mesh& m : s.meshes) mesh_tangents(m);   // TriangleMesh::preCalc (texture-mapped meshes)
    s.obj_mesh.clear();
    s.obj_tri.clear();
    s.obj_inst.clear();
    // world objects in add order: a world mesh's triangles (makeMeshObjs), a ProxyObject
    for (int32_t g : s.groups) {
        if (g >= 0) {
            if (s.mesh_blas[g] >= 0) continue;
            for (int32_t t = 0; t < s.meshes[g].nt(); t++) {
                s.obj_mesh.push_back(g);
                s.obj_tri.push_back(t);
                s.obj_inst.push_back(-1);
            }
        } else {
            s.obj_mesh.push_back(-1);
            s.obj_tri.push_back(-1);
            s.obj_inst.push_back(~g);
        }
    }
    if (s.obj_mesh.empty()) {
        err = "scene has no triangles";
        return MRT_ERR_BUILD;
    }
    // instance hit ids follow the world objects; every id must fit mrt_hit.prim
    // (int32) -- the reference's 201 x 201 proxy grid (src/main.cpp:37-51) of a
    // >53k-triangle BLAS would not
    int64_t base = (int64_t)s.obj_mesh.size();
    for (Instance& I : s.instances) {
        if (base > (int64_t)INT32_MAX) break;
        I.hit_base = (int32_t)base;
        base += (int64_t)s.blas[I.blas].obj_mesh.size();
    }
    if (base - 1 > (int64_t)INT32_MAX) {
        err = "world objects + instances x BLAS objects exceed 2^31 hit ids (" + std::to_string(base) + ")";
        return MRT_ERR_INVALID;
    }
    Builder b(s, s.obj_mesh, s.obj_tri, &s.obj_inst, s.nodes, s.leaves, build_threads());
    int rc = b.run(err);
    if (rc != MRT_OK) return rc;
    auto t1 = std::chrono::steady_clock::now();
    s.info.nodes = (int32_t)s.nodes.size();
    s.info.leaves = (int32_t)s.leaves.size();
    s.info.prims = (int32_t)s.obj_mesh.size();
    s.info.bin_nodes = b.bin_nodes();
    s.info.bin_leaves = b.bin_leaves;
    s.info.max_depth = b.q_depth;
    s.info.build_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    s.built = true;
    s.dev_dirty = true;
    return MRT_OK;
}

// ProxyObject::setupMultiProxy (src/ProxyObject.cpp:149-167) + BVH::build
int make_blas(Scene& s, const int32_t* meshes, int n_meshes, std::string& err) {
    if (!meshes || n_meshes <= 0) { err = "no meshes"; return MRT_ERR_INVALID; }
    Blas B;
    for (int j = 0; j < n_meshes; j++) {
        const int32_t m = meshes[j];
        if (m < 0 || m >= (int32_t)s.meshes.size() || s.mesh_blas[m] >= 0 || std::count(meshes, meshes + j, m)) {
            err = "bad mesh id, or the mesh already belongs to a BLAS";
            return MRT_ERR_INVALID;
        }
        B.meshes.push_back(m);
        for (int32_t t = s.meshes[m].nt() - 1; t >= 0; t--) {
            B.obj_mesh.push_back(m);
            B.obj_tri.push_back(t);
        }
    }
    if (B.obj_mesh.empty()) { err = "BLAS has no triangles"; return MRT_ERR_BUILD; }
    Builder b(s, B.obj_mesh, B.obj_tri, nullptr, B.nodes, B.leaves, build_threads());
    const int rc = b.run(err);
    if (rc != MRT_OK) return rc;
    const int32_t id = (int32_t)s.blas.size();
    for (int32_t m : B.meshes) s.mesh_blas[m] = id;
    s.blas.push_back(std::move(B));
    s.built = false;
    s.dev_dirty = true;
    return id;
}

// new ProxyObject(objects, bvh, M) with its ProxyMatrix (src/ProxyObject.cpp:5-12,
// src/ProxyMatrix.cpp:3-8) and ProxyObject::getAABB (src/ProxyObject.cpp:45-72):
// the BLAS root box (QBVH_Node::getAABB: the union of all four slots, unused ones
// included as zero boxes, src/BVH.cpp:107-112,416-424), corners A..F, bbMin,
// bbMax through multiplyAndDivideByW, grown in that order.
int add_instance(Scene& s, int32_t blas, const float* m16, std::string& err) {
    if (!m16 || blas < 0 || blas >= (int32_t)s.blas.size()) { err = "bad BLAS id or matrix"; return MRT_ERR_INVALID; }
    Instance I{};
    Mat4 M;
    memcpy(M.m, m16, sizeof M.m);
    const Mat4 inv = inverse(M), inv_t = transpose(inverse(M));
    memcpy(I.m, M.m, sizeof I.m);
    memcpy(I.inv, inv.m, sizeof I.inv);
    memcpy(I.inv_t, inv_t.m, sizeof I.inv_t);
    I.blas = blas;
    const QNode& r = s.blas[blas].nodes[0];
    Box t = empty_box();
    for (int k = 0; k < 4; k++)
        t = merge(t, Box{{r.box[0 + k], r.box[4 + k], r.box[8 + k]}, {r.box[12 + k], r.box[16 + k], r.box[20 + k]}});
    const v3 P[8] = {mk(t.mn[0], t.mn[1], t.mx[2]), mk(t.mn[0], t.mx[1], t.mn[2]), mk(t.mx[0], t.mn[1], t.mn[2]),
                     mk(t.mn[0], t.mx[1], t.mx[2]), mk(t.mx[0], t.mx[1], t.mn[2]), mk(t.mx[0], t.mn[1], t.mx[2]),
                     mk(t.mn[0], t.mn[1], t.mn[2]), mk(t.mx[0], t.mx[1], t.mx[2])};
    Box nb = empty_box();
    for (const v3& p : P) {
        const v3 q = xform_point(M, p);
        nb = merge(nb, Box{{q.x, q.y, q.z}, {q.x, q.y, q.z}});
    }
    for (int k = 0; k < 3; k++) {
        I.box[k] = nb.mn[k];
        I.box[3 + k] = nb.mx[k];
    }
    s.instances.push_back(I);
    s.groups.push_back(~(int32_t)(s.instances.size() - 1));
    s.built = false;
    s.dev_dirty = true;
    return (int)s.instances.size() - 1;
}

}  // namespace mrt
