// mrt_bin.h -- ray binning: a permutation of a ray batch that puts rays of
// similar direction and origin next to each other, so the 64 lanes of a trace
// wave walk nearly the same nodes (incoherent dome / GI / path rays).
//
// Each ray is traced on its own with the reference's tests, so the order in
// which a trace kernel takes its rays changes no answer, no visit count and no
// pixel; it only changes which rays share a wave.  The key is a counting-sort
// key of at most kBinBits bits: the octahedral cell of the direction (dbits per
// axis, major) and the Morton code of the origin's cell in the scene box (obits
// per axis, minor).  Three launches: per-block LDS histograms (+ the key per
// ray), one exclusive scan of the bins, a block-aggregated scatter.  Rays of a
// bin keep approximately their slot order (pixel order), which adds image-space
// locality within a bin.  Invalid slots (past a pixel's ray count) are dropped:
// the permutation lists valid rays only and `total` counts them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrt_types.h"

namespace mrt {

static constexpr int kBinBits = 12;                 // at most 4096 bins (16 KB LDS histogram)
static constexpr uint16_t kBinInvalid = 0xFFFFu;

struct BinArgs {
    const float4* o;          // ray i: origin o[i] (w unused), direction d[i]
    const float4* d;
    // items: n, or with a device count  min(n, min(cap1, *n_dev * mul1 - sub) * mul2)
    uint32_t n;
    const uint32_t* n_dev;
    uint32_t mul1, sub, cap1, mul2;
    const uint8_t* nrays;     // slot i valid iff i % m < nrays[i / m] (null: every item is valid)
    uint32_t m;
    float lo[3], inv[3];      // origin cell = (o - lo) * inv, clamped to [0, 2^obits)
    int dbits, obits;         // 2 * dbits + 3 * obits <= kBinBits
    // instance-major keys (instanced scenes' shadow rays): a ray whose pixel's primary hit
    // lies on ProxyObject instance i gets key 1 << 11 | inst_class[i] << 4 | direction cell
    // (inst_class: instances ranked by BLAS, then index, scaled to 7 bits), so the rays a
    // wave (and an XCD's band) traces leave the same instance and walk one BLAS first;
    // other rays keep the direction / origin-cell key below 1 << 11.  null: plain keys.
    const float4* hits;       // per pixel slot (ray i's pixel = i / m): t, a, b, prim bits
    const int32_t* hit_base;  // per instance: its first hit id (ascending)
    const uint16_t* inst_class;
    int32_t n_inst, n_world;
    // object-space keys (bin_inst 2): 1 << 11 | BLAS bit << 10 | the Morton code of the ray
    // origin's cell in its BLAS's box (4 cells per axis, in object space: the same region of
    // one BLAS across every instance of it) << 4 | direction cell.  Per instance two float4:
    // (BLAS box lo, BLAS bit), (4 / box extent, 0); the world -> object matrices from insts.
    const float4* inst_cell;
    const DevInstance* insts;
    int bits;                 // key bits (set by bin_rays)
    uint16_t* keys;           // [n] scratch
    uint32_t* hist;           // [2^bits + 1] scratch; word 2^bits receives the valid count
    uint32_t* perm;           // [n] out: valid rays, binned
};

// The three launches on `stream` (grid: workgroups of the count / scatter
// passes).  A.hist must hold 2^bits + 1 words.
int bin_rays(const BinArgs& A, int grid, hipStream_t stream);

}  // namespace mrt
