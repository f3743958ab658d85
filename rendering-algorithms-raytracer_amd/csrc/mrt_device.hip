// mrt_device.hip -- kernels + C-ABI of libmrt (MI355X / gfx950).
//
// Render kernel: persistent workgroups of 4 waves; a wave renders one 8x8
// pixel tile per step (one lane per pixel), so a wave's rays are coherent.
// Per lane: camera ray (Camera::eyeRayAdaptive, src/Camera.cpp:116-157) ->
// closest-hit traversal -> Lambert/Blinn shading (src/Lambert.cpp:19-53,
// src/Blinn.cpp:91-237) with PointLight / RectangleLight shadow rays traced
// any-hit (same occlusion boolean as the reference's closest-hit shadow rays)
// -> float RGB (+ Image::Map 8-bit).  The rcp/rsqrt tables (8 KB) and the
// traversal stacks live in LDS.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "mrt_bin.h"
#include "mrt_kernels.h"
#include "mrt_scene.h"
#include "mrt_texture.h"
#include "mrt_shader.h"

namespace mrt {

static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }

#define HIP_OK(expr)                                                                    \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));               \
            return MRT_ERR_HIP;                                                         \
        }                                                                               \
    } while (0)

// Kernel 2b: every wavefront shadow ray of the frame, any-hit (the occlusion
// answer of Shader::occluded).  Slots past a pixel's ray count are skipped.
//   sched 0: grid-stride, one ray per lane per iteration.
//   sched 1: XCD bands -- the ray slots are cut into 8 contiguous bands (slot
//            order is pixel order, so a band is a band of the image) and
//            workgroup b, which runs on XCD b mod 8, takes 64-slot chunks of band
//            b mod 8 from that band's counter, then steals from the others: the
//            rays one XCD traces touch the geometry of one image band, so its
//            4 MB L2 holds that band's share of the hierarchy.
//   sched 2: sched 1 + lane refill: a lane whose ray is done (an any-hit ray
//            ends at its first accepted triangle) or whose slot is empty takes
//            a new slot as soon as `refill_min` lanes of its wave are idle;
//            traversal runs one node visit per wave step (anyhit_step; in
//            special-leaf scenes anyhit_step_inst, which defers ProxyObject
//            lanes onto the stack), so the wave no longer waits for its longest
//            ray.
// Every ray is traced with traverse()'s box and triangle tests (the same
// visit order, except the deferred instance walks of sched 2, which an
// any-hit answer does not depend on), so the answers are identical under
// every schedule.
static constexpr int kShadowChunk = 64;
// REFILL: sched 2 (its own kernel, so the chunked schedules' nested traversal
// does not set its register budget); CHECK: the lane-refill step of a
// special-leaf scene handles alpha-mapped / motion-blurred lanes.
template <bool COUNT, bool FAST, bool INST, bool REFILL, bool CHECK, int MINW = 1>
__global__ void __launch_bounds__(kWG, MINW) shadow_kernel(RenderParams P, size_t n_rays, int sched, int refill_min) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    load_tables(P.tables, s_tab, 1024);
    const int tid = threadIdx.x, lane = tid & 63;
    Trav T{P.nodes, P.fast_box != 0, P.scalar_nodes, P.leaves, s_tab, s_stack + tid,
           P.gstack + (blockIdx.x * kWG + tid), P.gstride};
    T.inst = P.insts;
    trav_alpha(T, P);
    TravStats st;
    unsigned long long wave_steps = 0;
    if (P.ch_ovf && *P.ch_ovf) return;   // a chain chunk past its estimated capacity (redone by its fallback)
    // chain levels: the entry count is on the device (n_rays is the capacity)
    if (P.sh_count) {
        const size_t nd = (size_t)*P.sh_count * (size_t)P.max_shadow;
        if (nd < n_rays) n_rays = nd;
    }
    // binned order (mrt_bin.h): position c traces slot perm[c]; the list holds valid slots only
    const uint32_t* perm = P.sh_perm;
    if (perm) n_rays = *P.sh_perm_n;
    // slot e = pixel slot * max_shadow + j (n_rays < 2^32, checked on the host: 32-bit division)
    const uint32_t m = (uint32_t)P.max_shadow, nr32 = (uint32_t)n_rays;
    auto valid = [&](size_t e64) {
        if (perm) return e64 < n_rays;
        // m through an empty asm: the division's reciprocal is formed here, per dequeue, instead of
        // once before the loop and held across the walk (it was the kernel's one spilled value)
        uint32_t mm = m;
        asm volatile("" : "+s"(mm));
        const uint32_t e = (uint32_t)e64, px = e / mm;
        return e64 < n_rays && e < nr32 && e - px * m < (uint32_t)P.nrays[px];
    };
    auto slot_at = [&](size_t c) -> size_t { return perm ? (size_t)perm[c] : c; };
    auto trace_one = [&](size_t e) __attribute__((always_inline)) {   // (inlined: see chain_trace_kernel)
        const float4 o = P.ray_o[e], d = P.ray_d[e];
        const DRay r = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), d.w);
        DHit h{o.w, 0.f, 0.f, -1};
        const uint32_t n0 = st.nodes;
        P.occl[e] = traverse<true, COUNT, FAST, INST, CHECK, false, !INST>(T, r, 0.001f, h, st) ? 1 : 0;
        return st.nodes - n0;
    };
    // per-XCD band of ray slots and its chunk counter (own 128-B line)
    const int home = blockIdx.x & 7;
    auto band_lo = [&](int k) { return n_rays * (size_t)k / 8; };
    int band = home, probes = 0;
    // wave-level dequeue of `want` consecutive slots of the current band (or
    // the next band with slots left); returns the first slot (lane 0's atomic,
    // broadcast) and the end of its band, or exhausted
    auto dequeue = [&](uint32_t want, size_t& first, size_t& end) {
        unsigned long long got = ~0ull, hi = 0;
        if (lane == 0) {
            while (probes < 8) {
                const size_t lo = band_lo(band), bend = band_lo(band + 1);
                const unsigned long long v = atomicAdd(reinterpret_cast<unsigned long long*>(P.queue + band * 32),
                                                       (unsigned long long)want);
                if (lo + v < bend) { got = lo + v; hi = bend; break; }
                band = (band + 1) & 7;
                probes++;
            }
        }
        got = __shfl(got, 0);
        hi = __shfl(hi, 0);
        first = (size_t)got;
        end = (size_t)hi;
        return got != ~0ull;
    };
    if constexpr (!REFILL) {
        if (sched == 0) {
            for (size_t e0 = (size_t)blockIdx.x * kWG + (tid & ~63); e0 < n_rays; e0 += (size_t)gridDim.x * kWG) {
                const size_t e = e0 + lane;
                uint32_t v = valid(e) ? trace_one(slot_at(e)) : 0u;
                if (COUNT) {
                    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor(v, off));
                    wave_steps += v;
                }
            }
        } else {   // XCD bands: wave-uniform chunks, one ray per lane
            size_t first, end;
            while (dequeue(kShadowChunk, first, end)) {
                const size_t e = first + lane;
                uint32_t v = (e < end && valid(e)) ? trace_one(slot_at(e)) : 0u;
                if (COUNT) {
                    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor(v, off));
                    wave_steps += v;
                }
            }
        }
    } else {   // lane refill
        bool exhausted = false;   // wave-uniform
        bool active = false;
        uint32_t e = 0;   // the lane's ray slot (n_rays < 2^32, checked on the host): one VGPR, not two
        float tmax = 0.f;
        AnyState as{};
        for (;;) {
            const unsigned long long idle = __ballot(!active);
            const int nidle = __popcll(idle);
            if (!exhausted && (nidle >= refill_min || nidle == 64)) {
                size_t first, end;
                if (!dequeue((uint32_t)nidle, first, end)) {
                    exhausted = true;
                } else if (!active) {
                    const size_t c = first + (size_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                    if (c < end && valid(c)) {
                        e = (uint32_t)slot_at(c);
                        const float4 o = P.ray_o[e], d = P.ray_d[e];
                        as.q = make_ray(mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), d.w);
                        tmax = o.w;
                        as.cur = 0;
                        as.sp = 0;
                        as.aoff = -1;
                        active = true;
                    }
                }
            }
            if (__ballot(active) == 0) {
                if (exhausted) break;
                continue;
            }
            if (COUNT) wave_steps++;
            if (active) {
                bool hit = false;
                bool done;
                if constexpr (INST) done = anyhit_step_inst<COUNT, FAST, CHECK>(T, 0.001f, tmax, as, P.ray_o, P.ray_d, e, hit, st);
                else done = (FAST && as.q.finite) ? anyhit_step<COUNT, true>(T, as.q, 0.001f, tmax, as.cur, as.sp, hit, st)
                                                  : anyhit_step<COUNT, false>(T, as.q, 0.001f, tmax, as.cur, as.sp, hit, st);
                if (done) {
                    P.occl[e] = hit ? 1 : 0;
                    active = false;
                }
            }
        }
    }
    if (COUNT) {
        unsigned long long nv = st.nodes, lv = st.leaves;
        for (int off = 32; off > 0; off >>= 1) {
            nv += __shfl_down(nv, off);
            lv += __shfl_down(lv, off);
        }
        if (lane == 0) {
            atomicAdd(&P.ctr[CTR_NODES], nv);
            atomicAdd(&P.ctr[CTR_LEAVES], lv);
            atomicAdd(&P.ctr[CTR_NODES_S], nv);
            atomicAdd(&P.ctr[CTR_WAVE_STEPS_S], wave_steps);
        }
    }
    if (st.overflow) atomicOr(&P.ctr[CTR_OVERFLOW], 1ull);
}


// Numerics probe (mrt_debug_libm): the device's acosf / atan2f / sinf / cosf / powf
// (mrt_libm.h) and rcp_nr (RCPSS emulation + Newton step, mrt_math.h; table from global
// memory).
__global__ void __launch_bounds__(256) libm_kernel(int fn, const float* x, const float* y, size_t n, float* out,
                                                   const uint16_t* rcpT) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        out[i] = fn == 0 ? fd_acosf(x[i]) : fn == 1 ? fd_atan2f(y[i], x[i]) : fn == 2 ? rcp_nr(x[i], rcpT)
               : fn == 3 ? gl_sinf(x[i]) : fn == 4 ? gl_cosf(x[i]) : gl_powf(x[i], y[i]);
}

// Batched Scene::trace: one lane per query ray.
template <bool ANY, bool INST = false>
__global__ void __launch_bounds__(kWG) trace_kernel(const QNode* nodes, const DLeaf* leaves, const uint16_t* tables,
                                                    int32_t* gstack, uint32_t gstride, const float* o, const float* d,
                                                    const float* tmin, const float* tmax, size_t n, mrt_hit* out,
                                                    unsigned long long* ctr, int fast_box,
                                                    const DevInstance* insts, Trav alpha) {
    __shared__ uint16_t s_tab[2048];
    __shared__ int32_t s_stack[kLdsStack * kWG];
    const int tid = threadIdx.x;
    for (int i = tid; i < 1024; i += kWG) reinterpret_cast<uint32_t*>(s_tab)[i] = reinterpret_cast<const uint32_t*>(tables)[i];
    __syncthreads();
    const uint32_t gtid = blockIdx.x * kWG + tid;
    Trav T{nodes, fast_box != 0, false, leaves, s_tab, s_stack + tid, gstack + gtid, gstride};
    T.inst = insts;
    T.aprims = alpha.aprims; T.apuv = alpha.apuv; T.auv = alpha.auv; T.amats = alpha.amats; T.atex = alpha.atex;
    T.pflags = alpha.pflags; T.verts = alpha.verts; T.verts2 = alpha.verts2;   // Ray time 0 (src/Ray.h:71)
    TravStats st;
    for (size_t i = (size_t)blockIdx.x * kWG + tid; i < n; i += (size_t)gridDim.x * kWG) {
        DRay r = make_ray(mk(o[3 * i], o[3 * i + 1], o[3 * i + 2]), mk(d[3 * i], d[3 * i + 1], d[3 * i + 2]));
        DHit h{tmax[i], 0.f, 0.f, -1};
        bool hit = traverse<ANY, false, false, INST>(T, r, tmin[i], h, st);
        mrt_hit res;
        res.t = h.t; res.a = h.a; res.b = h.b; res.prim = hit ? (ANY ? 0 : h.prim) : -1;
        res.inst = (hit && !ANY) ? h.inst : -1;
        if (ANY && hit) res.prim = 1;  // any-hit: occluded flag only
        out[i] = res;
    }
    if (st.overflow) atomicOr(&ctr[CTR_OVERFLOW], 1ull);
}

// Bucket tiles -> frames.  Item id = frame * buckets_per_frame + bucket; frame f
// of the output starts at f * W * H pixels.  Float tiles (nullable) go to
// `frames`; 8-bit pixels come from tiles8 when given, else from the LUT.
// One 256-thread workgroup per item (a 32x32 tile), a thread per 4 consecutive
// pixels of a tile row: 48 B of float RGB as three 16-B loads and stores and 12 B
// of 8-bit RGB as three dword stores when the frame width is a multiple of 4
// and the buffers are 16-B / 4-B aligned (every 4-pixel group then is too);
// otherwise, and for groups the frame's right edge cuts, pixel by pixel.
__global__ void __launch_bounds__(256) unpack_kernel(const int32_t* items, int32_t n_items, const float* tiles,
                                                     const uint8_t* tiles8, int32_t W, int32_t H, int32_t buckets_x,
                                                     int32_t buckets_per_frame, int32_t n_frames, float* frames,
                                                     uint8_t* frames8, const uint8_t* gamma) {
    const int bslot = blockIdx.x;
    if (bslot >= n_items) return;
    const uint32_t id = (uint32_t)items[bslot];
    const uint32_t f = id / (uint32_t)buckets_per_frame, b = id % (uint32_t)buckets_per_frame;
    const int row = threadIdx.x >> 3, px = (threadIdx.x & 7) * 4;
    const int x = (int)(b % buckets_x) * 32 + px, y = (int)(b / buckets_x) * 32 + row;
    if (f >= (uint32_t)n_frames || x >= W || y >= H) return;  // ids outside the batch are ignored
    const size_t i = (size_t)bslot * 1024 + (size_t)(row * 32 + px);   // first pixel of the group in the tiles
    const size_t q = (size_t)f * W * H + (size_t)y * W + x;            // ... and in the frames
    const bool aligned = (((uintptr_t)tiles | (uintptr_t)frames) & 15) == 0 && (((uintptr_t)tiles8 | (uintptr_t)frames8) & 3) == 0;
    if ((W & 3) == 0 && aligned) {   // x + 3 < W: the whole group, aligned
        float v[12];
        if (tiles) {
            const float4* t4 = reinterpret_cast<const float4*>(tiles + 3 * i);
            const float4 a = t4[0], c = t4[1], d = t4[2];
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y;
            v[6] = c.z; v[7] = c.w; v[8] = d.x; v[9] = d.y; v[10] = d.z; v[11] = d.w;
            if (frames) {
                float4* o4 = reinterpret_cast<float4*>(frames + 3 * q);
                o4[0] = a; o4[1] = c; o4[2] = d;
            }
        }
        if (frames8) {
            uint32_t w[3];
            if (tiles8) {
                const uint32_t* t = reinterpret_cast<const uint32_t*>(tiles8 + 3 * i);
                w[0] = t[0]; w[1] = t[1]; w[2] = t[2];
            } else {
                uint32_t c8[12];
#pragma unroll
                for (int k = 0; k < 12; k++) c8[k] = map8(gamma, v[k]);
#pragma unroll
                for (int k = 0; k < 3; k++)
                    w[k] = c8[4 * k] | c8[4 * k + 1] << 8 | c8[4 * k + 2] << 16 | c8[4 * k + 3] << 24;
            }
            uint32_t* o = reinterpret_cast<uint32_t*>(frames8 + 3 * q);
            o[0] = w[0]; o[1] = w[1]; o[2] = w[2];
        }
        return;
    }
    for (int k = 0; k < 4 && x + k < W; k++) {
        const size_t ik = i + k, qk = q + k;
        if (tiles && frames) {
            frames[3 * qk] = tiles[3 * ik]; frames[3 * qk + 1] = tiles[3 * ik + 1]; frames[3 * qk + 2] = tiles[3 * ik + 2];
        }
        if (frames8) {
            if (tiles8) {
                frames8[3 * qk] = tiles8[3 * ik]; frames8[3 * qk + 1] = tiles8[3 * ik + 1];
                frames8[3 * qk + 2] = tiles8[3 * ik + 2];
            } else {
                frames8[3 * qk] = map8(gamma, tiles[3 * ik]); frames8[3 * qk + 1] = map8(gamma, tiles[3 * ik + 1]);
                frames8[3 * qk + 2] = map8(gamma, tiles[3 * ik + 2]);
            }
        }
    }
}

// ------------------------------------------------------------------ device state
// Launch scratch of one stream: everything a render / trace launch writes
// besides the caller's outputs.  Two launches on different streams never share
// one, so frames can overlap (the tail of one persistent launch with the start
// of the next).
struct StreamCtx {
    hipStream_t stream = nullptr;
    int32_t* gstack = nullptr;               // traversal-stack spill columns
    unsigned long long* ctr = nullptr;       // statistics + tile counters
    unsigned long long* wave_log = nullptr;  // 2 launches x grid x 4 waves x kLogWords u64 (diagnostics)
    int log_waves[2] = {0, 0};               // waves of the last logged primary / shade launch
    float4* hitbuf = nullptr;                // kernel 1 -> kernel 2 hand-off (per output slot)
    size_t hit_slots = 0;
    float4* rays = nullptr;                  // wavefront shadow rays: origin+tMax | direction
    uint8_t* occl = nullptr;                 // per ray: occluded
    uint8_t* nrays = nullptr;                // per output slot: rays written
    size_t ray_cap = 0, nrays_cap = 0;
    float* lvl = nullptr;                    // REC kernels: chain level records (RenderParams::lvl)
    size_t lvl_cap = 0;                      //   floats
    void* chain = nullptr;                   // wavefront chain engine scratch (mrt_chain.hip)
    size_t chain_bytes = 0;
    uint64_t chain_budget = 0;               // the chunk budget of its last chain-engine frame (bytes)
    uint32_t chain_chunks = 0;               //   and the chunks that frame ran
    void* adapt = nullptr;                   // chain-engine adaptive supersampling: means, pixel lists, unit colours
    size_t adapt_bytes = 0;
    // chain level capacities: per pass index (adapt_n, 0 = no supersampling) and level, the
    // largest entries per path a chunk on this stream needed (x 65536, + 1; 0 = not seen,
    // all ones = unknown) -- on the device (atomicMax by chain_merge), its last copy on the
    // host (pinned, in flight until est_ev), and the host's view used to size chunks
    uint32_t* est_dev = nullptr;
    uint32_t* est_pinned = nullptr;
    hipEvent_t est_ev = nullptr;
    bool est_pending = false;
    std::vector<uint32_t> est;
    bool last_was_render = false;
    bool fused = false;                      // the last render ran frame1_kernel (one launch)
    bool chain_used = false;                 // the last render's shading ran the wavefront chain engine
    uint16_t* bin_keys = nullptr;            // ray binning (mrt_bin.h): per-ray keys, two permutations
    uint32_t* bin_perm = nullptr;            //   [2][bin_cap] (0: shadow rays, 1: chain closest-hit entries)
    uint32_t* bin_hist = nullptr;            //   [2][kBinHist] bins + valid count
    size_t bin_cap = 0;
    float4* ray_e = nullptr;                 // dome-light replay (RenderParams::ray_e / lrec)
    uint32_t* lrec = nullptr;
    size_t ray_e_cap = 0, lrec_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evm = nullptr;
};
static constexpr int kMaxStreamCtx = 16;

// persistent buffers of one bucket share of mrt_render over several devices
struct ShareBuf {
    int32_t* items = nullptr;
    float* tiles = nullptr;
    size_t items_cap = 0, tiles_cap = 0;
    hipEvent_t done = nullptr;   // the share's tiles are in the caller's gather buffer
};

struct DeviceState {
    int device = -1;
    QNode* nodes = nullptr;
    DLeaf* leaves = nullptr;
    PrimShade* prims = nullptr;
    float4* verts = nullptr;
    float4* normals = nullptr;
    DevMaterial* mats = nullptr;
    DevLight* lights = nullptr;
    DevDome* domes = nullptr;
    DevInstance* insts = nullptr;
    int n_insts = 0, n_world = 0;
    int32_t* inst_hit_base = nullptr;   // per instance: hit_base (ascending), for the instance-major bin keys
    uint16_t* inst_class = nullptr;     //   and its 7-bit class (BLAS-major rank)
    float4* inst_cell = nullptr;        //   object-space bin cells: BLAS box lo + BLAS bit, 4 / extent (2 per instance)
    DevTexture* texs = nullptr;   // material-map textures (bufs hold their data)
    uint4* puv = nullptr;         // per prim texture-coordinate indices (nullptr: no texture-mapped mesh)
    float2* uvs = nullptr;
    float4* tans = nullptr;       // per normal: tangent / bitangent (texture-mapped meshes)
    float4* btans = nullptr;
    bool has_maps = false, has_alpha = false;
    uint8_t* pflags = nullptr;    // motion blur: per world prim bit 0 = MBObject lane
    float4* verts2 = nullptr;     //   time-1 vertices parallel to verts (copies of verts for static meshes)
    bool has_mb = false;
    bool special = false;         // instances, alpha maps or motion blur: leaf packets with special lanes (INST kernels)
    std::vector<void*> bufs;     // textures and dome tables (freed with the state)
    const float* env = nullptr;  // environment texture (one of bufs)
    uint16_t* tables = nullptr;
    uint8_t* gamma = nullptr;
    float* gammaF = nullptr;
    uint32_t gthreads = 0;
    // scratch for the synchronous API
    float* d_rgb = nullptr;
    uint8_t* d_rgb8 = nullptr;
    size_t frame_px = 0;
    int grid = 0;                // upper bound of any launch (kMaxBlocksPerCU per CU)
    bool boxes_finite = false;
    bool boxes_ordered = false;  // every used slot box has lo <= hi per axis (octant-ordered box test)
    bool lds_ok = false;         // the world hierarchy has kLdsNodes nodes for the LDS top-node walk (renumbered)
    std::atomic<int> lds_pick{-1};   // the last one-light frame ran the LDS top-node walk: 1 yes, 0 no, -1 none yet
    float bb_lo[3] = {0, 0, 0}, bb_hi[3] = {0, 0, 0};   // world root box (ray-binning origin cells)
    int cus = 0;
    bool point_only = false;
    bool dome = false;           // a dome light (incoherent shadow rays)
    int recursive = 0;           // chain shading (Shader REC): 1 reflection / refraction, 2 + path tracing
    bool disperse = false;       // a dispersive Blinn material with secondary rays: the fused (tree) engine
    bool transparent = false;    // a rect / dome light with transparent shadows: fused kernels only
    bool pow_spec = false;       // a Blinn material with specExp != 1 (frame1 / shade1 kernels with pow)
    int wall_khz = 0;            // wall_clock64() rate
    size_t bytes = 0;
    // per-stream launch scratch: frames on different streams are in flight at once
    std::mutex mu;
    std::vector<StreamCtx*> ctxs;
    StreamCtx* last = nullptr;   // context of the most recent launch (stats, wave log)
    std::vector<hipStream_t> share_streams;  // mrt_render over several devices: one stream per bucket share
    std::vector<ShareBuf*> share_bufs;       //   and its persistent item / tile buffers (+ copy-done event)
    hipStream_t gather_stream = nullptr;     //   the caller's device: frame assembly stream,
    float* g_tiles = nullptr;                //   every share's tiles gathered here,
    int32_t* g_items = nullptr;              //   their bucket ids
    size_t g_tiles_cap = 0, g_items_cap = 0;
};

// Tuning knobs (mrt_set_tuning): A/B switches for performance work.
static int g_fast_box = 1;        // hardware min/max box test when its precondition holds
static int g_primary_waves = 7;   // launch-bounds occupancy target of the primary kernel: 0 (none), 6, 7, 8
// shade1_kernel (the two-launch one-light shading) runs at 5 waves: 96 VGPRs, -2.5% vs 6 (round 2)
static int g_sched = 2;           // TileSched mode 0..3 (2 measured fastest)
static int g_batch_tpw = 2;       // bucket batches: tiles per wave the launch's grid is sized for when the batch is
                                  // smaller than the persistent grid (a 1/4 or 1/8 split share): 2 -- C3 share model
                                  // 2.98 -> 3.17x at N = 4, 4.69 -> 4.74x at N = 8; 4: 3.99x at N = 8
                                  // (profiles/r04_share_tpw_ab.txt)
static int g_wave_log = 0;        // 1: timing-only wave log on uninstrumented launches (diagnostics)
static int g_scalar_nodes = 7;    // scalar-cache fetch of wave-uniform nodes (bit 0) and triangles (bit 1); bit 2:
                                  // octant-ordered box test for waves whose rays share an octant (box_test_oct)
static int g_shade1 = 1;          // specialised shade kernel for one point light and one path
static int g_wavefront = 1;       // general shading: gen / trace / resolve kernels instead of one fused kernel
static int g_shadow_sched = -1;   // shadow_kernel schedule: 0 grid-stride, 1 XCD bands, 2 bands + lane refill,
                                  // -1 auto: refill for dome-light (incoherent) rays, else bands
// shadow_kernel's launch-bounds occupancy target is 8 waves (C4 / C5 -5.5% against none)
static int g_primary_inst_waves = 5;   // primary kernel of special-leaf scenes: 1 (none), 5, 6 (r02: 6 beat 1 by 5% on C5;
                                       // r03: 5 = 6 within 0.3% with binned shadow rays, and 96 VGPRs spill less)
// the resolve pass (kernel 2c) of dome-light scenes runs at 4 waves (D1 -4%, C5 -1.2 ms against none;
// special-leaf scenes at 3, without scratch);
// the direct-lighting adaptive kernel at 6 (unbounded it takes 256 VGPRs: A3 30.7 -> 12.8 ms)
static int g_adapt_refill = 32;   // adaptive_kernel pixel refill: idle lanes that trigger a dequeue (0: tiles; 32: A3 -13%)
static int g_chain_shadow_step = 0;   // instanced chain levels: shadow rays walk with anyhit_step_inst (deferred proxies)
// chain_trace_kernel of plain scenes runs at 8 waves (P4 -17%, R3 -3.5% against none)
static int g_near_first = -1;     // any-hit walks take the nearest hit child first: 0 off, 1 on, -1 auto
                                  // (auto: on in the chunked shadow kernel of plain scenes only -- C4 shade
                                  // -12.6%; off in the refill one, C5 +4.5%, the instanced chunked one,
                                  // C5 +15%, and the fused kernels, C3 +5%, A3 / R3 +2%)
static constexpr int kRefillMin = 40;   // lane refill: idle lanes of a wave that trigger a dequeue
static int g_chain_shadow_refill = 0;   // instanced chain levels: shadow rays on the lane-refill kernel (FS: 6% slower, profiles/r04_fs_chain_shadow_refill_ab.txt)
static int g_chain = 1;           // REC scenes: wavefront chain engine (mrt_chain.hip) instead of the fused kernel
static int g_chain_est = 1;       // chain levels sized by the entries earlier chunks needed (0: worst case, 3^ceil(k/2))
static int g_chain_est_pct = 125; //   headroom over the largest count per path seen, percent
static int g_chain_mb = 8192;     // chain scratch per stream (MB), at most 80% of the device's free memory; larger frames
                                  // run in chunks of work items.  With estimated level capacities 8 GB costs G3 3% against
                                  // 48 GB and R3 / P4 / FS nothing (profiles/r04_chain_mb_est_ab.txt)
static int g_fused = 1;           // one point light, one path: frame1_kernel (primary + shading in one launch)
static int g_walk_exit = 1;       // the walk loop of frame1_kernel / primary_kernel: 1 one exit (a stack overflow
                                  // empties the stack and leaves at the pop test), 0 two (the overflow returns).
                                  // One exit issues 19% fewer SALU per wave step (C3 -7%, C4 -6%); round 5's
                                  // 12-16% loss on the bunny scenes was the frame latency of a few heavy
                                  // top-row tiles with only 4 frames in flight (walk exit), gone
                                  // with 8 hardware queues: one exit everywhere, no probe (round 6)
static int g_walk_latch = 1;      // frame1_kernel's camera-ray walk: 1 one latch (the popping lanes pick their next node
                                  // by select in the same step), 0 nested (two latches: lanes that pop wait for the
                                  // wave's longest descent).  Round-6 A/B (profiles/r06_walk_latch_ab.txt): one latch
                                  // C2 -11%, C3L -4.4%, C3 +1.5%; config C3 runs 0 (miro/scenes.py)
static int g_lds_nodes = 0;       // frame1_kernel's LDS top-node walk (LN), 0 off / 1 on: with 4 frames in flight C2
                                  // -4.1%, C3 +9%, C3L +11% (profiles/r05_lds_nodes_ab_*.txt); no probe separated them
                                  // reliably (single-frame kernel times are equal on C2), so it is off unless asked for
static int g_frame1_waves = 7;    // frame1_kernel launch-bounds occupancy target: 1 (none), 5..8 (7: -0.9% per frame with
                                  // 4 frames in flight, +0.8% single-frame latency; profiles/r03_c3_scalar_waves_ab.txt)
static int g_bin = -1;            // ray binning (mrt_bin.h) before tracing: bit 0 the wavefront shadow pass (kernel 2b),
                                  // bit 1 the chain levels' closest-hit entries, bit 2 the chain levels' shadow rays;
                                  // -1 auto (bin_mode): chain levels of path-traced scenes (P4 -18% frame; the
                                  // coherent mirror / glass levels of R3 / G3 lose their pixel order: +22% / +44%)
                                  // and the dome shadow rays of instanced scenes, in the frame shadow pass (C5 -2.6%;
                                  // D1 +2%) and in the chain levels (FS -29% per frame, profiles/r04_fs_bin_ab.txt),
                                  // and the chain levels' shadow rays of dispersive scenes, whose three refraction
                                  // children per split diverge (G3 -5% with 4 frames in flight; R3's coherent
                                  // mirror levels +7%: off; profiles/r04_g3_bin_ab.txt)
static int g_chain_bands = -1;    // chain_trace_kernel: XCD-banded chunk queue (binned rays: one XCD's L2 holds its share);
                                  // -1 auto: on when the level is binned (P4 -3.4%; unbinned R3 +5.7%, G3 +3%)
static int g_dome_replay = 1;      // dome-light resolve (2c) sums 2a's recorded samples instead of sampling again
static int g_bin_inst = 0;        // off: C5 shade pass +0.8% (profiles/r04_c5_bin_inst_primary_waves_ab.txt); instanced scenes' shadow-ray bins: instance-major keys (the ray's origin instance, BLAS-major)
static constexpr int kBinBlocks = 4;   // binning launches: workgroups per CU (each reserves its range of every bin atomically)
static int g_bin_dbits = 2;       // binning key: direction cells per octahedral axis = 2^dbits
static int g_bin_obits = 2;       //   origin cells per scene-box axis = 2^obits (2 dbits + 3 obits <= 12);
                                  //   sweep of 12 pairs: (2, 2) best on P4 (-18%) and C5 (-2.6%), finer
                                  //   direction cells lose (P4 (6, 0) -11%), profiles/r03_bin_sweep.txt

static inline int fast_box(const DeviceState& d);

static void free_ctx(StreamCtx* c) {
    void* ptrs[] = {c->gstack, c->ctr, c->wave_log, c->hitbuf, c->rays, c->occl, c->nrays, c->lvl, c->chain,
                    c->adapt, c->bin_keys, c->bin_perm, c->bin_hist, c->ray_e, c->lrec};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->est_dev) (void)hipFree(c->est_dev);
    if (c->est_pinned) (void)hipHostFree(c->est_pinned);
    if (c->est_ev) (void)hipEventDestroy(c->est_ev);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->evm) (void)hipEventDestroy(c->evm);
    delete c;
}

static void free_device(DeviceState* d) {
    if (!d) return;
    if (d->device >= 0) (void)hipSetDevice(d->device);
    (void)hipDeviceSynchronize();   // no launch may still use the scratch below
    for (StreamCtx* c : d->ctxs) free_ctx(c);
    for (hipStream_t st : d->share_streams) (void)hipStreamDestroy(st);
    if (d->gather_stream) (void)hipStreamDestroy(d->gather_stream);
    for (ShareBuf* b : d->share_bufs) {
        if (b->items) (void)hipFree(b->items);
        if (b->tiles) (void)hipFree(b->tiles);
        if (b->done) (void)hipEventDestroy(b->done);
        delete b;
    }
    if (d->g_tiles) (void)hipFree(d->g_tiles);
    if (d->g_items) (void)hipFree(d->g_items);
    void* ptrs[] = {d->nodes, d->leaves, d->prims, d->verts, d->normals, d->mats, d->lights, d->domes, d->insts,
                    d->inst_hit_base, d->inst_class, d->inst_cell, d->tables,
                    d->gamma, d->gammaF, d->d_rgb, d->d_rgb8, d->texs, d->puv, d->uvs, d->tans, d->btans,
                    d->pflags, d->verts2};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (void* p : d->bufs)
        if (p) (void)hipFree(p);
    delete d;
}

// Scratch context of `stream` (created on first use, at most kMaxStreamCtx).
static int get_ctx(DeviceState& d, hipStream_t stream, StreamCtx*& out) {
    std::lock_guard<std::mutex> g(d.mu);
    for (StreamCtx* c : d.ctxs)
        if (c->stream == stream) { out = c; return MRT_OK; }
    if ((int)d.ctxs.size() >= kMaxStreamCtx) { set_error("too many streams on one scene (max 16)"); return MRT_ERR_INVALID; }
    StreamCtx* c = new StreamCtx();
    c->stream = stream;
    d.ctxs.push_back(c);   // owned by d from here (freed with it even if an allocation below fails)
    HIP_OK(hipMalloc((void**)&c->gstack, (size_t)kGlobalStack * d.gthreads * sizeof(int32_t)));
    HIP_OK(hipMalloc((void**)&c->ctr, kCtrBytes));
    HIP_OK(hipMalloc((void**)&c->wave_log, (size_t)2 * d.grid * (kWG / 64) * kLogWords * sizeof(unsigned long long)));
    HIP_OK(hipEventCreate(&c->ev0));
    HIP_OK(hipEventCreate(&c->ev1));
    HIP_OK(hipEventCreate(&c->evm));
    out = c;
    return MRT_OK;
}

template <typename T>
static int upload(T*& dst, const void* src, size_t bytes, size_t& total) {
    HIP_OK(hipMalloc((void**)&dst, bytes ? bytes : 16));
    if (bytes) HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    total += bytes;
    return MRT_OK;
}

static int upload_scene(Scene& s, DeviceState& d, int device);

static void free_replicas(Scene& s) {
    for (DeviceState* d : s.devs) free_device(d);
    s.devs.clear();
    s.dev = nullptr;
}

// The scene's replica on `device` (uploaded on first use; all replicas are
// dropped when the host scene changed) becomes s.dev.
static int ensure_device(Scene& s, int device) {
    if (!s.built) { set_error("scene not built"); return MRT_ERR_NOT_BUILT; }
    if (s.dev_dirty) { free_replicas(s); s.dev_dirty = false; }
    for (DeviceState* d : s.devs)
        if (d->device == device) { s.dev = d; return MRT_OK; }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) { set_error("no HIP device"); return MRT_ERR_NO_DEVICE; }
    if (device < 0 || device >= n) { set_error("bad device ordinal"); return MRT_ERR_INVALID; }
    if (s.lights.size() > (size_t)kMaxLights) { set_error("too many lights"); return MRT_ERR_INVALID; }
    DeviceState* d = new DeviceState();
    const int rc = upload_scene(s, *d, device);
    if (rc) { free_device(d); return rc; }
    s.devs.push_back(d);
    s.dev = d;
    return MRT_OK;
}

static int upload_scene(Scene& s, DeviceState& d, int device) {
    d.device = device;
    HIP_OK(hipSetDevice(device));
    // shading arrays: concatenate meshes
    std::vector<float4> V, N;
    std::vector<uint32_t> vbase(s.meshes.size()), nbase(s.meshes.size());
    for (size_t m = 0; m < s.meshes.size(); m++) {
        vbase[m] = (uint32_t)V.size();
        nbase[m] = (uint32_t)N.size();
        for (auto& p : s.meshes[m].verts) V.push_back(make_float4(p.x, p.y, p.z, 1.f));
        for (auto& p : s.meshes[m].normals) N.push_back(make_float4(p.x, p.y, p.z, 0.f));
    }
    // PrimShade: the world objects (a ProxyObject's own slot stays zero), then each BLAS's objects
    auto shade_rec = [&](int32_t mesh, int32_t tri) {
        PrimShade p{};
        if (mesh < 0) return p;
        const Mesh& m = s.meshes[mesh];
        const size_t t = (size_t)tri;
        for (int k = 0; k < 3; k++) {
            p.v[k] = vbase[mesh] + m.vidx[3 * t + k];
            p.n[k] = nbase[mesh] + m.nidx[3 * t + k];
        }
        p.mat = (uint32_t)m.material;
        return p;
    };
    // texture coordinates of texture-mapped meshes: (u, v) pairs, per-prim indices,
    // per-normal tangent frames (TriangleMesh::preCalc, host_texture.cpp)
    bool any_uv = false;
    for (const Mesh& m : s.meshes) any_uv |= !m.tidx.empty();
    std::vector<float2> UV;
    std::vector<float4> TN, BTN;
    std::vector<uint32_t> ubase(s.meshes.size(), 0);
    if (any_uv) {
        TN.assign(N.size(), make_float4(0.f, 0.f, 0.f, 0.f));
        BTN.assign(N.size(), make_float4(0.f, 0.f, 0.f, 0.f));
        for (size_t m = 0; m < s.meshes.size(); m++) {
            const Mesh& M = s.meshes[m];
            ubase[m] = (uint32_t)UV.size();
            if (M.tidx.empty()) continue;
            for (size_t i = 0; i + 1 < M.uv.size(); i += 2) UV.push_back(make_float2(M.uv[i], M.uv[i + 1]));
            for (size_t i = 0; i < M.tan.size(); i++) {
                TN[nbase[m] + i] = make_float4(M.tan[i].x, M.tan[i].y, M.tan[i].z, 0.f);
                BTN[nbase[m] + i] = make_float4(M.btan[i].x, M.btan[i].y, M.btan[i].z, 0.f);
            }
        }
    }
    auto uv_rec = [&](int32_t mesh, int32_t tri) {
        uint4 u = make_uint4(0u, 0u, 0u, 0u);
        if (mesh < 0 || s.meshes[mesh].tidx.empty()) return u;
        const uint32_t* t = &s.meshes[mesh].tidx[3 * (size_t)tri];
        return make_uint4(ubase[mesh] + t[0], ubase[mesh] + t[1], ubase[mesh] + t[2], 1u);
    };
    std::vector<PrimShade> PS;
    std::vector<uint4> PUV;
    for (size_t i = 0; i < s.obj_mesh.size(); i++) {
        PS.push_back(shade_rec(s.obj_mesh[i], s.obj_tri[i]));
        if (any_uv) PUV.push_back(uv_rec(s.obj_mesh[i], s.obj_tri[i]));
    }
    std::vector<int32_t> shade_base(s.blas.size());
    for (size_t b = 0; b < s.blas.size(); b++) {
        shade_base[b] = (int32_t)PS.size();
        for (size_t i = 0; i < s.blas[b].obj_mesh.size(); i++) {
            PS.push_back(shade_rec(s.blas[b].obj_mesh[i], s.blas[b].obj_tri[i]));
            if (any_uv) PUV.push_back(uv_rec(s.blas[b].obj_mesh[i], s.blas[b].obj_tri[i]));
        }
    }
    // materials with maps; world leaf packets holding alpha-mapped triangles
    d.has_maps = false;
    std::vector<char> alpha_mat(s.materials.size(), 0);
    for (size_t m = 0; m < s.materials.size(); m++) {
        const int32_t* mp = s.materials[m].maps;
        d.has_maps |= mp[kMapColor] >= 0 || mp[kMapNormal] >= 0 || mp[kMapSpecular] >= 0 || mp[kMapReflect] >= 0 ||
                      mp[kMapRefract] >= 0;
        alpha_mat[m] = mp[kMapAlpha] >= 0;
    }
    auto alpha_obj = [&](int32_t p) {
        return p >= 0 && (size_t)p < s.obj_mesh.size() && s.obj_mesh[p] >= 0 &&
               alpha_mat[(size_t)s.meshes[s.obj_mesh[p]].material];
    };
    // MBObject world triangles (meshes with time-1 vertices)
    auto mb_obj = [&](int32_t p) {
        return p >= 0 && (size_t)p < s.obj_mesh.size() && s.obj_mesh[p] >= 0 &&
               (s.obj_inst.empty() || s.obj_inst[(size_t)p] < 0) && !s.meshes[s.obj_mesh[p]].verts2.empty();
    };
    std::vector<uint8_t> PF(s.obj_mesh.size(), 0);
    d.has_mb = false;
    for (size_t i = 0; i < PF.size(); i++)
        if (mb_obj((int32_t)i)) { PF[i] = 1; d.has_mb = true; }
    d.has_alpha = false;
    std::vector<uint16_t> tab(4096);
    memcpy(tab.data(), host_rcp_table(), 4096);
    memcpy(tab.data() + 2048, host_rsqrt_table(), 4096);
    size_t total = 0;
    int rc;
    // device node / leaf arrays: the world hierarchy, then each BLAS (indices
    // offset).  Leaf slots carry their packet's object count and a ProxyObject
    // bit (leaf_child); a ProxyObject lane's prim is -2 - instance.
    size_t n_leaves = s.leaves.size();
    for (const Blas& B : s.blas) n_leaves += B.leaves.size();
    if (n_leaves >= (size_t(1) << 27)) { set_error("too many leaf packets"); return MRT_ERR_OVERFLOW; }
    std::vector<QNode> DN;
    std::vector<DLeaf> DL;
    auto append = [&](const std::vector<QNode>& nodes, const std::vector<QLeaf>& leaves,
                      const std::vector<int32_t>* oi, const Blas* B) -> int32_t {
        const int32_t nb = (int32_t)DN.size(), lb = (int32_t)DL.size();
        auto proxy_of = [&](int32_t p) { return (oi && p >= 0 && (size_t)p < oi->size()) ? (*oi)[p] : -1; };
        for (QNode q : nodes) {
            for (int k = 0; k < 4; k++) {
                const int32_t c = q.child[k];
                if (c == kEmptySlot) continue;
                if (c >= 0) { q.child[k] = c + nb; continue; }
                const QLeaf& L = leaves[(size_t)~c];
                int cnt = 0;
                bool proxy = false, alpha = false;
                for (int j = 0; j < 4; j++)
                    if (L.prim[j] >= 0) {  // zero-filled lanes below cnt are rejected by det = 0
                        cnt = j + 1;
                        proxy |= proxy_of(L.prim[j]) >= 0;
                        alpha |= oi != nullptr && proxy_of(L.prim[j]) < 0 &&
                                 (alpha_obj(L.prim[j]) || mb_obj(L.prim[j]));   // world: alpha / motion blur
                        alpha |= B != nullptr && (size_t)L.prim[j] < B->obj_mesh.size() &&
                                 alpha_mat[(size_t)s.meshes[B->obj_mesh[(size_t)L.prim[j]]].material];   // BLAS: alpha
                    }
                d.has_alpha |= alpha;
                q.child[k] = leaf_child((uint32_t)(~c + lb), cnt < 1 ? 1 : cnt, proxy, alpha);
            }
            DN.push_back(q);
        }
        for (const QLeaf& L : leaves) {
            DLeaf D{};
            for (int k = 0; k < 4; k++) {
                for (int c = 0; c < 9; c++) D.tri[k][c] = L.t[4 * c + k];
                const int32_t pi = proxy_of(L.prim[k]);
                D.prim[k] = pi >= 0 ? -2 - pi : L.prim[k];
            }
            DL.push_back(D);
        }
        return nb;
    };
    append(s.nodes, s.leaves, &s.obj_inst, nullptr);
    std::vector<int32_t> blas_root(s.blas.size());
    for (size_t b = 0; b < s.blas.size(); b++) blas_root[b] = append(s.blas[b].nodes, s.blas[b].leaves, nullptr, &s.blas[b]);
    // The world hierarchy's first kLdsNodes nodes in breadth-first order get device
    // numbers 0 .. kLdsNodes - 1 (frame1_kernel<LN> stages them in LDS).  Device node
    // numbers are internal: the visit order follows the child slots, not the numbers.
    const size_t nw = s.nodes.size();
    d.lds_ok = nw >= (size_t)kLdsNodes;
    if (d.lds_ok) {
        // (an imported hierarchy may share a node between parents: each is numbered once)
        std::vector<int32_t> bfs{0};
        std::vector<int32_t> perm(DN.size(), -1);
        perm[0] = 0;
        for (size_t q = 0; q < bfs.size() && bfs.size() < (size_t)kLdsNodes; q++)
            for (int k = 0; k < 4 && bfs.size() < (size_t)kLdsNodes; k++) {
                const int32_t ch = DN[(size_t)bfs[q]].child[k];
                if (ch >= 0 && (size_t)ch < nw && perm[(size_t)ch] < 0) {
                    perm[(size_t)ch] = (int32_t)bfs.size();
                    bfs.push_back(ch);
                }
            }
        d.lds_ok = bfs.size() == (size_t)kLdsNodes;
        int32_t next = (int32_t)bfs.size();
        for (size_t i = 0; i < nw; i++)
            if (perm[i] < 0) perm[i] = next++;
        for (size_t i = nw; i < DN.size(); i++) perm[i] = (int32_t)i;
        std::vector<QNode> R(DN.size());
        for (size_t i = 0; i < DN.size(); i++) {
            QNode q = DN[i];
            for (int k = 0; k < 4; k++)
                if (q.child[k] >= 0) q.child[k] = perm[(size_t)q.child[k]];
            R[(size_t)perm[i]] = q;
        }
        DN.swap(R);
        for (int32_t& br : blas_root) br = perm[(size_t)br];
    }
    for (QNode& q : DN) q.pad[0] = slot_kinds(q.child);   // the walks read the slot kinds (node_kinds)
    if ((rc = upload(d.nodes, DN.data(), DN.size() * sizeof(QNode), total))) return rc;
    std::vector<DevInstance> DI(s.instances.size());
    for (size_t i = 0; i < DI.size(); i++) {
        const Instance& I = s.instances[i];
        memcpy(DI[i].inv, I.inv, sizeof DI[i].inv);
        memcpy(DI[i].inv_t, I.inv_t, sizeof DI[i].inv_t);  // rows 0-2
        DI[i].root = blas_root[I.blas];
        DI[i].hit_base = I.hit_base;
        DI[i].shade_base = shade_base[I.blas];
        DI[i].pad = 0;
    }
    if ((rc = upload(d.insts, DI.data(), DI.size() * sizeof(DevInstance), total))) return rc;
    d.n_insts = (int)DI.size();
    {   // instance-major ray-bin keys (mrt_bin.h): hit bases, and instances ranked by BLAS then index
        std::vector<int32_t> hb(DI.size());
        std::vector<uint32_t> order(DI.size());
        for (size_t i = 0; i < DI.size(); i++) { hb[i] = DI[i].hit_base; order[i] = (uint32_t)i; }
        std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return DI[a].root < DI[b].root; });
        std::vector<uint16_t> cls(DI.size());
        for (size_t r = 0; r < order.size(); r++) cls[order[r]] = (uint16_t)std::min<size_t>(127, r * 128 / order.size());
        if ((rc = upload(d.inst_hit_base, hb.data(), hb.size() * sizeof(int32_t), total))) return rc;
        if ((rc = upload(d.inst_class, cls.data(), cls.size() * sizeof(uint16_t), total))) return rc;
        // object-space cells: each instance's BLAS root box (its finite child boxes), 4 cells per axis
        std::vector<float4> cell(2 * DI.size());
        for (size_t i = 0; i < DI.size(); i++) {
            const QNode& R = DN[(size_t)DI[i].root];
            float lo3[3] = {0, 0, 0}, hi3[3] = {0, 0, 0};
            bool any3[3] = {false, false, false};
            for (int k = 0; k < 4; k++) {
                if (R.child[k] == kEmptySlot) continue;
                for (int a = 0; a < 3; a++) {
                    const float l = R.box[a * 4 + k], h = R.box[12 + a * 4 + k];
                    if (!std::isfinite(l) || !std::isfinite(h)) continue;
                    lo3[a] = any3[a] ? std::min(lo3[a], l) : l;
                    hi3[a] = any3[a] ? std::max(hi3[a], h) : h;
                    any3[a] = true;
                }
            }
            auto sc = [&](int a) { return hi3[a] > lo3[a] ? 4.0f / (hi3[a] - lo3[a]) : 0.0f; };
            cell[2 * i] = make_float4(lo3[0], lo3[1], lo3[2], (float)(s.instances[i].blas & 1));
            cell[2 * i + 1] = make_float4(sc(0), sc(1), sc(2), 0.f);
        }
        if ((rc = upload(d.inst_cell, cell.data(), cell.size() * sizeof(float4), total))) return rc;
    }
    d.n_world = (int)s.obj_mesh.size();
    if ((rc = upload(d.leaves, DL.data(), DL.size() * sizeof(DLeaf), total))) return rc;
    if ((rc = upload(d.prims, PS.data(), PS.size() * sizeof(PrimShade), total))) return rc;
    if ((rc = upload(d.verts, V.data(), V.size() * sizeof(float4), total))) return rc;
    if ((rc = upload(d.normals, N.data(), N.size() * sizeof(float4), total))) return rc;
    if ((rc = upload(d.mats, s.materials.data(), s.materials.size() * sizeof(DevMaterial), total))) return rc;
    if ((rc = upload(d.lights, s.lights.data(), s.lights.size() * sizeof(DevLight), total))) return rc;
    if ((rc = upload(d.tables, tab.data(), tab.size() * sizeof(uint16_t), total))) return rc;
    if ((rc = upload(d.gamma, host_gamma_lut(), 32769, total))) return rc;
    if ((rc = upload(d.gammaF, host_gamma_float_lut(), 32769 * sizeof(float), total))) return rc;
    // textures, then each dome light's tables (DomeLight::setTexture products)
    auto upload_floats = [&](const std::vector<float>& v, const float*& dst) -> int {
        float* p = nullptr;
        const int r = upload(p, v.data(), v.size() * sizeof(float), total);
        d.bufs.push_back(p);
        dst = p;
        return r;
    };
    std::vector<const float*> dtex(s.textures.size(), nullptr);
    for (size_t i = 0; i < s.textures.size(); i++)
        if ((rc = upload_floats(s.textures[i].rgb, dtex[i]))) return rc;
    std::vector<DevDome> DD(s.domes.size());
    for (size_t i = 0; i < s.domes.size(); i++) {
        const DomeTables& t = s.domes[i];
        DevDome& g = DD[i];
        if ((rc = upload_floats(t.cdf_u, g.cdf_u)) || (rc = upload_floats(t.func_u, g.func_u)) ||
            (rc = upload_floats(t.cdf_v, g.cdf_v)) || (rc = upload_floats(t.func_v, g.func_v)) ||
            (rc = upload_floats(t.inv_int_v, g.inv_int_v)) || (rc = upload_floats(t.cos_u, g.cos_u)) ||
            (rc = upload_floats(t.sin_u, g.sin_u)) || (rc = upload_floats(t.cos_v, g.cos_v)) ||
            (rc = upload_floats(t.sin_v, g.sin_v)))
            return rc;
        float *rad = nullptr, *gu = nullptr, *gv = nullptr;
        if ((rc = upload(rad, t.rad.data(), t.rad.size() * sizeof(float), total)) ||
            (rc = upload(gu, t.guide_u.data(), t.guide_u.size() * sizeof(int32_t), total)) ||
            (rc = upload(gv, t.guide_v.data(), t.guide_v.size() * sizeof(int32_t), total)))
            return rc;
        for (float* p : {rad, gu, gv}) d.bufs.push_back(p);
        g.rad = rad;
        g.guide_u = reinterpret_cast<const int32_t*>(gu);
        g.guide_v = reinterpret_cast<const int32_t*>(gv);
        g.tex = dtex[t.tex];
        g.inv_int_u = t.inv_int_u;
        g.nu = t.nu;
        g.nv = t.nv;
    }
    if ((rc = upload(d.domes, DD.data(), DD.size() * sizeof(DevDome), total))) return rc;
    d.env = s.env_tex >= 0 ? dtex[s.env_tex] : nullptr;
    std::vector<DevTexture> DT(s.textures.size());
    for (size_t i = 0; i < DT.size(); i++) DT[i] = DevTexture{dtex[i], s.textures[i].W, s.textures[i].H, s.textures[i].type, 0};
    if ((rc = upload(d.texs, DT.data(), DT.size() * sizeof(DevTexture), total))) return rc;
    if (any_uv) {
        if ((rc = upload(d.puv, PUV.data(), PUV.size() * sizeof(uint4), total))) return rc;
        if ((rc = upload(d.uvs, UV.data(), UV.size() * sizeof(float2), total))) return rc;
        if ((rc = upload(d.tans, TN.data(), TN.size() * sizeof(float4), total))) return rc;
        if ((rc = upload(d.btans, BTN.data(), BTN.size() * sizeof(float4), total))) return rc;
    }
    if (d.has_mb) {
        std::vector<float4> V2 = V;
        for (size_t m = 0; m < s.meshes.size(); m++)
            for (size_t i = 0; i < s.meshes[m].verts2.size(); i++) {
                const v3& p = s.meshes[m].verts2[i];
                V2[vbase[m] + i] = make_float4(p.x, p.y, p.z, 1.f);
            }
        if ((rc = upload(d.verts2, V2.data(), V2.size() * sizeof(float4), total))) return rc;
        if ((rc = upload(d.pflags, PF.data(), PF.size(), total))) return rc;
    }
    d.special = d.n_insts > 0 || d.has_alpha || d.has_mb;
    d.bytes = total;
    // persistent grid: resident workgroups on every CU
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device));
    d.cus = prop.multiProcessorCount;
    if (hipDeviceGetAttribute(&d.wall_khz, hipDeviceAttributeWallClockRate, device) != hipSuccess) d.wall_khz = 0;
    d.grid = d.cus * kMaxBlocksPerCU;
    d.boxes_finite = true;
    d.boxes_ordered = true;
    for (const QNode& q : DN) {
        for (int k = 0; k < 24; k++) d.boxes_finite &= std::isfinite(q.box[k]);
        for (int i = 0; i < 4; i++)
            if (q.child[i] != kEmptySlot)
                for (int a = 0; a < 3; a++) d.boxes_ordered &= q.box[a * 4 + i] <= q.box[12 + a * 4 + i];
    }
    for (int a = 0; a < 3; a++) d.bb_lo[a] = d.bb_hi[a] = 0.f;
    if (!DN.empty()) {   // union of the root's used slot boxes (finite values only, per axis)
        bool any[3] = {false, false, false};
        for (int i = 0; i < 4; i++) {
            if (DN[0].child[i] == kEmptySlot) continue;
            for (int a = 0; a < 3; a++) {
                const float lo = DN[0].box[a * 4 + i], hi = DN[0].box[12 + a * 4 + i];
                if (!std::isfinite(lo) || !std::isfinite(hi)) continue;
                d.bb_lo[a] = any[a] ? std::min(d.bb_lo[a], lo) : lo;
                d.bb_hi[a] = any[a] ? std::max(d.bb_hi[a], hi) : hi;
                any[a] = true;
            }
        }
    }
    d.point_only = true;
    d.dome = false;
    for (const DevLight& l : s.lights) {
        d.point_only &= (l.type == MRT_POINT_LIGHT);
        d.dome |= l.type == MRT_DOME_LIGHT;
    }
    d.recursive = 0;
    for (const DevMaterial& m : s.materials)
        if (m.type == MRT_BLINN && (m.reflect > 0.f || m.refract > 0.f || m.gloss < 1.f || m.translucency > 0.01f)) d.recursive = 1;
    if (s.path_trace) d.recursive = 2;
    d.disperse = false;
    // transparent shadows: the walk is compiled into the fused chain kernels only (it
    // needs a closest-hit traversal in the shading, which would cost the direct
    // kernels occupancy), and they shade a scene without secondary rays identically
    d.transparent = false;
    for (const DevLight& l : s.lights) d.transparent |= l.transparent != 0;
    if (d.transparent && !d.recursive) d.recursive = 1;
    d.pow_spec = false;
    for (const DevMaterial& m : s.materials) d.pow_spec |= m.type == MRT_BLINN && m.spec_exp != 1.0f;
    for (const DevMaterial& m : s.materials)
        d.disperse |= m.type == MRT_BLINN && m.disperse && (m.reflect > 0.f || m.refract > 0.f);
    d.gthreads = (uint32_t)d.grid * kWG;
    s.info.device_bytes = total;
    return MRT_OK;
}

static int host_camera(const mrt_camera* c, int W, int H, CamParams& out) {
    if (!c || W <= 0 || H <= 0) { set_error("bad camera/frame"); return MRT_ERR_INVALID; }
    const uint16_t* RS = host_rsqrt_table();
    // Camera::setEye/setLookAt/setUp (src/Camera.h:82-124), eyeRayAdaptive basis
    v3 eye = mk(c->eye[0], c->eye[1], c->eye[2]);
    v3 viewDir = normalized(sub(mk(c->look_at[0], c->look_at[1], c->look_at[2]), eye), RS);
    v3 up = normalized(mk(c->up[0], c->up[1], c->up[2]), RS);
    v3 w = normalized(neg(viewDir), RS);
    v3 u = normalized(cross(up, w), RS);
    v3 v = cross(w, u);
    float aspect = (float)W / (float)H;
    const float DegToRad = 3.1415926f / 180.0f, Half = DegToRad / 2.0f;
    float top = tanf(c->fov_deg * Half);
    float right = aspect * top;
    out.eye[0] = eye.x; out.eye[1] = eye.y; out.eye[2] = eye.z;
    out.u[0] = u.x; out.u[1] = u.y; out.u[2] = u.z;
    out.v[0] = v.x; out.v[1] = v.y; out.v[2] = v.z;
    out.w[0] = w.x; out.w[1] = w.y; out.w[2] = w.z;
    out.top = top; out.right = right; out.bottom = -top; out.left = -right;
    out.W = W; out.H = H;
    out.aperture = c->aperture;
    out.focus = c->focus_plane;
    out.shutter = c->shutter_speed;
    return MRT_OK;
}

static void fill_params(const Scene& s, RenderParams& P) {
    const DeviceState& d = *s.dev;
    P.nodes = d.nodes; P.leaves = d.leaves; P.prims = d.prims; P.verts = d.verts; P.normals = d.normals;
    P.mats = d.mats; P.lights = d.lights; P.tables = d.tables; P.gamma = d.gamma;
    P.gammaF = d.gammaF;
    P.min_subdivs = s.min_subdivs;
    P.max_subdivs = s.max_subdivs;
    P.noise = s.noise_threshold;
    P.domes = d.domes;
    P.insts = d.insts;
    P.texs = d.texs;
    P.puv = d.puv;
    P.uvs = d.uvs;
    P.tans = d.tans;
    P.btans = d.btans;
    P.has_maps = d.has_maps ? 1 : 0;
    P.pflags = d.pflags;
    P.verts2 = d.verts2;
    P.has_mb = d.has_mb ? 1 : 0;
    P.n_insts = d.n_insts;
    P.n_world = d.n_world;
    P.env = d.env;
    P.env_w = d.env ? s.textures[s.env_tex].W : 0;
    P.env_h = d.env ? s.textures[s.env_tex].H : 0;
    P.env_exposure = s.env_exposure;
    P.gstride = d.gthreads;
    P.bg[0] = s.bg[0]; P.bg[1] = s.bg[1]; P.bg[2] = s.bg[2];
    P.n_lights = (int32_t)s.lights.size();
    P.num_paths = s.num_paths;
    P.path_trace = s.path_trace ? 1 : 0;
    P.max_bounces = s.max_bounces;
    P.sample_env = s.sample_env ? 1 : 0;
    P.mat_env = 0;
    for (const DevMaterial& m : s.materials) P.mat_env |= m.env >= 0 ? 1 : 0;
}

// chain levels of the REC kernels: reflection / refraction bounces (< 5) plus
// the GI bounces (giBounces < m_maxBounces - 1)
static int chain_levels(const Scene& s) { return 6 + (s.path_trace ? s.max_bounces : 0); }
// words of a level record: reflect / refract 3; GI 12 + 3 per light; a
// dispersive split in the fused engine 26 + the IOR history (Shader::level)
static constexpr int kDispWords = 26 + kIorCap;
static int level_words(const Scene& s) {
    const int w = s.path_trace ? 12 + 3 * (int)s.lights.size() : 3;
    return s.dev && s.dev->disperse ? std::max(w, kDispWords) : w;
}

static int ensure_levels(StreamCtx& c, size_t floats) {
    if (floats <= c.lvl_cap) return MRT_OK;
    if (c.lvl) { HIP_OK(hipStreamSynchronize(c.stream)); (void)hipFree(c.lvl); }
    c.lvl = nullptr; c.lvl_cap = 0;
    HIP_OK(hipMalloc((void**)&c.lvl, floats * sizeof(float)));
    c.lvl_cap = floats;
    return MRT_OK;
}

static inline int fast_box(const DeviceState& d) { return (g_fast_box && d.boxes_finite) ? 1 : 0; }

// wavefront shadow-ray buffers of a stream context (grown, never shrunk)
static int ensure_rays(StreamCtx& c, size_t slots, size_t per_slot) {
    const size_t n = slots * per_slot;
    if (n <= c.ray_cap && slots <= c.nrays_cap) return MRT_OK;
    HIP_OK(hipStreamSynchronize(c.stream));  // the previous launch may still read them
    void* ptrs[] = {c.rays, c.occl, c.nrays};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    c.rays = nullptr; c.occl = nullptr; c.nrays = nullptr; c.ray_cap = c.nrays_cap = 0;
    HIP_OK(hipMalloc((void**)&c.rays, 2 * n * sizeof(float4)));
    HIP_OK(hipMalloc((void**)&c.occl, n));
    HIP_OK(hipMalloc((void**)&c.nrays, slots));
    c.ray_cap = n;
    c.nrays_cap = slots;
    return MRT_OK;
}

// Dome-light replay scratch of a stream: n ray slots, calls call records.
static int ensure_replay(StreamCtx& c, size_t n, size_t calls) {
    if (n <= c.ray_e_cap && calls <= c.lrec_cap) return MRT_OK;
    HIP_OK(hipStreamSynchronize(c.stream));   // the previous launch may still read them
    if (c.ray_e) (void)hipFree(c.ray_e);
    if (c.lrec) (void)hipFree(c.lrec);
    c.ray_e = nullptr; c.lrec = nullptr; c.ray_e_cap = c.lrec_cap = 0;
    HIP_OK(hipMalloc((void**)&c.ray_e, n * sizeof(float4)));
    HIP_OK(hipMalloc((void**)&c.lrec, calls * sizeof(uint32_t)));
    c.ray_e_cap = n;
    c.lrec_cap = calls;
    return MRT_OK;
}

// The binning switches in effect for a scene (g_bin, or the auto choice).
static int bin_mode(const DeviceState& d) {
    if (g_bin >= 0) return g_bin;
    return (d.recursive == 2 ? 6 : 0) | (d.n_insts > 0 && d.dome ? 5 : 0) | (d.disperse ? 4 : 0);
}

// Ray-binning scratch of a stream (mrt_bin.h) for batches of up to n rays.
static constexpr size_t kBinHist = (size_t(1) << kBinBits) + 64;   // bins + the valid count, padded
static int ensure_bin(StreamCtx& c, size_t n) {
    if (n <= c.bin_cap) return MRT_OK;
    HIP_OK(hipStreamSynchronize(c.stream));   // the previous launch may still read them
    void* ptrs[] = {c.bin_keys, c.bin_perm, c.bin_hist};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    c.bin_keys = nullptr; c.bin_perm = nullptr; c.bin_hist = nullptr; c.bin_cap = 0;
    HIP_OK(hipMalloc((void**)&c.bin_keys, n * sizeof(uint16_t)));
    HIP_OK(hipMalloc((void**)&c.bin_perm, 2 * n * sizeof(uint32_t)));
    HIP_OK(hipMalloc((void**)&c.bin_hist, 2 * kBinHist * sizeof(uint32_t)));
    c.bin_cap = n;
    return MRT_OK;
}

// Binning of a ray batch o[i] / d[i], i < n (host bound), into permutation
// `which` of the stream's scratch; keys from the scene box and the tuning
// knobs.  The caller sets the validity / device-count fields, then bins.
static BinArgs bin_args(const DeviceState& d, const StreamCtx& c, int which, const float4* o, const float4* dd, size_t n) {
    BinArgs A{};
    A.o = o; A.d = dd; A.n = (uint32_t)n;
    A.mul1 = 1; A.cap1 = 0xFFFFFFFFu; A.mul2 = 1; A.m = 1;
    A.dbits = g_bin_dbits; A.obits = g_bin_obits;
    for (int a = 0; a < 3; a++) {
        const float ext = d.bb_hi[a] - d.bb_lo[a];
        A.lo[a] = d.bb_lo[a];
        A.inv[a] = ext > 0.f ? (float)(1 << A.obits) / ext : 0.f;
    }
    A.keys = c.bin_keys;
    A.hist = c.bin_hist + (size_t)which * kBinHist;
    A.perm = c.bin_perm + (size_t)which * c.bin_cap;
    return A;
}
static const uint32_t* bin_total(const BinArgs& A) {
    return A.hist + (size_t(1) << (A.hits ? kBinBits : 2 * A.dbits + 3 * A.obits));
}
static int bin_grid(const DeviceState& d, size_t n) {   // fewer blocks: fewer per-bin global atomics
    return (int)std::max<size_t>(1, std::min<size_t>((size_t)d.cus * (size_t)kBinBlocks, (n + 255) / 256));
}

static int ensure_slots(StreamCtx& c, size_t slots) {
    if (slots <= c.hit_slots) return MRT_OK;
    // the old buffer may still be read by this stream's previous launch
    if (c.hitbuf) { HIP_OK(hipStreamSynchronize(c.stream)); (void)hipFree(c.hitbuf); }
    c.hitbuf = nullptr; c.hit_slots = 0;
    HIP_OK(hipMalloc((void**)&c.hitbuf, slots * sizeof(float4)));
    c.hit_slots = slots;
    return MRT_OK;
}



// Resident workgroups per CU of one kernel instantiation (occupancy API, cached).
// An over-estimate only queues blocks behind the resident ones: the tile
// schedule (sched 2/3) keeps late blocks useful.
static int blocks_per_cu(KernelFn f, size_t lds) {
    static std::mutex mu;
    static std::map<std::pair<const void*, size_t>, int> cache;
    std::lock_guard<std::mutex> g(mu);
    const auto key = std::make_pair(reinterpret_cast<const void*>(f), lds);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(f), kWG, lds) != hipSuccess) n = 1;
    n = std::max(1, std::min(n, kMaxBlocksPerCU));
    cache[key] = n;
    return n;
}

template <int W, bool I = false, bool CHK = true, bool X = false>
static KernelFn primary_fn(bool c, bool f) {
    return c ? (f ? primary_kernel<true, W, true, I, CHK, X> : primary_kernel<true, W, false, I, CHK, X>)
             : (f ? primary_kernel<false, W, true, I, CHK, X> : primary_kernel<false, W, false, I, CHK, X>);
}
// check: the special-leaf scene has alpha-mapped or motion-blurred lanes; scenes with
// instances only take the variants without those tests (no noinline calls: C5's nested
// instance walk at 5 waves spills 28 B instead of 256 B per lane)
// xone: the one-exit walk loop (non-instanced scenes; the instanced walk keeps its exits:
// C5's primary launch measured 36% slower with one)
static KernelFn pick_primary(int w, bool c, bool f, bool inst, bool check = true, bool xone = false) {
    if (inst && !check) {
        switch (g_primary_inst_waves) {
            case 4: return primary_fn<4, true, false>(c, f);
            case 6: return primary_fn<6, true, false>(c, f);
            case 1: return primary_fn<1, true, false>(c, f);
            default: return primary_fn<5, true, false>(c, f);
        }
    }
    if (inst) {   // special-leaf scenes (instances: nested BLAS walks)
        switch (g_primary_inst_waves) {
            case 4: return primary_fn<4, true>(c, f);   // 128 VGPRs: the nested instance walk without spills
            case 5: return primary_fn<5, true>(c, f);
            case 6: return primary_fn<6, true>(c, f);
            default: return primary_fn<1, true>(c, f);
        }
    }
    if (xone) {
        switch (w) {
            case 6: return primary_fn<6, false, true, true>(c, f);
            case 7: return primary_fn<7, false, true, true>(c, f);
            case 8: return primary_fn<8, false, true, true>(c, f);
            default: return primary_fn<1, false, true, true>(c, f);
        }
    }
    switch (w) {
        case 6: return primary_fn<6>(c, f);
        case 7: return primary_fn<7>(c, f);
        case 8: return primary_fn<8>(c, f);
        default: return primary_fn<1>(c, f);
    }
}
// bound: the dome-light resolve pass at 4 waves (~240 VGPRs unbounded)
template <int MODE>
static KernelFn shade_mode_fn(bool c, bool po, bool inst, bool bound = false) {   // kGen / kResolve: no traversal, FAST unused
    if (!c && MODE == kResolve && bound) {
        // special-leaf scenes at 3 waves: 168 VGPRs and no scratch (152 B / 40 spills at 4 waves);
        // C5's resolve pass -0.7% (profiles/r06_c5_resolve_waves_ab.txt)
        if (inst) return shade_kernel<false, false, false, true, MODE, 0, 3>;
        return po ? shade_kernel<false, true, false, false, MODE, 0, 4> : shade_kernel<false, false, false, false, MODE, 0, 4>;
    }
    if (inst) return c ? shade_kernel<true, false, false, true, MODE> : shade_kernel<false, false, false, true, MODE>;
    if (po) return c ? shade_kernel<true, true, false, false, MODE> : shade_kernel<false, true, false, false, MODE>;
    return c ? shade_kernel<true, false, false, false, MODE> : shade_kernel<false, false, false, false, MODE>;
}
using ShadowFn = void (*)(RenderParams, size_t, int, int);
// MINW: launch-bounds occupancy target of the timed (COUNT = false) variants
template <bool INST, bool REFILL, bool CHECK, int MINW = 1>
static ShadowFn shadow_fn(bool c, bool f) {
    return c ? (f ? shadow_kernel<true, true, INST, REFILL, CHECK> : shadow_kernel<true, false, INST, REFILL, CHECK>)
             : (f ? shadow_kernel<false, true, INST, REFILL, CHECK, MINW> : shadow_kernel<false, false, INST, REFILL, CHECK, MINW>);
}
template <bool INST, bool REFILL, bool CHECK>
static ShadowFn shadow_fn_w(bool c, bool f) { return shadow_fn<INST, REFILL, CHECK, 8>(c, f); }
// check: the scene has alpha-mapped or motion-blurred lanes (child-word bit 3), which the
// refill step must test as such
static ShadowFn pick_shadow(bool c, bool f, bool inst, bool refill, bool check) {
    if (!refill) return inst ? shadow_fn<true, false, true>(c, f) : shadow_fn_w<false, false, false>(c, f);
    if (!inst) return shadow_fn_w<false, true, false>(c, f);
    return check ? shadow_fn<true, true, true>(c, f) : shadow_fn_w<true, true, false>(c, f);
}
// shadow rays per pixel at most: num_paths x (1 per point light, m_numSamples per area / dome light)
static int max_shadow_rays(const Scene& s) {
    int per_path = 0;
    for (const DevLight& l : s.lights) per_path += l.type == MRT_POINT_LIGHT ? 1 : std::max(1, l.samples);
    return s.num_paths * per_path;
}

// rec: Shader REC (0 direct, 1 reflection / refraction chains, 2 + path tracing)
static KernelFn pick_shade(bool c, bool po, bool f, bool inst, int rec) {
    if (rec) return pick_shade_rec(c, po, f, inst, rec);
    return pick4<ShadeK, 0>(c, po, f, inst);
}

// The wavefront chain engine (mrt_chain.hip) for the shading of a REC scene:
// per chunk of work units (eye rays), level 0 of every path (gen, shadow rays,
// resolve), then per level compact / trace / gen / shadow rays / resolve, the
// per-level folds and the per-unit finish.  P holds the primary launch's
// parameters (hits, outputs, cameras, work items, or an adaptive pass's units);
// the chunks are sized so the per-level arrays fit g_chain_mb.
static constexpr int kMaxChainLevels = 63;   // < the 64 level counts (level L's count stays 0)
// shadow rays one chain level of one path traces at most: every light's
// samples for the direct term, again for translucency, again for the last GI
// bounce (0: more than the u8 ray count holds -> fused kernel)
static int chain_shadow_rays(const Scene& s) {
    int per = 0;
    for (const DevLight& l : s.lights) per += l.type == MRT_POINT_LIGHT ? 1 : std::max(1, l.samples);
    bool tr = false;
    for (const DevMaterial& m : s.materials) tr |= m.type == MRT_BLINN && m.translucency > 0.01f;
    const int m = per * (1 + (tr ? 1 : 0) + (s.path_trace ? 1 : 0));
    return m <= 255 ? std::max(1, m) : 0;
}
// Entries of chain level k per path at most: one child per level, except a
// dispersive split's three (src/Blinn.cpp:275-301).  Split children are
// refraction rays, which do not split again, so splits are at least two levels
// apart: 3^ceil(k/2).  (Dispersion with path tracing -- GI levels without a
// bounce bound on splits -- stays on the fused kernel.)
static uint64_t level_mult(const Scene& s, int k) {
    uint64_t m = 1;
    if (s.dev->disperse)
        for (int i = 0; i < (k + 1) / 2; i++) m *= 3;
    return m;
}
// (Transparent shadows: the walk's answer is an attenuation, not the one bit the
// wavefront shadow passes carry -- such scenes shade in the fused kernels.)
static bool use_chain(const Scene& s) {
    return s.dev->recursive && g_chain && chain_levels(s) <= kMaxChainLevels && chain_shadow_rays(s) > 0 &&
           !(s.dev->disperse && s.path_trace) && !s.dev->transparent;
}
// One chunk of the engine over units [Q.unit_base, Q.unit_base + Q.n_units) of
// Q's pass (the chunk layout -- ch_lofs, arrays -- is set by the caller).
static int chain_chunk(Scene& s, StreamCtx& c, RenderParams& Q, bool count, hipStream_t stream, size_t ctl,
                       unsigned int* queues) {
    DeviceState& d = *s.dev;
    const int L = Q.ch_levels;
    const bool inst = d.special;
    const KernelFn g0 = pick_chain0(false, d.point_only, inst, d.recursive), r0 = pick_chain0(true, d.point_only, inst, d.recursive);
    const KernelFn gk = pick_chain_shade(false, d.point_only, inst, d.recursive),
                   rk = pick_chain_shade(true, d.point_only, inst, d.recursive);
    const KernelFn kc = pick_chain_compact(), kt = pick_chain_trace(count, Q.fast_box != 0, inst,
                                                                           g_chain_shadow_step ? (d.has_alpha || d.has_mb ? 2 : 1) : 0),
                   kf = pick_chain_finish(), kd = pick_chain_fold();
    auto go = [&](KernelFn f, int g) -> int {
        void* args[] = {&Q};
        HIP_OK(hipLaunchKernel(reinterpret_cast<const void*>(f), dim3(std::max(1, g)), dim3(kWG), args, 0, stream));
        return MRT_OK;
    };
    auto full = [&](KernelFn f) { return std::min(d.grid, d.cus * blocks_per_cu(f, 0)); };
    const int ug = (int)std::min<uint64_t>((uint64_t)full(r0), ((uint64_t)Q.n_units + kWG - 1) / kWG);
    int rc;
    // ray binning before each trace launch (g_bin bits 1 / 2): level k's closest-hit entries
    // and level k - 1's shadow rays, each in its own permutation
    const uint32_t m = (uint32_t)Q.max_shadow;
    auto lcap_h = [&](int k) { return (size_t)Q.ch_lofs[k + 1] - Q.ch_lofs[k]; };
    const int bm = bin_mode(d);
    if (bm & 6) {
        size_t need = 1;
        for (int k = 0; k < L; k++) need = std::max(need, std::max(lcap_h(k), lcap_h(k) * m));
        if ((rc = ensure_bin(c, need))) return rc;
    }
    // instanced scenes: the levels' shadow rays on the lane-refill kernel (their own launch)
    const bool refill_sh = inst && g_chain_shadow_refill;
    const ShadowFn ksh = refill_sh ? pick_shadow(count, Q.fast_box != 0, true, true, d.has_alpha || d.has_mb) : nullptr;
    int gsh = refill_sh ? std::max(8, std::min(d.grid, d.cus * blocks_per_cu(reinterpret_cast<KernelFn>(ksh), 0))) & ~7 : 0;
    auto trace = [&](int k) -> int {   // Q.ch_level == k
        if ((bm & 2) && k < L) {
            const size_t lo = Q.ch_lofs[k], cap = lcap_h(k);
            BinArgs A = bin_args(d, c, 1, Q.ch_ray + 2 * lo, Q.ch_ray + 2 * lo + cap, cap);
            A.n_dev = Q.ch_cnt + k;
            int r2;
            if ((r2 = bin_rays(A, bin_grid(d, cap), stream))) return r2;
            Q.tr_perm = A.perm;
        }
        if (bm & 4) {
            const size_t lo = Q.ch_lofs[k - 1], nb = lcap_h(k - 1) * m;
            BinArgs B = bin_args(d, c, 0, Q.ray_o + lo * m, Q.ray_d + lo * m, nb);
            B.nrays = Q.nrays + lo;
            B.m = m;
            if (k - 1 > 0) {
                B.n_dev = Q.ch_cnt + (k - 1);
                B.mul2 = m;
            } else if (Q.unit_cnt) {   // adaptive pass: chunk_units on the device
                B.n_dev = Q.unit_cnt;
                B.mul1 = Q.adapt_n > 1 ? (uint32_t)(Q.adapt_n * Q.adapt_n) : 1u;
                B.sub = Q.unit_base;
                B.cap1 = Q.n_units;
                B.mul2 = (uint32_t)Q.num_paths * m;
            } else {
                const uint32_t units = Q.units_total > Q.unit_base ? std::min(Q.n_units, Q.units_total - Q.unit_base) : 0u;
                B.n = (uint32_t)std::min<uint64_t>(nb, (uint64_t)units * (uint64_t)Q.num_paths * m);
            }
            int r2;
            if ((r2 = bin_rays(B, bin_grid(d, nb), stream))) return r2;
            Q.sh_perm = B.perm;
            Q.sh_perm_n = bin_total(B);
        }
        int r3 = MRT_OK;
        if (refill_sh) {
            // instanced scenes: level k - 1's shadow rays on the lane-refill any-hit kernel
            // (shadow_kernel sched 2: a finished lane takes the next ray, proxy lanes deferred
            // onto the stack), the entries' closest hits in chain_trace below.  Same rays,
            // same answers; level 0's ray counts of units past the chunk are zeroed at its start.
            RenderParams S = Q;
            const size_t sbase = (size_t)Q.ch_lofs[k - 1] * m;
            S.ray_o = Q.ray_o + sbase;
            S.ray_d = Q.ray_d + sbase;
            S.occl = Q.occl + sbase;
            S.nrays = Q.nrays + Q.ch_lofs[k - 1];
            S.sh_count = k - 1 > 0 ? Q.ch_cnt + (k - 1) : nullptr;
            S.near_first = 0;
            S.queue = queues + (size_t)(L + 2 + k) * 256;
            size_t n_rays = lcap_h(k - 1) * m;
            int sched = 2, refill = kRefillMin;
            void* sargs[] = {&S, &n_rays, &sched, &refill};
            r3 = MRT_OK;
            if (hipLaunchKernel(reinterpret_cast<const void*>(ksh), dim3(gsh), dim3(kWG), sargs, 0, stream) != hipSuccess) {
                set_error("chain shadow launch"); r3 = MRT_ERR_HIP;
            }
            Q.ch_skip_shadow = 1;
        }
        if (r3 == MRT_OK) r3 = go(kt, full(kt));
        Q.ch_skip_shadow = 0;
        Q.tr_perm = nullptr;
        Q.sh_perm = nullptr;
        Q.sh_perm_n = nullptr;
        return r3;
    };
    HIP_OK(hipMemsetAsync(Q.ch_cnt, 0, ctl, stream));
    if (refill_sh) HIP_OK(hipMemsetAsync(Q.nrays + Q.ch_lofs[0], 0, lcap_h(0), stream));   // level 0: only live units' counts
    Q.queue = queues;
    if (Q.uhits) {   // adaptive pass: the chunk's eye rays and their closest hits (counted in the frame's
                     // statistics: they run before any level can outgrow its capacity)
        const KernelFn ke = pick_unit_eye(count, Q.fast_box != 0, inst);
        unsigned long long* cc = Q.ctr;
        Q.ctr = Q.ctr_out;
        rc = go(ke, (int)std::min<uint64_t>((uint64_t)full(ke), ((uint64_t)Q.n_units + kWG - 1) / kWG));
        Q.ctr = cc;
        if (rc) return rc;
    }
    Q.ch_level = 0;
    if ((rc = go(g0, ug))) return rc;                 // level 0: shadow rays + children
    for (int k = 0; k + 1 < L; k++) {
        Q.ch_level = k;
        if ((rc = go(kc, full(kc)))) return rc;        // children of level k -> entries of level k + 1
        Q.ch_level = k + 1;
        if ((rc = trace(k + 1))) return rc;            // their closest hits + level k's shadow rays
        if ((rc = go(gk, full(gk)))) return rc;        // level k + 1: shadow rays + children
    }
    Q.ch_level = L;
    if ((rc = trace(L))) return rc;                    // the last level's shadow rays
    Q.queue = queues + 256;
    if ((rc = go(r0, ug))) return rc;                  // resolve level 0, then levels 1 .. L - 1
    if ((rc = go(rk, full(rk)))) return rc;
    for (int k = L - 2; k >= 0; k--) {                 // fold the values up, deepest level first
        Q.ch_level = k;
        if ((rc = go(kd, full(kd)))) return rc;
    }
    if ((rc = go(kf, ug))) return rc;                  // per unit: paths averaged, pixel / unit colour
    // the chunk's statistics and capacity counts; a chunk that outgrew a level: its units again,
    // fused (counted in the frame's statistics directly)
    void* margs[] = {&Q};
    HIP_OK(hipLaunchKernel(reinterpret_cast<const void*>(pick_chain_merge()), dim3(1), dim3(64), margs, 0, stream));
    const KernelFn kfb = pick_chain_fallback(d.point_only, inst, d.recursive, count);
    unsigned long long* cc = Q.ctr;
    Q.ctr = Q.ctr_out;
    rc = go(kfb, std::min(full(kfb), ug));
    Q.ctr = cc;
    return rc;
}

// The chain engine over a pass of `units_max` units (at most; the adaptive
// passes' counts live on the device): the scratch layout for `per_chunk`
// units, then the chunks.
static constexpr int kEstPasses = 17;   // capacity estimates: pass index 0 (no supersampling), 1 .. 16
static int launch_chain(Scene& s, StreamCtx& c, const RenderParams& P0, bool count, hipStream_t stream,
                        uint64_t units_max, int unit_align) {
    DeviceState& d = *s.dev;
    const int L = chain_levels(s), W = level_words(s), m = chain_shadow_rays(s), split = d.disperse ? 3 : 1;
    const uint64_t np = (uint64_t)P0.num_paths;
    // Level capacities in entries per path x 65536.  Worst case: level k holds 3^ceil(k/2)
    // entries per path where dispersive splits can occur, else one.  With chain_est, a level
    // this stream has seen (this pass index) gets the largest count per path any chunk needed
    // x chain_est_pct + 1/32: a chunk that outgrows it sets ch_ovf, its remaining launches
    // return at once and chain_fallback renders its units with the fused chain shading --
    // the same frame, at the fused kernel's speed for that chunk only.
    const int pi = std::min(P0.adapt_n, kEstPasses - 1);
    if (g_chain_est && !c.est_dev) {
        HIP_OK(hipMalloc((void**)&c.est_dev, kEstPasses * 64 * sizeof(uint32_t)));
        HIP_OK(hipMemsetAsync(c.est_dev, 0, kEstPasses * 64 * sizeof(uint32_t), stream));
        HIP_OK(hipHostMalloc((void**)&c.est_pinned, kEstPasses * 64 * sizeof(uint32_t)));
        HIP_OK(hipEventCreateWithFlags(&c.est_ev, hipEventDisableTiming));
        c.est.assign(kEstPasses * 64, 0u);
    }
    if (c.est_pending && hipEventQuery(c.est_ev) == hipSuccess) {   // the last copy has landed: no wait
        std::copy(c.est_pinned, c.est_pinned + kEstPasses * 64, c.est.begin());
        c.est_pending = false;
    }
    std::vector<uint64_t> capr(L);
    uint64_t capr_sum = 0, capr_max = 0;
    for (int k = 0; k < L; k++) {
        const uint64_t worst = level_mult(s, k) << 16;
        uint64_t r = worst;
        const uint32_t e = g_chain_est && k > 0 ? c.est[(size_t)pi * 64 + k] : 0u;
        if (e != 0u && e != 0xFFFFFFFFu) r = std::min(worst, (uint64_t)(e - 1) * (uint64_t)g_chain_est_pct / 100 + 2048);
        capr[k] = r;
        capr_sum += r;
        capr_max = std::max(capr_max, r);
    }
    // per path over all levels: ray + ior 2 x 32 B, hit 16, value 16, record 4 W, child map 4 split,
    // shadow rays m x (32 B + occlusion byte) + ray count; sparse spawn slots 65 B x split x the widest level
    const uint64_t entry_bytes = 32 + 32 + 16 + 16 + 4 * (uint64_t)W + 4 * (uint64_t)split + (uint64_t)m * 33 + 1;
    const uint64_t path_bytes = (capr_sum * entry_bytes + capr_max * (uint64_t)split * 65 + 65535) >> 16;
    const uint64_t unit_bytes = np * path_bytes + (P0.adapt_n ? 16 : 0);
    uint64_t budget = (uint64_t)g_chain_mb << 20;
    size_t mem_free = 0, mem_total = 0;   // this stream's current chunk can be reused: count it as free
    if (hipMemGetInfo(&mem_free, &mem_total) == hipSuccess) {
        budget = std::min<uint64_t>(budget, ((uint64_t)mem_free + c.chain_bytes) / 5 * 4);
        // every stream of this scene may hold a chunk at once: each gets at most its share of 80% of the
        // device (frames in flight on 4 streams cannot claim the whole device between them)
        size_t live = 1;
        {
            std::lock_guard<std::mutex> g(d.mu);
            live = std::max<size_t>(1, d.ctxs.size());
        }
        budget = std::min<uint64_t>(budget, (uint64_t)mem_total / 5 * 4 / live);
    }
    c.chain_budget = budget;
    uint64_t per = std::max<uint64_t>(1, budget / unit_bytes);
    per = std::max<uint64_t>(unit_align, per / unit_align * unit_align);
    per = std::min<uint64_t>(per, (units_max + unit_align - 1) / unit_align * unit_align);
    const uint64_t paths = per * np;
    std::vector<uint64_t> lcap(L);
    uint64_t entries = 0, lmax = 0;
    for (int k = 0; k < L; k++) {
        // whole 64-entry groups: every array's level slice stays aligned (the u64 statistics
        // after the maps need 8-byte alignment) and a wave's 64 entries share a group
        lcap[k] = k == 0 ? paths : std::max<uint64_t>(64, (((paths * capr[k] + 65535) >> 16) + 63) / 64 * 64);
        entries += lcap[k];
        lmax = std::max(lmax, lcap[k]);
    }
    const uint64_t spcap = lmax * (uint64_t)split;
    if (entries * (uint64_t)m >= (uint64_t(1) << 32) || spcap >= (uint64_t(1) << 32)) {
        set_error("chain chunk too large"); return MRT_ERR_INVALID;
    }
    int rc;
    if ((rc = ensure_rays(c, entries, (size_t)m))) return rc;   // every level keeps its shadow rays
    // layout: ray | ior (2 per entry) | hit | val | spawn (4 per slot) | uhits (float4), rec (float),
    // map (u32), control (counts, trace + resolve + chain shadow-launch queues, the chunk's
    // statistics, its overflow flag), flag (u8)
    const size_t ctl_q = 256 + (size_t)(2 * L + 3) * 1024;
    const size_t ctl = ctl_q + 256 + 64;
    const uint64_t n4 = 2 * entries + 2 * entries + entries + entries + 4 * spcap + (P0.adapt_n ? per : 0);
    const uint64_t bytes = n4 * 16 + entries * (uint64_t)W * 4 + entries * (uint64_t)split * 4 + ctl + spcap;
    if (bytes > c.chain_bytes) {
        if (c.chain) { HIP_OK(hipStreamSynchronize(c.stream)); (void)hipFree(c.chain); }
        c.chain = nullptr; c.chain_bytes = 0;
        HIP_OK(hipMalloc(&c.chain, bytes));
        c.chain_bytes = bytes;
    }
    RenderParams Q = P0;
    float4* f4 = static_cast<float4*>(c.chain);
    Q.ch_ray = f4; f4 += 2 * entries;
    Q.ch_ior = f4; f4 += 2 * entries;
    Q.ch_hit = f4; f4 += entries;
    Q.ch_val = f4; f4 += entries;
    Q.ch_sp = f4; f4 += 4 * spcap;
    Q.uhits = P0.adapt_n ? f4 : nullptr; f4 += P0.adapt_n ? per : 0;
    Q.ch_rec = reinterpret_cast<float*>(f4);
    Q.ch_map = reinterpret_cast<uint32_t*>(Q.ch_rec + entries * (uint64_t)W);
    Q.ch_cnt = Q.ch_map + entries * (uint64_t)split;           // 64 counts, then L + 2 queues
    unsigned int* queues = reinterpret_cast<unsigned int*>(reinterpret_cast<char*>(Q.ch_cnt) + 256);
    Q.ctr_out = P0.ctr;
    Q.ctr = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(Q.ch_cnt) + ctl_q);
    Q.ch_ovf = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(Q.ch_cnt) + ctl_q + 256);
    Q.ch_est = g_chain_est ? c.est_dev + (size_t)pi * 64 : nullptr;
    if (reinterpret_cast<uintptr_t>(Q.ctr) % 8 != 0) { set_error("chain layout misaligned"); return MRT_ERR_INVALID; }
    Q.ch_flag = reinterpret_cast<uint8_t*>(Q.ch_cnt) + ctl;
    Q.ch_spcap = (uint32_t)spcap;
    Q.ch_split = split;
    Q.ch_levels = L;
    uint64_t off = 0;
    for (int k = 0; k <= L; k++) {
        Q.ch_lofs[k] = (uint32_t)off;
        if (k < L) off += lcap[k];
    }
    Q.lvl_words = W;
    Q.ch_bands = g_chain_bands > 0 || (g_chain_bands < 0 && (bin_mode(d) & 6));
    Q.wave_log = nullptr;
    Q.ray_o = c.rays;
    Q.ray_d = c.rays + entries * (uint64_t)m;
    Q.occl = c.occl;
    Q.nrays = c.nrays;
    Q.max_shadow = m;
    Q.n_units = (uint32_t)per;
    c.chain_chunks += (uint32_t)((units_max + per - 1) / per);
    for (uint64_t b = 0; b < units_max; b += per) {
        Q.unit_base = (uint32_t)b;
        if ((rc = chain_chunk(s, c, Q, count, stream, ctl, queues))) return rc;
    }
    if (g_chain_est) {   // this pass's estimates to the host, read by a later frame once they have landed
        HIP_OK(hipMemcpyAsync(c.est_pinned, c.est_dev, kEstPasses * 64 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
        HIP_OK(hipEventRecord(c.est_ev, stream));
        c.est_pending = true;
    }
    return MRT_OK;
}

// Adaptive supersampling of a REC scene on the chain engine: passes n = 1 ..
// max_subdivs over the pixels still refining (each pass: the units' eye rays,
// the chain engine, then adapt_combine's running mean + stop test, which lists
// the next pass's pixels or writes the pixel).
static int launch_chain_adaptive(Scene& s, StreamCtx& c, RenderParams& P, bool count, hipStream_t stream) {
    DeviceState& d = *s.dev;
    const uint64_t lanes = (uint64_t)P.n_tiles * 64;   // pixels of the frame / batch (work-item lanes)
    const int maxs = std::max(P.min_subdivs, P.max_subdivs);
    // per stream: running means, two pixel lists + counts, unit colours of the largest pass
    const uint64_t ucol_n = lanes * (uint64_t)maxs * (uint64_t)maxs;
    const uint64_t bytes = lanes * 16 + 2 * lanes * 4 + 256 + ucol_n * 16;
    if (bytes > c.adapt_bytes) {
        if (c.adapt) { HIP_OK(hipStreamSynchronize(c.stream)); (void)hipFree(c.adapt); }
        c.adapt = nullptr; c.adapt_bytes = 0;
        HIP_OK(hipMalloc(&c.adapt, bytes));
        c.adapt_bytes = bytes;
    }
    float4* res = static_cast<float4*>(c.adapt);
    float4* ucol = res + lanes;
    uint32_t* lists = reinterpret_cast<uint32_t*>(ucol + ucol_n);
    uint32_t* cnts = lists + 2 * lanes;   // 2 counts (own 256 B)
    P.adapt_res = res;
    P.ucol = ucol;
    int cur = 0, rc;
    const KernelFn kcomb = pick_adapt_combine();
    for (int n = 1; n <= maxs; n++) {
        const int nxt = cur ^ 1;
        P.adapt_n = n;
        P.units = n == 1 ? nullptr : lists + (size_t)cur * lanes;
        P.unit_cnt = n == 1 ? nullptr : cnts + cur;
        P.units_total = (uint32_t)lanes;
        P.next_units = lists + (size_t)nxt * lanes;
        P.next_cnt = cnts + nxt;
        HIP_OK(hipMemsetAsync(cnts + nxt, 0, 4, stream));
        if ((rc = launch_chain(s, c, P, count, stream, lanes * (uint64_t)n * (uint64_t)n, 64))) return rc;
        void* args[] = {&P};
        const int g = std::min<int>(d.grid, (int)((lanes + kWG - 1) / kWG));
        HIP_OK(hipLaunchKernel(reinterpret_cast<const void*>(kcomb), dim3(std::max(1, g)), dim3(kWG), args, 0, stream));
        cur = nxt;
    }
    return MRT_OK;
}

// Two launches on `stream`: primary rays -> hit records, then shading with
// shadow rays.  Events bracket both (kernel_ms covers the whole frame).  With
// adaptive supersampling (subdivs > 1) one fused launch (kernel 3) instead.
static int launch_render(Scene& s, RenderParams& P, size_t slots, bool count, hipStream_t stream, bool want_hits) {
    DeviceState& d = *s.dev;
    StreamCtx* cp = nullptr;
    int rc = get_ctx(d, stream, cp);
    if (rc) return rc;
    StreamCtx& c = *cp;
    s.stats_final = false;
    if ((rc = ensure_slots(c, slots))) return rc;
    if (d.recursive) {
        P.lvl_words = level_words(s);
        if ((rc = ensure_levels(c, (size_t)d.gthreads * chain_levels(s) * P.lvl_words))) return rc;
        P.lvl = c.lvl;
    }
    P.hits = c.hitbuf;
    P.gstack = c.gstack;
    P.ctr = c.ctr;
    P.fast_box = fast_box(d);
    P.sched = g_sched;
    P.cus = d.cus;
    P.scalar_nodes = g_scalar_nodes & (d.boxes_ordered ? 7 : 3);
    P.near_first = g_near_first > 0 ? 1 : 0;
    c.chain_chunks = 0;
    c.chain_budget = 0;
    const bool inst = d.special;   // instances or alpha maps: the special-leaf kernels
    const bool adaptive = P.min_subdivs > 1 || P.max_subdivs > 1;
    const bool one = g_shade1 && d.point_only && P.n_lights == 1 && P.num_paths == 1 && !P.env && !inst && !d.recursive &&
                     !d.has_maps;
    const size_t log_stride = (size_t)d.grid * (kWG / 64) * kLogWords;
    const bool logw = count || g_wave_log;   // wave log: count mode, or timing-only on the timed kernels
    HIP_OK(hipMemsetAsync(c.ctr, 0, kCtrBytes, stream));
    unsigned int* qbase = reinterpret_cast<unsigned int*>(reinterpret_cast<char*>(c.ctr) + CTR_N * sizeof(unsigned long long));
    P.queue = qbase;
    // workgroups: at most one per 4 tiles (a tile per wave); bucket batches (P.mode 1) may ask for
    // g_batch_tpw tiles per wave, so a small share's waves take several tiles each
    const int tpw = P.mode == 1 ? g_batch_tpw : 1;
    const int items = (int)(((int64_t)P.n_tiles + 4 * tpw - 1) / (4 * tpw));
    if (logw) HIP_OK(hipMemsetAsync(c.wave_log, 0, 2 * log_stride * sizeof(unsigned long long), stream));
    int which = 0;
    auto launch = [&](KernelFn f) -> int {
        const int g = std::max(1, std::min(std::min(d.grid, d.cus * blocks_per_cu(f, 0)), items));
        P.wave_log = logw && which < 2 ? c.wave_log + which * log_stride : nullptr;  // primary + first shade
        P.n_waves = g * (kWG / 64);
        if (logw && which < 2) c.log_waves[which] = g * (kWG / 64);
        which++;
        void* args[] = {&P};
        HIP_OK(hipLaunchKernel(reinterpret_cast<const void*>(f), dim3(g), dim3(kWG), args, 0, stream));
        return MRT_OK;
    };
    HIP_OK(hipEventRecord(c.ev0, stream));
    const bool fb = P.fast_box != 0;
    c.chain_used = false;
    if (adaptive) {
        HIP_OK(hipEventRecord(c.evm, stream));   // primary_ms = 0: one launch
        P.refill_min = g_adapt_refill;
        if (use_chain(s)) {     // secondary rays: passes over the chain engine
            c.chain_used = true;
            if ((rc = launch_chain_adaptive(s, c, P, count, stream))) return rc;
        } else if ((rc = launch(pick_adaptive(count, d.point_only, fb, inst, d.recursive)))) {
            return rc;
        }
        c.last_was_render = true;
        HIP_OK(hipGetLastError());
        HIP_OK(hipEventRecord(c.ev1, stream));
        d.last = &c;
        s.last = mrt_stats{};
        return MRT_OK;
    }
    c.fused = one && g_fused;
    if (c.fused) {   // one launch: camera rays, closest hits, shading, shadow rays
        if (!want_hits) P.hits = nullptr;
        // LDS top-node walk (tuning "lds_nodes"; both walks give the same bits)
        const bool ln = fb && d.lds_ok && g_lds_nodes > 0;
        d.lds_pick = ln ? 1 : 0;
        const int walk = ln ? 2 : g_walk_exit == 0 ? 0 : g_walk_latch ? 3 : 1;
        if ((rc = launch(pick_frame1(g_frame1_waves, count, fb, d.pow_spec, walk)))) return rc;
        HIP_OK(hipEventRecord(c.evm, stream));
        c.last_was_render = true;
        HIP_OK(hipGetLastError());
        HIP_OK(hipEventRecord(c.ev1, stream));
        d.last = &c;
        s.last = mrt_stats{};
        return MRT_OK;
    }
    const bool chk = d.has_alpha || d.has_mb;
    if ((rc = launch(pick_primary(g_primary_waves, count, fb, inst, chk, g_walk_exit == 1)))) return rc;
    HIP_OK(hipEventRecord(c.evm, stream));
    P.queue = qbase + 8 * 32;
    const int max_sh = max_shadow_rays(s);
    // secondary rays and their shadow rays depend on hits along the path: fused kernel
    const bool wave = !one && g_wavefront && max_sh > 0 && max_sh <= kMaxWaveShadow && !d.recursive && !d.transparent;
    if (use_chain(s)) {
        c.chain_used = true;
        P.units = nullptr;
        P.unit_cnt = nullptr;
        P.adapt_n = 0;
        P.units_total = (uint32_t)P.n_tiles * 64u;
        if ((rc = launch_chain(s, c, P, count, stream, (uint64_t)P.n_tiles * 64, 64))) return rc;
    } else if (one || !wave) {
        if ((rc = launch(one ? pick_shade1(count, fb, d.pow_spec) : pick_shade(count, d.point_only, fb, inst, d.recursive)))) return rc;
    } else {
        if ((rc = ensure_rays(c, slots, (size_t)max_sh))) return rc;
        P.ray_o = c.rays;
        P.ray_d = c.rays + slots * (size_t)max_sh;
        P.occl = c.occl;
        P.nrays = c.nrays;
        P.max_shadow = max_sh;
        int ndome = 0;
        for (const DevLight& l : s.lights) ndome += l.type == MRT_DOME_LIGHT ? 1 : 0;
        const bool dome = ndome > 0;
        if (dome && g_dome_replay) {   // 2a records the dome samples, 2c replays them
            P.lcalls = P.num_paths * ndome;
            if ((rc = ensure_replay(c, slots * (size_t)max_sh, slots * (size_t)P.lcalls))) return rc;
            P.ray_e = c.ray_e;
            P.lrec = c.lrec;
        }
        if ((rc = launch(shade_mode_fn<kGen>(count, d.point_only, inst)))) return rc;
        // lane refill for dome-light (incoherent) rays: D1 -7%, C5 -13% shade pass; coherent
        // area-light rays keep the bands (C4: refill +9%)
        int sched = g_shadow_sched >= 0 ? g_shadow_sched : (dome ? 2 : 1), refill = kRefillMin;
        ShadowFn sf = pick_shadow(count, fb, inst, sched == 2, d.has_alpha || d.has_mb);
        int g = std::max(1, std::min(d.grid, d.cus * blocks_per_cu(reinterpret_cast<KernelFn>(sf), 0)));
        if (sched && (g & 7)) g &= ~7;          // XCD bands need a whole number of workgroups per XCD
        if (g < 8) {                            // too few workgroups for the bands: grid-stride
            sched = 0;
            sf = pick_shadow(count, fb, inst, false, d.has_alpha || d.has_mb);
        }
        size_t n_rays = slots * (size_t)max_sh;
        if (n_rays >= (size_t(1) << 32)) { set_error("too many wavefront shadow-ray slots (2^32)"); return MRT_ERR_INVALID; }
        P.near_first = g_near_first >= 0 ? g_near_first : (sched == 2 || inst ? 0 : 1);
        if (bin_mode(d) & 1) {   // the rays in binned order (valid slots only)
            if ((rc = ensure_bin(c, n_rays))) return rc;
            BinArgs A = bin_args(d, c, 0, P.ray_o, P.ray_d, n_rays);
            A.nrays = P.nrays;
            A.m = (uint32_t)max_sh;
            if (g_bin_inst && d.n_insts > 0 && A.dbits == 2 && A.obits == 2) {   // instance-major keys
                A.hits = P.hits;
                A.hit_base = d.inst_hit_base;
                A.inst_class = d.inst_class;
                A.inst_cell = g_bin_inst == 2 ? d.inst_cell : nullptr;   // 2: object-space cells
                A.insts = d.insts;
                A.n_inst = d.n_insts;
                A.n_world = d.n_world;
            }
            if ((rc = bin_rays(A, bin_grid(d, n_rays), stream))) return rc;
            P.sh_perm = A.perm;
            P.sh_perm_n = bin_total(A);
        }
        void* args[] = {&P, &n_rays, &sched, &refill};
        P.wave_log = nullptr;
        P.queue = qbase + 24 * 32;
        HIP_OK(hipLaunchKernel(reinterpret_cast<const void*>(sf), dim3(g), dim3(kWG), args, 0, stream));
        P.sh_perm = nullptr;
        P.sh_perm_n = nullptr;
        P.queue = qbase + 16 * 32;
        // dome-light resolve passes run faster at 4 waves (D1 -4%, C5 -1.2 ms), the rect-light one not (C4 +2%)
        if ((rc = launch(shade_mode_fn<kResolve>(count, d.point_only, inst, dome)))) return rc;
        P.ray_e = nullptr;
        P.lrec = nullptr;
        P.lcalls = 0;
    }
    c.last_was_render = true;
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(c.ev1, stream));
    d.last = &c;
    s.last = mrt_stats{};
    return MRT_OK;
}

}  // namespace mrt

using namespace mrt;

// ================================================================== C ABI
extern "C" {

const char* mrt_last_error(void) { return g_err.c_str(); }
int mrt_abi_version(void) { return MRT_ABI_VERSION; }
int mrt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

mrt_scene* mrt_scene_create(void) { return new (std::nothrow) mrt_scene(); }
void mrt_scene_destroy(mrt_scene* s) {
    if (!s) return;
    free_replicas(s->impl);
    delete s;
}

int mrt_scene_add_material(mrt_scene* s, const mrt_material* m) {
    if (!s || !m || (m->type != MRT_LAMBERT && m->type != MRT_BLINN)) { set_error("bad material"); return MRT_ERR_INVALID; }
    if (s->impl.materials.size() >= (size_t)kMaxMaterials) { set_error("too many materials"); return MRT_ERR_INVALID; }
    DevMaterial d;
    d.type = m->type;
    memcpy(d.kd, m->kd, 12); memcpy(d.ka, m->ka, 12); memcpy(d.ks, m->ks, 12);
    d.spec_exp = m->spec_exp; d.spec_amt = m->spec_amt;
    d.reflect = 0.f; d.refract = 0.f; d.ior = 1.5f; d.gloss = 1.f;   // Blinn defaults (src/Blinn.h:11-22)
    d.disperse = 0; d.ior3[0] = d.ior3[1] = d.ior3[2] = 1.5f;
    d.translucency = 0.f;
    memcpy(d.le, m->le, 12);
    d.emitted = m->emitted;
    d.sample_env = 1;                                                 // Material::Material, src/Material.cpp:6
    d.env = -1;                                                       // m_envMap NULL, m_envExposure 1 (:4)
    d.env_exposure = 1.f;
    for (int k = 0; k < 6; k++) d.maps[k] = -1;                       // no maps (src/Material.cpp:4-5)
    d.emitter = (d.emitted > 0.0f || (d.le[0] + d.le[1]) + d.le[2] > 0.0f) ? 1 : 0;   // src/Blinn.cpp:47
    if (m->type != MRT_BLINN) { d.le[0] = d.le[1] = d.le[2] = 0.f; d.emitted = 0.f; d.emitter = 0; }
    s->impl.materials.push_back(d);
    s->impl.dev_dirty = true;
    return (int)s->impl.materials.size() - 1;
}

int mrt_scene_add_light(mrt_scene* s, const mrt_light* l) {
    if (!s || !l || (l->type != MRT_POINT_LIGHT && l->type != MRT_RECT_LIGHT && l->type != MRT_DOME_LIGHT)) {
        set_error("bad light");
        return MRT_ERR_INVALID;
    }
    if (s->impl.lights.size() >= (size_t)kMaxLights) { set_error("too many lights"); return MRT_ERR_INVALID; }
    // Light::setFastShadows(false).  A point light's "full method" (src/PointLight.cpp:49-70)
    // sets sampleHit.t = distance and then loops while sampleHit.t < distance: it never
    // traces, so the light casts no shadow -- exactly cast_shadows = 0.  The rectangle and
    // dome lights walk through refractive hits (src/RectangleLight.cpp:93-116,
    // src/DomeLight.cpp:123-145; Shader::transmit).
    DevLight d;
    memset(&d, 0, sizeof d);
    d.dome = -1;
    if (l->type == MRT_DOME_LIGHT) {
        // DomeLight::setTexture (src/DomeLight.cpp:8-78): tables built now, on the host
        if (l->texture < 0 || l->texture >= (int32_t)s->impl.textures.size() ||
            tex_channels(s->impl.textures[l->texture].type) != 3) {
            set_error("dome light needs an RGB / HDR texture id from mrt_scene_add_texture");
            return MRT_ERR_INVALID;
        }
        DomeTables t;
        std::string err;
        const int rc = build_dome(s->impl.textures[l->texture], t, err);
        if (rc) { set_error(err); return rc; }
        t.tex = l->texture;
        d.dome = (int32_t)s->impl.domes.size();
        s->impl.domes.push_back(std::move(t));
    }
    d.type = l->type;
    memcpy(d.pos, l->pos, 12); memcpy(d.v1, l->v1, 12); memcpy(d.v2, l->v2, 12); memcpy(d.v3, l->v3, 12);
    d.samples = l->samples < 1 ? 1 : l->samples;
    d.noise = l->noise_threshold;
    d.cast_shadows = l->cast_shadows && !(l->transparent_shadows && l->type == MRT_POINT_LIGHT);
    d.transparent = l->transparent_shadows && l->type != MRT_POINT_LIGHT ? 1 : 0;
    d.power = l->power;
    if (l->type == MRT_RECT_LIGHT) {
        // RectangleLight::setPower (src/RectangleLight.cpp:14-40)
        const uint16_t* RS = host_rsqrt_table();
        v3 v1 = mk(l->v1[0], l->v1[1], l->v1[2]);
        v3 e0 = sub(mk(l->v2[0], l->v2[1], l->v2[2]), v1), e1 = sub(mk(l->v3[0], l->v3[1], l->v3[2]), v1);
        float recip = 1.0f, sq;
        if (fabsf(dot(e0, e1)) < 0.001f) sq = dot(e0, e0) * dot(e1, e1);
        else { v3 c = cross(e0, e1); sq = dot(c, c); }
        if (sq > 0.001f) recip = rsqrt_nr(sq, RS);
        d.power = l->power * recip;
    }
    s->impl.lights.push_back(d);
    s->impl.dev_dirty = true;
    return (int)s->impl.lights.size() - 1;
}

int mrt_scene_make_blas(mrt_scene* s, const int32_t* meshes, int32_t n_meshes) {
    if (!s) { set_error("null scene"); return MRT_ERR_INVALID; }
    std::string err;
    const int rc = make_blas(s->impl, meshes, n_meshes, err);
    if (rc < 0) set_error(err);
    return rc;
}

int mrt_scene_add_instance(mrt_scene* s, int32_t blas, const float* m16) {
    if (!s) { set_error("null scene"); return MRT_ERR_INVALID; }
    std::string err;
    const int rc = add_instance(s->impl, blas, m16, err);
    if (rc < 0) set_error(err);
    return rc;
}

int mrt_scene_blas_info(const mrt_scene* s, int32_t blas, int32_t* nodes, int32_t* leaves, int32_t* prims) {
    if (!s || !nodes || !leaves || !prims || blas < 0 || blas >= (int32_t)s->impl.blas.size()) {
        set_error("bad BLAS id / argument");
        return MRT_ERR_INVALID;
    }
    const Blas& B = s->impl.blas[blas];
    *nodes = (int32_t)B.nodes.size();
    *leaves = (int32_t)B.leaves.size();
    *prims = (int32_t)B.obj_mesh.size();
    return MRT_OK;
}

int mrt_scene_blas_export(const mrt_scene* s, int32_t blas, float* node_boxes, int32_t* node_child, float* leaf_tris,
                          int32_t* leaf_prims) {
    if (!s || !node_boxes || !node_child || !leaf_tris || !leaf_prims || blas < 0 ||
        blas >= (int32_t)s->impl.blas.size()) {
        set_error("bad BLAS id / argument");
        return MRT_ERR_INVALID;
    }
    const Blas& B = s->impl.blas[blas];
    for (size_t i = 0; i < B.nodes.size(); i++) {
        memcpy(node_boxes + 24 * i, B.nodes[i].box, 24 * sizeof(float));
        memcpy(node_child + 4 * i, B.nodes[i].child, 4 * sizeof(int32_t));
    }
    for (size_t i = 0; i < B.leaves.size(); i++) {
        memcpy(leaf_tris + 36 * i, B.leaves[i].t, 36 * sizeof(float));
        memcpy(leaf_prims + 4 * i, B.leaves[i].prim, 4 * sizeof(int32_t));
    }
    return MRT_OK;
}

int mrt_hdr_info(const char* path, int32_t* width, int32_t* height) {
    if (!path || !width || !height) { set_error("bad argument"); return MRT_ERR_INVALID; }
    int W = 0, H = 0;
    std::string err;
    const int rc = load_hdr(path, W, H, nullptr, err);
    if (rc) { set_error(err); return rc; }
    *width = W;
    *height = H;
    return MRT_OK;
}

int mrt_hdr_load(const char* path, float* rgb, int32_t width, int32_t height) {
    if (!path || !rgb) { set_error("bad argument"); return MRT_ERR_INVALID; }
    int W = 0, H = 0;
    std::string err;
    std::vector<float> buf;
    const int rc = load_hdr(path, W, H, &buf, err);
    if (rc) { set_error(err); return rc; }
    if (W != width || H != height) { set_error("HDR size differs from width x height (see mrt_hdr_info)"); return MRT_ERR_INVALID; }
    memcpy(rgb, buf.data(), buf.size() * sizeof(float));
    return MRT_OK;
}

int mrt_image_info(const char* path, int32_t* width, int32_t* height, int32_t* type) {
    if (!path || !width || !height || !type) { set_error("bad argument"); return MRT_ERR_INVALID; }
    int W = 0, H = 0, T = 0;
    std::string err;
    const int rc = load_image(path, W, H, T, nullptr, err);
    if (rc) { set_error(err); return rc; }
    *width = W;
    *height = H;
    *type = T;
    return MRT_OK;
}

int mrt_image_load(const char* path, float* data, int32_t width, int32_t height) {
    if (!path || !data) { set_error("bad argument"); return MRT_ERR_INVALID; }
    int W = 0, H = 0, T = 0;
    std::string err;
    std::vector<float> buf;
    const int rc = load_image(path, W, H, T, &buf, err);
    if (rc) { set_error(err); return rc; }
    if (W != width || H != height) { set_error("image size differs from width x height (see mrt_image_info)"); return MRT_ERR_INVALID; }
    memcpy(data, buf.data(), buf.size() * sizeof(float));
    return MRT_OK;
}

int mrt_scene_add_texture_typed(mrt_scene* s, const float* data, int32_t width, int32_t height, int32_t type) {
    if (!s || !data || width <= 0 || height <= 0 || (int64_t)width * height > (int64_t(1) << 28) ||
        (type != kTexHDR && type != kTexGray && type != kTexRGB && type != kTexRGBA)) {
        set_error("bad texture");
        return MRT_ERR_INVALID;
    }
    if (s->impl.textures.size() >= (size_t)kMaxTextures) { set_error("too many textures"); return MRT_ERR_INVALID; }
    Texture t;
    t.W = width;
    t.H = height;
    t.type = type;
    t.rgb.assign(data, data + (size_t)width * height * tex_channels(type));
    s->impl.textures.push_back(std::move(t));
    s->impl.dev_dirty = true;
    return (int)s->impl.textures.size() - 1;
}

int mrt_scene_set_material_maps(mrt_scene* s, int material, const int32_t maps[6]) {
    if (!s || !maps || material < 0 || material >= (int)s->impl.materials.size()) { set_error("bad material"); return MRT_ERR_INVALID; }
    for (int k = 0; k < 6; k++)
        if (maps[k] < -1 || maps[k] >= (int32_t)s->impl.textures.size()) { set_error("bad texture id"); return MRT_ERR_INVALID; }
    for (int k = 0; k < 6; k++) s->impl.materials[material].maps[k] = maps[k];
    s->impl.built = false;   // alpha maps change which leaf packets need the alpha test
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_add_texture(mrt_scene* s, const float* rgb, int32_t width, int32_t height) {
    if (!s || !rgb || width <= 0 || height <= 0 || (int64_t)width * height > (int64_t(1) << 28)) {
        set_error("bad texture");
        return MRT_ERR_INVALID;
    }
    if (s->impl.textures.size() >= (size_t)kMaxTextures) { set_error("too many textures"); return MRT_ERR_INVALID; }
    Texture t;
    t.W = width;
    t.H = height;
    t.rgb.assign(rgb, rgb + (size_t)width * height * 3);
    s->impl.textures.push_back(std::move(t));
    s->impl.dev_dirty = true;
    return (int)s->impl.textures.size() - 1;
}

int mrt_scene_set_material_env_map(mrt_scene* s, int material, int32_t texture, float exposure) {
    if (!s || material < 0 || material >= (int)s->impl.materials.size()) { set_error("bad material id"); return MRT_ERR_INVALID; }
    if (texture < -1 || texture >= (int32_t)s->impl.textures.size() ||
        (texture >= 0 && tex_channels(s->impl.textures[texture].type) != 3)) {
        set_error("bad texture id (an environment map needs an RGB / HDR texture)");
        return MRT_ERR_INVALID;
    }
    DevMaterial& m = s->impl.materials[(size_t)material];
    m.env = texture;
    m.env_exposure = exposure;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_env_map(mrt_scene* s, int32_t texture, float exposure) {
    if (!s || texture < -1 || texture >= (int32_t)s->impl.textures.size() ||
        (texture >= 0 && tex_channels(s->impl.textures[texture].type) != 3)) {
        set_error("bad texture id (the environment map needs an RGB / HDR texture)");
        return MRT_ERR_INVALID;
    }
    s->impl.env_tex = texture;
    s->impl.env_exposure = exposure;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

static const DomeTables* dome_of(const mrt_scene* s, int32_t light) {
    if (!s || light < 0 || light >= (int32_t)s->impl.lights.size() || s->impl.lights[light].dome < 0) return nullptr;
    return &s->impl.domes[s->impl.lights[light].dome];
}

int mrt_scene_dome_info(const mrt_scene* s, int32_t light, int32_t* nu, int32_t* nv) {
    const DomeTables* t = dome_of(s, light);
    if (!t || !nu || !nv) { set_error("not a dome light"); return MRT_ERR_INVALID; }
    *nu = t->nu;
    *nv = t->nv;
    return MRT_OK;
}

int mrt_scene_dome_export(const mrt_scene* s, int32_t light, float* cdf_u, float* func_u, float* cdf_v,
                          float* func_v, float* func_int, float* cos_u, float* sin_u, float* cos_v, float* sin_v) {
    const DomeTables* t = dome_of(s, light);
    if (!t || !cdf_u || !func_u || !cdf_v || !func_v || !func_int || !cos_u || !sin_u || !cos_v || !sin_v) {
        set_error("not a dome light / bad argument");
        return MRT_ERR_INVALID;
    }
    auto put = [](const std::vector<float>& v, float* dst) { memcpy(dst, v.data(), v.size() * sizeof(float)); };
    put(t->cdf_u, cdf_u); put(t->func_u, func_u); put(t->cdf_v, cdf_v); put(t->func_v, func_v);
    put(t->int_v, func_int);
    func_int[t->nu] = t->int_u;
    put(t->cos_u, cos_u); put(t->sin_u, sin_u); put(t->cos_v, cos_v); put(t->sin_v, sin_v);
    return MRT_OK;
}

int mrt_scene_add_obj(mrt_scene* s, const char* path, const float* ctm16, int material) {
    if (!s || !path) { set_error("bad argument"); return MRT_ERR_INVALID; }
    Mesh m;
    std::string err;
    int rc = load_obj(path, ctm16, m, err);
    if (rc != MRT_OK) { set_error(err); return rc; }
    m.material = material;
    s->impl.push_mesh(std::move(m));
    s->impl.built = false;
    return (int)s->impl.meshes.size() - 1;
}

int mrt_scene_add_mesh(mrt_scene* s, const mrt_mesh* mesh, int material) {
    if (!s || !mesh || mesh->nv < 0 || mesh->nn < 0 || mesh->nt < 0) { set_error("bad mesh"); return MRT_ERR_INVALID; }
    const int vs = mesh->vert_stride ? mesh->vert_stride : 3, ns = mesh->normal_stride ? mesh->normal_stride : 3;
    if (vs < 3 || ns < 3 || (mesh->nv && !mesh->verts) || (mesh->nn && !mesh->normals) ||
        (mesh->nt && (!mesh->vidx || !mesh->nidx))) {
        set_error("bad mesh: null array or stride < 3"); return MRT_ERR_INVALID;
    }
    Mesh m;
    m.material = material;
    for (int i = 0; i < mesh->nv; i++) {
        const float* v = mesh->verts + (size_t)vs * i;
        m.verts.push_back(mk(v[0], v[1], v[2]));
    }
    for (int i = 0; i < mesh->nn; i++) {
        const float* v = mesh->normals + (size_t)ns * i;
        m.normals.push_back(mk(v[0], v[1], v[2]));
    }
    m.vidx.assign(mesh->vidx, mesh->vidx + 3 * (size_t)mesh->nt);
    m.nidx.assign(mesh->nidx, mesh->nidx + 3 * (size_t)mesh->nt);
    for (size_t i = 0; i < m.vidx.size(); i++)
        if (m.vidx[i] >= (uint32_t)mesh->nv || m.nidx[i] >= (uint32_t)mesh->nn) { set_error("mesh index out of range"); return MRT_ERR_INVALID; }
    s->impl.push_mesh(std::move(m));
    s->impl.built = false;
    return (int)s->impl.meshes.size() - 1;
}

int mrt_scene_mesh_info(const mrt_scene* s, int mesh, int32_t* nv, int32_t* nn, int32_t* nt) {
    if (!s || mesh < 0 || mesh >= (int)s->impl.meshes.size()) { set_error("bad mesh id"); return MRT_ERR_INVALID; }
    const Mesh& m = s->impl.meshes[mesh];
    *nv = (int32_t)m.verts.size(); *nn = (int32_t)m.normals.size(); *nt = m.nt();
    return MRT_OK;
}

int mrt_scene_mesh_export(const mrt_scene* s, int mesh, float* verts, float* normals, uint32_t* vidx, uint32_t* nidx) {
    if (!s || mesh < 0 || mesh >= (int)s->impl.meshes.size()) { set_error("bad mesh id"); return MRT_ERR_INVALID; }
    const Mesh& m = s->impl.meshes[mesh];
    for (size_t i = 0; i < m.verts.size(); i++) { verts[3*i] = m.verts[i].x; verts[3*i+1] = m.verts[i].y; verts[3*i+2] = m.verts[i].z; }
    for (size_t i = 0; i < m.normals.size(); i++) { normals[3*i] = m.normals[i].x; normals[3*i+1] = m.normals[i].y; normals[3*i+2] = m.normals[i].z; }
    memcpy(vidx, m.vidx.data(), m.vidx.size() * 4);
    memcpy(nidx, m.nidx.data(), m.nidx.size() * 4);
    return MRT_OK;
}

int mrt_scene_mesh_set_texcoords(mrt_scene* s, int mesh, const float* uv, int32_t n_texcoords, const uint32_t* tidx) {
    if (!s || mesh < 0 || mesh >= (int)s->impl.meshes.size() || !uv || !tidx || n_texcoords <= 0) {
        set_error("bad texcoords");
        return MRT_ERR_INVALID;
    }
    Mesh& m = s->impl.meshes[mesh];
    for (size_t i = 0; i < m.vidx.size(); i++)
        if (tidx[i] >= (uint32_t)n_texcoords) { set_error("texture-coordinate index out of range"); return MRT_ERR_INVALID; }
    m.uv.assign(uv, uv + 2 * (size_t)n_texcoords);
    m.tidx.assign(tidx, tidx + m.vidx.size());
    s->impl.built = false;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_mesh_motion(mrt_scene* s, int mesh, const float* verts2) {
    if (!s || mesh < 0 || mesh >= (int)s->impl.meshes.size() || !verts2) { set_error("bad mesh id"); return MRT_ERR_INVALID; }
    Mesh& m = s->impl.meshes[mesh];
    m.verts2.resize(m.verts.size());
    for (size_t i = 0; i < m.verts.size(); i++) m.verts2[i] = v3{verts2[3*i], verts2[3*i+1], verts2[3*i+2]};
    s->impl.built = false;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_mesh_texcoords(const mrt_scene* s, int mesh, int32_t* n_texcoords, float* uv, uint32_t* tidx) {
    if (!s || mesh < 0 || mesh >= (int)s->impl.meshes.size() || !n_texcoords) { set_error("bad mesh id"); return MRT_ERR_INVALID; }
    const Mesh& m = s->impl.meshes[mesh];
    *n_texcoords = m.tidx.empty() ? 0 : (int32_t)(m.uv.size() / 2);
    if (*n_texcoords && uv) memcpy(uv, m.uv.data(), m.uv.size() * sizeof(float));
    if (*n_texcoords && tidx) memcpy(tidx, m.tidx.data(), m.tidx.size() * sizeof(uint32_t));
    return MRT_OK;
}

int mrt_scene_set_background(mrt_scene* s, const float rgb[3]) {
    if (!s || !rgb) { set_error("bad argument"); return MRT_ERR_INVALID; }
    memcpy(s->impl.bg, rgb, 12);
    return MRT_OK;
}

int mrt_scene_set_num_paths(mrt_scene* s, int num_paths) {
    if (!s || num_paths < 1 || num_paths > 1024) { set_error("bad num_paths (1..1024)"); return MRT_ERR_INVALID; }
    s->impl.num_paths = num_paths;
    return MRT_OK;
}

int mrt_scene_set_material_emission(mrt_scene* s, int material, float emitted, const float le[3]) {
    if (!s || !le || material < 0 || material >= (int)s->impl.materials.size()) {
        set_error("bad material / emission"); return MRT_ERR_INVALID;
    }
    DevMaterial& m = s->impl.materials[(size_t)material];
    if (m.type != MRT_BLINN) { set_error("only Blinn materials emit (src/Blinn.h:44-45)"); return MRT_ERR_INVALID; }
    memcpy(m.le, le, 12);
    m.emitted = emitted;
    m.emitter = (m.emitted > 0.0f || (m.le[0] + m.le[1]) + m.le[2] > 0.0f) ? 1 : 0;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_material_sample_env(mrt_scene* s, int material, int sample_env) {
    if (!s || material < 0 || material >= (int)s->impl.materials.size()) { set_error("bad material"); return MRT_ERR_INVALID; }
    s->impl.materials[(size_t)material].sample_env = sample_env ? 1 : 0;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_path_trace(mrt_scene* s, int enable, int max_bounces, int sample_env) {
    if (!s || max_bounces < 1 || max_bounces > 64) { set_error("bad path trace settings (1 <= max_bounces <= 64)"); return MRT_ERR_INVALID; }
    s->impl.path_trace = enable != 0;
    s->impl.max_bounces = max_bounces;
    s->impl.sample_env = sample_env != 0;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_prim_object(const mrt_scene* s, int32_t prim, int32_t* mesh, int32_t* tri, int32_t* inst) {
    if (!s || !mesh || !tri || !inst) { set_error("bad argument"); return MRT_ERR_INVALID; }
    const Scene& S = s->impl;
    if (!S.built) { set_error("scene not built"); return MRT_ERR_NOT_BUILT; }
    if (prim < 0) { set_error("prim id out of range"); return MRT_ERR_INVALID; }
    if ((size_t)prim < S.obj_mesh.size()) {   // a world object (a ProxyObject's own slot never hits)
        *mesh = S.obj_mesh[prim]; *tri = S.obj_tri[prim]; *inst = S.obj_inst[prim];
        return MRT_OK;
    }
    int lo = 0, hi = (int)S.instances.size() - 1;   // the last instance with hit_base <= prim
    if (hi < 0) { set_error("prim id out of range"); return MRT_ERR_INVALID; }
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (S.instances[mid].hit_base <= prim) lo = mid; else hi = mid - 1;
    }
    const Blas& B = S.blas[S.instances[lo].blas];
    const int64_t k = (int64_t)prim - S.instances[lo].hit_base;
    if (k < 0 || k >= (int64_t)B.obj_mesh.size()) { set_error("prim id out of range"); return MRT_ERR_INVALID; }
    *mesh = B.obj_mesh[k]; *tri = B.obj_tri[k]; *inst = lo;
    return MRT_OK;
}

int mrt_scene_set_material_optics(mrt_scene* s, int material, float reflect_amt, float refract_amt, float ior) {
    if (!s || material < 0 || material >= (int)s->impl.materials.size() || !(reflect_amt >= 0.f) ||
        !(refract_amt >= 0.f) || !(ior > 0.f)) {
        set_error("bad material optics: need a valid material, reflect / refract >= 0 and ior > 0");
        return MRT_ERR_INVALID;
    }
    DevMaterial& m = s->impl.materials[(size_t)material];
    m.reflect = reflect_amt;
    m.refract = refract_amt;
    m.ior = ior;
    m.ior3[1] = ior;   // one m_ior[3] in the reference: m_ior[1] is both the optics and the middle dispersion IOR
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_material_dispersion(mrt_scene* s, int material, int disperse, const float ior[3]) {
    if (!s || material < 0 || material >= (int)s->impl.materials.size() || !ior || !(ior[0] > 0.f) ||
        !(ior[1] > 0.f) || !(ior[2] > 0.f)) {
        set_error("bad dispersion: need a valid material and three IORs > 0");
        return MRT_ERR_INVALID;
    }
    DevMaterial& m = s->impl.materials[(size_t)material];
    m.disperse = disperse ? 1 : 0;
    for (int i = 0; i < 3; i++) m.ior3[i] = ior[i];
    m.ior = ior[1];   // m_ior[1]: the IOR of the non-dispersive refraction
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_material_translucency(mrt_scene* s, int material, float translucency) {
    if (!s || material < 0 || material >= (int)s->impl.materials.size() || !(translucency >= 0.f)) {
        set_error("bad translucency: need a valid material and translucency >= 0");
        return MRT_ERR_INVALID;
    }
    s->impl.materials[(size_t)material].translucency = translucency;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_material_gloss(mrt_scene* s, int material, float gloss) {
    if (!s || material < 0 || material >= (int)s->impl.materials.size() || !(gloss >= 0.f && gloss <= 1.f)) {
        set_error("bad gloss: need a valid material and 0 <= gloss <= 1");
        return MRT_ERR_INVALID;
    }
    s->impl.materials[(size_t)material].gloss = gloss;
    s->impl.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_set_subdivs(mrt_scene* s, int min_subdivs, int max_subdivs, float noise_threshold) {
    if (!s || min_subdivs < 1 || max_subdivs < min_subdivs || max_subdivs > 16 || !(noise_threshold >= 0.f)) {
        set_error("bad subdivs: need 1 <= min <= max <= 16 and noise >= 0");
        return MRT_ERR_INVALID;
    }
    s->impl.min_subdivs = min_subdivs;
    s->impl.max_subdivs = max_subdivs;
    s->impl.noise_threshold = noise_threshold;
    return MRT_OK;
}

int mrt_scene_build_bvh(mrt_scene* s) {
    if (!s) { set_error("null scene"); return MRT_ERR_INVALID; }
    for (auto& m : s->impl.meshes)
        if (m.material < 0 || m.material >= (int)s->impl.materials.size()) { set_error("mesh references unknown material"); return MRT_ERR_INVALID; }
    std::string err;
    int rc = build_qbvh(s->impl, err);
    if (rc != MRT_OK) set_error(err);
    return rc;
}

int mrt_scene_bvh_info(const mrt_scene* s, mrt_bvh_info* info) {
    if (!s || !info) { set_error("bad argument"); return MRT_ERR_INVALID; }
    if (!s->impl.built) { set_error("scene not built"); return MRT_ERR_NOT_BUILT; }
    *info = s->impl.info;
    return MRT_OK;
}

int mrt_scene_bvh_export(const mrt_scene* s, float* node_boxes, int32_t* node_child, float* leaf_tris, int32_t* leaf_prims) {
    if (!s) { set_error("null scene"); return MRT_ERR_INVALID; }
    if (!s->impl.built) { set_error("scene not built"); return MRT_ERR_NOT_BUILT; }
    for (size_t i = 0; i < s->impl.nodes.size(); i++) {
        memcpy(node_boxes + 24 * i, s->impl.nodes[i].box, 96);
        memcpy(node_child + 4 * i, s->impl.nodes[i].child, 16);
    }
    for (size_t i = 0; i < s->impl.leaves.size(); i++) {
        memcpy(leaf_tris + 36 * i, s->impl.leaves[i].t, 144);
        memcpy(leaf_prims + 4 * i, s->impl.leaves[i].prim, 16);
    }
    return MRT_OK;
}

int mrt_scene_bvh_import(mrt_scene* s, int32_t nodes, int32_t leaves, const float* node_boxes, const int32_t* node_child,
                         const float* leaf_tris, const int32_t* leaf_prims) {
    if (!s || nodes < 1 || leaves < 0) { set_error("bad argument"); return MRT_ERR_INVALID; }
    Scene& S = s->impl;
    if (!S.built) { set_error("build the scene first (prim ids come from it)"); return MRT_ERR_NOT_BUILT; }
    std::vector<QNode> N((size_t)nodes);
    std::vector<QLeaf> L((size_t)leaves);
    for (int i = 0; i < nodes; i++) {
        memset(&N[i], 0, sizeof(QNode));
        memcpy(N[i].box, node_boxes + 24 * (size_t)i, 96);
        memcpy(N[i].child, node_child + 4 * (size_t)i, 16);
        for (int k = 0; k < 4; k++) {
            int32_t c = N[i].child[k];
            if (c == kEmptySlot) continue;
            if ((c >= 0 && c >= nodes) || (c < 0 && ~c >= leaves)) { set_error("child index out of range"); return MRT_ERR_INVALID; }
        }
    }
    for (int i = 0; i < leaves; i++) {
        memcpy(L[i].t, leaf_tris + 36 * (size_t)i, 144);
        memcpy(L[i].prim, leaf_prims + 4 * (size_t)i, 16);
        for (int k = 0; k < 4; k++)
            if (L[i].prim[k] >= S.info.prims) { set_error("prim id out of range"); return MRT_ERR_INVALID; }
    }
    S.nodes.swap(N);
    S.leaves.swap(L);
    S.info.nodes = nodes;
    S.info.leaves = leaves;
    S.dev_dirty = true;
    return MRT_OK;
}

int mrt_scene_upload(mrt_scene* s, int device) {
    if (!s) { set_error("null scene"); return MRT_ERR_INVALID; }
    return ensure_device(s->impl, device);
}

int mrt_render_frame_async(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts, float* d_rgb,
                           uint8_t* d_rgb8, void* stream) {
    if (!s || !cam || !opts || !d_rgb) { set_error("bad argument"); return MRT_ERR_INVALID; }
    Scene& S = s->impl;
    int rc = ensure_device(S, opts->device);
    if (rc) return rc;
    HIP_OK(hipSetDevice(opts->device));
    RenderParams P{};
    fill_params(S, P);
    if ((rc = host_camera(cam, opts->width, opts->height, P.cam[0]))) return rc;
    P.seed = opts->seed ? opts->seed : 0x5EEDu;
    P.mode = 0;
    P.tiles_x = (opts->width + 7) / 8;
    P.n_tiles = P.tiles_x * ((opts->height + 7) / 8);
    P.out_rgb = d_rgb;
    P.out_rgb8 = d_rgb8;
    rc = launch_render(S, P, (size_t)opts->width * opts->height, opts->count_visits != 0, (hipStream_t)stream,
                       opts->want_hits != 0);
    S.last.primary_rays = (uint64_t)opts->width * opts->height;
    return rc;
}

static int render_batch(mrt_scene* s, const mrt_camera* cams, int32_t n_cams, const mrt_render_opts* opts,
                        const int32_t* d_items, int32_t n_items, float* d_out, uint8_t* d_out8, void* stream,
                        bool frame_out) {
    if (!s || !cams || !opts || n_items < 0 || (n_items && !d_items) || (!d_out && !d_out8)) {
        set_error("bad argument"); return MRT_ERR_INVALID;
    }
    if (n_cams < 1 || n_cams > kMaxBatch) { set_error("n_cams must be 1..16"); return MRT_ERR_INVALID; }
    Scene& S = s->impl;
    int rc = ensure_device(S, opts->device);
    if (rc) return rc;
    HIP_OK(hipSetDevice(opts->device));
    RenderParams P{};
    fill_params(S, P);
    for (int f = 0; f < n_cams; f++)
        if ((rc = host_camera(cams + f, opts->width, opts->height, P.cam[f]))) return rc;
    P.seed = opts->seed ? opts->seed : 0x5EEDu;
    P.mode = 1;
    P.frame_out = frame_out ? 1 : 0;
    P.buckets = d_items;
    P.buckets_x = (opts->width + 31) / 32;
    P.buckets_per_frame = P.buckets_x * ((opts->height + 31) / 32);
    P.n_cams = n_cams;
    P.n_tiles = n_items * 16;
    P.out_rgb = d_out;
    P.out_rgb8 = d_out8;
    if (n_items == 0) return MRT_OK;
    rc = launch_render(S, P, (size_t)n_items * 1024, opts->count_visits != 0, (hipStream_t)stream, opts->want_hits != 0);
    S.last.primary_rays = 0;
    return rc;
}

int mrt_render_batch_async(mrt_scene* s, const mrt_camera* cams, int32_t n_cams, const mrt_render_opts* opts,
                           const int32_t* d_items, int32_t n_items, float* d_tiles, uint8_t* d_tiles8, void* stream) {
    return render_batch(s, cams, n_cams, opts, d_items, n_items, d_tiles, d_tiles8, stream, false);
}

int mrt_render_batch_frames_async(mrt_scene* s, const mrt_camera* cams, int32_t n_cams, const mrt_render_opts* opts,
                                  const int32_t* d_items, int32_t n_items, float* d_frames, uint8_t* d_frames8,
                                  void* stream) {
    return render_batch(s, cams, n_cams, opts, d_items, n_items, d_frames, d_frames8, stream, true);
}

// ---- device memory shared between processes (the multi-GPU split's frame assembly)
int mrt_ipc_export(const void* d_ptr, mrt_ipc_handle* out) {
    if (!d_ptr || !out) { set_error("bad argument"); return MRT_ERR_INVALID; }
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    HIP_OK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)d_ptr));
    hipIpcMemHandle_t h;
    HIP_OK(hipIpcGetMemHandle(&h, (void*)base));
    static_assert(sizeof(h) <= sizeof(out->handle), "hipIpcMemHandle_t does not fit mrt_ipc_handle");
    memset(out, 0, sizeof(*out));
    memcpy(out->handle, &h, sizeof(h));
    out->offset = (uint64_t)((const char*)d_ptr - (const char*)base);
    out->size = (uint64_t)size;
    return MRT_OK;
}

static std::mutex g_ipc_mu;
static std::vector<std::pair<void*, void*>> g_ipc_maps;   // (pointer handed out, mapping base)

int mrt_ipc_open(const mrt_ipc_handle* h, int device, void** d_ptr) {
    if (!h || !d_ptr || h->offset > h->size) { set_error("bad argument"); return MRT_ERR_INVALID; }
    HIP_OK(hipSetDevice(device));
    hipIpcMemHandle_t hh;
    memcpy(&hh, h->handle, sizeof(hh));
    void* base = nullptr;
    HIP_OK(hipIpcOpenMemHandle(&base, hh, hipIpcMemLazyEnablePeerAccess));
    *d_ptr = (char*)base + h->offset;
    std::lock_guard<std::mutex> g(g_ipc_mu);
    g_ipc_maps.emplace_back(*d_ptr, base);
    return MRT_OK;
}

int mrt_ipc_close(void* d_ptr) {
    void* base = nullptr;
    {
        std::lock_guard<std::mutex> g(g_ipc_mu);
        for (size_t i = 0; i < g_ipc_maps.size(); i++)
            if (g_ipc_maps[i].first == d_ptr) {
                base = g_ipc_maps[i].second;
                g_ipc_maps.erase(g_ipc_maps.begin() + (long)i);
                break;
            }
    }
    if (!base) { set_error("not a pointer from mrt_ipc_open"); return MRT_ERR_INVALID; }
    HIP_OK(hipIpcCloseMemHandle(base));
    return MRT_OK;
}

int mrt_render_buckets_async(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts, const int32_t* d_buckets,
                             int32_t n_buckets, float* d_tiles, void* stream) {
    if (!d_tiles) { set_error("bad argument"); return MRT_ERR_INVALID; }
    return mrt_render_batch_async(s, cam, 1, opts, d_buckets, n_buckets, d_tiles, nullptr, stream);
}

int mrt_unpack_batch_async(const int32_t* d_items, int32_t n_items, const float* d_tiles, const uint8_t* d_tiles8,
                           int32_t width, int32_t height, int32_t n_frames, float* d_frames, uint8_t* d_frames8,
                           const mrt_scene* s_for_lut, void* stream) {
    if ((n_items && !d_items) || n_items < 0 || width <= 0 || height <= 0 || n_frames < 1 || (!d_frames && !d_frames8)) {
        set_error("bad argument"); return MRT_ERR_INVALID;
    }
    if (d_frames && !d_tiles) { set_error("float frames need float tiles"); return MRT_ERR_INVALID; }
    if (d_frames8 && !d_tiles8 && !d_tiles) { set_error("rgb8 frames need tiles"); return MRT_ERR_INVALID; }
    const bool need_lut = d_frames8 && !d_tiles8;
    if (need_lut && (!s_for_lut || !s_for_lut->impl.dev)) { set_error("rgb8 needs an uploaded scene for the LUT"); return MRT_ERR_INVALID; }
    if (n_items == 0) return MRT_OK;
    const uint8_t* lut = need_lut ? s_for_lut->impl.dev->gamma : nullptr;
    const int bx = (width + 31) / 32, bpf = bx * ((height + 31) / 32);
    hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)n_items), dim3(256), 0, (hipStream_t)stream, d_items,
                       n_items, d_tiles, d_tiles8, width, height, bx, bpf, n_frames, d_frames, d_frames8, lut);
    HIP_OK(hipGetLastError());
    return MRT_OK;
}

int mrt_unpack_buckets_async(const int32_t* d_buckets, int32_t n_buckets, const float* d_tiles, int32_t width,
                             int32_t height, float* d_frame, uint8_t* d_frame8, const mrt_scene* s_for_lut, void* stream) {
    if (!d_tiles || !d_frame) { set_error("bad argument"); return MRT_ERR_INVALID; }
    return mrt_unpack_batch_async(d_buckets, n_buckets, d_tiles, nullptr, width, height, 1, d_frame, d_frame8,
                                  s_for_lut, stream);
}

// HitInfo of a device hit record (t, a, b, prim bits): m_proxy from the id
static mrt_hit to_hit(const Scene& S, const float4& v) {
    mrt_hit h;
    h.t = v.x; h.a = v.y; h.b = v.z;
    h.prim = __builtin_bit_cast(int32_t, v.w);
    h.inst = -1;
    if (h.prim >= (int32_t)S.obj_mesh.size() && !S.instances.empty()) {
        int lo = 0, hi = (int)S.instances.size() - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (S.instances[mid].hit_base <= h.prim) lo = mid; else hi = mid - 1;
        }
        h.inst = lo;
    }
    return h;
}

// mrt_render over several devices: bucket b of the frame's 32x32 grid
// (src/Scene.cpp:90-95) -> share b mod n, share k rendered on devices[k] from
// that device's scene replica (own stream, persistent item / tile buffers).  The
// frame is assembled on the caller's device: every share's float tiles are
// copied into one gather buffer there (a peer copy over xGMI from another
// device, a device copy from the same one), the caller's stream waits for them
// and one unpack launch scatters them into the frame (+ Image::Map 8-bit), which
// is copied to the caller's host buffers once.  Each pixel is a pure function of
// (scene, camera, pixel, seed), so the frame is bit-identical to a one-device
// render.  Hit records (want_hits, debug / parity) still come back per share.
static int ensure_buf(void*& p, size_t& cap, size_t bytes, hipStream_t sync_on) {
    if (bytes <= cap) return MRT_OK;
    if (p) { HIP_OK(hipStreamSynchronize(sync_on)); (void)hipFree(p); }
    p = nullptr; cap = 0;
    HIP_OK(hipMalloc(&p, bytes ? bytes : 16));
    cap = bytes;
    return MRT_OK;
}
static int render_shared(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts, float* rgb, uint8_t* rgb8,
                         mrt_hit* hits) {
    Scene& S = s->impl;
    const int n = opts->n_devices, W = opts->width, H = opts->height;
    const int bx = (W + 31) / 32, bpf = bx * ((H + 31) / 32);
    const size_t tile_f = 1024 * 3;   // floats per 32x32 bucket tile
    int rc;
    // the caller's device: gather buffer, item list, frame, its own stream
    if ((rc = ensure_device(S, opts->device))) return rc;
    DeviceState& dc = *S.dev;
    HIP_OK(hipSetDevice(dc.device));
    if (!dc.gather_stream) HIP_OK(hipStreamCreateWithFlags(&dc.gather_stream, hipStreamNonBlocking));
    const hipStream_t gs = dc.gather_stream;
    const size_t px = (size_t)W * H;
    if (px > dc.frame_px) {
        HIP_OK(hipStreamSynchronize(gs));
        if (dc.d_rgb) (void)hipFree(dc.d_rgb);
        if (dc.d_rgb8) (void)hipFree(dc.d_rgb8);
        dc.d_rgb = nullptr; dc.d_rgb8 = nullptr; dc.frame_px = 0;
        HIP_OK(hipMalloc((void**)&dc.d_rgb, px * 12));
        HIP_OK(hipMalloc((void**)&dc.d_rgb8, px * 3));
        dc.frame_px = px;
    }
    if ((rc = ensure_buf(reinterpret_cast<void*&>(dc.g_tiles), dc.g_tiles_cap, (size_t)bpf * tile_f * sizeof(float), gs)) ||
        (rc = ensure_buf(reinterpret_cast<void*&>(dc.g_items), dc.g_items_cap, (size_t)bpf * sizeof(int32_t), gs)))
        return rc;
    struct Share {
        int device = -1;
        DeviceState* d = nullptr;
        hipStream_t stream = nullptr;
        ShareBuf* buf = nullptr;
        size_t first = 0, ni = 0;   // its items' offset in the gathered list
        std::vector<float4> hitrec;
    };
    std::vector<Share> sh((size_t)n);
    std::vector<int32_t> all;   // the gathered item list: share 0's buckets, then share 1's, ...
    all.reserve((size_t)bpf);
    for (int k = 0; k < n; k++) {
        sh[k].first = all.size();
        for (int b = k; b < bpf; b += n) all.push_back(b);
        sh[k].ni = all.size() - sh[k].first;
    }
    HIP_OK(hipMemcpyAsync(dc.g_items, all.data(), all.size() * sizeof(int32_t), hipMemcpyHostToDevice, gs));
    rc = MRT_OK;
    for (int k = 0; k < n && rc == MRT_OK; k++) {
        Share& q = sh[k];
        q.device = opts->devices[k];
        if ((rc = ensure_device(S, q.device))) break;
        q.d = S.dev;
        int slot = 0;
        for (int j = 0; j < k; j++) slot += sh[j].device == q.device;
        if (hipSetDevice(q.device) != hipSuccess) { set_error("hipSetDevice"); rc = MRT_ERR_HIP; break; }
        while ((int)q.d->share_streams.size() <= slot) {
            hipStream_t st;
            if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { set_error("stream"); rc = MRT_ERR_HIP; break; }
            q.d->share_streams.push_back(st);
        }
        if (rc) break;
        while ((int)q.d->share_bufs.size() <= slot) q.d->share_bufs.push_back(new ShareBuf());
        q.stream = q.d->share_streams[slot];
        q.buf = q.d->share_bufs[slot];
        if (!q.buf->done && hipEventCreateWithFlags(&q.buf->done, hipEventDisableTiming) != hipSuccess) {
            set_error("event"); rc = MRT_ERR_HIP; break;
        }
        if (q.ni == 0) continue;
        const size_t tb = q.ni * tile_f * sizeof(float);
        if ((rc = ensure_buf(reinterpret_cast<void*&>(q.buf->items), q.buf->items_cap, q.ni * sizeof(int32_t), q.stream)) ||
            (rc = ensure_buf(reinterpret_cast<void*&>(q.buf->tiles), q.buf->tiles_cap, tb, q.stream)))
            break;
        if (hipMemcpyAsync(q.buf->items, all.data() + q.first, q.ni * sizeof(int32_t), hipMemcpyHostToDevice, q.stream) !=
            hipSuccess) {
            set_error("hipMemcpyAsync"); rc = MRT_ERR_HIP; break;
        }
        mrt_render_opts o = *opts;
        o.device = q.device; o.devices = nullptr; o.n_devices = 0;
        o.want_hits = hits ? 1 : 0;
        if ((rc = mrt_render_batch_async(s, cam, 1, &o, q.buf->items, (int32_t)q.ni, q.buf->tiles, nullptr, q.stream))) break;
        // the share's tiles into the caller's gather buffer: over xGMI from a peer, a device copy on the same device
        float* dst = dc.g_tiles + q.first * tile_f;
        hipError_t e;
        if (q.device == dc.device) {
            e = hipMemcpyAsync(dst, q.buf->tiles, tb, hipMemcpyDeviceToDevice, q.stream);
        } else {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, q.device, dc.device) == hipSuccess && can) {
                const hipError_t pe = hipDeviceEnablePeerAccess(dc.device, 0);
                if (pe == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
            }
            e = hipMemcpyPeerAsync(dst, dc.device, q.buf->tiles, q.device, tb, q.stream);
        }
        if (e != hipSuccess || hipEventRecord(q.buf->done, q.stream) != hipSuccess) {
            set_error(std::string("share tile copy: ") + hipGetErrorString(e)); rc = MRT_ERR_HIP; break;
        }
    }
    // the caller's stream: wait for every share's tiles, one unpack, one copy back
    if (rc == MRT_OK) {
        HIP_OK(hipSetDevice(dc.device));
        for (Share& q : sh)
            if (q.ni) HIP_OK(hipStreamWaitEvent(gs, q.buf->done, 0));
        hipLaunchKernelGGL(unpack_kernel, dim3((unsigned)bpf), dim3(256), 0, gs, dc.g_items,
                           (int32_t)bpf, dc.g_tiles, (const uint8_t*)nullptr, W, H, bx, bpf, 1, dc.d_rgb,
                           rgb8 ? dc.d_rgb8 : nullptr, dc.gamma);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(rgb, dc.d_rgb, px * 12, hipMemcpyDeviceToHost, gs));
        if (rgb8) HIP_OK(hipMemcpyAsync(rgb8, dc.d_rgb8, px * 3, hipMemcpyDeviceToHost, gs));
    }
    mrt_stats total{};
    for (int k = 0; k < n && rc == MRT_OK; k++) {
        Share& q = sh[k];
        if (q.ni == 0) continue;
        if (hipSetDevice(q.device) != hipSuccess) { set_error("hipSetDevice"); rc = MRT_ERR_HIP; break; }
        StreamCtx* c = nullptr;
        if ((rc = get_ctx(*q.d, q.stream, c))) break;
        if (hits) {   // debug / parity: the share's hit records to the host
            q.hitrec.resize(q.ni * 1024);
            if (hipMemcpyAsync(q.hitrec.data(), c->hitbuf, q.ni * 1024 * sizeof(float4), hipMemcpyDeviceToHost, q.stream) !=
                hipSuccess) {
                set_error("hipMemcpyAsync"); rc = MRT_ERR_HIP; break;
            }
        }
        if (hipStreamSynchronize(q.stream) != hipSuccess) { set_error("hipStreamSynchronize"); rc = MRT_ERR_HIP; break; }
        // this share's counters (the share's own stream context)
        q.d->last = c;
        S.dev = q.d;
        mrt_stats st{};
        const int src = mrt_scene_last_stats(s, &st);
        if (src && src != MRT_ERR_OVERFLOW) { rc = src; break; }
        total.shadow_rays += st.shadow_rays; total.secondary_rays += st.secondary_rays;
        total.node_visits += st.node_visits; total.leaf_visits += st.leaf_visits;
        total.primary_node_visits += st.primary_node_visits; total.primary_leaf_visits += st.primary_leaf_visits;
        total.primary_hits += st.primary_hits; total.primary_wave_steps += st.primary_wave_steps;
        total.primary_uniform_visits += st.primary_uniform_visits;
        total.kernel_ms = std::max(total.kernel_ms, st.kernel_ms);
        total.fused = st.fused;
        total.chain = st.chain;
        total.max_stack = std::max(total.max_stack, st.max_stack);
        if (src == MRT_ERR_OVERFLOW) rc = src;
        if (hits)
            for (size_t i = 0; i < q.ni; i++) {
                const int b = all[q.first + i], x0 = (b % bx) * 32, y0 = (b / bx) * 32;
                for (int ly = 0; ly < 32 && y0 + ly < H; ly++)
                    for (int lx = 0; lx < 32 && x0 + lx < W; lx++)
                        hits[(size_t)(y0 + ly) * W + x0 + lx] = to_hit(S, q.hitrec[i * 1024 + ly * 32 + lx]);
            }
    }
    // every share and the assembly are done before the caller's buffers are returned
    for (Share& q : sh) {
        if (q.device >= 0) (void)hipSetDevice(q.device);
        if (q.stream) (void)hipStreamSynchronize(q.stream);
    }
    (void)hipSetDevice(dc.device);
    if (hipStreamSynchronize(gs) != hipSuccess && rc == MRT_OK) { set_error("frame assembly"); rc = MRT_ERR_HIP; }
    // the scene's current replica goes back to the caller's device (mrt_trace /
    // mrt_trace_async launch on S.dev->device), not the last share's
    for (DeviceState* d : S.devs)
        if (d->device == opts->device) S.dev = d;
    if (rc && rc != MRT_ERR_OVERFLOW) return rc;
    total.primary_rays = (uint64_t)W * H;
    S.last = total;
    S.stats_final = true;
    S.last_rc = rc;
    if (rc) set_error("traversal stack overflow");
    return rc;
}

int mrt_render(mrt_scene* s, const mrt_camera* cam, const mrt_render_opts* opts, float* rgb, uint8_t* rgb8, mrt_hit* hits) {
    if (!s || !cam || !opts || !rgb || opts->width <= 0 || opts->height <= 0) { set_error("bad argument"); return MRT_ERR_INVALID; }
    if (opts->n_devices < 0 || (opts->n_devices > 0 && !opts->devices)) { set_error("bad device list"); return MRT_ERR_INVALID; }
    if (opts->n_devices > 1 || (opts->n_devices == 1 && opts->devices[0] != opts->device)) {
        if (opts->n_devices > 64) { set_error("at most 64 bucket shares"); return MRT_ERR_INVALID; }
        return render_shared(s, cam, opts, rgb, rgb8, hits);
    }
    Scene& S = s->impl;
    int rc = ensure_device(S, opts->device);
    if (rc) return rc;
    HIP_OK(hipSetDevice(opts->device));
    DeviceState& d = *S.dev;
    size_t px = (size_t)opts->width * opts->height;
    if (px > d.frame_px) {
        if (d.d_rgb) (void)hipFree(d.d_rgb);
        if (d.d_rgb8) (void)hipFree(d.d_rgb8);
        d.d_rgb = nullptr; d.d_rgb8 = nullptr; d.frame_px = 0;
        HIP_OK(hipMalloc((void**)&d.d_rgb, px * 12));
        HIP_OK(hipMalloc((void**)&d.d_rgb8, px * 3));
        d.frame_px = px;
    }
    RenderParams P{};
    fill_params(S, P);
    if ((rc = host_camera(cam, opts->width, opts->height, P.cam[0]))) return rc;
    P.seed = opts->seed ? opts->seed : 0x5EEDu;
    P.mode = 0;
    P.tiles_x = (opts->width + 7) / 8;
    P.n_tiles = P.tiles_x * ((opts->height + 7) / 8);
    P.out_rgb = d.d_rgb;
    P.out_rgb8 = d.d_rgb8;
    if ((rc = launch_render(S, P, px, opts->count_visits != 0, nullptr, hits != nullptr || opts->want_hits))) return rc;
    HIP_OK(hipMemcpy(rgb, d.d_rgb, px * 12, hipMemcpyDeviceToHost));
    if (rgb8) HIP_OK(hipMemcpy(rgb8, d.d_rgb8, px * 3, hipMemcpyDeviceToHost));
    if (hits) {
        std::vector<float4> rec(px);
        HIP_OK(hipMemcpy(rec.data(), d.last->hitbuf, px * sizeof(float4), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < px; i++) hits[i] = to_hit(S, rec[i]);
    }
    S.last.primary_rays = px;
    mrt_stats tmp;
    if ((rc = mrt_scene_last_stats(s, &tmp))) return rc;
    return MRT_OK;
}

int mrt_scene_walk_info(const mrt_scene* cs, int32_t* lds_nodes, int32_t* walk_exits) {
    if (!cs) { set_error("bad argument"); return MRT_ERR_INVALID; }
    const Scene& S = cs->impl;
    const DeviceState* d = S.dev;
    if (lds_nodes) *lds_nodes = d ? (int32_t)d->lds_pick.load() : -1;
    if (walk_exits) {
        *walk_exits = g_walk_exit ? 1 : 2;
    }
    return MRT_OK;
}

int mrt_scene_last_stats(const mrt_scene* cs, mrt_stats* out) {
    if (!cs || !out) { set_error("bad argument"); return MRT_ERR_INVALID; }
    mrt_scene* s = const_cast<mrt_scene*>(cs);
    Scene& S = s->impl;
    if (S.stats_final) {   // multi-device mrt_render: the shares' counters, summed
        *out = S.last;
        if (S.last_rc) set_error("traversal stack overflow");
        return S.last_rc;
    }
    if (!S.dev) { set_error("nothing rendered"); return MRT_ERR_INVALID; }
    DeviceState& d = *S.dev;
    if (!d.last) { set_error("nothing rendered"); return MRT_ERR_INVALID; }
    const StreamCtx& x = *d.last;
    HIP_OK(hipSetDevice(d.device));
    HIP_OK(hipEventSynchronize(x.ev1));
    unsigned long long c[CTR_N];
    HIP_OK(hipMemcpy(c, x.ctr, sizeof c, hipMemcpyDeviceToHost));
    float ms = 0.f, ms1 = 0.f, ms2 = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, x.ev0, x.ev1));
    if (x.last_was_render) {
        HIP_OK(hipEventElapsedTime(&ms1, x.ev0, x.evm));
        HIP_OK(hipEventElapsedTime(&ms2, x.evm, x.ev1));
    }
    S.last.primary_ms = ms1;
    S.last.shade_ms = ms2;
    S.last.primary_node_visits = c[CTR_NODES_P];
    S.last.primary_leaf_visits = c[CTR_LEAVES_P];
    S.last.shadow_rays = c[CTR_SHADOW];
    S.last.primary_hits = c[CTR_HITS];
    if (c[CTR_RAYS_P]) S.last.primary_rays = c[CTR_RAYS_P];
    S.last.secondary_rays = c[CTR_SECONDARY];   // adaptive supersampling: eye rays traced
    S.last.primary_wave_steps = c[CTR_WAVE_STEPS_P];
    S.last.primary_uniform_visits = c[CTR_UNIFORM_P];
    S.last.node_visits = c[CTR_NODES];
    S.last.leaf_visits = c[CTR_LEAVES];
    S.last.max_stack = (int32_t)c[CTR_MAXSP];
    S.last.shadow_wave_steps = c[CTR_WAVE_STEPS_S];
    S.last.shadow_node_visits = c[CTR_NODES_S];
    if (x.last_was_render && c[CTR_TP + 3]) {   // count mode: wave ramp / tail (wall clock)
        const double us = d.wall_khz > 0 ? 1e3 / d.wall_khz : 0.0;
        for (int k = 0; k < 2; k++) {
            // the fused frame kernel is one launch: its span is the primary record's
            const unsigned long long* t = c + ((k && !x.fused) ? CTR_TS : CTR_TP);
            const double s0 = (double)~t[0], s1 = (double)t[1], e0 = (double)~t[2], e1 = (double)t[3];
            float* o = k ? &S.last.shade_span_us : &S.last.primary_span_us;
            o[0] = (float)((e1 - s0) * us);   // first wave start -> last wave end
            o[1] = (float)((s1 - s0) * us);   // ramp: first -> last wave start
            o[2] = (float)((e1 - e0) * us);   // tail: first -> last wave end
        }
    }
    S.last.kernel_ms = ms;
    S.last.fused = x.last_was_render && x.fused ? 1 : 0;
    S.last.chain = x.last_was_render && x.chain_used ? 1 : 0;
    S.last.chain_budget_bytes = x.chain_budget;
    S.last.chain_chunks = x.chain_chunks;
    S.last.chain_fallbacks = (int32_t)c[CTR_FALLBACK];
    *out = S.last;
    if (c[CTR_OVERFLOW]) { set_error("traversal stack overflow"); return MRT_ERR_OVERFLOW; }
    return MRT_OK;
}

int mrt_trace_async(mrt_scene* s, const float* d_o, const float* d_d, const float* d_tmin, const float* d_tmax, size_t n,
                    int any_hit, mrt_hit* d_out, void* stream) {
    if (!s || (n && (!d_o || !d_d || !d_tmin || !d_tmax || !d_out))) { set_error("bad argument"); return MRT_ERR_INVALID; }
    Scene& S = s->impl;
    int dev = S.dev ? S.dev->device : 0;
    int rc = ensure_device(S, dev);
    if (rc) return rc;
    HIP_OK(hipSetDevice(dev));
    DeviceState& d = *S.dev;
    if (n == 0) return MRT_OK;
    StreamCtx* cp = nullptr;
    if ((rc = get_ctx(d, (hipStream_t)stream, cp))) return rc;
    StreamCtx& c = *cp;
    S.stats_final = false;
    HIP_OK(hipMemsetAsync(c.ctr, 0, CTR_N * sizeof(unsigned long long), (hipStream_t)stream));
    c.last_was_render = false;
    int grid = (int)std::min<size_t>((size_t)d.grid, (n + kWG - 1) / kWG);
    HIP_OK(hipEventRecord(c.ev0, (hipStream_t)stream));
    auto kern = any_hit ? (d.special ? trace_kernel<true, true> : trace_kernel<true, false>)
                        : (d.special ? trace_kernel<false, true> : trace_kernel<false, false>);
    Trav alpha{};
    alpha.aprims = d.prims; alpha.apuv = d.puv; alpha.auv = d.uvs; alpha.amats = d.mats; alpha.atex = d.texs;
    alpha.pflags = d.pflags; alpha.verts = d.verts; alpha.verts2 = d.verts2;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kWG), 0, (hipStream_t)stream, d.nodes, d.leaves, d.tables, c.gstack,
                       d.gthreads, d_o, d_d, d_tmin, d_tmax, n, d_out, c.ctr, fast_box(d), d.insts, alpha);
    HIP_OK(hipGetLastError());
    HIP_OK(hipEventRecord(c.ev1, (hipStream_t)stream));
    d.last = &c;
    return MRT_OK;
}

int mrt_trace(mrt_scene* s, const float* o, const float* d, const float* tmin, const float* tmax, size_t n, int any_hit,
              mrt_hit* out) {
    if (!s || (n && (!o || !d || !tmin || !tmax || !out))) { set_error("bad argument"); return MRT_ERR_INVALID; }
    Scene& S = s->impl;
    int dev = S.dev ? S.dev->device : 0;
    int rc = ensure_device(S, dev);
    if (rc) return rc;
    if (n == 0) return MRT_OK;
    HIP_OK(hipSetDevice(dev));
    float *bo = nullptr, *bd = nullptr, *bmin = nullptr, *bmax = nullptr;
    mrt_hit* bout = nullptr;
    HIP_OK(hipMalloc((void**)&bo, n * 12));
    HIP_OK(hipMalloc((void**)&bd, n * 12));
    HIP_OK(hipMalloc((void**)&bmin, n * 4));
    HIP_OK(hipMalloc((void**)&bmax, n * 4));
    HIP_OK(hipMalloc((void**)&bout, n * sizeof(mrt_hit)));
    HIP_OK(hipMemcpy(bo, o, n * 12, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(bd, d, n * 12, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(bmin, tmin, n * 4, hipMemcpyHostToDevice));
    HIP_OK(hipMemcpy(bmax, tmax, n * 4, hipMemcpyHostToDevice));
    rc = mrt_trace_async(s, bo, bd, bmin, bmax, n, any_hit, bout, nullptr);
    if (rc == MRT_OK) {
        HIP_OK(hipMemcpy(out, bout, n * sizeof(mrt_hit), hipMemcpyDeviceToHost));
        unsigned long long c[CTR_N];
        HIP_OK(hipMemcpy(c, S.dev->last->ctr, sizeof c, hipMemcpyDeviceToHost));
        if (c[CTR_OVERFLOW]) { set_error("traversal stack overflow"); rc = MRT_ERR_OVERFLOW; }
    }
    (void)hipFree(bo); (void)hipFree(bd); (void)hipFree(bmin); (void)hipFree(bmax); (void)hipFree(bout);
    return rc;
}

int mrt_debug_wave_log(const mrt_scene* cs, int launch, uint64_t* out, int32_t max_waves) {
    if (!cs || !out || launch < 0 || launch > 1 || max_waves < 0) { set_error("bad argument"); return MRT_ERR_INVALID; }
    const Scene& S = cs->impl;
    if (!S.dev) { set_error("nothing rendered"); return MRT_ERR_INVALID; }
    const DeviceState& d = *S.dev;
    HIP_OK(hipSetDevice(d.device));
    if (!d.last) { set_error("nothing rendered"); return MRT_ERR_INVALID; }
    HIP_OK(hipEventSynchronize(d.last->ev1));
    const int n = std::min(max_waves, d.last->log_waves[launch]);
    const size_t log_stride = (size_t)d.grid * (kWG / 64) * kLogWords;
    if (n > 0)
        HIP_OK(hipMemcpy(out, d.last->wave_log + launch * log_stride, (size_t)n * kLogWords * sizeof(uint64_t),
                         hipMemcpyDeviceToHost));
    return n;
}

int mrt_device_wall_clock_khz(const mrt_scene* cs) {
    if (!cs || !cs->impl.dev) { set_error("scene not on a device"); return MRT_ERR_INVALID; }
    return cs->impl.dev->wall_khz;
}

int mrt_set_tuning(const char* key, int value) {
    if (!key) { set_error("null key"); return MRT_ERR_INVALID; }
    std::string k(key);
    if (k == "fast_box") g_fast_box = value ? 1 : 0;
    else if (k == "primary_waves") {
        if (value != 0 && value != 1 && (value < 6 || value > 8)) { set_error("primary_waves must be 0 or 6..8"); return MRT_ERR_INVALID; }
        g_primary_waves = value;
    } else if (k == "scalar_nodes") {   // bit 0 nodes, bit 1 triangles (1 = round 3's nodes only), bit 2 octant box test
        if (value < 0 || value > 7) { set_error("scalar_nodes must be 0..7"); return MRT_ERR_INVALID; }
        g_scalar_nodes = value;
    } else if (k == "batch_tpw") {
        if (value < 1 || value > 64) { set_error("batch_tpw must be 1..64"); return MRT_ERR_INVALID; }
        g_batch_tpw = value;
    } else if (k == "wave_log") {
        g_wave_log = value ? 1 : 0;
    } else if (k == "shade1") {
        g_shade1 = value ? 1 : 0;
    } else if (k == "wavefront") {
        g_wavefront = value ? 1 : 0;
    } else if (k == "chain") {
        g_chain = value ? 1 : 0;
    } else if (k == "chain_mb") {
        if (value < 1 || value > 1 << 20) { set_error("chain_mb out of range"); return MRT_ERR_INVALID; }
        g_chain_mb = value;
    } else if (k == "shadow_sched") {
        if (value < -1 || value > 2) { set_error("shadow_sched must be -1..2"); return MRT_ERR_INVALID; }
        g_shadow_sched = value;
    } else if (k == "primary_inst_waves") {
        if (value != 1 && value != 4 && value != 5 && value != 6) {
            set_error("primary_inst_waves must be 1, 4, 5 or 6"); return MRT_ERR_INVALID;
        }
        g_primary_inst_waves = value;
    } else if (k == "adapt_refill") {
        if (value < 0 || value > 64) { set_error("adapt_refill must be 0..64"); return MRT_ERR_INVALID; }
        g_adapt_refill = value;
    } else if (k == "chain_shadow_step") {
        g_chain_shadow_step = value ? 1 : 0;
    } else if (k == "near_first") {
        if (value < -1 || value > 1) { set_error("near_first must be -1..1"); return MRT_ERR_INVALID; }
        g_near_first = value;
    } else if (k == "fused") {
        g_fused = value ? 1 : 0;
    } else if (k == "chain_est") {
        g_chain_est = value ? 1 : 0;
    } else if (k == "chain_est_pct") {
        if (value < 1 || value > 100000) { set_error("chain_est_pct must be 1..100000"); return MRT_ERR_INVALID; }
        g_chain_est_pct = value;
    } else if (k == "chain_shadow_refill") {
        g_chain_shadow_refill = value ? 1 : 0;
    } else if (k == "bin_inst") {
        if (value < 0 || value > 2) { set_error("bin_inst must be 0..2"); return MRT_ERR_INVALID; }
        g_bin_inst = value;
    } else if (k == "chain_bands") {
        if (value < -1 || value > 1) { set_error("chain_bands must be -1..1"); return MRT_ERR_INVALID; }
        g_chain_bands = value;
    } else if (k == "dome_replay") {
        g_dome_replay = value ? 1 : 0;
    } else if (k == "bin") {
        if (value < -1 || value > 7) { set_error("bin must be -1 (auto) or 0..7"); return MRT_ERR_INVALID; }
        g_bin = value;
    } else if (k == "bin_dbits") {   // the pair is checked when a batch is binned (2 dbits + 3 obits = 1..12)
        if (value < 0 || value > 6) { set_error("bin_dbits must be 0..6"); return MRT_ERR_INVALID; }
        g_bin_dbits = value;
    } else if (k == "bin_obits") {
        if (value < 0 || value > 4) { set_error("bin_obits must be 0..4"); return MRT_ERR_INVALID; }
        g_bin_obits = value;
    } else if (k == "walk_latch") {
        if (value < 0 || value > 1) { set_error("walk_latch must be 0 or 1"); return MRT_ERR_INVALID; }
        g_walk_latch = value;
    } else if (k == "walk_exit") {
        if (value < 0 || value > 1) { set_error("walk_exit must be 0 or 1"); return MRT_ERR_INVALID; }
        g_walk_exit = value;
    } else if (k == "lds_nodes") {
        if (value < 0 || value > 1) { set_error("lds_nodes must be 0 or 1"); return MRT_ERR_INVALID; }
        g_lds_nodes = value;
    } else if (k == "frame1_waves") {
        if (value != 1 && (value < 5 || value > 8)) { set_error("frame1_waves must be 1 or 5..8"); return MRT_ERR_INVALID; }
        g_frame1_waves = value;
    } else if (k == "sched") {
        if (value < 0 || value > 3) { set_error("sched must be 0..3"); return MRT_ERR_INVALID; }
        g_sched = value;
    } else { set_error("unknown tuning key " + k); return MRT_ERR_INVALID; }
    return MRT_OK;
}

int mrt_debug_libm(int fn, const float* x, const float* y, size_t n, float* out) {
    if (fn < 0 || fn > 5 || !x || !out || ((fn == 1 || fn == 5) && !y)) { set_error("bad libm probe arguments"); return MRT_ERR_INVALID; }
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || nd <= 0) { set_error("no HIP device"); return MRT_ERR_NO_DEVICE; }
    if (n == 0) return MRT_OK;
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    uint16_t* dt = nullptr;
    const size_t b = n * sizeof(float);
    int rc = MRT_OK;
    auto run = [&]() -> int {
        HIP_OK(hipMalloc((void**)&dx, b));
        HIP_OK(hipMalloc((void**)&dy, b));
        HIP_OK(hipMalloc((void**)&dout, b));
        HIP_OK(hipMalloc((void**)&dt, 2048 * sizeof(uint16_t)));
        HIP_OK(hipMemcpy(dx, x, b, hipMemcpyHostToDevice));
        if (fn == 1 || fn == 5) HIP_OK(hipMemcpy(dy, y, b, hipMemcpyHostToDevice));
        HIP_OK(hipMemcpy(dt, host_rcp_table(), 2048 * sizeof(uint16_t), hipMemcpyHostToDevice));
        const int blocks = (int)std::min<size_t>((n + 255) / 256, 65536);
        hipLaunchKernelGGL(libm_kernel, dim3(blocks), dim3(256), 0, 0, fn, dx, dy, n, dout, dt);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpy(out, dout, b, hipMemcpyDeviceToHost));
        return MRT_OK;
    };
    rc = run();
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    if (dout) (void)hipFree(dout);
    if (dt) (void)hipFree(dt);
    return rc;
}

float mrt_rcp_nr(float x) { return rcp_nr(x, host_rcp_table()); }
float mrt_rsqrt_nr(float x) { return rsqrt_nr(x, host_rsqrt_table()); }

}  // extern "C"
