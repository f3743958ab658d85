// mrt_bin.hip -- ray binning (see mrt_bin.h): counting sort of a ray batch by
// direction cell and origin cell.  Three launches, no library sort: one pass
// over the rays for per-block histograms, one scan of at most 4096 bins, one
// pass that scatters each block's rays into its reserved ranges.
#include <string>

#include "../../include/mrt.h"
#include "mrt_bin.h"

namespace mrt {

void set_error(const std::string& m);

static constexpr int kBinWG = 256;

__device__ __forceinline__ uint32_t bin_items(const BinArgs& A) {
    if (!A.n_dev) return A.n;
    uint64_t v = (uint64_t)*A.n_dev * A.mul1;
    v = v > A.sub ? v - A.sub : 0;
    if (v > A.cap1) v = A.cap1;
    v *= A.mul2;
    return v < A.n ? (uint32_t)v : A.n;
}

// block b's contiguous item range (both passes use the same split)
__device__ __forceinline__ void bin_range(uint32_t n, uint32_t& lo, uint32_t& hi) {
    const uint32_t per = ((n + gridDim.x - 1) / gridDim.x + (kBinWG - 1)) & ~(uint32_t)(kBinWG - 1);
    lo = min(n, (uint32_t)blockIdx.x * per);
    hi = min(n, lo + per);
}

__device__ __forceinline__ int bin_cell(float x, int n) {
    const float c = fminf(fmaxf(x, 0.0f), (float)(n - 1));   // NaN -> 0 (fmaxf returns the number)
    return (int)c;
}

__device__ __forceinline__ uint32_t bin_key(const BinArgs& A, float4 o, float4 d) {
    // octahedral map of the direction to [-1, 1]^2 (lower hemisphere folded)
    const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    const float is = s > 0.0f ? 1.0f / s : 0.0f;
    float u = d.x * is, v = d.y * is;
    if (d.z < 0.0f) {
        const float u2 = (1.0f - fabsf(v)) * (u >= 0.0f ? 1.0f : -1.0f);
        v = (1.0f - fabsf(u)) * (v >= 0.0f ? 1.0f : -1.0f);
        u = u2;
    }
    const int nd = 1 << A.dbits, no = 1 << A.obits;
    const uint32_t iu = (uint32_t)bin_cell((u * 0.5f + 0.5f) * (float)nd, nd);
    const uint32_t iv = (uint32_t)bin_cell((v * 0.5f + 0.5f) * (float)nd, nd);
    const uint32_t cx = (uint32_t)bin_cell((o.x - A.lo[0]) * A.inv[0], no);
    const uint32_t cy = (uint32_t)bin_cell((o.y - A.lo[1]) * A.inv[1], no);
    const uint32_t cz = (uint32_t)bin_cell((o.z - A.lo[2]) * A.inv[2], no);
    uint32_t mort = 0;
    for (int b = 0; b < A.obits; b++)
        mort |= (((cx >> b) & 1u) << (3 * b)) | (((cy >> b) & 1u) << (3 * b + 1)) | (((cz >> b) & 1u) << (3 * b + 2));
    return (((iu << A.dbits) | iv) << (3 * A.obits)) | mort;
}

// instance-major key of ray i (BinArgs::hits): 1 << 11 | class << 4 | direction cell
// (2 x 2 bits) when its pixel's primary hit is on an instance, else the plain key
// (which stays below 1 << 11: dbits = obits = 2)
__device__ __forceinline__ uint32_t bin_key_inst(const BinArgs& A, uint32_t i, float4 o, float4 d) {
    const int32_t prim = __float_as_int(A.hits[i / A.m].w);
    if (prim < A.n_world) return bin_key(A, o, d);
    int lo = 0, hi = A.n_inst - 1;   // the last instance whose hit_base <= prim
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (A.hit_base[mid] <= prim) lo = mid; else hi = mid - 1;
    }
    const uint32_t dir = bin_key(A, o, d) >> (3 * A.obits);   // the direction cell
    if (A.inst_cell) {   // object-space cell of the origin in its BLAS
        const float* M = A.insts[lo].inv;
        const float4 c0 = A.inst_cell[2 * lo], c1 = A.inst_cell[2 * lo + 1];
        const float ox = M[0] * o.x + M[1] * o.y + M[2] * o.z + M[3];
        const float oy = M[4] * o.x + M[5] * o.y + M[6] * o.z + M[7];
        const float oz = M[8] * o.x + M[9] * o.y + M[10] * o.z + M[11];
        const uint32_t cx = (uint32_t)min(3, max(0, (int)((ox - c0.x) * c1.x)));
        const uint32_t cy = (uint32_t)min(3, max(0, (int)((oy - c0.y) * c1.y)));
        const uint32_t cz = (uint32_t)min(3, max(0, (int)((oz - c0.z) * c1.z)));
        const uint32_t morton = (cx & 1u) | (cy & 1u) << 1 | (cz & 1u) << 2 | (cx >> 1) << 3 | (cy >> 1) << 4 | (cz >> 1) << 5;
        return (1u << 11) | ((c0.w != 0.f) ? 1u << 10 : 0u) | morton << 4 | dir;
    }
    return (1u << 11) | ((uint32_t)A.inst_class[lo] << (2 * A.dbits)) | dir;
}

__device__ __forceinline__ bool bin_valid(const BinArgs& A, uint32_t i) {
    if (!A.nrays) return true;
    const uint32_t px = i / A.m;
    return i - px * A.m < (uint32_t)A.nrays[px];
}

__global__ void __launch_bounds__(kBinWG) bin_count_kernel(BinArgs A) {
    __shared__ uint32_t h[1 << kBinBits];
    const int K = 1 << A.bits;
    for (int i = threadIdx.x; i < K; i += kBinWG) h[i] = 0;
    __syncthreads();
    uint32_t lo, hi;
    bin_range(bin_items(A), lo, hi);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kBinWG) {
        uint16_t k = kBinInvalid;
        if (bin_valid(A, i)) {
            k = (uint16_t)(A.hits ? bin_key_inst(A, i, A.o[i], A.d[i]) : bin_key(A, A.o[i], A.d[i]));
            atomicAdd(&h[k], 1u);
        }
        A.keys[i] = k;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < K; i += kBinWG)
        if (h[i]) atomicAdd(&A.hist[i], h[i]);
}

// one workgroup: exclusive scan of the bin counts (in place: each bin's first
// position, the scatter's cursor) and the total
__global__ void __launch_bounds__(1024) bin_scan_kernel(BinArgs A) {
    __shared__ uint32_t part[1024];
    const int K = 1 << A.bits;
    const int per = (K + 1023) / 1024, t = threadIdx.x, b0 = t * per;
    uint32_t s = 0;
    for (int j = 0; j < per; j++)
        if (b0 + j < K) s += A.hist[b0 + j];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {   // inclusive Hillis-Steele scan of the thread sums
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = t ? part[t - 1] : 0u;
    for (int j = 0; j < per; j++) {
        if (b0 + j >= K) break;
        const uint32_t c = A.hist[b0 + j];
        A.hist[b0 + j] = run;
        run += c;
    }
    if (t == 1023) A.hist[K] = part[1023];
}

__global__ void __launch_bounds__(kBinWG) bin_scatter_kernel(BinArgs A) {
    __shared__ uint32_t h[1 << kBinBits];
    const int K = 1 << A.bits;
    for (int i = threadIdx.x; i < K; i += kBinWG) h[i] = 0;
    __syncthreads();
    uint32_t lo, hi;
    bin_range(bin_items(A), lo, hi);
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kBinWG) {
        const uint16_t k = A.keys[i];
        if (k != kBinInvalid) atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < K; i += kBinWG)   // this block's range in each bin
        if (h[i]) h[i] = atomicAdd(&A.hist[i], h[i]);
    __syncthreads();
    for (uint32_t i = lo + threadIdx.x; i < hi; i += kBinWG) {
        const uint16_t k = A.keys[i];
        if (k != kBinInvalid) A.perm[atomicAdd(&h[k], 1u)] = i;
    }
}

int bin_rays(const BinArgs& A0, int grid, hipStream_t stream) {
    BinArgs A = A0;
    A.bits = A.hits ? kBinBits : 2 * A.dbits + 3 * A.obits;
    if (A.hits && (A.dbits != 2 || A.obits != 2 || A.n_inst < 1 || !A.hit_base || !A.inst_class || A.m < 1)) {
        set_error("instance-major ray-bin keys need dbits = obits = 2 and the instance tables");
        return MRT_ERR_INVALID;
    }
    const int bits = A.bits;
    if (A.dbits < 0 || A.obits < 0 || bits < 1 || bits > kBinBits) { set_error("bad ray-bin key bits"); return MRT_ERR_INVALID; }
    const int K = 1 << bits;
    hipError_t e = hipMemsetAsync(A.hist, 0, (size_t)(K + 1) * sizeof(uint32_t), stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(bin_count_kernel, dim3(grid), dim3(kBinWG), 0, stream, A);
        hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(1024), 0, stream, A);
        hipLaunchKernelGGL(bin_scatter_kernel, dim3(grid), dim3(kBinWG), 0, stream, A);
        e = hipGetLastError();
    }
    if (e != hipSuccess) { set_error(std::string("bin_rays: ") + hipGetErrorString(e)); return MRT_ERR_HIP; }
    return MRT_OK;
}

}  // namespace mrt
