// Issue cost of packed f32 VALU (v_pk_add_f32 / v_pk_mul_f32) against the scalar
// v_add_f32 / v_mul_f32 doing the same lanes' work, on gfx950: every lane runs
// ITER iterations of 8 independent (sub, mul) chains -- the box test's slab form,
// (p - o) * id -- as 16 scalar pairs or 8 packed pairs.  Prints ns per launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int ITER = 4096;

__global__ void __launch_bounds__(256) scalar_k(const float* in, float* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    float a[16], o = in[i & 1023], id = in[(i + 7) & 1023];
#pragma unroll
    for (int k = 0; k < 16; k++) a[k] = in[(i + k) & 1023];
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int k = 0; k < 16; k++) a[k] = (a[k] - o) * id;
        asm volatile("" : "+v"(o), "+v"(id));
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k++) s += a[k];
    out[i] = s;
}
__global__ void __launch_bounds__(256) packed_k(const float* in, float* out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    f2v a[8];
    f2v o = {in[i & 1023], in[i & 1023]}, id = {in[(i + 7) & 1023], in[(i + 7) & 1023]};
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = (f2v){in[(i + 2 * k) & 1023], in[(i + 2 * k + 1) & 1023]};
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) a[k] = (a[k] - o) * id;
        asm volatile("" : "+v"(o), "+v"(id));
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k].x + a[k].y;
    out[i] = s;
}

int main() {
    float *in, *out;
    const int blocks = 256 * 4 * 8 / 4;   // 8 waves per SIMD
    hipMalloc(&in, 1024 * 4);
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    float h[1024];
    for (int k = 0; k < 1024; k++) h[k] = 1.0f + k * 1e-3f;
    hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; rep++) {
        for (int v = 0; v < 2; v++) {
            hipEventRecord(e0);
            if (v == 0) scalar_k<<<blocks, 256>>>(in, out);
            else packed_k<<<blocks, 256>>>(in, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // 32 slab ops (16 sub + 16 mul) per lane per iteration either way
            const double ops = (double)blocks * 256 * ITER * 32;
            printf("%s: %.3f ms  %.1f Gop/s per lane-op  (%.2f cyc per wave-instr-equiv @2.4GHz/1024 SIMD)\n",
                   v ? "packed" : "scalar", ms, ops / ms / 1e6,
                   ms * 1e-3 * 2.4e9 * 1024 / ((double)blocks * 4 * ITER * (v ? 16 : 32)));
        }
    }
    return 0;
}
