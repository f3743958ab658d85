// Sweep of the product's rcp_nr (libmrt.so, host build of csrc/mrt_math.h) against the
// oracle's (oracle/mrt_oracle.c) over every stride-th float bit pattern from `start`:
//   rcp_sweep <libmrt.so> <libmrt_oracle.so> <stride> [start]
// Prints "checked N mismatches M" (and the first mismatches).
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef float (*fn_t)(float);

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    void* a = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    void* b = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
    if (!a || !b) { printf("dlopen: %s\n", dlerror()); return 2; }
    fn_t prod = (fn_t)dlsym(a, "mrt_rcp_nr"), orc = (fn_t)dlsym(b, "oro_rcp_nr");
    if (!prod || !orc) { printf("dlsym failed\n"); return 2; }
    const uint64_t stride = strtoull(argv[3], 0, 10), start = argc > 4 ? strtoull(argv[4], 0, 10) : 0;
    uint64_t n = 0, bad = 0;
    for (uint64_t v = start; v < (1ull << 32); v += stride) {
        uint32_t u = (uint32_t)v, p, q;
        float x;
        memcpy(&x, &u, 4);
        float fp = prod(x), fq = orc(x);
        memcpy(&p, &fp, 4);
        memcpy(&q, &fq, 4);
        n++;
        if (p != q) {
            if (bad < 8) printf("MISMATCH x=%08x prod=%08x oracle=%08x\n", u, p, q);
            bad++;
        }
    }
    printf("checked %llu mismatches %llu\n", (unsigned long long)n, (unsigned long long)bad);
    return bad != 0;
}
