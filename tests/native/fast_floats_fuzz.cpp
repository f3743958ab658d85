// Fuzz harness: fast_floats (csrc/host_build.cpp) against glibc sscanf("%f %f %f").

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <random>
// @FAST_FLOATS@ (spliced from csrc/host_build.cpp by tests/test_obj_loader.py)
int main(int argc, char** argv) {
  std::mt19937_64 g(12345);
  long bad = 0, fast = 0, n = argc > 1 ? atol(argv[1]) : 1000000;
  char buf[128];
  for (long it = 0; it < n; it++) {
    int kind = g() % 6;
    double x;
    uint64_t r = g();
    switch (kind) {
      case 0: x = (double)(int64_t)(r % 2000000001) / 1e6 - 1000; snprintf(buf, sizeof buf, "%.6f", x); break;
      case 1: { float f; uint32_t b = (uint32_t)r; memcpy(&f, &b, 4); if (!(f == f)) f = 1; snprintf(buf, sizeof buf, "%.9g", f); break; }
      case 2: { float f; uint32_t b = (uint32_t)r; memcpy(&f, &b, 4); if (!(f == f)) f = 1; snprintf(buf, sizeof buf, "%.8e", f); break; }
      case 3: snprintf(buf, sizeof buf, "%llu.%llue%d", (unsigned long long)(r % 100000000), (unsigned long long)(g() % 1000000000), (int)(g() % 60) - 30); break;
      case 4: snprintf(buf, sizeof buf, "%.17g", (double)(r % 100000) * 1e-5 + 0.5); break;
      default: { double d = (double)(r >> 11) * (1.0 / 9007199254740992.0); snprintf(buf, sizeof buf, "%.*f", (int)(g() % 12) + 1, d * 100); }
    }
    char line[160];
    snprintf(line, sizeof line, " %.40s %.40s -%.40s\n", buf, buf, buf);
    float a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
    sscanf(line, "%f %f %f\n", &a[0], &a[1], &a[2]);
    if (fast_floats(line, 3, b)) {
      fast++;
      if (memcmp(a, b, sizeof a)) { if (bad < 10) printf("MISMATCH '%s' %a %a\n", buf, a[0], b[0]); bad++; }
    }
  }
  printf("fast-path %ld of %ld, mismatches %ld\n", fast, n, bad);
}
