// mrt_rec.hip -- instantiations of the fused chain kernels (Shader REC 1 / 2:
// Blinn reflection / refraction chains and path tracing traced inline) and of
// the adaptive supersampling kernels.  A translation unit of its own so the
// library's kernels compile in parallel (the shading code is mrt_shader.h).
#include "mrt_shader.h"

namespace mrt {

template <bool C, bool PO, bool F, bool I, int REC>
struct AdaptK { static constexpr KernelFn fn = adaptive_kernel<C, PO, F, I, REC>; };

KernelFn pick_shade_rec(bool c, bool po, bool f, bool inst, int rec) {
    if (rec == 2) return pick4<ShadeK, 2>(c, po, f, inst);
    return pick4<ShadeK, 1>(c, po, f, inst);
}

// direct-lighting adaptive kernels (timed variants) at an occupancy target:
// unbounded, the compiler gives them all 256 VGPRs (one wave per SIMD)
template <int W, int REC = 0>
static KernelFn adapt_direct(bool po, bool f, bool inst) {
    if (inst) return f ? adaptive_kernel<false, false, true, true, REC, W> : adaptive_kernel<false, false, false, true, REC, W>;
    if (po) return f ? adaptive_kernel<false, true, true, false, REC, W> : adaptive_kernel<false, true, false, false, REC, W>;
    return f ? adaptive_kernel<false, false, true, false, REC, W> : adaptive_kernel<false, false, false, false, REC, W>;
}

KernelFn pick_adaptive(bool c, bool po, bool f, bool inst, int rec) {
    if (rec == 0 && !c) return adapt_direct<6>(po, f, inst);   // 4 / 5 waves measured 6% / 1% slower on A3
    // (REC 1 / 2 kernels bounded to 2 or 3 waves still end at one: no variants)
    if (rec == 2) return pick4<AdaptK, 2>(c, po, f, inst);
    if (rec == 1) return pick4<AdaptK, 1>(c, po, f, inst);
    return pick4<AdaptK, 0>(c, po, f, inst);
}

}  // namespace mrt
