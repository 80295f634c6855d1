// ngrtd_gen_disp.hip -- the generic log-prob instances for plans with a dispersion component
// (MIX bits 6 and 7: the channel table and the per-age aux staged in LDS, the exact age sum
// split over the unit's theta and RTD waves; ngrtd_gen.hip holds the others).  A translation
// unit of its own, compiled in parallel.
#include <hip/hip_runtime.h>

#include "../../include/ngrtd.h"
#define NGRTD_FUSED_ONLY
#include "ngrtd_kernels.hpp"

namespace ngrtd {

template <int C, bool FULL, int MIX>
static hipError_t launch_gen(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                             const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&logp_fused_kernel<C, FULL, 2, MIX>), hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)max_lds);
    (void)attr;
    const unsigned nb = (unsigned)((W + WB - 1) / WB);
    hipLaunchKernelGGL((logp_fused_kernel<C, FULL, 2, MIX>), dim3(nb), dim3(64 * kFusedWaves * 2), lds, st, a, u, WB,
                       logp, da);
    return hipGetLastError();
}

hipError_t launch_fused_gen_disp_instance(int C, bool full, int mix, const RtdArgs& a, const UnitArgs& u, int WB,
                                          int64_t W, double* logp, const DemcAccept& da, size_t lds, size_t max_lds,
                                          hipStream_t st) {
    mix &= ~128;
    if (full) {
        switch (mix) {
        case 64: return launch_gen<5, true, 192>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 68: return launch_gen<5, true, 196>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 96: return launch_gen<5, true, 224>(a, u, WB, W, logp, da, lds, max_lds, st);
        default: return launch_gen<5, true, 228>(a, u, WB, W, logp, da, lds, max_lds, st);
        }
    }
    if (mix == 96) {
        if (C == 4) return launch_gen<4, false, 224>(a, u, WB, W, logp, da, lds, max_lds, st);
        return launch_gen<5, false, 224>(a, u, WB, W, logp, da, lds, max_lds, st);
    }
    switch (C) {
    case 1: return launch_gen<1, false, 192>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 2: return launch_gen<2, false, 192>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 3: return launch_gen<3, false, 192>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 4: return launch_gen<4, false, 192>(a, u, WB, W, logp, da, lds, max_lds, st);
    default: return launch_gen<5, false, 192>(a, u, WB, W, logp, da, lds, max_lds, st);
    }
}

}  // namespace ngrtd
