// ngrtd_dz_lw.hip -- the single-launch DEMetropolisZ instances with the sampled CFC12
// half-life (logp_fused_kernel MIX bit 5, lw_decay): their own translation unit (compiled
// like ngrtd_dz.hip, without machine LICM) so that the instances build in parallel.
#include <hip/hip_runtime.h>

#include "../../include/ngrtd.h"
#define NGRTD_FUSED_ONLY
#include "ngrtd_kernels.hpp"

namespace ngrtd {

template <int MIX>
static hipError_t launch_dz_lw_mix(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                   const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&logp_fused_kernel<5, true, 2, MIX>), hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)max_lds);
    (void)attr;
    const unsigned nb = (unsigned)((W + WB - 1) / WB);
    hipLaunchKernelGGL((logp_fused_kernel<5, true, 2, MIX>), dim3(nb), dim3(64 * kFusedWaves * 2), lds, st, a, u, WB,
                       logp, da);
    return hipGetLastError();
}

// 32 | 8 | EPM 2 | Jacobian 4 | per-well chains 16 (ngrtd_dz.hip fused_dz_instance_exists)
hipError_t launch_fused_dz_lw_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                       const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    switch (mix) {
    case 40: return launch_dz_lw_mix<40>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 42: return launch_dz_lw_mix<42>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 44: return launch_dz_lw_mix<44>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 46: return launch_dz_lw_mix<46>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 56: return launch_dz_lw_mix<56>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 58: return launch_dz_lw_mix<58>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 60: return launch_dz_lw_mix<60>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 62: return launch_dz_lw_mix<62>(a, u, WB, W, logp, da, lds, max_lds, st);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace ngrtd
