// ngrtd_dz_gen.hip -- the single-launch DEMetropolisZ instances of logp_fused_kernel for the generic
// model pairs without a dispersion component: MIX 8 (the step) | 64 (generic components, run_age_mcmc.py:61-70 pairs
// without a specialised instance) | 4 (PyMC3's transformed space) | 16 (per-well chains), on the
// c4 shape (C = 5, FULL).  Compiled with machine LICM off like ngrtd_dz.hip (__graft_entry__.py).
#include <hip/hip_runtime.h>

#include "../../include/ngrtd.h"
#define NGRTD_FUSED_ONLY
#include "ngrtd_kernels.hpp"

namespace ngrtd {

template <int MIX>
static hipError_t launch_dz_gen(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
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

hipError_t launch_fused_dz_gen_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                       const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    switch (mix) {
    case 72: return launch_dz_gen<72>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 76: return launch_dz_gen<76>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 88: return launch_dz_gen<88>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 92: return launch_dz_gen<92>(a, u, WB, W, logp, da, lds, max_lds, st);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace ngrtd
