// ngrtd_lw.hip -- the log-prob instances of logp_fused_kernel with the sampled CFC12
// half-life (MIX bit 5, lw_decay; the reference's savenum-123 runs, run_age_mcmc.py:180-198):
// a translation unit of their own so that they compile in parallel with ngrtd.hip.
#include <hip/hip_runtime.h>

#include "../../include/ngrtd.h"
#define NGRTD_FUSED_ONLY
#include "ngrtd_kernels.hpp"

namespace ngrtd {

template <int C, bool FULL, int MIX>
static hipError_t launch_lw(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
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

template <int C>
static hipError_t launch_lw_partial(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                    const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    switch (mix) {
    case 32: return launch_lw<C, false, 32>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 33: return launch_lw<C, false, 33>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 34: return launch_lw<C, false, 34>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 35: return launch_lw<C, false, 35>(a, u, WB, W, logp, da, lds, max_lds, st);
    default: return hipErrorInvalidValue;
    }
}

// The LW log-prob instance (channels C, FULL: the joint plan, mix: 32 | piston 1 | EPM 2 |
// Jacobian 4 (FULL only)): FULL at C = 5 (32..36, 38), the other plans at C = 4, 5 (32..35).
hipError_t launch_fused_lw_instance(int C, bool full, int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W,
                                    double* logp, const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    if (full) {
        if (C != 5) return hipErrorInvalidValue;
        switch (mix) {
        case 32: return launch_lw<5, true, 32>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 33: return launch_lw<5, true, 33>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 34: return launch_lw<5, true, 34>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 35: return launch_lw<5, true, 35>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 36: return launch_lw<5, true, 36>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 38: return launch_lw<5, true, 38>(a, u, WB, W, logp, da, lds, max_lds, st);
        default: return hipErrorInvalidValue;
        }
    }
    if (C == 4) return launch_lw_partial<4>(mix, a, u, WB, W, logp, da, lds, max_lds, st);
    if (C == 5) return launch_lw_partial<5>(mix, a, u, WB, W, logp, da, lds, max_lds, st);
    return hipErrorInvalidValue;
}

}  // namespace ngrtd
