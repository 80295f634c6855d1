// ngrtd_gen.hip -- the generic log-prob instances of logp_fused_kernel (MIX bit 6,
// gen_component): the model pairs of run_age_mcmc.py:61-70 without a specialised instance --
// a piston or dispersion first component, and BMMs whose second component is exponential,
// exp_pist_flow or dispersion.  A translation unit of its own (compiled in parallel with
// ngrtd.hip).
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

// The instances: FULL (the joint plan) at C = 5 with / without the Jacobians and the sampled
// CFC12 half-life (64, 68, 96, 100); the other plans (RTD-only, forward()) at C = 1..5 (64)
// and, with the half-life, C = 4, 5 (96) -- the channel counts of the reference's tracer sets.
// Each also with MIX bit 7 (+128): plans with a dispersion component (ngrtd_gen_disp.hip).
bool gen_instance_exists(int C, bool full, int mix) {
    mix &= ~128;
    if (full) return C == 5 && (mix == 64 || mix == 68 || mix == 96 || mix == 100);
    if (mix == 64) return C >= 1 && C <= 5;
    return mix == 96 && (C == 4 || C == 5);
}
hipError_t launch_fused_gen_disp_instance(int C, bool full, int mix, const RtdArgs& a, const UnitArgs& u, int WB,
                                          int64_t W, double* logp, const DemcAccept& da, size_t lds, size_t max_lds,
                                          hipStream_t st);

hipError_t launch_fused_gen_instance(int C, bool full, int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W,
                                     double* logp, const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    if (!gen_instance_exists(C, full, mix)) return hipErrorInvalidValue;
    if (mix & 128) return launch_fused_gen_disp_instance(C, full, mix, a, u, WB, W, logp, da, lds, max_lds, st);
    if (full) {
        switch (mix) {
        case 64: return launch_gen<5, true, 64>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 68: return launch_gen<5, true, 68>(a, u, WB, W, logp, da, lds, max_lds, st);
        case 96: return launch_gen<5, true, 96>(a, u, WB, W, logp, da, lds, max_lds, st);
        default: return launch_gen<5, true, 100>(a, u, WB, W, logp, da, lds, max_lds, st);
        }
    }
    if (mix == 96) {
        if (C == 4) return launch_gen<4, false, 96>(a, u, WB, W, logp, da, lds, max_lds, st);
        return launch_gen<5, false, 96>(a, u, WB, W, logp, da, lds, max_lds, st);
    }
    switch (C) {
    case 1: return launch_gen<1, false, 64>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 2: return launch_gen<2, false, 64>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 3: return launch_gen<3, false, 64>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 4: return launch_gen<4, false, 64>(a, u, WB, W, logp, da, lds, max_lds, st);
    default: return launch_gen<5, false, 64>(a, u, WB, W, logp, da, lds, max_lds, st);
    }
}

}  // namespace ngrtd
