// ngrtd_dz.hip -- the single-launch DEMetropolisZ instances of logp_fused_kernel (MIX bit 3),
// in a translation unit of their own so that they compile with machine LICM off
// (__graft_entry__.py): a launch runs many steps of its chains (the DemcAccept::Sched loop),
// and hoisting the log-prob body's loop-invariant constants and addresses out of that loop
// held them in registers for the whole launch and spilled to scratch (257 VGPRs of scratch
// spills with it; 0 without).  The plain log-prob instances stay in ngrtd.hip with the
// default pipeline, so their code does not change.
#include <hip/hip_runtime.h>

#include "../../include/ngrtd.h"
#define NGRTD_FUSED_ONLY
#include "ngrtd_kernels.hpp"

namespace ngrtd {

template <int MIX>
static hipError_t launch_dz_mix(const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
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

hipError_t launch_fused_dz_lw_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                       const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st);
hipError_t launch_fused_dz_gen_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                        const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st);
hipError_t launch_fused_dz_gen_disp_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W,
                                             double* logp, const DemcAccept& da, size_t lds, size_t max_lds,
                                             hipStream_t st);

// The DZ instances: 8 | piston 1 | EPM 2 | Jacobian 4 (13 / 15: the transformed-space BMMs) |
// per-well chains 16 | the sampled
// CFC12 half-life 32 (ngrtd_dz_lw.hip; the BMM ones exceed kDzMaxP rows at the c4 shape) |
// generic components 64 (+ 128: a dispersion component; ngrtd_dz_gen*.hip, no half-life).
bool fused_dz_instance_exists(int mix) {
    switch (mix & ~16) {
    case 8: case 9: case 10: case 11: case 12: case 13: case 14: case 15: return true;
    case 40: case 42: case 44: case 46: return true;
    case 72: case 76: case 200: case 204: return true;
    default: return false;
    }
}
// The DZ instance `mix` over W chains in blocks of WB (fused_dz_instance_exists(mix)).
hipError_t launch_fused_dz_instance(int mix, const RtdArgs& a, const UnitArgs& u, int WB, int64_t W, double* logp,
                                    const DemcAccept& da, size_t lds, size_t max_lds, hipStream_t st) {
    if (mix & 32) return launch_fused_dz_lw_instance(mix, a, u, WB, W, logp, da, lds, max_lds, st);
    if (mix & 128) return launch_fused_dz_gen_disp_instance(mix, a, u, WB, W, logp, da, lds, max_lds, st);
    if (mix & 64) return launch_fused_dz_gen_instance(mix, a, u, WB, W, logp, da, lds, max_lds, st);
    switch (mix) {
    case 8: return launch_dz_mix<8>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 9: return launch_dz_mix<9>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 10: return launch_dz_mix<10>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 11: return launch_dz_mix<11>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 12: return launch_dz_mix<12>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 13: return launch_dz_mix<13>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 14: return launch_dz_mix<14>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 15: return launch_dz_mix<15>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 24: return launch_dz_mix<24>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 25: return launch_dz_mix<25>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 26: return launch_dz_mix<26>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 27: return launch_dz_mix<27>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 28: return launch_dz_mix<28>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 29: return launch_dz_mix<29>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 30: return launch_dz_mix<30>(a, u, WB, W, logp, da, lds, max_lds, st);
    case 31: return launch_dz_mix<31>(a, u, WB, W, logp, da, lds, max_lds, st);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace ngrtd

#ifdef NGRTD_SECTION_PROBE
// this translation unit's probe buffer (the DZ instances stamp it; tools/section_probe.py)
extern "C" int ngrtd_probe_read_dz(unsigned long long* dst, int64_t n) {
    using ngrtd::g_probe;
    if (n > (int64_t)(sizeof(g_probe) / sizeof(g_probe[0]))) n = sizeof(g_probe) / sizeof(g_probe[0]);
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_probe), (size_t)n * sizeof(unsigned long long)) == hipSuccess ? 0 : -2;
}
#endif
