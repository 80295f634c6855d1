// ngrtd_dzc.hip -- the lane-chain DEMetropolisZ instances (ngrtd_dzc.hpp): the reference's
// RTD-only model (1 or 4 tracers: C = 1 or 4 channels; exponential / exp_pist_flow, with or
// without a piston second component; the sampled CFC12 half-life at C = 4) and its CE-only
// model, natural or transformed space.  Compiled like ngrtd_dz.hip, without machine LICM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../../include/ngrtd.h"
#define NGRTD_FUSED_ONLY
#include "ngrtd_dzc.hpp"

namespace ngrtd {

template <int C, int MIX, bool TW>
static hipError_t launch_dzc_tw(const RtdArgs& a, const UnitArgs& u, const DemcAccept& da, unsigned blocks,
                                unsigned threads, size_t lds, size_t max_lds, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&dz_chain_kernel<C, MIX, TW>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)max_lds);
    (void)attr;
    hipLaunchKernelGGL((dz_chain_kernel<C, MIX, TW>), dim3(blocks), dim3(threads), lds, st, a, u, da);
    return hipGetLastError();
}

template <int C, int MIX>
static hipError_t launch_dzc(const RtdArgs& a, const UnitArgs& u, const DemcAccept& da, int64_t U, size_t lds,
                             size_t max_lds, hipStream_t st) {
    // one chain wave + its theta wave per block (da.theta_wave: <= 64 chains)
    if (da.theta_wave) return launch_dzc_tw<C, MIX, true>(a, u, da, (unsigned)((U + 63) / 64), 128, lds, max_lds, st);
    // threads per block: NT, or the waves the chains need when they are fewer -- the
    // reference's own runs are 3 chains (1 well) or 4 (CE): one wave alone on its SIMD instead
    // of 8 waves of shadow lanes, two per SIMD, issuing the same step (NGRTD_DZC_MIN_THREADS:
    // a floor, for A/B runs)
    constexpr int NT = dzc_threads(MIX);
    static const int min_t = [] {
        const char* e = getenv("NGRTD_DZC_MIN_THREADS");
        const int v = e ? atoi(e) : 64;
        return v < 64 ? 64 : v > NT ? NT : v / 64 * 64;
    }();
    int tb = (int)std::min<int64_t>(NT, (U + 63) / 64 * 64);
    tb = std::max(tb, min_t);
    return launch_dzc_tw<C, MIX, false>(a, u, da, (unsigned)((U + tb - 1) / tb), (unsigned)tb, lds, max_lds, st);
}

#define NGRTD_DZC_RTD(CC)                                                                          \
    switch (mix) {                                                                                 \
    case 0: return launch_dzc<CC, 0>(a, u, da, U, lds, max_lds, st);                               \
    case 1: return launch_dzc<CC, 1>(a, u, da, U, lds, max_lds, st);                               \
    case 2: return launch_dzc<CC, 2>(a, u, da, U, lds, max_lds, st);                               \
    case 3: return launch_dzc<CC, 3>(a, u, da, U, lds, max_lds, st);                               \
    case 4: return launch_dzc<CC, 4>(a, u, da, U, lds, max_lds, st);                               \
    case 5: return launch_dzc<CC, 5>(a, u, da, U, lds, max_lds, st);                               \
    case 6: return launch_dzc<CC, 6>(a, u, da, U, lds, max_lds, st);                               \
    case 7: return launch_dzc<CC, 7>(a, u, da, U, lds, max_lds, st);                               \
    default: break;                                                                                \
    }

// Instances: C = 1 and C = 4 (mix 0..7: piston 1 | EPM 2 | transformed 4), C = 4 with the
// sampled CFC12 half-life (+32), the CE-only model (mix 64 | 4).
bool dz_chain_instance_exists(int C, int mix) {
    if (mix & 64) return (mix & ~4) == 64;
    if (mix & 32) return C == 4 && (mix & ~7) == 32;
    return (C == 1 || C == 4) && mix >= 0 && mix <= 7;
}

hipError_t launch_dz_chain(int C, int mix, const RtdArgs& a, const UnitArgs& u, const DemcAccept& da, int64_t U,
                           size_t lds, size_t max_lds, hipStream_t st) {
    if (mix == 64) return launch_dzc<1, 64>(a, u, da, U, lds, max_lds, st);
    if (mix == 68) return launch_dzc<1, 68>(a, u, da, U, lds, max_lds, st);
    if (C == 1) { NGRTD_DZC_RTD(1) }
    if (C == 4 && !(mix & 32)) { NGRTD_DZC_RTD(4) }
    if (C == 4 && (mix & 32)) {
        switch (mix) {
        case 32: return launch_dzc<4, 32>(a, u, da, U, lds, max_lds, st);
        case 33: return launch_dzc<4, 33>(a, u, da, U, lds, max_lds, st);
        case 34: return launch_dzc<4, 34>(a, u, da, U, lds, max_lds, st);
        case 35: return launch_dzc<4, 35>(a, u, da, U, lds, max_lds, st);
        case 36: return launch_dzc<4, 36>(a, u, da, U, lds, max_lds, st);
        case 37: return launch_dzc<4, 37>(a, u, da, U, lds, max_lds, st);
        case 38: return launch_dzc<4, 38>(a, u, da, U, lds, max_lds, st);
        case 39: return launch_dzc<4, 39>(a, u, da, U, lds, max_lds, st);
        default: break;
        }
    }
    return hipErrorInvalidValue;
}

}  // namespace ngrtd

#ifdef NGRTD_SECTION_PROBE
// this translation unit's probe buffer (the lane-chain step's sections; tools/dzc_probe.py)
extern "C" int ngrtd_probe_read_dzc(unsigned long long* dst, int64_t n) {
    using ngrtd::g_probe;
    if (n > (int64_t)(sizeof(g_probe) / sizeof(g_probe[0]))) n = sizeof(g_probe) / sizeof(g_probe[0]);
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_probe), (size_t)n * sizeof(unsigned long long)) == hipSuccess ? 0 : -2;
}
#endif
