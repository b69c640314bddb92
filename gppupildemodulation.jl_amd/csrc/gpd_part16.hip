// Split build, units 16-19 (gpd_kernels.hpp GPD_OWNS, GPD_U_EXACT64): the exact-evaluator fit
// with one wave per series (k_fit_exact WGT = 64, two waves per SIMD) for short spans, two
// instances per unit (FAINT × OFFS; both PHBUF forms).  gpd_part17-19.hip include this file with
// their own GPD_PART.
#ifndef GPD_PART
#define GPD_PART 16
#endif
#include "gpd_kernels.hpp"

namespace gpd {
#if GPD_PART == 16
#define GPD_FA false
#define GPD_OF false
#elif GPD_PART == 17
#define GPD_FA true
#define GPD_OF false
#elif GPD_PART == 18
#define GPD_FA false
#define GPD_OF true
#else
#define GPD_FA true
#define GPD_OF true
#endif
__attribute__((used)) void *const k_fit_exact64_units[] = {
    (void *)&k_fit_exact<GPD_FA, GPD_OF, false, 2, 64>,
    (void *)&k_fit_exact<GPD_FA, GPD_OF, true, 2, 64>};
#undef GPD_FA
#undef GPD_OF
}  // namespace gpd
