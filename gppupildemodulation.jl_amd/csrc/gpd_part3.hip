// Split build, units 3, 4, 7 and 8 (gpd_kernels.hpp GPD_OWNS): the exact-evaluator fit
// k_fit_exact, two instances per unit (FAINT × OFFS; both PHBUF forms) — the exact path's
// inlined NEWUOA and Julia-libm batches make these the slowest kernels to compile.
// gpd_part4/7/8.hip include this file with their own GPD_PART.
#ifndef GPD_PART
#define GPD_PART 3
#endif
#include "gpd_kernels.hpp"

namespace gpd {
#if GPD_PART == 3
#define GPD_FA false
#define GPD_OF false
#elif GPD_PART == 4
#define GPD_FA true
#define GPD_OF false
#elif GPD_PART == 7
#define GPD_FA false
#define GPD_OF true
#else
#define GPD_FA true
#define GPD_OF true
#endif
__attribute__((used)) void *const k_fit_exact_units[] = {
    (void *)&k_fit_exact<GPD_FA, GPD_OF, false>, (void *)&k_fit_exact<GPD_FA, GPD_OF, true>};
#undef GPD_FA
#undef GPD_OF
}  // namespace gpd
