// Split build, units 3, 4, 7, 8 (MINB 1) and 12-15 (MINB 2) (gpd_kernels.hpp GPD_OWNS): the
// exact-evaluator fit k_fit_exact, two instances per unit (FAINT × OFFS × MINB; both PHBUF forms)
// — the exact path's inlined NEWUOA and Julia-libm batches make these the slowest kernels to
// compile.  gpd_part4/7/8/12-15.hip include this file with their own GPD_PART.
#ifndef GPD_PART
#define GPD_PART 3
#endif
#include "gpd_kernels.hpp"

namespace gpd {
#if GPD_PART == 3 || GPD_PART == 12
#define GPD_FA false
#define GPD_OF false
#elif GPD_PART == 4 || GPD_PART == 13
#define GPD_FA true
#define GPD_OF false
#elif GPD_PART == 7 || GPD_PART == 14
#define GPD_FA false
#define GPD_OF true
#else
#define GPD_FA true
#define GPD_OF true
#endif
#define GPD_MB (GPD_PART >= 12 ? 2 : 1)
__attribute__((used)) void *const k_fit_exact_units[] = {
    (void *)&k_fit_exact<GPD_FA, GPD_OF, false, GPD_MB>,
    (void *)&k_fit_exact<GPD_FA, GPD_OF, true, GPD_MB>};
#undef GPD_FA
#undef GPD_OF
#undef GPD_MB
}  // namespace gpd
