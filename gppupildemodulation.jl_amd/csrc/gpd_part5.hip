// Split build, units 5, 9, 10 and 11 (gpd_kernels.hpp GPD_OWNS): the exact evaluator's
// one-point kernels — k_chi2_exact (the lkl functor as a batch), two instances per unit
// (FAINT × OFFS; both PHBUF forms), and k_refine_exact in unit 5.
// gpd_part9/10/11.hip include this file with their own GPD_PART.
#ifndef GPD_PART
#define GPD_PART 5
#endif
#include "gpd_kernels.hpp"

namespace gpd {
#if GPD_PART == 5
#define GPD_FA false
#define GPD_OF false
#elif GPD_PART == 9
#define GPD_FA true
#define GPD_OF false
#elif GPD_PART == 10
#define GPD_FA false
#define GPD_OF true
#else
#define GPD_FA true
#define GPD_OF true
#endif
__attribute__((used)) void *const k_chi2_exact_units[] = {
    (void *)&k_chi2_exact<GPD_FA, GPD_OF, false>, (void *)&k_chi2_exact<GPD_FA, GPD_OF, true>,
#if GPD_PART == 5
    (void *)&k_refine_exact<false>,
#endif
};
#undef GPD_FA
#undef GPD_OF
}  // namespace gpd
