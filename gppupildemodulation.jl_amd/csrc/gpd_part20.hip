// Split build, units 20-23 (gpd_kernels.hpp GPD_OWNS, GPD_U_EXACT512): the exact-evaluator fit
// in the split form (k_fit_exact WGT = 512: two threads per canonical chain, G = 8 parts per
// series, one workgroup of two waves per SIMD per CU), two instances per unit (FAINT × OFFS;
// both PHBUF forms).  gpd_part21-23.hip include this file with their own GPD_PART.
#ifndef GPD_PART
#define GPD_PART 20
#endif
#include "gpd_kernels.hpp"

namespace gpd {
#if GPD_PART == 20
#define GPD_FA false
#define GPD_OF false
#elif GPD_PART == 21
#define GPD_FA true
#define GPD_OF false
#elif GPD_PART == 22
#define GPD_FA false
#define GPD_OF true
#else
#define GPD_FA true
#define GPD_OF true
#endif
__attribute__((used)) void *const k_fit_exact512_units[] = {
    (void *)&k_fit_exact<GPD_FA, GPD_OF, false, 1, 512>,
    (void *)&k_fit_exact<GPD_FA, GPD_OF, true, 1, 512>};
#undef GPD_FA
#undef GPD_OF
}  // namespace gpd
