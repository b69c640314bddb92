// Split build, unit 1 (gpd_kernels.hpp GPD_OWNS): the harmonic-path fit kernels
// k_fit_harmonic and k_chi2_harmonic.
#define GPD_PART 1
#include "gpd_kernels.hpp"

namespace gpd {
__attribute__((used)) void *const k_fit_harmonic_units[] = {
    (void *)&k_fit_harmonic<1, false>, (void *)&k_fit_harmonic<2, false>,
    (void *)&k_fit_harmonic<4, false>, (void *)&k_fit_harmonic<8, false>,
    (void *)&k_fit_harmonic<2, true>,  (void *)&k_fit_harmonic<4, true>,
    (void *)&k_fit_harmonic<8, true>};
}  // namespace gpd
