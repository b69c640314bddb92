// Split build, unit 1 (gpd_kernels.hpp GPD_OWNS): the harmonic-path fit kernels
// k_fit_harmonic and k_chi2_harmonic.
#define GPD_PART 1
#include "gpd_kernels.hpp"
