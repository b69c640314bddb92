// Split build, units 2 and 6 (gpd_kernels.hpp GPD_OWNS): the producer/consumer moment kernel
// k_moments_ws, Float64-storage instances here (unit 2) or Float32-storage ones (unit 6,
// gpd_part6.hip includes this file); the diagnostics build adds the timing variants.
#ifndef GPD_PART
#define GPD_PART 2
#endif
#include "gpd_kernels.hpp"

namespace gpd {
#if GPD_PART == 2
__attribute__((used)) void *const k_moments_ws_c64_units[] = {
    (void *)&k_moments_ws<0, false, c64, 2>,              // production (mixed precision)
    (void *)&k_moments_ws<0, false, c64, 2, false>,       // all-f64 (option mix = 0)
    (void *)&k_moments_ws<0, false, c64, 2, true, true>,  // faint series
    (void *)&k_moments_ws<0, false, c64, 2, false, true>,
    (void *)&k_moments_ws<0, true>,                       // UNIT mode (harmonic fitoffsets)
    (void *)&k_moments_ws<0, true, c64, 0, false>,
#ifdef GPD_DIAG
    (void *)&k_moments_ws<1>, (void *)&k_moments_ws<2>, (void *)&k_moments_ws<5>,
    (void *)&k_moments_ws<6>, (void *)&k_moments_ws<7>, (void *)&k_moments_ws<8>,
    (void *)&k_moments_ws<9, false, c64, 2, true, true>,   // faint without the fused statistics
    (void *)&k_moments_ws<10, false, c64, 2, true, true>,  // faint, producers without masking
#endif
};
#else
__attribute__((used)) void *const k_moments_ws_c32_units[] = {
    (void *)&k_moments_ws<0, false, c32, 2>,
    (void *)&k_moments_ws<0, false, c32, 2, false>,
    (void *)&k_moments_ws<0, false, c32, 2, true, true>,
    (void *)&k_moments_ws<0, false, c32, 2, false, true>,
    (void *)&k_moments_ws<0, true, c32>,
    (void *)&k_moments_ws<0, true, c32, 0, false>,
};
#endif
}  // namespace gpd
