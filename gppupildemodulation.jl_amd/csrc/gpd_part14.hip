// Split build, unit 14: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 14
#include "gpd_part3.hip"
