// Split build, unit 8: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 8
#include "gpd_part3.hip"
