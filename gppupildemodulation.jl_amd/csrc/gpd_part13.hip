// Split build, unit 13: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 13
#include "gpd_part3.hip"
