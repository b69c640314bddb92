// Split build, unit 12: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 12
#include "gpd_part3.hip"
