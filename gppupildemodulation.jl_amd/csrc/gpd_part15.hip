// Split build, unit 15: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 15
#include "gpd_part3.hip"
