// Split build, unit 11: k_chi2_exact instances (see gpd_part5.hip).
#define GPD_PART 11
#include "gpd_part5.hip"
