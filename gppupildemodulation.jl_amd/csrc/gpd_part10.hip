// Split build, unit 10: k_chi2_exact instances (see gpd_part5.hip).
#define GPD_PART 10
#include "gpd_part5.hip"
