// Split build, unit 9: k_chi2_exact instances (see gpd_part5.hip).
#define GPD_PART 9
#include "gpd_part5.hip"
