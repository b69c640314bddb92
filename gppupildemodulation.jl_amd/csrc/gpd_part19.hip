// Split build, unit 19: k_fit_exact one wave per series (see gpd_part16.hip).
#define GPD_PART 19
#include "gpd_part16.hip"
