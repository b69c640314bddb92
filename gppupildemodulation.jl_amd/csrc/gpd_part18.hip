// Split build, unit 18: k_fit_exact one wave per series (see gpd_part16.hip).
#define GPD_PART 18
#include "gpd_part16.hip"
