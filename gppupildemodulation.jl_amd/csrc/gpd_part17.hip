// Split build, unit 17: k_fit_exact one wave per series (see gpd_part16.hip).
#define GPD_PART 17
#include "gpd_part16.hip"
