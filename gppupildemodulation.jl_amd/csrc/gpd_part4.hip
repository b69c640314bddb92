// Split build, unit 4: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 4
#include "gpd_part3.hip"
