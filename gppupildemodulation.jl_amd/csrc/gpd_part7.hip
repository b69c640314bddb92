// Split build, unit 7: k_fit_exact instances (see gpd_part3.hip).
#define GPD_PART 7
#include "gpd_part3.hip"
