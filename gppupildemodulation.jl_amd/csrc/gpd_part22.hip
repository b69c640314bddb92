// Split build, unit 22: k_fit_exact split form (see gpd_part20.hip).
#define GPD_PART 22
#include "gpd_part20.hip"
