// Split build, unit 23: k_fit_exact split form (see gpd_part20.hip).
#define GPD_PART 23
#include "gpd_part20.hip"
