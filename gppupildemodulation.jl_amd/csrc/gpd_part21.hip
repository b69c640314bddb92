// Split build, unit 21: k_fit_exact split form (see gpd_part20.hip).
#define GPD_PART 21
#include "gpd_part20.hip"
