// Split build, unit 6: k_moments_ws instances on Float32 storage (see gpd_part2.hip).
#define GPD_PART 6
#include "gpd_part2.hip"
