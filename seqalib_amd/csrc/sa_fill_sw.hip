// Fill-kernel instantiations for SA_SW (one translation unit per algorithm: parallel builds).
#include "sa_fill_impl.h"

namespace sa {
hipError_t launch_fill_sw(const FillVariant& v, const FillParams& p, uint32_t grid, hipStream_t s) {
    return launch_fill_alg<SA_SW>(v, p, grid, s);
}
SA_SPLIT_STATS_ACCESSOR(sa_debug_split_stats_sw)
SA_FILL_STATS_ACCESSOR(sa_debug_fill_stats_sw)
}  // namespace sa
