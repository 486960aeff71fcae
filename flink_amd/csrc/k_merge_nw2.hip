// k_merge_nw2.hip -- k_merge_fire instantiations for 2 accumulator word(s) per entry
#include "fw_merge_hopb.h"

namespace fw {
template hipError_t merge_nw<2>(const MergeArgs& a, hipStream_t s);
}  // namespace fw
