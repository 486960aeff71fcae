// k_merge_nw1.hip -- k_merge_fire instantiations for 1 accumulator word(s) per entry
#include "fw_merge_hopb.h"

namespace fw {
template hipError_t merge_nw<1>(const MergeArgs& a, hipStream_t s);
}  // namespace fw
