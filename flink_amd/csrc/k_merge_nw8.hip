// k_merge_nw8.hip -- k_merge_fire instantiations for 8 accumulator word(s) per entry
#include "fw_merge_hopb.h"

namespace fw {
template hipError_t merge_nw<8>(const MergeArgs& a, hipStream_t s);
}  // namespace fw
