// k_ingest_nv2.hip -- k_ingest instantiations for 2 loaded value column slot(s)
#include "fw_ingest_impl.h"

namespace fw {
template hipError_t ingest_nv<2>(const IngestArgs& a, hipStream_t s, KTimer* t);
}  // namespace fw
