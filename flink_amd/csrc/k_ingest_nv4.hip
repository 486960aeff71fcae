// k_ingest_nv4.hip -- k_ingest instantiations for 4 loaded value column slot(s)
#include "fw_ingest_impl.h"

namespace fw {
template hipError_t ingest_nv<4>(const IngestArgs& a, hipStream_t s, KTimer* t);
}  // namespace fw
