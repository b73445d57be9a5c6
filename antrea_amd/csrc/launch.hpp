// Internal launch entry of the classification kernel (classify.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "core.hpp"
#include "gpc.h"

namespace gpc {
int launch_classify(const ImageHdr* d_hdr, const uint32_t* d_blob, const gpc_pkt_soa& pk, uint64_t n, gpc_verdict* out,
                    unsigned long long* counters, int count, hipStream_t stream);
}
