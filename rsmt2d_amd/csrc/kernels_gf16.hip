// kernels_gf16.hip -- Leopard GF(2^16) kernels (k > 128): not yet implemented in
// this build; the runtime maps this to RSM_EUNSUPPORTED (never a CPU fallback).
#include <hip/hip_runtime.h>
#include "rsm_kernels.hpp"

namespace rsm {
hipError_t launch_encode_gf16(const CodewordSet&, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_decode_gf16(const DecodeSet&, hipStream_t) { return hipErrorNotSupported; }
}  // namespace rsm
