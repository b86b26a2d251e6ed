// k_verify_strict.hip -- verify kernels, strict mode (one translation unit per mode).
#include "k_verify.inc"

namespace nt {
template hipError_t launch_verify_m<kStrict>(uint64_t, const uint8_t*, const uint8_t*, const uint8_t*,
                                        const uint64_t*, const uint64_t*, uint64_t, const uint32_t*, void*,
                                        uint64_t*, hipStream_t);
}  // namespace nt
