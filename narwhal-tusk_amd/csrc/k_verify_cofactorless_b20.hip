// k_verify_cofactorless_b20.hip -- verify kernels, cofactorless mode, 20-bit comb of B (one translation
// unit per mode and comb width, so the build compiles them in parallel).
#include "k_verify.inc"

namespace nt {
template hipError_t launch_verify_m<kCofactorless, kBCombFallback>(uint64_t, const uint8_t*, const uint8_t*, const uint8_t*, uint64_t,
                                              const uint64_t*, const uint64_t*, uint64_t, const uint32_t*, void*,
                                              uint64_t*, hipStream_t, int);
}  // namespace nt
