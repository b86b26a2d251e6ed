// k_keyset_strict_w18.hip -- key-cache kernels, strict mode, 18-bit key combs
// (one translation unit per mode and comb width: the build compiles them in parallel).
#include "k_keyset.inc"

namespace nt {
template hipError_t launch_keyset_m<kStrict, 18>(const KsPlan&, const uint32_t*, const uint8_t*, const uint8_t*,
                                             const uint64_t*, const uint64_t*, uint64_t, const uint32_t*,
                                             const uint32_t*, const uint32_t*, uint32_t, const uint32_t*,
                                             void*, uint64_t*, const uint32_t*, uint8_t*, uint32_t*, hipStream_t);
}  // namespace nt
