// k_keyset_cofactorless.hip -- keyset kernels, cofactorless mode (one translation unit per mode).
#include "k_keyset.inc"

namespace nt {
template hipError_t launch_keyset_m<kCofactorless>(uint64_t, const uint32_t*, const uint8_t*, const uint8_t*,
                                        const uint64_t*, const uint64_t*, uint64_t, const uint32_t*,
                                        const uint32_t*, const uint32_t*, uint32_t, const uint32_t*,
                                        void*, uint64_t*, hipStream_t);
}  // namespace nt
