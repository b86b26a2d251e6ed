// k_keyset_cofactorless_w21.hip -- key-cache kernels, cofactorless mode, 21-bit reduced-scalar key combs, for
// both widths of the comb of B (one translation unit per mode and key-comb width:
// the build compiles them in parallel).
#include "k_keyset.inc"

#define NT_KS_INST(WB)                                                                                          \
  template hipError_t launch_keyset_m<kCofactorless, 21, WB>(                                                          \
      const KsPlan&, const uint32_t*, const uint8_t*, const uint8_t*, uint64_t, const uint64_t*, const uint64_t*,  \
      uint64_t, const uint32_t*, const uint32_t*, const uint32_t*, uint32_t, const uint32_t*, void*,            \
      const uint32_t*, const KsVerdict&, uint32_t*, hipStream_t);
namespace nt {
NT_KS_INST(kBCombBits)
NT_KS_INST(kBCombFallback)
}  // namespace nt
