// lane_shim.cpp -- TEST INFRASTRUCTURE: C entry points over the product's
// small-call host lane (narwhal-tusk_amd/csrc/cpu_lane.cpp, compiled from the
// same source into libntlane.so) so CPU-only tests can pin it to the golden
// corpus without a GPU.  Never linked into libntcrypto.so.
#include <cstdint>

#include "../../narwhal-tusk_amd/csrc/cpu_lane.hpp"
#include "../../narwhal-tusk_amd/csrc/nt_common.hpp"

extern "C" {
void ntl_init(int threads) { nt::cpu::init(threads); }
void ntl_sha512_trunc32_many(const uint8_t* data, const uint64_t* off, const uint64_t* len, uint64_t n, uint8_t* out32,
                             int threads) {
  nt::cpu::parallel_for(n, threads, [&](uint64_t i) { nt::cpu::sha512_trunc32(data + off[i], len[i], out32 + 32 * i); });
}
// mode 0 = verify_strict, 1 = cofactorless; out: one byte per item
void ntl_verify_many(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, const uint64_t* off,
                     const uint64_t* len, uint64_t n, uint8_t* out, int threads) {
  nt::cpu::init(threads);
  nt::cpu::parallel_for(n, threads, [&](uint64_t i) {
    out[i] = nt::cpu::verify(mode == 0 ? nt::kStrict : nt::kCofactorless, pk + 32 * i, sig + 64 * i, msg + off[i],
                             len[i]);
  });
}
}
