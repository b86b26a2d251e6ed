// nt_host_harness.cpp -- TEST INFRASTRUCTURE: the exact device arithmetic of
// narwhal-tusk_amd/csrc/*.hpp compiled for the host (g++, NT_HD empty) so that
// CPU-only tests can (a) stress the radix-2^25.5 bound discipline with
// adversarial limb values against Python big integers, (b) replay the golden
// corpus through the same verify_one<> the kernels run, and (c) count field
// multiplies per operation (profiles/opcount.json, the roofline numerator).
// Never linked into libntcrypto.so.
#define NT_OPCOUNT 1
#include <cstring>

#include "../../narwhal-tusk_amd/csrc/ed25519_ops.hpp"

namespace nt {
unsigned long long g_fe_mul = 0, g_fe_sq = 0;
}

using namespace nt;

namespace {
struct HostATab {
  ge_cached e[9];
  void store(uint32_t j, const ge_cached& c) { e[j] = c; }
  void load(uint32_t j, ge_cached& c) const { c = e[j]; }
};
struct HostBTab {
  ge_niels e[129];
  bool ready = false;
  void load(uint32_t j, ge_niels& q) const { q = e[j]; }
};
HostBTab& btab() {
  static HostBTab t;
  if (!t.ready) {
    for (uint32_t j = 0; j < 129; ++j) btab_entry(t.e[j], j);
    t.ready = true;
  }
  return t;
}
void words(uint32_t w[8], const uint8_t* b) { std::memcpy(w, b, 32); }
}  // namespace

extern "C" {

void nth_fe_mul(const uint32_t* f, const uint32_t* g, uint32_t* out) {
  fe a, b, c;
  std::memcpy(a.v, f, 40);
  std::memcpy(b.v, g, 40);
  fe_mul(c, a, b);
  std::memcpy(out, c.v, 40);
}
void nth_fe_sq(const uint32_t* f, uint32_t* out) {
  fe a, c;
  std::memcpy(a.v, f, 40);
  fe_sq(c, a);
  std::memcpy(out, c.v, 40);
}
void nth_fe_carry(const uint32_t* f, uint32_t* out) {
  fe a;
  std::memcpy(a.v, f, 40);
  fe_carry(a);
  std::memcpy(out, a.v, 40);
}
void nth_fe_tobytes(const uint32_t* f, uint8_t* out32) {
  fe a;
  std::memcpy(a.v, f, 40);
  uint32_t w[8];
  fe_tobytes_w(w, a);
  std::memcpy(out32, w, 32);
}
void nth_fe_frombytes(const uint8_t* in32, uint32_t* out) {
  uint32_t w[8];
  words(w, in32);
  fe a;
  fe_frombytes_w(a, w);
  std::memcpy(out, a.v, 40);
}
void nth_sc_reduce512(const uint8_t* in64, uint8_t* out32) {
  uint32_t x[16], r[8];
  std::memcpy(x, in64, 64);
  sc_reduce512(r, x);
  std::memcpy(out32, r, 32);
}
void nth_sc_muladd(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out32) {
  uint32_t wa[8], wb[8], wc[8], r[8];
  words(wa, a);
  words(wb, b);
  words(wc, c);
  sc_muladd(r, wa, wb, wc);
  std::memcpy(out32, r, 32);
}
void nth_sha512(const uint8_t* msg, uint64_t len, uint8_t* out64) {
  uint64_t st[8];
  sha512_prefixed<0>(st, nullptr, msg, len);
  uint32_t w[16];
  sha512_out_words(w, st, 16);
  std::memcpy(out64, w, 64);
}
int nth_verify(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t len) {
  uint32_t A[8], R[8], S[8];
  words(A, pk);
  words(R, sig);
  words(S, sig + 32);
  HostATab at;
  if (mode == 0) return (int)verify_one<kStrict>(A, R, S, msg, len, at, btab());
  return (int)verify_one<kCofactorless>(A, R, S, msg, len, at, btab());
}
void nth_sign(const uint8_t* seed, const uint8_t* msg, uint64_t len, uint8_t* pk, uint8_t* sig) {
  uint32_t sw[8], A[8], R[8], s[8];
  words(sw, seed);
  sign_one(A, R, s, sw, msg, len, btab());
  std::memcpy(pk, A, 32);
  std::memcpy(sig, R, 32);
  std::memcpy(sig + 32, s, 32);
}
void nth_counts_reset() { g_fe_mul = g_fe_sq = 0; btab(); g_fe_mul = g_fe_sq = 0; }
unsigned long long nth_count_mul() { return g_fe_mul; }
unsigned long long nth_count_sq() { return g_fe_sq; }
}
