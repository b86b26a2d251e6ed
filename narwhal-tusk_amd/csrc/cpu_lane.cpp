// cpu_lane.cpp -- host build of the device arithmetic for the small-call path
// (see cpu_lane.hpp).  Compiled by g++ (NT_HD empty): the same verify_one<>,
// wcomb_acc<> and sha512_prefixed<> the gfx950 kernels run, with per-call
// tables on the stack and a 12-bit host comb of B.
#include "cpu_lane.hpp"

#include <stdint.h>

#include <cstring>
#include <mutex>
#include <vector>

// The device headers are compiled here into a namespace of their own (nt_lane),
// with the host-lane field multiply (NT_HOST_FAST_FE, fe25519.hpp): no inline
// definition of this TU can be merged with -- or interposed by -- the device
// arithmetic's host build in any other object or library.
#define NT_HOST_FAST_FE 1
#define nt nt_lane
#include "ed25519_ops.hpp"
#undef nt

namespace nt {
namespace cpu {
namespace {
using namespace nt_lane;

constexpr int kHostBBits = 12;
using HG = CombGeom<kHostBBits>;

std::vector<uint32_t>* g_comb = nullptr;
std::once_flag g_once;

// [pos][entry][kWStride words] as on the device (ed25519_ops.hpp wide combs)
struct HostComb {
  static constexpr int kBits = kHostBBits;
  const uint32_t* base;
  void load(uint32_t pos, uint32_t idx, ge_niels& q) const {
    const uint32_t* e = base + ((size_t)pos * HG::kEntries + idx) * kWStride;
    for (int i = 0; i < 10; ++i) {
      q.ypx.v[i] = e[i];
      q.ymx.v[i] = e[10 + i];
      q.xy2d.v[i] = e[20 + i];
    }
  }
};

// the lane's j*(+-A), j*(-R) tables (entries 0..8, 9..17)
struct HostATab {
  ge_cached e[18];
  void store(uint32_t j, const ge_cached& c) { e[j] = c; }
  void load(uint32_t j, ge_cached& c) const { c = e[j]; }
};

void build(int threads) {
  auto* comb = new std::vector<uint32_t>(HG::kWordsPerPoint, 0u);
  uint32_t enc[8];
  for (int i = 0; i < 8; ++i) enc[i] = kBaseEnc[i];
  ge_p3 B;
  ge_frombytes_w(B, enc);
  std::vector<uint32_t> bases((size_t)HG::kPos * 40);
  wcomb_bases<kHostBBits>(bases.data(), B);
  parallel_for((uint64_t)HG::kPos * HG::kChunks, threads, [&](uint64_t t) {
    const uint32_t pos = (uint32_t)(t / HG::kChunks), c = (uint32_t)(t % HG::kChunks);
    uint32_t tmp[kWChunk * 10];
    uint32_t* dst = comb->data() + ((size_t)pos * HG::kEntries + 1 + (size_t)kWChunk * c) * kWStride;
    wcomb_fill<kHostBBits>(dst, tmp, bases.data() + (size_t)pos * 40, c);
  });
  g_comb = comb;
}

}  // namespace

void init(int threads) {
  std::call_once(g_once, [threads] { build(threads); });
}

bool ready() { return g_comb != nullptr; }

void sha512_trunc32(const uint8_t* msg, uint64_t len, uint8_t out32[32]) {
  uint64_t st[8];
  sha512_prefixed<0>(st, nullptr, msg, len);
  uint32_t w[8];
  sha512_out_words(w, st, 8);
  std::memcpy(out32, w, 32);
}

bool verify(int mode, const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t* msg, uint64_t len) {
  uint32_t A[8], R[8], S[8];
  std::memcpy(A, pk32, 32);
  std::memcpy(R, sig64, 32);
  std::memcpy(S, sig64 + 32, 32);
  HostATab at;
  const HostComb wb{g_comb->data()};
  const uint32_t ok = mode == nt_lane::kStrict ? verify_one<nt_lane::kStrict>(A, R, S, msg, len, at, wb)
                                               : verify_one<nt_lane::kCofactorless>(A, R, S, msg, len, at, wb);
  return ok != 0;
}

}  // namespace cpu
}  // namespace nt
