// cpu_lane.hpp -- the small-call path of the C ABI (SURVEY.md H3, §8(b)
// "CPU-fallback threshold").
//
// The reference's callers are latency-bound, not throughput-bound: Core::run
// verifies one certificate (1 strict + 67 batch signatures) per message
// (primary/src/core.rs:349-411) and each Processor hashes ONE ~508 KB batch per
// call (worker/src/processor.rs:36-38).  On the GPU such a call costs a launch
// plus one lane's serial chain (a lone 508,052-B digest: 16.8 ms; a lone
// verify: ~1.5 ms) -- far more than the host needs.  Below a cost crossover the
// C ABI therefore runs the SAME arithmetic (fe25519 / ge25519 / sc25519 /
// sha512 / ed25519_ops .hpp, compiled for the host by g++) on host threads.
//
// This is product code, not the oracle (oracle/ is the independent checker and
// is never linked here), and it is not a fallback: it only runs inside a
// context that owns a gfx950 device (nt_init still fails without one), only
// when the caller enables it (nt_set_small_call_path), and only below the
// crossover.  The B table of the host lane is a 12-bit wide comb (22 x 2049
// affine niels entries = 5.8 MB, built once by wcomb_bases / wcomb_fill on the
// host) instead of the device's 872 MB 20-bit comb.
#pragma once
#include <cstddef>
#include <cstdint>

namespace nt {
namespace cpu {

// Builds the host B comb (idempotent, thread-safe); `threads` host threads.
void init(int threads);
bool ready();

// Digest = SHA-512(msg)[..32]
void sha512_trunc32(const uint8_t* msg, uint64_t len, uint8_t out32[32]);

// mode: nt::kStrict (dalek verify_strict) or nt::kCofactorless (one entry of
// verify_batch under SURVEY A.3).  Requires init().
bool verify(int mode, const uint8_t pk32[32], const uint8_t sig64[64], const uint8_t* msg, uint64_t len);

// fn(i) for i in [0, n) on up to `threads` threads (the caller's thread included).
template <class F>
void parallel_for(uint64_t n, int threads, F&& fn);

}  // namespace cpu
}  // namespace nt

#include <thread>
#include <vector>

template <class F>
void nt::cpu::parallel_for(uint64_t n, int threads, F&& fn) {
  const uint64_t T = threads < 1 ? 1 : (uint64_t)threads < n ? (uint64_t)threads : n;
  if (T <= 1) {
    for (uint64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  auto work = [&](uint64_t t) {
    for (uint64_t i = n * t / T; i < n * (t + 1) / T; ++i) fn(i);
  };
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (uint64_t t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}
