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
// host) instead of the device's 11.8 GB 24-bit comb.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>

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

// the 32-byte encoding decodes to a curve point (ge_frombytes_w, as the
// device's key tables decide it; the key registry admits only such keys)
bool key_decodes(const uint8_t pk32[32]);

// threads the worker pool runs with the caller (min(64, hardware threads)): the
// most parallelism a host-lane call gets
int pool_threads();

// fn(i) for i in [0, n) on the lane's persistent worker pool plus the calling
// thread (threads <= 1 or n <= 1: inline).  Safe to call from several threads
// at once: each call is a job the pool's workers share with its caller.
void parallel_for_fn(uint64_t n, int threads, const std::function<void(uint64_t)>& fn);
template <class F>
void parallel_for(uint64_t n, int threads, F&& fn) {
  if (threads <= 1 || n <= 1) {
    for (uint64_t i = 0; i < n; ++i) fn(i);
    return;
  }
  parallel_for_fn(n, threads, std::function<void(uint64_t)>(fn));
}

}  // namespace cpu
}  // namespace nt
