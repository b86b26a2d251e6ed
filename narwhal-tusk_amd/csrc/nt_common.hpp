// nt_common.hpp -- shared definitions for the gfx950 crypto backend.
//
// Device code is written as plain C++ with NT_HD (= __host__ __device__ under
// hipcc) so that the exact same arithmetic can be exercised on the host by the
// bound-stress test in tests/cpp/ (compiled with g++, NT_HD empty).  The
// product library (libntcrypto.so) only ever runs it on the GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define NT_HD __host__ __device__
#define NT_D __device__
#define NT_INLINE __attribute__((always_inline)) inline
#else
#define NT_HD
#define NT_D
#define NT_INLINE inline
struct uint4 {
  uint32_t x, y, z, w;
};
#endif

namespace nt {

// Kernel-facing verification modes (see include/ntcrypto.h).
enum VerifyMode : int {
  kStrict = 0,        // dalek verify_strict (crypto/src/lib.rs:200-204)
  kCofactorless = 1,  // per-entry rule of dalek verify_batch, SURVEY.md A.3
  kMixed = 2,         // key-cache only: per signature, key_idx bit 31 set = strict, clear = cofactorless
};

// Digit widths of the committee-key combs (ed25519_ops.hpp, wide combs)
constexpr int kKeyCombReduced = 21;  // 12 additions per [k]A (k reduced to |k| <= L/2), 1.61 GB per key: used when they fit
constexpr int kKeyCombWide = 20;    // 13 additions per [k]A, 872 MB per key
constexpr int kKeyCombMid = 18;     // 15 additions, 252 MB per key (NT_KEYSET_COMB_BITS=18, A/B)
constexpr int kKeyCombNarrow = 16;  // 16 additions, 67 MB per key

// Digit widths of the comb of the base point B (one per device ordinal): 24 bits
// by measurement, 20 bits when the context's HBM budget or the
// device's free memory cannot hold 11.8 GB (ntcrypto.cpp: comb_b_for).  Every
// kernel that reads it is compiled for both; the launchers dispatch on the width
// of the comb the device entry holds.
#ifndef NT_BCOMB_WIDE
#define NT_BCOMB_WIDE 24  // A/B builds: -DNT_BCOMB_WIDE=26 (10 additions, 43 GB)
#endif
constexpr int kBCombBits = NT_BCOMB_WIDE;  // 24: 11 additions per [s]B, 11.8 GB (the host harness builds this one)
constexpr int kBCombFallback = 20;  // 13 additions, 872 MB

// Message i of a launch is msg[off[i] .. off[i] + len[i]) of a buffer of
// `bytes` bytes.  Every kernel that reads caller messages takes the slice
// through msg_slice: out of bounds (off > bytes, or len > bytes - off -- no
// overflow) it gets an empty slice at the buffer's start and ok = 0, and the
// item is rejected (verification, signing) or gets a zero digest and is counted
// (SHA-512); the kernel never dereferences the caller's offset.  (Round 4's
// fault r04e: a key-cache launch read offsets another stream had not written
// yet, and the wild offset faulted the card.)
struct MsgSlice {
  uint64_t off, len;
  uint32_t ok;
};
NT_HD NT_INLINE MsgSlice msg_slice(uint64_t off, uint64_t len, uint64_t bytes) {
  const uint32_t ok = off <= bytes && len <= bytes - off;
  return MsgSlice{ok ? off : 0u, ok ? len : 0u, ok};
}

}  // namespace nt
