// key_table.hpp -- the host-side index of the key registry (host-only; shared by
// ntcrypto.cpp and the host test harness).
//
// The registry (ntcrypto.cpp, include/ntcrypto.h nt_set_key_cache) keeps the
// committee key cache behind the unchanged entry points: nt_ed25519_verify_strict
// and nt_ed25519_verify_batch_groups carry raw 32-byte keys (the crate's
// `PublicKey`, crypto/src/lib.rs:65-119), and every call maps each key to its
// registry index here, on host threads, before the keys cross PCIe.  A vote
// then travels as a 4-byte index + its 64-byte signature (68 B, as through the
// key-set entry points) instead of 96 B, and a key the registry does not hold
// comes back as kKeyMiss (verified by the uncached kernel).
//
// A KeyTable is immutable once built: the registry publishes a new one with
// every admission, and a call keeps the table it started with.  Open
// addressing with linear probing at load <= 1/4; a slot holds the key index and
// the key's first 8 bytes (most probes are rejected without touching the
// encodings); the hash multiplies those 8 bytes by a per-table odd constant.
#pragma once
#include <stdint.h>

#include <cstring>
#include <vector>

namespace nt {

constexpr uint32_t kKeyMiss = 0xffffffffu;

struct KeyTable {
  uint32_t nkeys = 0;         // keys 0 .. nkeys - 1 of `enc` are indexed
  uint32_t shift = 64;        // 64 - log2(slots)
  uint32_t mask = 0;          // slots - 1
  uint64_t mult = 0x9e3779b97f4a7c15ull;
  std::vector<uint32_t> idx;  // per slot: key index or kKeyMiss (empty)
  std::vector<uint64_t> head; // per slot: the key's first 8 bytes
  std::vector<uint8_t> enc;   // nkeys x 32: the key encodings, in index order

  static uint64_t load64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
  }
  uint32_t home(uint64_t h0) const { return nkeys ? (uint32_t)((h0 * mult) >> shift) : 0u; }

  // index of the 32-byte key, or kKeyMiss
  uint32_t find(const uint8_t* pk) const {
    if (nkeys == 0) return kKeyMiss;
    const uint64_t h0 = load64(pk);
    for (uint32_t s = home(h0);; s = (s + 1) & mask) {
      const uint32_t k = idx[s];
      if (k == kKeyMiss) return kKeyMiss;
      if (head[s] == h0) {
        const uint8_t* e = enc.data() + 32ull * k;  // the other 24 bytes as three words
        if (((load64(e + 8) ^ load64(pk + 8)) | (load64(e + 16) ^ load64(pk + 16)) | (load64(e + 24) ^ load64(pk + 24))) == 0)
          return k;
      }
    }
  }

  // index over keys[0 .. n) (distinct 32-byte encodings; a repeated key keeps
  // its first index).  seed varies the multiplier between tables.
  void build(const uint8_t* keys, uint32_t n, uint64_t seed = 0) {
    nkeys = n;
    enc.assign(keys, keys + 32ull * n);
    uint32_t bits = 4;
    while ((1ull << bits) < 4ull * (n ? n : 1)) ++bits;
    shift = 64 - bits;
    mask = (1u << bits) - 1;
    mult = (0x9e3779b97f4a7c15ull ^ (seed * 0xbf58476d1ce4e5b9ull)) | 1ull;
    idx.assign((size_t)mask + 1, kKeyMiss);
    head.assign((size_t)mask + 1, 0);
    for (uint32_t k = 0; k < n; ++k) {
      const uint8_t* pk = enc.data() + 32ull * k;
      const uint64_t h0 = load64(pk);
      uint32_t s = home(h0);
      bool dup = false;
      for (; idx[s] != kKeyMiss; s = (s + 1) & mask)
        if (head[s] == h0 && std::memcmp(enc.data() + 32ull * idx[s], pk, 32) == 0) {
          dup = true;
          break;
        }
      if (dup) continue;
      idx[s] = k;
      head[s] = h0;
    }
  }
};

}  // namespace nt
