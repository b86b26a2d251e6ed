// sc25519.hpp -- scalars mod L = 2^252 + 27742317777372353535851937790883648493
// (little-endian 32-bit words), plus the signed fixed-window recodings the
// SIMT double-scalar ladder uses.
//
// Semantics restated from the pinned crates:
//   Scalar::from_hash      -> sc_reduce512 of the 64-byte SHA-512 output
//   check_scalar (s decode) -> sc_is_canonical: accept iff s < L
#pragma once
#include "constants.hpp"
#include "nt_common.hpp"

namespace nt {

// a >= b over n words
template <int N>
NT_HD NT_INLINE uint32_t bn_ge(const uint32_t* a, const uint32_t* b) {
  uint32_t gt = 0, eq = 1;
#pragma unroll
  for (int i = N - 1; i >= 0; --i) {
    gt |= eq & (a[i] > b[i]);
    eq &= (a[i] == b[i]);
  }
  return gt | eq;
}

// a -= b (mod 2^(32N)), returns borrow
template <int N>
NT_HD NT_INLINE uint32_t bn_sub(uint32_t* a, const uint32_t* b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t t = (uint64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)t;
    br = (t >> 63) & 1;
  }
  return (uint32_t)br;
}

// out[0..NA+NB) = a * b  (schoolbook, v_mad_u64_u32 chains)
template <int NA, int NB>
NT_HD NT_INLINE void bn_mul(uint32_t* out, const uint32_t* a, const uint32_t* b) {
#pragma unroll
  for (int i = 0; i < NA + NB; ++i) out[i] = 0;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const uint64_t t = (uint64_t)a[i] * b[j] + out[i + j] + c;
      out[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    out[i + NB] = (uint32_t)c;
  }
}

// x (16 words, < 2^512) mod L -> out (8 words).  Barrett (HAC 14.42, b=2^32, k=8).
NT_HD NT_INLINE void sc_reduce512(uint32_t out[8], const uint32_t x[16]) {
  uint32_t q2[18], t[17], r[9];
  bn_mul<9, 9>(q2, x + 7, kScMu);          // floor(x / b^7) * mu
  bn_mul<9, 8>(t, q2 + 9, kScL);           // q3 * L, q3 = floor(q2 / b^9)
#pragma unroll
  for (int i = 0; i < 9; ++i) r[i] = x[i];
  bn_sub<9>(r, t);                          // (x - q3 L) mod b^9, in [0, 3L)
  uint32_t L9[9];
#pragma unroll
  for (int i = 0; i < 8; ++i) L9[i] = kScL[i];
  L9[8] = 0;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    uint32_t s[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) s[i] = r[i];
    const uint32_t ge = bn_ge<9>(r, L9);
    bn_sub<9>(s, L9);
#pragma unroll
    for (int i = 0; i < 9; ++i) r[i] = ge ? s[i] : r[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) out[i] = r[i];
}

// reduce a 256-bit value mod L
NT_HD NT_INLINE void sc_reduce256(uint32_t out[8], const uint32_t a[8]) {
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) { x[i] = a[i]; x[8 + i] = 0; }
  sc_reduce512(out, x);
}

// (a * b + c) mod L; a, b < 2^256 with a*b + c < 2^512
NT_HD NT_INLINE void sc_muladd(uint32_t out[8], const uint32_t a[8], const uint32_t b[8],
                               const uint32_t c[8]) {
  uint32_t p[16];
  bn_mul<8, 8>(p, a, b);
  uint64_t cy = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint64_t t = (uint64_t)p[i] + (i < 8 ? c[i] : 0u) + cy;
    p[i] = (uint32_t)t;
    cy = t >> 32;
  }
  sc_reduce512(out, p);
}

// dalek check_scalar: accept iff s < L (bit 255 set -> reject)
NT_HD NT_INLINE uint32_t sc_is_canonical(const uint32_t s[8]) {
  return (bn_ge<8>(s, kScL) ^ 1u);
}

// Signed radix-16 recoding: 64 digits in [-8, 7], packed as two's-complement
// nibbles (digit i in bits 4(i%8).. of word i/8).  Requires s < 2^255 - 2^251.
NT_HD NT_INLINE void sc_recode_w4(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t v = ((s[w] >> (4 * j)) & 15u) + carry;
      carry = v >= 8u;
      const uint32_t d = (v - (carry << 4)) & 15u;  // two's-complement nibble
      acc |= d << (4 * j);
    }
    out[w] = acc;
  }
}

// Signed radix-256 recoding: 32 digits in [-128, 127] as two's-complement bytes.
// Requires s < 2^255 - 2^247 (all our inputs are < L).
NT_HD NT_INLINE void sc_recode_w8(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    uint32_t acc = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t v = ((s[w] >> (8 * j)) & 255u) + carry;
      carry = v >= 128u;
      const uint32_t d = (v - (carry << 8)) & 255u;
      acc |= d << (8 * j);
    }
    out[w] = acc;
  }
}

// Signed radix-2^16 recoding: 16 digits in [-2^15, 2^15) as two's-complement
// halfwords (digit i in bits 16(i%2).. of word i/2).  Exact for s < 2^255 - 2^239
// (every scalar < L); for larger s (non-canonical signature scalars, rejected
// anyway) the final carry is dropped, and every |digit| stays <= 2^15.
NT_HD NT_INLINE void sc_recode_w16(uint32_t out[8], const uint32_t s[8]) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < 8; ++w) {
    const uint32_t lo = (s[w] & 0xffffu) + carry;
    carry = lo >= 0x8000u;
    const uint32_t hi = (s[w] >> 16) + carry;
    const uint32_t dlo = (lo - (carry << 16)) & 0xffffu;
    carry = hi >= 0x8000u;
    const uint32_t dhi = (hi - (carry << 16)) & 0xffffu;
    out[w] = dlo | (dhi << 16);
  }
}

}  // namespace nt
