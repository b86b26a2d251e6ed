// fe_inv_vt.hpp -- variable-time inversion in GF(2^255-19) by binary GCD.
//
// Verification handles public data only, so the key-cache kernel's one field
// inversion per wave batch (Montgomery's trick over a wave's rows, ~0.8 of a
// signature row of issue time as 254 squarings + 11 multiplies) can be a
// variable-time algorithm.  This is the optimized binary GCD of T. Pornin,
// "Optimized Binary GCD for Modular Inversion" (2020), Algorithm 2 with
// k = 31, restated for SIMT lanes:
//   * a = z, b = p, u = 1, v = 0  (invariants a 2^(30 i) = u z, b 2^(30 i) = v z mod p)
//   * 17 outer iterations (ceil((2 * 255 - 1) / 30)); each takes 62-bit
//     approximations of a and b (the low 30 bits exactly, the top 32 bits at
//     the larger of the two lengths), runs 30 exact-parity binary-GCD steps on
//     them recording a 2x2 matrix of 31-bit signed entries, applies it to the
//     full a, b (exact division by 2^30; a negative result is negated together
//     with its matrix row) and to u, v modulo p (no division: the result
//     carries 2^510, removed by one multiply at the end).
//   * at the end b = gcd(z, p) = 1 for z != 0 and v = z^-1 2^510; z = 0 gives 0
//     (as z^(p-2) does).
// Every lane runs the same schedule (30 steps per iteration, selects instead of
// branches), so lanes never diverge; the wave leaves the loop once a = 0 in all
// of its lanes (13-14 iterations instead of 17) and applies the remaining
// iterations' factor 2^30 each directly.  Numbers are 9 limbs of 30 bits; the
// matrix application is one v_mad_i64_i32 per limb and entry.
#pragma once
#include "ge25519.hpp"

namespace nt {

constexpr uint32_t kM30 = 0x3fffffffu;
constexpr int kGcdOuter = 17;  // ceil((2 * 255 - 1) / 30)
constexpr int kGcdInner = 30;  // k - 1
// -DNT_GCD_EARLY_EXIT=0 (A/B): all 17 iterations in every wave
#ifndef NT_GCD_EARLY_EXIT
#define NT_GCD_EARLY_EXIT 1
#endif
constexpr bool kGcdEarlyExit = NT_GCD_EARLY_EXIT != 0;

NT_HD NT_INLINE uint32_t clz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (uint32_t)__clz((int)x);
#else
  return x ? (uint32_t)__builtin_clz(x) : 32u;
#endif
}

// any lane of the wave (the host build: this lane)
NT_HD NT_INLINE bool gcd_wave_any(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(x != 0) != 0;
#else
  return x != 0;
#endif
}

// bit length of a nonnegative 9-limb value (0 for 0)
NT_HD NT_INLINE uint32_t gcd_len(const uint32_t x[9]) {
  uint32_t L = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) L = x[i] ? 30u * (uint32_t)i + 32u - clz32(x[i]) : L;
  return L;
}

// bits [s, s + 32) of a 9-limb value, 30 <= s < 270 (per-lane s: N-way selects)
NT_HD NT_INLINE uint32_t gcd_bits32(const uint32_t x[9], uint32_t s) {
  const uint32_t q = s / 30u, r = s - 30u * q;
  uint32_t x0 = 0, x1 = 0, x2 = 0;
#pragma unroll
  for (int i = 1; i < 9; ++i) {
    const bool hit = q == (uint32_t)i;
    x0 = hit ? x[i] : x0;
    x1 = hit ? (i + 1 < 9 ? x[i + 1] : 0u) : x1;
    x2 = hit ? (i + 2 < 9 ? x[i + 2] : 0u) : x2;
  }
  // r + 32 <= 61: of x2 only its lowest bit can be inside the window
  const uint64_t w = (uint64_t)x0 | ((uint64_t)x1 << 30) | ((uint64_t)(x2 & 1u) << 60);
  return (uint32_t)(w >> r);
}

// out = (a f + b g) / 2^30 for a, b < 2^255 (|f| + |g| <= 2^30, the low 30 bits
// of a f + b g are zero by construction); a negative result is negated and 1
// returned.  |result| <= 2^255: 9 limbs.
NT_HD NT_INLINE uint32_t gcd_lincomb_shift(uint32_t out[9], const uint32_t a[9], const uint32_t b[9], int32_t f,
                                           int32_t g) {
  int64_t t = (int64_t)(int32_t)a[0] * f;
  t += (int64_t)(int32_t)b[0] * g;
  t >>= 30;
#pragma unroll
  for (int i = 1; i < 9; ++i) {  // two v_mad_i64_i32 per limb
    t += (int64_t)(int32_t)a[i] * f;
    t += (int64_t)(int32_t)b[i] * g;
    out[i - 1] = (uint32_t)t & kM30;
    t >>= 30;
  }
  out[8] = (uint32_t)t & kM30;  // bits 240..269; t >> 30 is now the sign (0 or -1)
  const uint32_t neg = (t >> 30) < 0 ? 1u : 0u;
  // A negative result needs a wrong comparison of the approximations: ~1 in 3,000
  // inversions (Python model of this loop), so the negation sits behind a branch
  // that a wave skips unless one of its lanes takes it.
  if (neg) {
    int64_t s = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {  // two's complement over 270 bits
      s -= (int64_t)out[i];
      out[i] = (uint32_t)s & kM30;
      s >>= 30;
    }
  }
  return neg;
}

// out = u f + v g (mod p), kept in [0, 2^257): u, v < 2^257 (limb 8 < 2^17),
// |f| + |g| <= 2^30.  The sum (< 2^288 in magnitude) is folded at 2^255
// (2^255 = 19 mod p) and 2p added so it stays nonnegative.
NT_HD NT_INLINE void gcd_lincomb_modp(uint32_t out[9], const uint32_t u[9], const uint32_t v[9], int32_t f,
                                      int32_t g) {
  uint32_t r[9];
  int64_t t = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    t += (int64_t)(int32_t)u[i] * f;
    t += (int64_t)(int32_t)v[i] * g;
    r[i] = (uint32_t)t & kM30;
    t >>= 30;
  }
  // value = L + H 2^255, L = r[0..7] + (r[8] mod 2^15) 2^240, H = t 2^15 + r[8] >> 15
  const int64_t H = t * 32768 + (int64_t)(r[8] >> 15);
  int64_t c = (int64_t)r[0] + 19 * H + 2 * (int64_t)(kM30 - 18u);  // + 2p, limb by limb
  out[0] = (uint32_t)c & kM30;
  c >>= 30;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    c += (int64_t)r[i] + 2 * (int64_t)kM30;
    out[i] = (uint32_t)c & kM30;
    c >>= 30;
  }
  out[8] = (uint32_t)(c + (int64_t)(r[8] & 0x7fffu) + 2 * 0x7fff);  // < 2^17: the value < 2^257
}

// z^-1 (0 for z = 0); output "R"
NT_HD NT_INLINE void fe_invert_vt(fe& out, const fe& z) {
  uint32_t w[8];
  fe_tobytes_w(w, z);  // canonical, < p
  uint32_t a[9], b[9], u[9], v[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) {  // 30-bit limbs of the canonical value
    const int bit = 30 * i, q = bit >> 5, r = bit & 31;
    uint64_t x = (uint64_t)w[q];
    if (q + 1 < 8) x |= (uint64_t)w[q + 1] << 32;
    a[i] = (uint32_t)(x >> r) & kM30;
    b[i] = i == 0 ? kM30 - 18u : (i < 8 ? kM30 : 0x7fffu);  // p = 2^255 - 19
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0u;
  }
  int it = 0;
#pragma unroll 1
  for (; it < kGcdOuter; ++it) {
    // a = 0 in every lane: nothing is left to reduce (a lane reaches it after 12-13
    // of the 17 iterations, a wave of 64 after 13-14: tools/isa/gcd_iterations.py)
    uint32_t anz = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) anz |= a[i];
    if (kGcdEarlyExit && !gcd_wave_any(anz)) break;
    uint32_t ab[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) ab[i] = a[i] | b[i];
    uint32_t nb = gcd_len(ab);  // max(len(a), len(b))
    nb = nb > 62u ? nb : 62u;
    uint64_t A = (uint64_t)a[0] | ((uint64_t)gcd_bits32(a, nb - 32u) << 30);
    uint64_t B = (uint64_t)b[0] | ((uint64_t)gcd_bits32(b, nb - 32u) << 30);
    // the update matrix rows packed as f + 2^32 g in one signed 64-bit word each
    // (|f|, |g| <= 2^30: the packing is linear, so a row subtraction or doubling
    // is one 64-bit operation)
    int64_t r0 = 1, r1 = (int64_t)1 << 32;
#pragma unroll
    for (int j = 0; j < kGcdInner; ++j) {
      const bool odd = (A & 1u) != 0;
      const bool sw = odd && A < B;
      const uint64_t A1 = sw ? B : A, B1 = sw ? A : B;
      const int64_t R0 = sw ? r1 : r0, R1 = sw ? r0 : r1;
      A = (odd ? A1 - B1 : A1) >> 1;
      B = B1;
      r0 = odd ? R0 - R1 : R0;
      r1 = R1 * 2;
    }
    int32_t f0 = (int32_t)(uint32_t)r0, f1 = (int32_t)(uint32_t)r1;
    int32_t g0 = (int32_t)((r0 - f0) >> 32), g1 = (int32_t)((r1 - f1) >> 32);
    uint32_t na[9], nbv[9];
    const uint32_t nega = gcd_lincomb_shift(na, a, b, f0, g0);
    const uint32_t negb = gcd_lincomb_shift(nbv, a, b, f1, g1);
    f0 = nega ? -f0 : f0;
    g0 = nega ? -g0 : g0;
    f1 = negb ? -f1 : f1;
    g1 = negb ? -g1 : g1;
    uint32_t nu[9], nv[9];
    gcd_lincomb_modp(nu, u, v, f0, g0);
    gcd_lincomb_modp(nv, u, v, f1, g1);
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      a[i] = na[i];
      b[i] = nbv[i];
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  // An iteration with a = 0 leaves b = 1 and multiplies v by 2^30 (its matrix
  // is f1 = 0, g1 = 2^30): the skipped ones, done directly, keep the 2^510 below
#pragma unroll 1
  for (; it < kGcdOuter; ++it) {
    uint32_t nv[9];
    gcd_lincomb_modp(nv, u, v, 0, 1 << 30);
#pragma unroll
    for (int i = 0; i < 9; ++i) v[i] = nv[i];
  }
  // v = z^-1 2^510 mod p, v < 2^257: radix-2^25.5 limbs (limb 9 takes bits 230..256, < 2^27)
  fe vf;
  constexpr int kW[11] = {0, 26, 51, 77, 102, 128, 153, 179, 204, 230, 257};
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int lo = kW[i], hi = kW[i + 1];
    const int q = lo / 30, r = lo % 30;
    uint64_t x = (uint64_t)v[q];
    if (q + 1 < 9) x |= (uint64_t)v[q + 1] << 30;
    vf.v[i] = (uint32_t)(x >> r) & ((1u << (hi - lo)) - 1u);
  }
  fe c;
  fe_const(c, kFeInv2e510);
  fe_mul(out, vf, c);
}

}  // namespace nt
