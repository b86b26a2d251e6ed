// sc25519.hpp -- scalars mod L = 2^252 + 27742317777372353535851937790883648493
// (little-endian 32-bit words), plus the signed fixed-window recodings the
// SIMT double-scalar ladder uses.
//
// Semantics restated from the pinned crates:
//   Scalar::from_hash      -> sc_reduce512 of the 64-byte SHA-512 output
//   check_scalar (s decode) -> sc_is_canonical: accept iff s < L
#pragma once
#include <math.h>

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

// ---------------------------------------------------------------------------
// Half-size scalars (lattice reduction in dimension 2 over Z / 8L).
//
// For k < L find (u, v), v odd and 0 < v < L, with u == v k (mod 8L) and
// |u|, v ~ 2^128.  Then for any points A, R of the curve (order | 8L) and any s:
//      [v]([s]B - [k]A - R) = [v s mod L]B - [u]A - [v]R
// and, because gcd(v, 8L) = 1, the left side is the identity iff
// [s]B - [k]A - R is.  This turns the 253-bit variable-base scalar into two
// ~128-bit ones (half the doublings) with EXACTLY the verdict of the
// full-size equation -- for every A and R, torsion components included (the
// lattice is taken mod 8L, not mod L, for that reason).
//
// Method: the extended Euclidean remainder sequence of (8L, k) (r_i == t_i k)
// stopped at the first r < 2^127.5 (then |t| <= 8L / r_prev < 2^127.5).
// Quotients are estimated from fp64 images of the remainders and rounded
// DOWN (a short quotient is just a partial step), so every basis the loop
// visits is an exact lattice basis with r0 |t1| + r1 |t0| = 8L and t0, t1 of
// opposite signs; the result is therefore valid whatever the rounding.  If
// the last t is even, the odd one of the two neighbouring vectors with fewer
// bits is used.  Anything unexpected (step cap, > 250 bits) falls back to the
// trivial vector (k, 1).  Returns max(bitlen|u|, bitlen v) (never an
// underestimate).  Per-lane loop lengths differ (~73 steps on average).
// Down to r1 ~ 2^136 the steps run in Lehmer batches (lat_lehmer_batch:
// ~20 quotients per fp64 run, one matrix update of the multiword state),
// landing on the same remainder pairs; the one-step loop finishes.
// ---------------------------------------------------------------------------
template <int N>
NT_HD NT_INLINE double bn_to_f64(const uint32_t* a) {
  double d = (double)a[N - 1];
#pragma unroll
  for (int i = N - 2; i >= 0; --i) d = fma(d, 4294967296.0, (double)a[i]);
  return d;
}

// bit length of a non-negative integer from its fp64 image (rounding can only
// overestimate by one)
NT_HD NT_INLINE int f64_bitlen(double d) {
  int e;
  frexp(d, &e);
  return d == 0.0 ? 0 : e;
}

// a < b over N words
template <int N>
NT_HD NT_INLINE uint32_t bn_lt(const uint32_t* a, const uint32_t* b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) br = ((uint64_t)a[i] - b[i] - br) >> 63;
  return (uint32_t)br;
}

// a -= q b over N words (caller guarantees no underflow)
template <int N>
NT_HD NT_INLINE void bn_submul1(uint32_t* a, const uint32_t* b, uint32_t q) {
  uint64_t c = 0;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t p = (uint64_t)q * b[i] + c;
    c = p >> 32;
    const uint64_t t = (uint64_t)a[i] - (uint32_t)p - br;
    a[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
}

// a += q b over N words (caller guarantees no overflow)
template <int N>
NT_HD NT_INLINE void bn_addmul1(uint32_t* a, const uint32_t* b, uint32_t q) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t p = (uint64_t)q * b[i] + a[i] + c;
    a[i] = (uint32_t)p;
    c = p >> 32;
  }
}

// floor(d0 / d1) rounded down by a 2^-40 margin, clamped to [1, 2^32 - 1]
NT_HD NT_INLINE uint32_t lat_quot(double d0, double d1) {
  const double qd = d0 / d1 * (1.0 - 0x1p-40);
  return qd >= 4294967295.0 ? 0xffffffffu : (qd < 1.0 ? 1u : (uint32_t)qd);
}

constexpr int kLatMaxSteps = 600;
constexpr double kLatStop = 0x1.6a09e667f3bcdp+127;  // 2^127.5

// n-word helpers of the Lehmer batches
// out[0..N] = a * m
template <int N>
NT_HD NT_INLINE void bn_mul1(uint32_t* out, const uint32_t* a, uint32_t m) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t p = (uint64_t)m * a[i] + c;
    out[i] = (uint32_t)p;
    c = p >> 32;
  }
  out[N] = (uint32_t)c;
}
// out = a - b over N words; returns the borrow
template <int N>
NT_HD NT_INLINE uint32_t bn_sub(uint32_t* out, const uint32_t* a, const uint32_t* b) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const uint64_t t = (uint64_t)a[i] - b[i] - br;
    out[i] = (uint32_t)t;
    br = (uint32_t)(t >> 63);
  }
  return br;
}
// a += b over N words; returns the carry
template <int N>
NT_HD NT_INLINE uint32_t bn_add(uint32_t* a, const uint32_t* b) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    c += (uint64_t)a[i] + b[i];
    a[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}

// Remainder-sequence state: r0 > r1 >= 0 (8 words), |t0|, |t1| (4 words, of
// opposite signs, t1neg = sign of t1), fp64 images d0, d1, steps taken.
struct LatState {
  uint32_t r0[8], r1[8], t0[4], t1[4];
  uint32_t t1neg;
  double d0, d1;
  int steps;
};

// One exact step: r0 -= q r1 with q = floor(d0 / d1) rounded down (a short
// quotient is a partial step), swap when r0 < r1.
NT_HD NT_INLINE void lat_exact_step(LatState& S) {
  const uint32_t q = lat_quot(S.d0, S.d1);
  bn_submul1<8>(S.r0, S.r1, q);
  bn_addmul1<4>(S.t0, S.t1, q);
  S.d0 = bn_to_f64<8>(S.r0);
  const uint32_t sw = bn_lt<8>(S.r0, S.r1);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t a = S.r0[i], b = S.r1[i];
    S.r0[i] = sw ? b : a;
    S.r1[i] = sw ? a : b;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t a = S.t0[i], b = S.t1[i];
    S.t0[i] = sw ? b : a;
    S.t1[i] = sw ? a : b;
  }
  const double e0 = S.d0;
  S.d0 = sw ? S.d1 : S.d0;
  S.d1 = sw ? e0 : S.d1;
  S.t1neg ^= sw;
  ++S.steps;
}

// Lehmer batch: Euclid on the leading 53 bits of (r0, r1) in fp64, then ONE
// 2x2 cofactor matrix applied to the 256-bit remainders and the t's, instead
// of a multiword update per quotient.  a = the 53-bit mantissa of d0 (r0 / 2^sh),
// b = floor(d1 / 2^sh); both are within E = 8 of the true r / 2^sh (seven fma
// roundings in bn_to_f64 + the floor).  After j steps with cofactor magnitudes
// (x, y) a truncated remainder differs from the exact one (/ 2^sh) by at most
// E (x + y), so a step is accepted only while its new remainder r exceeds that
// bound and b - r exceeds the bound of both rows: then the exact remainders stay
// positive and ordered, i.e. every accepted quotient IS the exact Euclid
// quotient and the batch lands on the same remainder pair the one-step loop
// visits.  Steps stop above 2^132 (the one-step loop finishes the last few).
// The applied state is re-validated (r0' > r1' >= 0, |t| in 4 words); an
// empty or invalid batch falls back to one exact step.
constexpr double kLehmerStop = 0x1p136;  // batches while r1 >= 2^136
constexpr int kLehmerMaxInner = 48;      // > the 37 all-ones quotients of 26 bits
NT_HD NT_INLINE void lat_lehmer_batch(LatState& S) {
  int e;
  frexp(S.d0, &e);
  const int sh = e - 53;  // d0 in [2^(e-1), 2^e): d0 / 2^sh is an integer in [2^52, 2^53)
  double a = ldexp(S.d0, -sh), b = floor(ldexp(S.d1, -sh));
  const double thr = ldexp(1.0, 132 - sh);
  double x0 = 1.0, y0 = 0.0, x1 = 0.0, y1 = 1.0;
  int n = 0;
#pragma unroll 1
  for (int it = 0; it < kLehmerMaxInner; ++it) {
    if (!(b >= 1.0)) break;
#if defined(__HIP_DEVICE_COMPILE__)
    // v_rcp_f64 (~1 ulp) instead of the IEEE division sequence: an estimate off
    // by more than the one correction below fails the acceptance test
    double q = floor(a * __builtin_amdgcn_rcp(b));
#else
    double q = floor(a / b);
#endif
    double r = fma(-q, b, a);  // exact: every operand and product < 2^53
    if (r < 0.0) {
      q -= 1.0;
      r += b;
    } else if (r >= b) {
      q += 1.0;
      r -= b;
    }
    const double x2 = fma(q, x1, x0), y2 = fma(q, y1, y0);
    if (!(r >= thr && r > 8.0 * (x2 + y2) && b - r > 8.0 * (x1 + y1 + x2 + y2))) break;
    a = b;
    b = r;
    x0 = x1;
    y0 = y1;
    x1 = x2;
    y1 = y2;
    ++n;
  }
  // (cofactors < 2^26 here: r > 8 (x + y) with r < 2^53)
  const uint32_t X0 = (uint32_t)x0, Y0 = (uint32_t)y0, X1 = (uint32_t)x1, Y1 = (uint32_t)y1;
  const uint32_t odd = (uint32_t)n & 1u;
  // remainder j of the batch = (-1)^j (x_j r0 - y_j r1): r0' is j = n, r1' is j = n + 1
  uint32_t P[9], Q[9], A[9], B[9], n0[9], n1[9];
  bn_mul1<8>(P, S.r0, X0);
  bn_mul1<8>(Q, S.r1, Y0);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    A[i] = odd ? Q[i] : P[i];
    B[i] = odd ? P[i] : Q[i];
  }
  uint32_t bad = bn_sub<9>(n0, A, B);
  bn_mul1<8>(P, S.r0, X1);
  bn_mul1<8>(Q, S.r1, Y1);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    A[i] = odd ? P[i] : Q[i];
    B[i] = odd ? Q[i] : P[i];
  }
  bad |= bn_sub<9>(n1, A, B);
  bad |= (n0[8] | n1[8]) != 0u;
  bad |= bn_lt<8>(n1, n0) ^ 1u;
  // |t_j| = x_j |t0| + y_j |t1| (t0, t1 of opposite signs)
  uint32_t m0[5], m1[5], w[5];
  bn_mul1<4>(m0, S.t0, X0);
  bn_mul1<4>(w, S.t1, Y0);
  bn_add<5>(m0, w);
  bn_mul1<4>(m1, S.t0, X1);
  bn_mul1<4>(w, S.t1, Y1);
  bn_add<5>(m1, w);
  bad |= (m0[4] | m1[4]) != 0u;
  if (n == 0 || bad) {
    lat_exact_step(S);
    return;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    S.r0[i] = n0[i];
    S.r1[i] = n1[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    S.t0[i] = m0[i];
    S.t1[i] = m1[i];
  }
  S.t1neg ^= odd;
  S.d0 = bn_to_f64<8>(S.r0);
  S.d1 = bn_to_f64<8>(S.r1);
  S.steps += n;
}

// LEHMER = false: the one-step loop only (the reference the tests compare the
// batched reduction with; the kernels use LEHMER = true).
template <bool LEHMER>
NT_HD NT_INLINE int sc_halfsize_t(uint32_t u[8], uint32_t& uneg, uint32_t v[8], const uint32_t k[8]) {
  LatState S;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    S.r0[i] = kSc8L[i];
    S.r1[i] = k[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) S.t0[i] = S.t1[i] = 0;
  S.t1[0] = 1;
  S.t1neg = 0;
  S.d0 = bn_to_f64<8>(S.r0);
  S.d1 = bn_to_f64<8>(S.r1);
  S.steps = 0;
  if (LEHMER) {
#pragma unroll 1
    while (S.d1 >= kLehmerStop && S.steps < kLatMaxSteps) lat_lehmer_batch(S);
  }
  // Inside the loop r1 >= 2^127.5, so |t0|, |t1| <= 8L / r1 < 2^128: 4 words.
#pragma unroll 1
  while (S.d1 >= kLatStop && S.steps < kLatMaxSteps) lat_exact_step(S);
  uint32_t(&r0)[8] = S.r0;
  uint32_t(&r1)[8] = S.r1;
  uint32_t(&t0)[4] = S.t0;
  uint32_t(&t1)[4] = S.t1;
  const uint32_t t1neg = S.t1neg;
  const double d0 = S.d0, d1 = S.d1;
  const int steps = S.steps;
  int bits;
  if (t1[0] & 1u) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      u[i] = r1[i];
      v[i] = i < 4 ? t1[i] : 0u;
    }
    uneg = t1neg;
    bits = f64_bitlen(d1);
    const int bt = f64_bitlen(bn_to_f64<4>(t1));
    bits = bt > bits ? bt : bits;
  } else {
    // t1 even => t0 odd (gcd(t0, t1) = 1).  Candidates with the sign of t0:
    // b0 = (r0, t0) and b2 = b0 - q b1 = (r0 - q r1, |t0| + q |t1|).
    uint32_t r2[8], t2[8], t1w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      r2[i] = r0[i];
      t2[i] = i < 4 ? t0[i] : 0u;
      t1w[i] = i < 4 ? t1[i] : 0u;
    }
    const uint32_t q = d1 > 0.0 ? lat_quot(d0, d1) : 1u;
    if (d1 > 0.0) bn_submul1<8>(r2, r1, q);
    bn_addmul1<8>(t2, t1w, q);
    const int b0r = f64_bitlen(d0), b0t = f64_bitlen(bn_to_f64<4>(t0));
    const int b2r = f64_bitlen(bn_to_f64<8>(r2)), b2t = f64_bitlen(bn_to_f64<8>(t2));
    const int c0 = b0r > b0t ? b0r : b0t;
    const int c2 = b2r > b2t ? b2r : b2t;
    const bool use2 = d1 > 0.0 && c2 < c0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      u[i] = use2 ? r2[i] : r0[i];
      v[i] = use2 ? t2[i] : (i < 4 ? t0[i] : 0u);
    }
    uneg = t1neg ^ 1u;
    bits = use2 ? c2 : c0;
  }
  if (steps >= kLatMaxSteps || bits > 250) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      u[i] = k[i];
      v[i] = 0;
    }
    v[0] = 1;
    uneg = 0;
    bits = 253;
  }
  return bits;
}
NT_HD NT_INLINE int sc_halfsize(uint32_t u[8], uint32_t& uneg, uint32_t v[8], const uint32_t k[8]) {
#ifdef NT_LAT_ONE_STEP  // A/B builds only
  return sc_halfsize_t<false>(u, uneg, v, k);
#else
  return sc_halfsize_t<true>(u, uneg, v, k);
#endif
}
NT_HD NT_INLINE int sc_halfsize_euclid(uint32_t u[8], uint32_t& uneg, uint32_t v[8], const uint32_t k[8]) {
  return sc_halfsize_t<false>(u, uneg, v, k);
}

// (v * s) mod L for v, s < 2^256
NT_HD NT_INLINE void sc_mul(uint32_t out[8], const uint32_t a[8], const uint32_t b[8]) {
  uint32_t p[16];
  bn_mul<8, 8>(p, a, b);
  sc_reduce512(out, p);
}

}  // namespace nt
