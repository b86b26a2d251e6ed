// ge25519.hpp -- twisted Edwards -x^2 + y^2 = 1 + d x^2 y^2 over GF(2^255-19).
//
// Coordinates (same model curve25519-dalek uses, restated):
//   p2        (X:Y:Z)               x = X/Z, y = Y/Z
//   p3        (X:Y:Z:T)             extended, T = XY/Z
//   completed (X:Y:Z:T)             x = X/Z, y = Y/T   (output of add/dbl)
//   cached    (Y+X, Y-X, 2Z, 2dT)   variable-base table entries
//   niels     (y+x, y-x, 2dxy)      affine base-point table entries
// Bounds are tracked per line against fe25519.hpp's contract.
#pragma once
#include "constants.hpp"
#include "fe25519.hpp"

namespace nt {

struct ge_p2 { fe X, Y, Z; };
struct ge_p3 { fe X, Y, Z, T; };
struct ge_cp { fe X, Y, Z, T; };
struct ge_cached { fe YpX, YmX, Z2, T2d; };
struct ge_niels { fe ypx, ymx, xy2d; };

NT_HD NT_INLINE void fe_const(fe& h, const uint32_t c[10]) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = c[i];
}

NT_HD NT_INLINE void ge_p3_0(ge_p3& h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); fe_0(h.T); }
NT_HD NT_INLINE void ge_p2_0(ge_p2& h) { fe_0(h.X); fe_1(h.Y); fe_1(h.Z); }
NT_HD NT_INLINE void ge_cached_0(ge_cached& h) {
  fe_1(h.YpX); fe_1(h.YmX); fe_0(h.Z2); h.Z2.v[0] = 2; fe_0(h.T2d);
}
NT_HD NT_INLINE void ge_niels_0(ge_niels& h) { fe_1(h.ypx); fe_1(h.ymx); fe_0(h.xy2d); }

// completed -> p2 (3M); every completed coordinate here is < 2^28.6 with
// X and Z "g-safe" (< 2^27.75) as produced below.
NT_HD NT_INLINE void ge_cp_to_p2(ge_p2& r, const ge_cp& p) {
  fe_mul(r.X, p.T, p.X);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.T, p.Z);
  NT_POINT_FENCE();
}
NT_HD NT_INLINE void ge_cp_to_p3(ge_p3& r, const ge_cp& p) {
  fe_mul(r.X, p.T, p.X);
  fe_mul(r.Y, p.Y, p.Z);
  fe_mul(r.Z, p.T, p.Z);
  fe_mul(r.T, p.Y, p.X);
  NT_POINT_FENCE();
}
NT_HD NT_INLINE void ge_p3_to_p2(ge_p2& r, const ge_p3& p) { r.X = p.X; r.Y = p.Y; r.Z = p.Z; }

// Cached entries are only ever g operands of fe_mul (ge_add_cached) or swapped /
// negated (ge_cached_cneg: T2d is a multiply output), so their sums need no carry:
// from "R" coordinates Y + X < 2^27 (even) / 2^26.01 (odd), Y + 2p - X < 2^27.58,
// 2Z < 2^27 -- all within fe_mul's g bound 2^27.75.  (The ladder's seed, which
// subtracts two of them, uses fe_sub4.)
#ifndef NT_CACHED_NOCARRY
#define NT_CACHED_NOCARRY 1
#endif
NT_HD NT_INLINE void ge_p3_to_cached(ge_cached& r, const ge_p3& p) {
  fe d2;
  fe_const(d2, kFeD2);
  fe_add(r.YpX, p.Y, p.X);
  fe_sub(r.YmX, p.Y, p.X);
  fe_add(r.Z2, p.Z, p.Z);
#if !NT_CACHED_NOCARRY
  fe_carry(r.YpX);
  fe_carry(r.YmX);
  fe_carry(r.Z2);
#endif
  fe_mul(r.T2d, p.T, d2);
  NT_POINT_FENCE();
}

// 2P from a p2 point with "R" coordinates (dalek ProjectivePoint::double).
NT_HD NT_INLINE void ge_dbl(ge_cp& r, const ge_p2& p) {
  fe XX, YY, ZZ, S, t;
  fe_sq(XX, p.X);
  fe_sq(YY, p.Y);
  fe_sq(ZZ, p.Z);
  fe_add(t, p.X, p.Y);        // < 2^27 (sq_wide input bound)
  fe_sq_wide(S, t);
  fe_add(r.Y, YY, XX);        // Y' = YY + XX           < 2^27
  fe_sub(r.Z, YY, XX);        // Z' = YY - XX (2p)      < 2^27.6
  fe_sub4(r.X, S, r.Y);       // X' = S - Y'  (4p)      < 2^28.6 -> carry
  fe_carry(r.X);
#ifndef NT_DBL_SUB4
#define NT_DBL_SUB4 0
#endif
#if NT_DBL_SUB4
  fe_dbl_sub4(r.T, ZZ, r.Z);  // T' = 2ZZ - Z' (4p)     < 2^28.6 (f-side only)
#else
  fe_add(ZZ, ZZ, ZZ);
  fe_sub4(r.T, ZZ, r.Z);
#endif
  NT_POINT_FENCE();
}

// P + Q (neg=0) or P - Q (neg=1), Q cached with "R" coordinates.
NT_HD NT_INLINE void ge_add_cached(ge_cp& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, PP, MM, TT, ZZ;
  fe_add(a, p.Y, p.X);        // < 2^27
  fe_sub(b, p.Y, p.X);        // < 2^27.6
  fe_mul(PP, a, q.YpX);
  fe_mul(MM, b, q.YmX);
  fe_mul(TT, p.T, q.T2d);
  fe_mul(ZZ, p.Z, q.Z2);
  fe_sub(r.X, PP, MM);
  fe_add(r.Y, PP, MM);
  fe_add(r.Z, ZZ, TT);
  fe_sub(r.T, ZZ, TT);
  NT_POINT_FENCE();
}

// P + Q, Q affine niels.  Split in two halves so a caller can issue its next
// table load as soon as the multiplies that read q have been issued.
NT_HD NT_INLINE void ge_add_niels_1(fe& PP, fe& MM, fe& TT, const ge_p3& p, const ge_niels& q) {
  fe a, b;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul(PP, a, q.ypx);
  fe_mul(MM, b, q.ymx);
  fe_mul(TT, p.T, q.xy2d);
  NT_POINT_FENCE();
}
NT_HD NT_INLINE void ge_add_niels_2(ge_cp& r, const fe& PP, const fe& MM, const fe& TT, const fe& Z) {
  fe ZZ;
  fe_add(ZZ, Z, Z);           // < 2^27
  fe_sub(r.X, PP, MM);
  fe_add(r.Y, PP, MM);
  fe_add(r.Z, ZZ, TT);
  fe_sub(r.T, ZZ, TT);        // ZZ + 2p - TT < 2^27.6
  NT_POINT_FENCE();
}
NT_HD NT_INLINE void ge_add_niels(ge_cp& r, const ge_p3& p, const ge_niels& q) {
  fe PP, MM, TT;
  ge_add_niels_1(PP, MM, TT, p, q);
  ge_add_niels_2(r, PP, MM, TT, p.Z);
}

// The first point of a comb sum that starts at the identity: an affine niels
// entry (y+x, y-x, 2dxy) taken as (2x : 2y : 2 : 2xy), T = (2dxy) / d -- one
// multiply instead of an addition to the identity (7).
NT_HD NT_INLINE void ge_p3_from_niels(ge_p3& r, const ge_niels& q) {
  fe dinv;
  fe_const(dinv, kFeDInv);
  fe_sub(r.X, q.ypx, q.ymx);
  fe_carry(r.X);
  fe_add(r.Y, q.ypx, q.ymx);
  fe_carry(r.Y);
  fe_0(r.Z);
  r.Z.v[0] = 2;
  fe_mul(r.T, q.xy2d, dinv);  // xy2d: niels (< 2^26) or its fe_neg (f side)
  NT_POINT_FENCE();
}

// Affine niels entry of the projective point (X:Y:Z), given zi = Z^-1.
NT_HD NT_INLINE void ge_niels_from(ge_niels& q, const fe& X, const fe& Y, const fe& zi) {
  fe x, y, d2;
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_add(q.ypx, y, x);
  fe_carry(q.ypx);
  fe_sub(q.ymx, y, x);
  fe_carry(q.ymx);
  fe_const(d2, kFeD2);
  fe_mul(q.xy2d, x, y);
  fe_mul(q.xy2d, q.xy2d, d2);
  NT_POINT_FENCE();
}

// Conditionally negate a cached entry in place: -(Y+X, Y-X, 2Z, 2dT) = (Y-X, Y+X, 2Z, -2dT)
NT_HD NT_INLINE void ge_cached_cneg(ge_cached& q, uint32_t neg) {
  fe n;
  fe_neg(n, q.T2d);           // < 2^27
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t a = q.YpX.v[i], b = q.YmX.v[i];
    q.YpX.v[i] = neg ? b : a;
    q.YmX.v[i] = neg ? a : b;
    q.T2d.v[i] = neg ? n.v[i] : q.T2d.v[i];
  }
}
NT_HD NT_INLINE void ge_niels_cneg(ge_niels& q, uint32_t neg) {
  fe n;
  fe_neg(n, q.xy2d);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t a = q.ypx.v[i], b = q.ymx.v[i];
    q.ypx.v[i] = neg ? b : a;
    q.ymx.v[i] = neg ? a : b;
    q.xy2d.v[i] = neg ? n.v[i] : q.xy2d.v[i];
  }
}

NT_HD NT_INLINE void ge_dbl_p2(ge_p2& r, const ge_p2& p) {
  ge_cp t;
  ge_dbl(t, p);
  ge_cp_to_p2(r, t);
}

// curve25519-dalek FieldElement::sqrt_ratio_i: returns 1 iff u/v is a nonzero
// square or u == 0; r = the nonnegative root.  u, v "R".
NT_HD NT_INLINE uint32_t fe_sqrt_ratio_i(fe& r, const fe& u, const fe& v) {
  fe v3, v7, t, check, negu, negu_i, sqm1, ri;
  fe_const(sqm1, kFeSqrtM1);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);          // v^3
  fe_sq(v7, v3);
  fe_mul(v7, v7, v);          // v^7
  fe_mul(t, u, v7);
  fe_pow22523(t, t);          // (u v^7)^((p-5)/8)
  fe_mul(t, t, v3);
  fe_mul(r, t, u);            // u v^3 (u v^7)^((p-5)/8)
  fe_sq(check, r);
  fe_mul(check, check, v);    // v r^2
  fe_neg(negu, u);            // <= 2p limbwise
  fe_mul(negu_i, negu, sqm1);
  const uint32_t correct = fe_eq(check, u);
  const uint32_t flipped = fe_eq(check, negu);
  const uint32_t flipped_i = fe_eq(check, negu_i);
  fe_mul(ri, r, sqm1);
  fe_cmov(r, ri, flipped | flipped_i);
  fe n;
  fe_neg(n, r);
  fe_cmov(r, n, fe_isneg(r));
  fe_carry(r);
  return correct | flipped;
}

// CompressedEdwardsY::decompress (dalek semantics: y not reduced/rejected,
// negative zero accepted).  w = 8 little-endian words of the encoding.
NT_HD NT_INLINE uint32_t ge_frombytes_w(ge_p3& h, const uint32_t w[8]) {
  fe u, v, yy, one, d;
  fe_frombytes_w(h.Y, w);
  fe_1(one);
  fe_const(d, kFeD);
  fe_1(h.Z);
  fe_sq(yy, h.Y);
  fe_sub(u, yy, one);
  fe_carry(u);                // u = y^2 - 1
  fe_mul(v, yy, d);
  fe_add(v, v, one);          // v = d y^2 + 1
  const uint32_t ok = fe_sqrt_ratio_i(h.X, u, v);
  fe n;
  fe_neg(n, h.X);
  fe_cmov(h.X, n, w[7] >> 31);
  fe_carry(h.X);
  fe_mul(h.T, h.X, h.Y);
  return ok;
}

// canonical compression of a p2 point (one inversion)
NT_HD NT_INLINE void ge_tobytes_w(uint32_t w[8], const ge_p2& p) {
  fe zi, x, y;
  fe_invert(zi, p.Z);
  fe_mul(x, p.X, zi);
  fe_mul(y, p.Y, zi);
  fe_tobytes_w(w, y);
  w[7] ^= fe_isneg(x) << 31;
}

NT_HD NT_INLINE uint32_t ge_p2_is_identity(const ge_p2& p) {
  return fe_iszero(p.X) & fe_eq(p.Y, p.Z);
}

// Small order from the canonical y alone: the 8 torsion points are exactly the
// curve points with y in {1, -1, 0, +-y8} (identity, order 2, the two of
// order 4, the four of order 8 -- and -(x, y) = (-x, y) keeps the set closed),
// so for a point ON the curve "[8]P == identity" (EdwardsPoint::is_small_order)
// is 5 word compares instead of 3 doublings.  y = canonical words (< p).
NT_HD NT_INLINE uint32_t torsion_y_words(const uint32_t y[8]) {
  uint32_t z = 1, one = 1, m1 = 1, a = 1, b = 1;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t pm1 = i == 0 ? 0xffffffecu : (i == 7 ? 0x7fffffffu : 0xffffffffu);  // p - 1
    z &= y[i] == 0u;
    one &= y[i] == (i == 0 ? 1u : 0u);
    m1 &= y[i] == pm1;
    a &= y[i] == kTorsionY8[i];
    b &= y[i] == kTorsionY8n[i];
  }
  return z | one | m1 | a | b;
}
// small order of a decoded point (ge_frombytes_w: Z = 1, Y = y, possibly >= p)
NT_HD NT_INLINE uint32_t ge_is_small_order_affine(const ge_p3& p) {
  uint32_t w[8];
  fe_tobytes_w(w, p.Y);
  return torsion_y_words(w);
}

// [8]P == identity  (EdwardsPoint::is_small_order), by doublings: any Z
NT_HD NT_INLINE uint32_t ge_is_small_order_p2(const ge_p2& p) {
  ge_p2 t = p;
#pragma unroll 1
  for (int i = 0; i < 3; ++i) ge_dbl_p2(t, t);
  return ge_p2_is_identity(t);
}
NT_HD NT_INLINE uint32_t ge_is_small_order(const ge_p3& p) {
  ge_p2 t;
  ge_p3_to_p2(t, p);
  return ge_is_small_order_p2(t);
}

// Projective equality of a p2 point with a p3 point whose Z = 1 (decompressed).
NT_HD NT_INLINE uint32_t ge_eq_affine(const ge_p2& p, const ge_p3& q) {
  fe a, b;
  fe_mul(a, q.X, p.Z);
  fe_mul(b, q.Y, p.Z);
  return fe_eq(p.X, a) & fe_eq(p.Y, b);
}

}  // namespace nt
