// ed25519_ops.hpp -- per-lane Ed25519 operations shared by the gfx950 kernels
// (kernels.hip) and the host-compiled bound/op-count harness (tools/opcount.cpp,
// tests/cpp/).  Table storage is abstracted:
//   ATab: store(entry, ge_cached) / load(entry, ge_cached&)   -- j*(-A), j = 0..8
//   BTab: load(idx, ge_niels&)                                 -- j*B,   j = 0..128
//
// Semantics (restated from ed25519-dalek 1.0.1 /
// curve25519-dalek 3.x):
//   verify_one<kStrict>       = PublicKey::verify_strict  (crypto/src/lib.rs:200-204)
//   verify_one<kCofactorless> = one entry of verify_batch under the deterministic
//                               rule A.3                   (crypto/src/lib.rs:206-219)
//   sign_one                  = Keypair::generate + sign   (crypto/src/lib.rs:163-191)
#pragma once
#include "fe25519.hpp"
#include "ge25519.hpp"
#include "sc25519.hpp"
#include "sha512.hpp"

namespace nt {

// [j]B as an affine-niels entry (j = 0 -> identity).
NT_HD NT_INLINE void btab_entry(ge_niels& q, uint32_t j) {
  if (j == 0) {
    ge_niels_0(q);
    return;
  }
  uint32_t enc[8];
  for (int i = 0; i < 8; ++i) enc[i] = kBaseEnc[i];
  ge_p3 B, P;
  ge_frombytes_w(B, enc);
  ge_cached Bc;
  ge_p3_to_cached(Bc, B);
  ge_p3_0(P);
  for (int bit = 7; bit >= 0; --bit) {
    ge_p2 t2;
    ge_cp t;
    ge_p3_to_p2(t2, P);
    ge_dbl(t, t2);
    ge_cp_to_p3(P, t);
    if ((j >> bit) & 1) {
      ge_add_cached(t, P, Bc);
      ge_cp_to_p3(P, t);
    }
  }
  fe zi, x, y, d2;
  fe_invert(zi, P.Z);
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  fe_add(q.ypx, y, x);
  fe_carry(q.ypx);
  fe_sub(q.ymx, y, x);
  fe_carry(q.ymx);
  fe_const(d2, kFeD2);
  fe_mul(q.xy2d, x, y);
  fe_mul(q.xy2d, q.xy2d, d2);
}

// acc = [s]B + [k](-A): 64 signed 4-bit windows of k, 32 signed 8-bit windows of s.
// Every lane follows the same schedule (no divergence).
template <class ATab, class BTab>
NT_HD NT_INLINE void ladder(ge_p2& acc, const uint32_t kd[8], const uint32_t sd[8], const ATab& at,
                            const BTab& bt) {
  uint32_t kw[8], sw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { kw[i] = kd[i]; sw[i] = sd[i]; }
  ge_p2_0(acc);
  ge_cp t;
  ge_p3 u;
#pragma unroll 1
  for (int wi = 7; wi >= 0; --wi) {
    const uint32_t kcur = kw[7], scur = sw[7];
#pragma unroll
    for (int m = 7; m > 0; --m) { kw[m] = kw[m - 1]; sw[m] = sw[m - 1]; }
#pragma unroll 1
    for (int j = 7; j >= 0; --j) {
#pragma unroll 1
      for (int r = 0; r < 3; ++r) ge_dbl_p2(acc, acc);
      ge_dbl(t, acc);
      ge_cp_to_p3(u, t);
      const int32_t dk = (int32_t)(((kcur >> (4 * j)) & 15u) ^ 8u) - 8;
      const uint32_t negk = dk < 0;
      ge_cached ce;
      at.load((uint32_t)(negk ? -dk : dk), ce);
      ge_cached_cneg(ce, negk);
      ge_add_cached(t, u, ce);
      if ((j & 1) == 0) {
        const int32_t ds = (int32_t)(((scur >> (4 * j)) & 255u) ^ 128u) - 128;
        const uint32_t negs = ds < 0;
        ge_niels ne;
        bt.load((uint32_t)(negs ? -ds : ds), ne);
        ge_niels_cneg(ne, negs);
        ge_cp_to_p3(u, t);
        ge_add_niels(t, u, ne);
      }
      ge_cp_to_p2(acc, t);
    }
  }
}

// Fixed-base [x]B (x < L) with 8-bit signed windows.
template <class BTab>
NT_HD NT_INLINE void base_mul(ge_p2& acc, const uint32_t x[8], const BTab& bt) {
  uint32_t sd[8];
  sc_recode_w8(sd, x);
  ge_p2_0(acc);
  ge_cp t;
  ge_p3 u;
#pragma unroll 1
  for (int wi = 7; wi >= 0; --wi) {
    const uint32_t scur = sd[7];
#pragma unroll
    for (int m = 7; m > 0; --m) sd[m] = sd[m - 1];
#pragma unroll 1
    for (int j = 3; j >= 0; --j) {
#pragma unroll 1
      for (int r = 0; r < 7; ++r) ge_dbl_p2(acc, acc);
      ge_dbl(t, acc);
      ge_cp_to_p3(u, t);
      const int32_t ds = (int32_t)(((scur >> (8 * j)) & 255u) ^ 128u) - 128;
      const uint32_t negs = ds < 0;
      ge_niels ne;
      bt.load((uint32_t)(negs ? -ds : ds), ne);
      ge_niels_cneg(ne, negs);
      ge_add_niels(t, u, ne);
      ge_cp_to_p2(acc, t);
    }
  }
}

// One verification. Aw = pk words, Rw/Sw = signature halves, msg/len = message.
// Order chosen to keep little state live across the ladder: A is decoded and
// checked first; R is only decoded after the ladder (its bytes are 8 words).
template <int MODE, class ATab, class BTab>
NT_HD NT_INLINE uint32_t verify_one(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                                    const uint8_t* msg, uint64_t len, ATab& at, const BTab& bt) {
  uint32_t ok = sc_is_canonical(Sw);
  {
    ge_p3 A;
    ok &= ge_frombytes_w(A, Aw);
    if (MODE == kStrict) ok &= ge_is_small_order(A) ^ 1u;
    // table j * (-A), j = 0..8
    ge_p3 An;
    fe_neg(An.X, A.X);
    fe_carry(An.X);
    An.Y = A.Y;
    An.Z = A.Z;
    fe_neg(An.T, A.T);
    fe_carry(An.T);
    ge_cached c0, c1;
    ge_cached_0(c0);
    at.store(0, c0);
    ge_p3_to_cached(c1, An);
    at.store(1, c1);
    ge_p3 cur = An;
#pragma unroll 1
    for (uint32_t j = 2; j < 9; ++j) {
      ge_cp t;
      ge_add_cached(t, cur, c1);
      ge_cp_to_p3(cur, t);
      ge_cached cj;
      ge_p3_to_cached(cj, cur);
      at.store(j, cj);
    }
  }
  uint32_t kd[8], sd[8];
  {
    // k = SHA-512(R || A || M) mod L over the raw encodings (Scalar::from_hash)
    uint32_t prefix[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) { prefix[q] = Rw[q]; prefix[8 + q] = Aw[q]; }
    uint64_t st[8];
    sha512_prefixed<16>(st, prefix, msg, len);
    uint32_t hw[16], k[8];
    sha512_out_words(hw, st, 16);
    sc_reduce512(k, hw);
    sc_recode_w4(kd, k);
    sc_recode_w8(sd, Sw);
  }
  ge_p2 Rp;
  ladder(Rp, kd, sd, at, bt);
  ge_p3 R;
  ok &= ge_frombytes_w(R, Rw);
  if (MODE == kStrict) ok &= ge_is_small_order(R) ^ 1u;
  ok &= ge_eq_affine(Rp, R);
  return ok;
}

// Keygen + RFC 8032 signature.  sw = 32-byte seed words.
template <class BTab>
NT_HD NT_INLINE void sign_one(uint32_t Aw[8], uint32_t Rw[8], uint32_t s[8], const uint32_t sw[8],
                              const uint8_t* msg, uint64_t len, const BTab& bt) {
  uint64_t st[8];
  sha512_prefixed<8>(st, sw, nullptr, 0);
  uint32_t h[16];
  sha512_out_words(h, st, 16);
  uint32_t a[8], pre[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) { a[q] = h[q]; pre[q] = h[8 + q]; }
  a[0] &= 0xfffffff8u;
  a[7] &= 0x3fffffffu;
  a[7] |= 0x40000000u;
  uint32_t ared[8];
  sc_reduce256(ared, a);
  ge_p2 P;
  base_mul(P, ared, bt);
  ge_tobytes_w(Aw, P);

  sha512_prefixed<8>(st, pre, msg, len);
  uint32_t hr[16], r[8];
  sha512_out_words(hr, st, 16);
  sc_reduce512(r, hr);
  base_mul(P, r, bt);
  ge_tobytes_w(Rw, P);

  uint32_t prefix[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) { prefix[q] = Rw[q]; prefix[8 + q] = Aw[q]; }
  sha512_prefixed<16>(st, prefix, msg, len);
  uint32_t hk[16], k[8];
  sha512_out_words(hk, st, 16);
  sc_reduce512(k, hk);
  sc_muladd(s, k, a, r);
}

}  // namespace nt

namespace nt {

// ---------------------------------------------------------------------------
// Committee key cache: fixed-base combs.
//   comb entry (i, j) = j * 256^i * P  as affine niels, i in [0, 32), j in [0, 128]
// With a comb for -A and one for B, [s]B + [k](-A) is 64 mixed additions and
// no doublings: 32 signed 8-bit digits of k and of s.
// ---------------------------------------------------------------------------
constexpr int kCombPos = 32;
constexpr int kCombEntries = 129;

// j * 256^i * P (P given as p3), returned affine-niels.
NT_HD NT_INLINE void comb_entry(ge_niels& q, const ge_p3& P, uint32_t i, uint32_t j) {
  if (j == 0) {
    ge_niels_0(q);
    return;
  }
  ge_cached Pc;
  ge_p3_to_cached(Pc, P);
  ge_p3 Q;
  ge_p3_0(Q);
  ge_cp t;
#pragma unroll 1
  for (int bit = 7; bit >= 0; --bit) {
    ge_p2 t2;
    ge_p3_to_p2(t2, Q);
    ge_dbl(t, t2);
    ge_cp_to_p3(Q, t);
    if ((j >> bit) & 1) {
      ge_add_cached(t, Q, Pc);
      ge_cp_to_p3(Q, t);
    }
  }
  ge_p2 q2;
  ge_p3_to_p2(q2, Q);
#pragma unroll 1
  for (uint32_t r = 0; r < 8 * i; ++r) ge_dbl_p2(q2, q2);
  fe zi, x, y, d2;
  fe_invert(zi, q2.Z);
  fe_mul(x, q2.X, zi);
  fe_mul(y, q2.Y, zi);
  fe_add(q.ypx, y, x);
  fe_carry(q.ypx);
  fe_sub(q.ymx, y, x);
  fe_carry(q.ymx);
  fe_const(d2, kFeD2);
  fe_mul(q.xy2d, x, y);
  fe_mul(q.xy2d, q.xy2d, d2);
}

// Key metadata bits produced at keyset build time.
enum : uint32_t { kKeyDecodes = 1u, kKeySmallOrder = 2u };

// One verification against a cached key.  CA: comb of -A, CB: comb of B;
// both expose load(pos, idx, ge_niels&).  meta: kKey* bits of the key.
template <int MODE, class CombA, class CombB>
NT_HD NT_INLINE uint32_t verify_one_cached(uint32_t meta, const uint32_t Aw[8], const uint32_t Rw[8],
                                           const uint32_t Sw[8], const uint8_t* msg, uint64_t len,
                                           const CombA& ca, const CombB& cb) {
  uint32_t ok = sc_is_canonical(Sw) & (meta & kKeyDecodes ? 1u : 0u);
  if (MODE == kStrict) ok &= (meta & kKeySmallOrder) ? 0u : 1u;
  uint32_t kd[8], sd[8];
  {
    uint32_t prefix[16];
#pragma unroll
    for (int q = 0; q < 8; ++q) { prefix[q] = Rw[q]; prefix[8 + q] = Aw[q]; }
    uint64_t st[8];
    sha512_prefixed<16>(st, prefix, msg, len);
    uint32_t hw[16], k[8];
    sha512_out_words(hw, st, 16);
    sc_reduce512(k, hw);
    sc_recode_w8(kd, k);
    sc_recode_w8(sd, Sw);
  }
  ge_p3 acc;
  ge_p3_0(acc);
  ge_cp t;
  // word w of kd/sd holds the digits of positions 4w..4w+3 (one byte each);
  // consume word 0 and shift the arrays down (no dynamic register indexing)
#pragma unroll 1
  for (int w = 0; w < 8; ++w) {
    const uint32_t kw = kd[0], sw = sd[0];
#pragma unroll
    for (int m = 0; m < 7; ++m) { kd[m] = kd[m + 1]; sd[m] = sd[m + 1]; }
#pragma unroll 1
    for (int b = 0; b < 4; ++b) {
      const uint32_t pos = 4 * w + b;
      const int32_t dk = (int32_t)(((kw >> (8 * b)) & 255u) ^ 128u) - 128;
      const int32_t ds = (int32_t)(((sw >> (8 * b)) & 255u) ^ 128u) - 128;
      ge_niels ne;
      ca.load(pos, (uint32_t)(dk < 0 ? -dk : dk), ne);
      ge_niels_cneg(ne, dk < 0);
      ge_add_niels(t, acc, ne);
      ge_cp_to_p3(acc, t);
      cb.load(pos, (uint32_t)(ds < 0 ? -ds : ds), ne);
      ge_niels_cneg(ne, ds < 0);
      ge_add_niels(t, acc, ne);
      ge_cp_to_p3(acc, t);
    }
  }
  ge_p3 R;
  ok &= ge_frombytes_w(R, Rw);
  if (MODE == kStrict) ok &= ge_is_small_order(R) ^ 1u;
  ge_p2 Rp;
  ge_p3_to_p2(Rp, acc);
  ok &= ge_eq_affine(Rp, R);
  return ok;
}

}  // namespace nt

namespace nt {

// ---------------------------------------------------------------------------
// Cached verification of TWO signatures per lane with one shared inversion.
//
// R is never decompressed.  For R' = [s]B - [k]A with affine (x', y'):
//   dalek accepts  <=>  R decodes to a point equal to R'
//                  <=>  y_R == y' (mod p)  and  (sign(R) == parity(x')  or  x' == 0)
// (R's y is taken mod p exactly as curve25519-dalek's from_bytes does; a valid
// R' makes R decodable whenever y matches; x' = 0 covers the accepted
// "negative zero" encodings).  In strict mode the small-order test of R is done
// on R' (equal points have equal order; if they differ the verdict is reject
// anyway).  The two Z^-1 come from one exponentiation (Montgomery's trick).
// ---------------------------------------------------------------------------
template <class CombA, class CombB>
NT_HD NT_INLINE void comb_ladder(ge_p3& acc, const uint32_t k[8], const uint32_t Sw[8], const CombA& ca,
                                 const CombB& cb) {
  uint32_t kd[8], sd[8];
  sc_recode_w8(kd, k);
  sc_recode_w8(sd, Sw);
  ge_p3_0(acc);
  ge_cp t;
#pragma unroll 1
  for (int w = 0; w < 8; ++w) {
    const uint32_t kw = kd[0], sw = sd[0];
#pragma unroll
    for (int m = 0; m < 7; ++m) { kd[m] = kd[m + 1]; sd[m] = sd[m + 1]; }
#pragma unroll 1
    for (int b = 0; b < 4; ++b) {
      const uint32_t pos = 4 * w + b;
      const int32_t dk = (int32_t)(((kw >> (8 * b)) & 255u) ^ 128u) - 128;
      const int32_t ds = (int32_t)(((sw >> (8 * b)) & 255u) ^ 128u) - 128;
      ge_niels ne;
      ca.load(pos, (uint32_t)(dk < 0 ? -dk : dk), ne);
      ge_niels_cneg(ne, dk < 0);
      ge_add_niels(t, acc, ne);
      ge_cp_to_p3(acc, t);
      cb.load(pos, (uint32_t)(ds < 0 ? -ds : ds), ne);
      ge_niels_cneg(ne, ds < 0);
      ge_add_niels(t, acc, ne);
      ge_cp_to_p3(acc, t);
    }
  }
}

NT_HD NT_INLINE void hram_scalar(uint32_t k[8], const uint32_t Rw[8], const uint32_t Aw[8], const uint8_t* msg,
                                 uint64_t len) {
  uint32_t prefix[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) { prefix[q] = Rw[q]; prefix[8 + q] = Aw[q]; }
  uint64_t st[8];
  sha512_prefixed<16>(st, prefix, msg, len);
  uint32_t hw[16];
  sha512_out_words(hw, st, 16);
  sc_reduce512(k, hw);
}

// compare affine (x, y) with the encoding Rw under dalek decode semantics
NT_HD NT_INLINE uint32_t enc_matches(const fe& x, const fe& y, const uint32_t Rw[8]) {
  fe yr;
  fe_frombytes_w(yr, Rw);  // bit 255 dropped, value taken mod p by the compare
  uint32_t a[8], b[8], xw[8];
  fe_tobytes_w(a, y);
  fe_tobytes_w(b, yr);
  fe_tobytes_w(xw, x);
  uint32_t same = 1, xz = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    same &= (a[i] == b[i]);
    xz |= xw[i];
  }
  const uint32_t sign = Rw[7] >> 31;
  return same & (((xw[0] & 1u) == sign) | (xz == 0));
}

template <int MODE, class CombA, class CombB>
NT_HD NT_INLINE void verify_two_cached(uint32_t ok[2], const uint32_t meta[2], const uint32_t Aw[2][8],
                                       const uint32_t Rw[2][8], const uint32_t Sw[2][8], const uint8_t* msg[2],
                                       const uint64_t len[2], const CombA ca[2], const CombB& cb) {
  ge_p2 P[2];
#pragma unroll 1
  for (int j = 0; j < 2; ++j) {
    ok[j] = sc_is_canonical(Sw[j]) & (meta[j] & kKeyDecodes ? 1u : 0u);
    if (MODE == kStrict) ok[j] &= (meta[j] & kKeySmallOrder) ? 0u : 1u;
    uint32_t k[8];
    hram_scalar(k, Rw[j], Aw[j], msg[j], len[j]);
    ge_p3 acc;
    comb_ladder(acc, k, Sw[j], ca[j], cb);
    ge_p3_to_p2(P[j], acc);
  }
  // Z0^-1, Z1^-1 from one inversion
  fe zz, inv, zi0, zi1;
  fe_mul(zz, P[0].Z, P[1].Z);
  fe_invert(inv, zz);
  fe_mul(zi0, inv, P[1].Z);
  fe_mul(zi1, inv, P[0].Z);
#pragma unroll 1
  for (int j = 0; j < 2; ++j) {
    fe x, y;
    fe_mul(x, P[j].X, j ? zi1 : zi0);
    fe_mul(y, P[j].Y, j ? zi1 : zi0);
    ok[j] &= enc_matches(x, y, Rw[j]);
    if (MODE == kStrict) ok[j] &= ge_is_small_order_p2(P[j]) ^ 1u;
  }
}

}  // namespace nt
