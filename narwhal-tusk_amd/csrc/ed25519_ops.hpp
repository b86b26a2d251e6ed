// ed25519_ops.hpp -- per-lane Ed25519 operations shared by the gfx950 kernels
// (k_*.hip) and the host-compiled harness (tests/cpp/nt_host_harness.cpp,
// tools/opcount.py).  Table storage is abstracted:
//   ATab:  store(entry, ge_cached) / load_signed(e0, d, ge_cached&)   j*(-A), j = 0..8, per lane
//          (load_signed: entry e0 + |d|, negated when d < 0)
//   WComb: load(pos, idx, ge_niels&)                            idx * 2^(16 pos) * P (wide comb)
//
// Semantics (restated from ed25519-dalek 1.0.1 /
// curve25519-dalek 3.x):
//   verify_n<kStrict>         = PublicKey::verify_strict  (crypto/src/lib.rs:200-204)
//   verify_n<kCofactorless>   = one entry of verify_batch under the deterministic
//                               rule A.3                   (crypto/src/lib.rs:206-219)
//   verify_cached_batch<..>   = the same two predicates against a committee key cache
//   sign_one                  = Keypair::generate + sign   (crypto/src/lib.rs:163-191)
#pragma once
#include "fe25519.hpp"
#include "fe_inv_vt.hpp"
#include "ge25519.hpp"
#include "sc25519.hpp"
#include "sha512.hpp"

namespace nt {

// a[j] for a loop index j without indexing a per-lane array dynamically (which
// would put the array in scratch memory): N-way select
template <int N, class T>
NT_HD NT_INLINE T pick(const T* a, int j) {
  T r = a[0];
#pragma unroll
  for (int q = 1; q < N; ++q)
    if (q == j) r = a[q];
  return r;
}

// 8 little-endian words from a 16-byte aligned pointer
NT_HD NT_INLINE void ld8(uint32_t w[8], const uint32_t* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4* q = (const uint4*)p;
  const uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
#else
  for (int i = 0; i < 8; ++i) w[i] = p[i];
#endif
}

// ---------------------------------------------------------------------------
// Wide combs: for a fixed point P and digit width W, entry (i, j) =
// j * 2^(W i) * P as affine niels, i in [0, pos), j in [0, 2^(W-1)].  [x]P is
// then `pos` mixed additions and no doublings (signed radix-2^W digits of x).
//   W = 24: 11 additions, 11.8 GB per point (the base point, one per device)
//   W = 20: 13 additions, 872 MB per point  (committee keys while they fit:
//           100 keys = 87 GB of the MI355X's 288 GB of HBM3E)
//   W = 16: 16 additions,  67 MB per point  (committee keys otherwise)
// Layout [pos][entry][kWStride words]; a table access type carries its W as
// `kBits` (WideComb<W> on the device, HostWComb<W> in the host harness).
// ---------------------------------------------------------------------------
constexpr int kWStride = 32;  // words per entry (30 used)
constexpr int kWChunk = 64;   // consecutive entries built by one thread
// (the widths of the comb of B, kBCombBits / kBCombFallback: nt_common.hpp)

template <int W>
struct CombGeom {
  static_assert(W >= 12 && W <= 26, "comb digit width");
  // Reduced-scalar combs (W == kKeyCombReduced, committee keys only): the
  // scalar is k or k - L, whichever is smaller in magnitude (|k'| <= (L - 1) / 2
  // < 2^251 + 2^124), so ceil(252 / W) digits; the top digit is taken unsigned
  // (it can reach 2^(W-1) + 1: one more chunk of 64 entries per position), and
  // the point's [L]P (the torsion part of [k - L]P's error: identity for a
  // torsion-free point) follows the positions as one niels entry.
  static constexpr bool kReduced = W == kKeyCombReduced;
  static constexpr int kPos = kReduced ? (252 + W - 1) / W : (254 + W - 1) / W;  // signed digits of the scalar
  static constexpr int kChunks = (1 << (W - 1)) / kWChunk + (kReduced ? 1 : 0);  // chunks per position: entries 1..
  static constexpr int kEntries = kChunks * kWChunk + 1;                         // |digit| in 0..2^(W-1) (+ 64)
  static constexpr size_t kCorrWord = (size_t)kPos * kEntries * kWStride;        // the [L]P entry (reduced)
  static constexpr size_t kWordsPerPoint = kCorrWord + (kReduced ? kWStride : 0);
  // the top digit of any x < 2^253 (every scalar of a passing check) never goes
  // negative, so no carry is lost: the bits above (kPos-1) W plus a carry are <= 2^(W-1)
  static_assert(kReduced || 253 - (kPos - 1) * W <= W - 1, "top comb digit must absorb the carry");
  // reduced: the top digit (bits (kPos-1) W .. 251 plus a carry) is at most 2^(W-1) + 1
  static_assert(!kReduced || (252 - (kPos - 1) * W == W && kChunks * kWChunk >= (1 << (W - 1)) + 1),
                "reduced comb: the unsigned top digit needs its extra chunk");
};

// Next signed radix-2^W digit of the scalar held in d (d >>= W), in
// [-2^(W-1)+1, 2^(W-1)] for ANY 256-bit input (an unchecked s >= L only yields
// a wrong point, never an out-of-range table index; its verdict is reject).
// top_unsigned: the top digit of a reduced-scalar comb, taken as is (no carry out).
template <int W>
NT_HD NT_INLINE int32_t wcomb_digit(uint32_t d[8], uint32_t& carry, bool top_unsigned = false) {
  const uint32_t raw = (d[0] & ((1u << W) - 1u)) + carry;
  carry = raw > (1u << (W - 1)) && !top_unsigned ? 1u : 0u;
#pragma unroll
  for (int m = 0; m < 7; ++m) d[m] = (d[m] >> W) | (d[m + 1] << (32 - W));
  d[7] >>= W;
  return (int32_t)raw - (int32_t)(carry << W);
}

// acc += [x]P with P's wide comb (kFromIdentity: acc = [x]P, the first entry
// taken as the starting point instead of added to the identity).  The table
// load of digit i+1 is issued right after the multiplies that consume entry i,
// so its latency (a random 128-B line) overlaps the rest of the addition.
#ifndef NT_COMB_FROM_ID
#define NT_COMB_FROM_ID 1
#endif
template <class WComb, bool kFromIdentity = false, int kSkipTop = 0>
NT_HD NT_INLINE void wcomb_acc(ge_p3& acc, const uint32_t x[8], const WComb& wc, uint32_t neg_all = 0) {
  // kSkipTop > 0: timing-only experiment builds (wrong results) that drop top positions
  // neg_all: acc += [-x]P (a reduced-scalar comb's k - L < 0): every digit's sign flipped
  constexpr int W = WComb::kBits, P = CombGeom<W>::kPos - kSkipTop;
  constexpr bool kRed = CombGeom<W>::kReduced;
  uint32_t d[8], carry = 0;
#pragma unroll
  for (int m = 0; m < 8; ++m) d[m] = x[m];
  int32_t dg = wcomb_digit<W>(d, carry);
  ge_niels ne;
  wc.load(0, (uint32_t)(dg < 0 ? -dg : dg), ne);
  int pos0 = 0;
  if (kFromIdentity && NT_COMB_FROM_ID) {
    ge_niels_cneg(ne, (dg < 0) ^ (neg_all != 0));
    ge_p3_from_niels(acc, ne);
    dg = wcomb_digit<W>(d, carry, kRed && P == 2);
    wc.load(1, (uint32_t)(dg < 0 ? -dg : dg), ne);
    pos0 = 1;
  } else if (kFromIdentity) {
    ge_p3_0(acc);  // -DNT_COMB_FROM_ID=0 (A/B builds): add the first entry to the identity
  }
#pragma unroll 1
  for (int pos = pos0; pos < P; ++pos) {
    ge_niels_cneg(ne, (dg < 0) ^ (neg_all != 0));
    fe PP, MM, TT;
    ge_add_niels_1(PP, MM, TT, acc, ne);
    // past the last position: a harmless in-range digit
    const int32_t dn = wcomb_digit<W>(d, carry, kRed && pos + 2 == P);
    const int nxt = pos + 1 < P ? pos + 1 : pos;   // last round reloads a valid entry
    wc.load(nxt, (uint32_t)(dn < 0 ? -dn : dn), ne);
    dg = dn;
    ge_cp t;
    ge_add_niels_2(t, PP, MM, TT, acc.Z);
    ge_cp_to_p3(acc, t);
  }
}

// [L]P as an affine niels entry (the reduced-scalar comb's correction), and
// whether P has a torsion component ([L]P != identity).  253 doublings and the
// additions of L's set bits, once per committee key.
NT_HD NT_INLINE uint32_t wcomb_corr(ge_niels& q, const ge_p3& P) {
  ge_cached Pc;
  ge_p3_to_cached(Pc, P);
  ge_p3 Q;
  ge_p3_0(Q);
  ge_cp t;
#pragma unroll 1
  for (int bit = 252; bit >= 0; --bit) {
    ge_p2 q2;
    ge_p3_to_p2(q2, Q);
    ge_dbl(t, q2);
    ge_cp_to_p3(Q, t);
    if ((kScL[bit >> 5] >> (bit & 31)) & 1u) {
      ge_add_cached(t, Q, Pc);
      ge_cp_to_p3(Q, t);
    }
  }
  fe zi;
  fe_invert(zi, Q.Z);
  ge_niels_from(q, Q.X, Q.Y, zi);
  // identity <=> X == 0 and Y == Z
  return (fe_iszero(Q.X) & fe_eq(Q.Y, Q.Z)) ^ 1u;
}

// k (< L) -> its magnitude when k - L is the smaller one: returns 1 and sets
// k = L - k iff k > (L - 1) / 2, so |k'| <= (L - 1) / 2 (reduced-scalar combs)
NT_HD NT_INLINE uint32_t sc_reduce_half(uint32_t k[8]) {
  uint32_t t[8];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {  // t = L - k
    const uint64_t v = (uint64_t)kScL[i] - k[i] - br;
    t[i] = (uint32_t)v;
    br = (v >> 63) & 1u;
  }
  // L - k < k  <=>  k > L / 2
  uint32_t lt = 0, eq = 1;
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    lt |= eq & (t[i] < k[i] ? 1u : 0u);
    eq &= t[i] == k[i] ? 1u : 0u;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) k[i] = lt ? t[i] : k[i];
  return lt;
}

// Wide-comb construction, step 1 (one thread per point): P_i = 2^(W i) P,
// stored as p3 limbs [i][X,Y,Z,T][10].
template <int W>
NT_HD NT_INLINE void wcomb_bases(uint32_t* out, const ge_p3& P0) {
  ge_p3 P = P0;
#pragma unroll 1
  for (int i = 0; i < CombGeom<W>::kPos; ++i) {
    uint32_t* o = out + 40 * i;
#pragma unroll
    for (int l = 0; l < 10; ++l) {
      o[l] = P.X.v[l]; o[10 + l] = P.Y.v[l]; o[20 + l] = P.Z.v[l]; o[30 + l] = P.T.v[l];
    }
    ge_p2 q;
    ge_p3_to_p2(q, P);
#pragma unroll 1
    for (int r = 0; r < W - 1; ++r) ge_dbl_p2(q, q);
    ge_cp t;
    ge_dbl(t, q);
    ge_cp_to_p3(P, t);
  }
}

// Step 2 (one thread per (position, chunk)): entries j0 .. j0+63 of position i
// with j0 = 1 + 64 c, written to dst (entry j0 first, kWStride words each);
// chunk 0 also writes entry 0 (identity) at dst - kWStride.  One inversion per
// chunk (Montgomery's trick); tmp holds the 64 prefix products (640 words).
template <int W>
NT_HD NT_INLINE void wcomb_fill(uint32_t* dst, uint32_t* tmp, const uint32_t* base, uint32_t c) {
  ge_p3 P;
#pragma unroll
  for (int l = 0; l < 10; ++l) {
    P.X.v[l] = base[l]; P.Y.v[l] = base[10 + l]; P.Z.v[l] = base[20 + l]; P.T.v[l] = base[30 + l];
  }
  ge_cached Pc;
  ge_p3_to_cached(Pc, P);
  // Q = j0 * P by double-and-add over the W bits of j0
  const uint32_t j0 = 1u + (uint32_t)kWChunk * c;
  ge_p3 Q;
  ge_p3_0(Q);
  ge_cp t;
#pragma unroll 1
  for (int bit = W - 1; bit >= 0; --bit) {
    ge_p2 q2;
    ge_p3_to_p2(q2, Q);
    ge_dbl(t, q2);
    ge_cp_to_p3(Q, t);
    if ((j0 >> bit) & 1u) {
      ge_add_cached(t, Q, Pc);
      ge_cp_to_p3(Q, t);
    }
  }
  // forward: projective X,Y,Z into the entry slots, prefix products of Z in tmp
  fe acc;
#pragma unroll 1
  for (int e = 0; e < kWChunk; ++e) {
    uint32_t* o = dst + (size_t)e * kWStride;
#pragma unroll
    for (int l = 0; l < 10; ++l) { o[l] = Q.X.v[l]; o[10 + l] = Q.Y.v[l]; o[20 + l] = Q.Z.v[l]; }
    if (e == 0) acc = Q.Z;
    else fe_mul(acc, acc, Q.Z);
#pragma unroll
    for (int l = 0; l < 10; ++l) tmp[10 * e + l] = acc.v[l];
    ge_add_cached(t, Q, Pc);
    ge_cp_to_p3(Q, t);
  }
  fe inv;
  fe_invert(inv, acc);
  // backward: Z_e^-1 = inv * prefix_{e-1}; inv *= Z_e
#pragma unroll 1
  for (int e = kWChunk - 1; e >= 0; --e) {
    uint32_t* o = dst + (size_t)e * kWStride;
    fe X, Y, Z, zi;
#pragma unroll
    for (int l = 0; l < 10; ++l) { X.v[l] = o[l]; Y.v[l] = o[10 + l]; Z.v[l] = o[20 + l]; }
    if (e > 0) {
      fe pre;
#pragma unroll
      for (int l = 0; l < 10; ++l) pre.v[l] = tmp[10 * (e - 1) + l];
      fe_mul(zi, inv, pre);
      fe_mul(inv, inv, Z);
    } else {
      zi = inv;
    }
    ge_niels q;
    ge_niels_from(q, X, Y, zi);
#pragma unroll
    for (int l = 0; l < 10; ++l) { o[l] = q.ypx.v[l]; o[10 + l] = q.ymx.v[l]; o[20 + l] = q.xy2d.v[l]; }
    o[30] = 0;
    o[31] = 0;
  }
  if (c == 0) {
    uint32_t* o = dst - kWStride;
    ge_niels z;
    ge_niels_0(z);
#pragma unroll
    for (int l = 0; l < 10; ++l) { o[l] = z.ypx.v[l]; o[10 + l] = z.ymx.v[l]; o[20 + l] = z.xy2d.v[l]; }
    o[30] = 0;
    o[31] = 0;
  }
}

// ---------------------------------------------------------------------------
// Variable-base part: [u](+-A) + [v](-R) with joint 4-bit signed windows
// over two per-lane tables (entries 0..8: j*(+-A), 9..17: j*(-R))
// ---------------------------------------------------------------------------
constexpr uint32_t kTabR = 9;  // first entry of the R table

// store j * (neg ? -P : P), j = 0..8, at entries e0 .. e0+8
#ifndef NT_TAB_DBL
#define NT_TAB_DBL 1
#endif
template <class ATab>
NT_HD NT_INLINE void ptab_build(const ge_p3& P, uint32_t neg, ATab& at, uint32_t e0) {
  ge_p3 Q;
  fe n;
  fe_neg(n, P.X);
  fe_carry(n);
  fe_cmov(n, P.X, neg ^ 1u);
  Q.X = n;
  fe_neg(n, P.T);
  fe_carry(n);
  fe_cmov(n, P.T, neg ^ 1u);
  Q.T = n;
  Q.Y = P.Y;
  Q.Z = P.Z;
  ge_cached c0, c1;
  ge_cached_0(c0);
  at.store(e0, c0);
  ge_p3_to_cached(c1, Q);
  at.store(e0 + 1, c1);
#if NT_TAB_DBL
  // 2Q, 4Q, 8Q by doubling (4S + 4M each instead of an 8M addition); right after
  // each, its odd neighbour from the point still in registers: 3Q = 2Q + Q,
  // 5Q = 4Q + Q, 7Q = 8Q - Q, and finally 6Q = 7Q - Q (no table reloads:
  // a store followed by a load of the same entry is a full memory round trip)
  {
    ge_cached cn = c1;
    ge_cached_cneg(cn, 1u);  // -Q
    ge_p3 cur = Q, nb;
#pragma unroll 1
    for (uint32_t j = 2; j <= 8; j <<= 1) {
      ge_p2 q;
      ge_p3_to_p2(q, cur);
      ge_cp t;
      ge_dbl(t, q);
      ge_cp_to_p3(cur, t);
      ge_cached c;
      ge_p3_to_cached(c, cur);
      at.store(e0 + j, c);
      ge_add_cached(t, cur, j == 8 ? cn : c1);
      ge_cp_to_p3(nb, t);
      ge_p3_to_cached(c, nb);
      at.store(e0 + (j == 8 ? 7u : j + 1u), c);
    }
    ge_cp t;
    ge_add_cached(t, nb, cn);  // 7Q - Q
    ge_cp_to_p3(nb, t);
    ge_cached c;
    ge_p3_to_cached(c, nb);
    at.store(e0 + 6, c);
  }
#else
  ge_p3 cur = Q;
#pragma unroll 1
  for (uint32_t j = 2; j < 9; ++j) {
    ge_cp t;
    ge_add_cached(t, cur, c1);
    ge_cp_to_p3(cur, t);
    ge_cached cj;
    ge_p3_to_cached(cj, cur);
    at.store(e0 + j, cj);
  }
#endif
}

// any lane of the wave (the host: this lane)
NT_HD NT_INLINE bool wave_any(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(x != 0) != 0;
#else
  return x != 0;
#endif
}

// wave-uniform maximum: every lane of a wave then runs the same window count
NT_HD NT_INLINE int wave_max(int x) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int y = __shfl_xor(x, o);
    x = x > y ? x : y;
  }
  return __builtin_amdgcn_readfirstlane(x);
#else
  return x;
#endif
}

// signed 4-bit digit wi of a sc_recode_w4 string (wi wave-uniform)
NT_HD NT_INLINE int32_t w4_digit(const uint32_t d[8], int wi) {
  return (int32_t)(((pick<8>(d, wi >> 3) >> (4 * (wi & 7))) & 15u) ^ 8u) - 8;
}

// acc (completed -> p3) + table entry e0 + |d| with the sign of d
// (ATab::load_signed: the entry of |d|, negated when d < 0)
template <class ATab>
NT_HD NT_INLINE void ladder_add(ge_cp& t, int32_t d, uint32_t e0, const ATab& at) {
  ge_cached ce;
  at.load_signed(e0, d, ce);  // latency overlaps the conversion
  ge_p3 u;
  ge_cp_to_p3(u, t);
  ge_add_cached(t, u, ce);
}

// t = [u](+-A) + [v](-R) (completed) for W-window digit strings ud, vd:
// 4(W-1) doublings and 2W - 1 additions.  The top A digit seeds the accumulator.
template <class ATab>
NT_HD NT_INLINE void ladder_ar(ge_cp& t, const uint32_t ud[8], const uint32_t vd[8], int W, const ATab& at) {
  {
    const int32_t d = w4_digit(ud, W - 1);
    ge_cached ce;
    at.load_signed(0, d, ce);
    // cached (Y+X, Y-X, 2Z, .) -> (2X : 2Y : 2Z) as a completed point with T = Z
    // (cached sums are not carried: subtract with 4p)
    fe_sub4(t.X, ce.YpX, ce.YmX);
    fe_carry(t.X);
    fe_add(t.Y, ce.YpX, ce.YmX);
    fe_carry(t.Y);
    t.Z = ce.Z2;
    t.T = ce.Z2;
    ladder_add(t, w4_digit(vd, W - 1), kTabR, at);
  }
#pragma unroll 1
  for (int wi = W - 2; wi >= 0; --wi) {
    ge_p2 acc;
    ge_cp_to_p2(acc, t);
#pragma unroll 1
    for (int r = 0; r < 3; ++r) ge_dbl_p2(acc, acc);
    ge_dbl(t, acc);
    ladder_add(t, w4_digit(ud, wi), 0, at);
    ladder_add(t, w4_digit(vd, wi), kTabR, at);
  }
}

// k = SHA-512(R || A || M) mod L over the raw encodings (Scalar::from_hash).
// kDigestFast: a 32-byte M (what every certificate, header and vote signs)
// hashes as one block built from registers (sha512_96) -- the key-cache
// kernels; the general verify kernel keeps one code path (config 2 signs 512-B
// messages, and its register budget is tight).
template <bool kDigestFast = false>
NT_HD NT_INLINE void hram_scalar(uint32_t k[8], const uint32_t Rw[8], const uint32_t Aw[8], const uint8_t* msg,
                                 uint64_t len) {
  uint32_t prefix[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) { prefix[q] = Rw[q]; prefix[8 + q] = Aw[q]; }
  uint64_t st[8];
  if (kDigestFast && len == 32) {
    uint32_t m[8];
    load_words<8>(m, msg);
    sha512_96(st, prefix, m);
  } else {
    sha512_prefixed<16>(st, prefix, msg, len);
  }
  uint32_t hw[16];
  sha512_out_words(hw, st, 16);
  sc_reduce512(k, hw);
}

// ---------------------------------------------------------------------------
// Final comparison without decompressing R (key-cache path).  For R' = [s]B - [k]A with affine
// (x', y'):
//   dalek accepts  <=>  R decodes to a point equal to R'
//                  <=>  y_R == y' (mod p)  and  (sign(R) == parity(x')  or  x' == 0)
// (R's y is taken mod p exactly as curve25519-dalek's from_bytes does; a valid
// R' makes R decodable whenever y matches; x' = 0 covers the accepted
// "negative zero" encodings).  In strict mode the small-order test of R is done
// on R' (equal points have equal order; if they differ the verdict is reject
// anyway).  verify_cached_batch gets the N Z^-1 of a lane from one inversion
// (Montgomery's trick).
// ---------------------------------------------------------------------------
// a = canonical words of y'
NT_HD NT_INLINE uint32_t enc_matches(const fe& x, const uint32_t a[8], const uint32_t Rw[8]) {
  fe yr;
  fe_frombytes_w(yr, Rw);  // bit 255 dropped, value taken mod p by the compare
  uint32_t b[8], xw[8];
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

// The check for a given lattice vector (u = (-1)^uneg |u|, v) of k with
// max(bitlen |u|, bitlen v) <= bits; any valid vector gives the same verdict
// (verify_one below uses sc_halfsize's; the tests also run the trivial (k, 1)).
template <int MODE, class ATab, class WComb>
NT_HD NT_INLINE uint32_t verify_uv(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                                   const uint32_t u[8], uint32_t uneg, const uint32_t v[8], int bits, ATab& at,
                                   const WComb& wb) {
  uint32_t ok = sc_is_canonical(Sw);
  {
    ge_p3 A;
    ok &= ge_frombytes_w(A, Aw);
    if (MODE == kStrict) ok &= ge_is_small_order_affine(A) ^ 1u;
    ptab_build(A, uneg ^ 1u, at, 0);  // -[u]A = [|u|](u < 0 ? A : -A)
  }
  {
    ge_p3 R;
    ok &= ge_frombytes_w(R, Rw);
    if (MODE == kStrict) ok &= ge_is_small_order_affine(R) ^ 1u;
    ptab_build(R, 1u, at, kTabR);
  }
  uint32_t w[8], ud[8], vd[8];
  sc_mul(w, v, Sw);
  sc_recode_w4(ud, u);
  sc_recode_w4(vd, v);
  const int W = wave_max((bits + 5) >> 2);  // 4W >= bits + 2: the signed top digit absorbs the carry
  ge_cp t;
  ladder_ar(t, ud, vd, W, at);
  ge_p3 acc;
  ge_cp_to_p3(acc, t);
  wcomb_acc(acc, w, wb);
  return ok & fe_iszero(acc.X) & fe_eq(acc.Y, acc.Z);
}

// One verification (A, R, s encodings as words), half-size scalars:
//   ok  <=>  s < L, A and R decode, (strict) neither is small order, and
//            [v s mod L]B - [u]A - [v]R == identity     (= [v]([s]B - [k]A - R))
// with (u, v) = sc_halfsize(k), k = SHA-512(R || A || M) mod L.  at holds this
// lane's tables, wb is the wide comb of B.
template <int MODE, class ATab, class WComb>
NT_HD NT_INLINE uint32_t verify_one(const uint32_t Aw[8], const uint32_t Rw[8], const uint32_t Sw[8],
                                    const uint8_t* msg, uint64_t len, ATab& at, const WComb& wb) {
  uint32_t u[8], v[8], uneg;
  int bits;
  {
    uint32_t k[8];
    hram_scalar(k, Rw, Aw, msg, len);
    bits = sc_halfsize(u, uneg, v, k);
  }
  return verify_uv<MODE>(Aw, Rw, Sw, u, uneg, v, bits, at, wb);
}

// N verifications per lane in turn.  A[j] = 8 pk words, sig[j] = 16 words
// (R || s), msg[j]/len[j] = message; at is this lane's table storage.
template <int MODE, int N, class ATab, class WComb>
NT_HD NT_INLINE void verify_n(uint32_t ok[N], const uint32_t* const A[N], const uint32_t* const sig[N],
                              const uint8_t* const msg[N], const uint64_t len[N], ATab& at, const WComb& wb) {
#pragma unroll 1
  for (int j = 0; j < N; ++j) {
    const uint32_t* sj = pick<N>(sig, j);
    uint32_t Aw[8], Rw[8], Sw[8];
    ld8(Aw, pick<N>(A, j));
    ld8(Rw, sj);
    ld8(Sw, sj + 8);
    const uint32_t okj = verify_one<MODE>(Aw, Rw, Sw, pick<N>(msg, j), pick<N>(len, j), at, wb);
#pragma unroll
    for (int q = 0; q < N; ++q)
      if (q == j) ok[q] = okj;
  }
}

// Key-cache variant.  meta = the key's kKey* bits.
// kKeyTorsion: the key has a torsion component ([L]A != identity; reduced-scalar combs add the
// key's [L](-A) entry when they use k - L)
enum : uint32_t { kKeyDecodes = 1u, kKeySmallOrder = 2u, kKeyTorsion = 4u };
// set by the kMixed loader in the meta it hands over: this signature is checked strictly
constexpr uint32_t kKeyWantStrict = 0x80000000u;
// strictness of one signature: the mode, or in kMixed mode the loader's per-signature bit
template <int MODE>
NT_HD NT_INLINE bool is_strict(uint32_t meta) {
  return MODE == kStrict || (MODE == kMixed && (meta & kKeyWantStrict));
}

// One cached verification up to R' = [s]B - [k]A (extended), no decompression
// of A and no doublings: 16 + 16 wide-comb additions.  Returns the s / key flags.
template <int MODE, class WCombA, class WCombB>
NT_HD NT_INLINE uint32_t cached_point(ge_p3& acc, uint32_t meta, const uint32_t Aw[8], const uint32_t Rw[8],
                                      const uint32_t Sw[8], const uint8_t* msg, uint64_t len, const WCombA& ca,
                                      const WCombB& cb) {
  uint32_t okj = sc_is_canonical(Sw) & (meta & kKeyDecodes ? 1u : 0u);
  if (is_strict<MODE>(meta)) okj &= (meta & kKeySmallOrder) ? 0u : 1u;
  uint32_t k[8];
  hram_scalar<true>(k, Rw, Aw, msg, len);
#ifdef NT_EXPERIMENT_KEY_SKIP
  wcomb_acc<WCombA, true, NT_EXPERIMENT_KEY_SKIP>(acc, k, ca);  // timing only: wrong verdicts
#else
  if (CombGeom<WCombA::kBits>::kReduced) {
    // [k](-A) = [k - L](-A) + [L](-A): one position fewer; the second term is
    // the identity unless A has a torsion component
    const uint32_t kneg = sc_reduce_half(k);
    wcomb_acc<WCombA, true>(acc, k, ca, kneg);
    const uint32_t corr = kneg & ((meta & kKeyTorsion) ? 1u : 0u);
    if (wave_any(corr)) {
      ge_niels c;
      ca.load_corr(c);
      if (!corr) ge_niels_0(c);
      fe PP, MM, TT;
      ge_add_niels_1(PP, MM, TT, acc, c);
      ge_cp t;
      ge_add_niels_2(t, PP, MM, TT, acc.Z);
      ge_cp_to_p3(acc, t);
    }
  } else {
    wcomb_acc<WCombA, true>(acc, k, ca);
  }
#endif
  wcomb_acc(acc, Sw, cb);
  return okj;
}

// Compare of one projective R' with the encoding Rw given zi = Z^-1 (see
// finish_compare); strict mode adds the small-order test on R'.
template <int MODE>
NT_HD NT_INLINE uint32_t compare_one(const ge_p2& P, const fe& zi, const uint32_t Rw[8], bool strict) {
  fe x, y;
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  uint32_t yw[8];
  fe_tobytes_w(yw, y);
  uint32_t r = enc_matches(x, yw, Rw);
  if (strict) r &= torsion_y_words(yw) ^ 1u;  // R' on the curve: small order <=> torsion y
  return r;
}

// The inversion of a key-cache batch (verification is public data): the
// variable-time binary GCD (fe_inv_vt.hpp) unless -DNT_INV_VT=0 (the Fermat
// chain, 254 squarings + 11 multiplies).
#ifndef NT_INV_VT
#define NT_INV_VT 1
#endif
NT_HD NT_INLINE void fe_invert_batch(fe& out, const fe& z) {
#if defined(NT_EXPERIMENT_NO_INV)
  out = z;  // timing only (wrong verdicts): what the batch inversion costs a launch
#elif NT_INV_VT
  fe_invert_vt(out, z);
#else
  fe_invert(out, z);
#endif
}

// N cached verifications per lane with ONE inversion (Montgomery's trick).
//   ld.get(j, meta, Aw, Rw, Sw, msg, len, ca)   inputs of signature j
//   st.put(j, P, prefix) / st.get_point(j, P) /  per-lane stash of R'_j and the
//   st.get_prefix(j, prefix)                     running product Z_0 .. Z_j
// Returns bit j = verdict of signature j (m <= 64).  The stash keeps the registers of a
// lane independent of N (the kernel's stash lives in global memory); m <= N
// signatures are run (the kernel's run-time per-lane count).
template <int MODE, int N, class Loader, class WCombB, class Stash>
NT_HD NT_INLINE uint64_t verify_cached_batch(const Loader& ld, const WCombB& cb, Stash& st, int m = N) {
  static_assert(N >= 1 && N <= 64, "verdict bits of a lane are one 64-bit word");
  uint64_t okbits = 0, strictbits = 0;
  fe acc;
#pragma unroll 1
  for (int j = 0; j < m; ++j) {
    uint32_t meta, Aw[8], Rw[8], Sw[8];
    const uint8_t* msg;
    uint64_t len;
    typename Loader::Comb ca;
    ld.get(j, meta, Aw, Rw, Sw, msg, len, ca);
    ge_p3 P;
    okbits |= (uint64_t)cached_point<MODE>(P, meta, Aw, Rw, Sw, msg, len, ca, cb) << j;
    strictbits |= (uint64_t)(is_strict<MODE>(meta) ? 1u : 0u) << j;
    if (j == 0) acc = P.Z;
    else fe_mul(acc, acc, P.Z);
    ge_p2 P2;
    ge_p3_to_p2(P2, P);
    st.put(j, P2, acc);
  }
  fe inv;
  fe_invert_batch(inv, acc);
#pragma unroll 1
  for (int j = m - 1; j >= 0; --j) {
    ge_p2 P;
    fe zi;
    st.get_point(j, P);
    if (j > 0) {
      fe pre;
      st.get_prefix(j - 1, pre);  // Z_0 .. Z_{j-1}
      fe_mul(zi, inv, pre);
      fe_mul(inv, inv, P.Z);
    } else {
      zi = inv;
    }
    uint32_t Rw[8];
    ld.rbytes(j, Rw);
    okbits &= ~((uint64_t)(compare_one<MODE>(P, zi, Rw, (strictbits >> j) & 1u) ^ 1u) << j);
  }
  return okbits;
}

// Keygen + RFC 8032 signature.  sw = 32-byte seed words; wb = wide comb of B.
template <class WComb>
NT_HD NT_INLINE void sign_one(uint32_t Aw[8], uint32_t Rw[8], uint32_t s[8], const uint32_t sw[8],
                              const uint8_t* msg, uint64_t len, const WComb& wb) {
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
  ge_p3 P;
  ge_p2 P2;
  wcomb_acc<WComb, true>(P, ared, wb);
  ge_p3_to_p2(P2, P);
  ge_tobytes_w(Aw, P2);

  sha512_prefixed<8>(st, pre, msg, len);
  uint32_t hr[16], r[8];
  sha512_out_words(hr, st, 16);
  sc_reduce512(r, hr);
  wcomb_acc<WComb, true>(P, r, wb);
  ge_p3_to_p2(P2, P);
  ge_tobytes_w(Rw, P2);

  uint32_t k[8];
  hram_scalar(k, Rw, Aw, msg, len);
  sc_muladd(s, k, a, r);
}

}  // namespace nt
