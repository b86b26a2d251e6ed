// nt_host_harness.cpp -- TEST INFRASTRUCTURE: the exact device arithmetic of
// narwhal-tusk_amd/csrc/*.hpp compiled for the host (g++, NT_HD empty) so that
// CPU-only tests can (a) stress the radix-2^25.5 bound discipline with
// adversarial limb values against Python big integers, (b) replay the golden
// corpus through the same verify_n<> / verify_cached_n<> the kernels run,
// (c) check the wide-comb construction (wcomb_bases/wcomb_fill) against an
// independent curve model, and (d) count field multiplies per operation
// (profiles/opcount.json, the roofline numerator).
// Never linked into libntcrypto.so.
#define NT_OPCOUNT 1
#include <cstring>
#include <unordered_map>

#include "../../narwhal-tusk_amd/csrc/ed25519_ops.hpp"
#include "../../narwhal-tusk_amd/csrc/fe_inv_vt.hpp"
#include "../../narwhal-tusk_amd/csrc/ks_plan.hpp"
#include "../../narwhal-tusk_amd/csrc/pipe_plan.hpp"
#include "../../narwhal-tusk_amd/csrc/key_table.hpp"
#include "../../narwhal-tusk_amd/csrc/small_model.hpp"

namespace nt {
unsigned long long g_fe_mul = 0, g_fe_sq = 0;
}

using namespace nt;

namespace {
struct HostATab {
  ge_cached e[18];
  void store(uint32_t j, const ge_cached& c) { e[j] = c; }
  void load(uint32_t j, ge_cached& c) const { c = e[j]; }
  void load_signed(uint32_t e0, int32_t d, ge_cached& c) const {
    c = e[e0 + (uint32_t)(d < 0 ? -d : d)];
    ge_cached_cneg(c, d < 0);
  }
};

// Wide comb of a point with entries computed on demand (and memoized) by
// plain double-and-add; table construction is not counted by NT_OPCOUNT.
template <int W>
struct HostWComb {
  static constexpr int kBits = W;
  ge_p3 base[CombGeom<W>::kPos];
  ge_niels corr;       // [L]P (reduced-scalar combs)
  uint32_t torsion = 0;
  mutable std::unordered_map<uint64_t, ge_niels> memo;
  void load_corr(ge_niels& q) const { q = corr; }
  void init(const ge_p3& P) {
    const unsigned long long m0 = g_fe_mul, s0 = g_fe_sq;
    torsion = CombGeom<W>::kReduced ? wcomb_corr(corr, P) : 0u;
    uint32_t w[CombGeom<W>::kPos * 40];
    wcomb_bases<W>(w, P);
    for (int i = 0; i < CombGeom<W>::kPos; ++i)
      for (int l = 0; l < 10; ++l) {
        base[i].X.v[l] = w[40 * i + l];
        base[i].Y.v[l] = w[40 * i + 10 + l];
        base[i].Z.v[l] = w[40 * i + 20 + l];
        base[i].T.v[l] = w[40 * i + 30 + l];
      }
    g_fe_mul = m0;
    g_fe_sq = s0;
  }
  void load(uint32_t pos, uint32_t idx, ge_niels& q) const {
    const uint64_t key = ((uint64_t)pos << 32) | idx;
    auto it = memo.find(key);
    if (it != memo.end()) {
      q = it->second;
      return;
    }
    const unsigned long long m0 = g_fe_mul, s0 = g_fe_sq;
    if (idx == 0) {
      ge_niels_0(q);
    } else {
      ge_cached Pc;
      ge_p3_to_cached(Pc, base[pos]);
      ge_p3 Q;
      ge_p3_0(Q);
      ge_cp t;
      for (int bit = W - 1; bit >= 0; --bit) {
        ge_p2 q2;
        ge_p3_to_p2(q2, Q);
        ge_dbl(t, q2);
        ge_cp_to_p3(Q, t);
        if ((idx >> bit) & 1u) {
          ge_add_cached(t, Q, Pc);
          ge_cp_to_p3(Q, t);
        }
      }
      fe zi;
      fe_invert(zi, Q.Z);
      ge_niels_from(q, Q.X, Q.Y, zi);
    }
    g_fe_mul = m0;
    g_fe_sq = s0;
    memo.emplace(key, q);
  }
};

using HostBComb = HostWComb<kBCombBits>;
using HostKeyComb = HostWComb<kKeyCombWide>;        // 13 positions
using HostKeyCombRed = HostWComb<kKeyCombReduced>;  // 12 positions, reduced scalars: the device's first choice

HostBComb& bcomb() {
  static HostBComb* c = [] {
    auto* w = new HostBComb;
    uint32_t enc[8];
    for (int i = 0; i < 8; ++i) enc[i] = kBaseEnc[i];
    ge_p3 B;
    ge_frombytes_w(B, enc);
    w->init(B);
    return w;
  }();
  return *c;
}

// kKey* bits and the comb of -A, as k_wcomb_bases builds them
template <class KC>
uint32_t key_comb(KC& c, const uint32_t Aw[8]) {
  ge_p3 P;
  const uint32_t ok = ge_frombytes_w(P, Aw);
  const uint32_t meta = (ok ? kKeyDecodes : 0u) | (ge_is_small_order(P) ? kKeySmallOrder : 0u);
  if (!ok) ge_p3_0(P);
  fe_neg(P.X, P.X);
  fe_carry(P.X);
  fe_neg(P.T, P.T);
  fe_carry(P.T);
  c.init(P);
  return meta | (c.torsion ? kKeyTorsion : 0u);
}

void words(uint32_t w[8], const uint8_t* b) { std::memcpy(w, b, 32); }
}  // namespace

extern "C" {

void nth_fe_mul(const uint32_t* f, const uint32_t* g, uint32_t* out) {
  fe a, b, c;
  std::memcpy(a.v, f, 40);
  std::memcpy(b.v, g, 40);
  fe_mul(c, a, b);
  std::memcpy(out, c.v, 40);
}
void nth_fe_sq(const uint32_t* f, uint32_t* out) {
  fe a, c;
  std::memcpy(a.v, f, 40);
  fe_sq(c, a);
  std::memcpy(out, c.v, 40);
}
void nth_fe_sq_wide(const uint32_t* f, uint32_t* out) {
  fe a, c;
  std::memcpy(a.v, f, 40);
  fe_sq_wide(c, a);
  std::memcpy(out, c.v, 40);
}
void nth_fe_carry(const uint32_t* f, uint32_t* out) {
  fe a;
  std::memcpy(a.v, f, 40);
  fe_carry(a);
  std::memcpy(out, a.v, 40);
}
void nth_fe_tobytes(const uint32_t* f, uint8_t* out32) {
  fe a;
  std::memcpy(a.v, f, 40);
  uint32_t w[8];
  fe_tobytes_w(w, a);
  std::memcpy(out32, w, 32);
}
void nth_fe_frombytes(const uint8_t* in32, uint32_t* out) {
  uint32_t w[8];
  words(w, in32);
  fe a;
  fe_frombytes_w(a, w);
  std::memcpy(out, a.v, 40);
}
void nth_sc_reduce512(const uint8_t* in64, uint8_t* out32) {
  uint32_t x[16], r[8];
  std::memcpy(x, in64, 64);
  sc_reduce512(r, x);
  std::memcpy(out32, r, 32);
}
void nth_sc_muladd(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* out32) {
  uint32_t wa[8], wb[8], wc[8], r[8];
  words(wa, a);
  words(wb, b);
  words(wc, c);
  sc_muladd(r, wa, wb, wc);
  std::memcpy(out32, r, 32);
}
// sc_halfsize on a 32-byte scalar k: u, v (32 B each), sign of u; returns bits
int nth_sc_halfsize(const uint8_t* k32, uint8_t* u32, uint8_t* v32, int* uneg) {
  uint32_t k[8], u[8], v[8], un;
  words(k, k32);
  const int bits = sc_halfsize(u, un, v, k);
  std::memcpy(u32, u, 32);
  std::memcpy(v32, v, 32);
  *uneg = (int)un;
  return bits;
}
// Batched (Lehmer) vs one-step lattice reduction on n scalars (32 bytes each):
// the number whose (u, v, sign, bits) differ.
int nth_halfsize_disagree(const uint8_t* ks, int n) {
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    uint32_t k[8], u0[8], v0[8], u1[8], v1[8], n0, n1;
    words(k, ks + 32 * (size_t)i);
    const int b0 = sc_halfsize(u0, n0, v0, k);
    const int b1 = sc_halfsize_euclid(u1, n1, v1, k);
    bad += (b0 != b1 || n0 != n1 || std::memcmp(u0, u1, 32) != 0 || std::memcmp(v0, v1, 32) != 0) ? 1 : 0;
  }
  return bad;
}
void nth_sha512(const uint8_t* msg, uint64_t len, uint8_t* out64, int one_site) {
  uint64_t st[8];
  if (one_site) sha512_prefixed_1site<0>(st, nullptr, msg, len);
  else sha512_prefixed<0>(st, nullptr, msg, len);
  uint32_t w[16];
  sha512_out_words(w, st, 16);
  std::memcpy(out64, w, 64);
}
// k = H(R || A || M) mod L through the general and the one-block (32-byte M) paths
void nth_hram(const uint8_t* sig, const uint8_t* pk, const uint8_t* msg, uint64_t len, int fast, uint8_t* out32) {
  alignas(16) uint32_t A[8], S[16], k[8];
  std::memcpy(A, pk, 32);
  std::memcpy(S, sig, 64);
  if (fast) hram_scalar<true>(k, S, A, msg, len);
  else hram_scalar<false>(k, S, A, msg, len);
  std::memcpy(out32, k, 32);
}
int nth_verify(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t len) {
  alignas(16) uint32_t A[8], S[16];
  std::memcpy(A, pk, 32);
  std::memcpy(S, sig, 64);
  const uint32_t* Ap[1] = {A};
  const uint32_t* Sp[1] = {S};
  const uint8_t* Mp[1] = {msg};
  const uint64_t Lp[1] = {len};
  uint32_t ok[1];
  HostATab at;
  if (mode == 0) verify_n<kStrict, 1>(ok, Ap, Sp, Mp, Lp, at, bcomb());
  else verify_n<kCofactorless, 1>(ok, Ap, Sp, Mp, Lp, at, bcomb());
  return (int)ok[0];
}
// The message bound of every kernel that reads caller messages (nt_common.hpp
// msg_slice): out3 = {off, len, ok} as the kernel takes the slice.
void nth_msg_slice(uint64_t off, uint64_t len, uint64_t bytes, uint64_t* out3) {
  const MsgSlice ms = msg_slice(off, len, bytes);
  out3[0] = ms.off;
  out3[1] = ms.len;
  out3[2] = ms.ok;
}
// One item of k_ed25519_verify's body: the slice of a `bytes`-byte message
// buffer, then the verification, the verdict ANDed with the bound (the kernel's
// act & ok).  An out-of-bounds slice is never read: the harness hands the
// arithmetic the clamped (empty) slice, exactly as the kernel does.
int nth_verify_item(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t bytes,
                    uint64_t off, uint64_t len) {
  const MsgSlice ms = msg_slice(off, len, bytes);
  return nth_verify(mode, pk, sig, msg + ms.off, ms.len) & (int)ms.ok;
}
// verify_uv with the trivial lattice vector (u, v) = (k, 1), 253-bit ladder:
// the path sc_halfsize falls back to, checked against the same corpus.
int nth_verify_trivial(int mode, const uint8_t* pk, const uint8_t* sig, const uint8_t* msg, uint64_t len) {
  alignas(16) uint32_t A[8], S[16];
  std::memcpy(A, pk, 32);
  std::memcpy(S, sig, 64);
  uint32_t k[8], v[8] = {1, 0, 0, 0, 0, 0, 0, 0};
  hram_scalar(k, S, A, msg, len);
  HostATab at;
  return (int)(mode == 0 ? verify_uv<kStrict>(A, S, S + 8, k, 0u, v, 253, at, bcomb())
                         : verify_uv<kCofactorless>(A, S, S + 8, k, 0u, v, 253, at, bcomb()));
}
// Two signatures through the two-per-lane path the kernel runs (shared inversion).
void nth_verify_pair(int mode, const uint8_t* pk64, const uint8_t* sig128, const uint8_t* m0, uint64_t l0,
                     const uint8_t* m1, uint64_t l1, int* out2) {
  alignas(16) uint32_t A[2][8], S[2][16];
  std::memcpy(A, pk64, 64);
  std::memcpy(S, sig128, 128);
  const uint32_t* Ap[2] = {A[0], A[1]};
  const uint32_t* Sp[2] = {S[0], S[1]};
  const uint8_t* Mp[2] = {m0, m1};
  const uint64_t Lp[2] = {l0, l1};
  uint32_t ok[2];
  HostATab at;
  if (mode == 0) verify_n<kStrict, 2>(ok, Ap, Sp, Mp, Lp, at, bcomb());
  else verify_n<kCofactorless, 2>(ok, Ap, Sp, Mp, Lp, at, bcomb());
  out2[0] = (int)ok[0];
  out2[1] = (int)ok[1];
}
// The key-cache path (combs of -A_j) for nsig in [1, 8] signatures (the kernel
// runs keyset_per_lane() = 8 per lane) through verify_cached_batch with a host stash.
constexpr int kHostKsMax = 8;
struct HostStash {
  ge_p2 P[kHostKsMax];
  fe pre[kHostKsMax];
  void put(int j, const ge_p2& p, const fe& a) { P[j] = p; pre[j] = a; }
  void get_point(int j, ge_p2& p) const { p = P[j]; }
  void get_prefix(int j, fe& a) const { a = pre[j]; }
};
}  // extern "C" (the key-cache helpers below are templates)
template <class KC>
struct HostCombRef {  // a comb by reference, with the WComb interface
  static constexpr int kBits = KC::kBits;
  const KC* c;
  void load(uint32_t pos, uint32_t idx, ge_niels& q) const { c->load(pos, idx, q); }
  void load_corr(ge_niels& q) const { c->load_corr(q); }
};
template <class KC>
struct HostLoader {
  using Comb = HostCombRef<KC>;
  const uint32_t (*A)[8];
  const uint32_t (*S)[16];
  const uint8_t* const* M;
  const uint64_t* L;
  const uint32_t* meta;
  KC* ca;
  void get(int j, uint32_t& m, uint32_t Aw[8], uint32_t Rw[8], uint32_t Sw[8], const uint8_t*& msg, uint64_t& len,
           Comb& c) const {
    m = meta[j];
    for (int q = 0; q < 8; ++q) { Aw[q] = A[j][q]; Rw[q] = S[j][q]; Sw[q] = S[j][8 + q]; }
    msg = M[j];
    len = L[j];
    c = Comb{&ca[j]};
  }
  void rbytes(int j, uint32_t Rw[8]) const {
    for (int q = 0; q < 8; ++q) Rw[q] = S[j][q];
  }
};
template <class KC>
int verify_cached_impl(int mode, int nsig, const uint8_t* pk, const uint8_t* sig, const uint8_t* const* msgs,
                       const uint64_t* lens, int* out) {
  if (nsig < 1 || nsig > kHostKsMax) return -1;
  alignas(16) uint32_t A[kHostKsMax][8], S[kHostKsMax][16];
  std::memcpy(A, pk, 32 * nsig);
  std::memcpy(S, sig, 64 * nsig);
  static KC ca[kHostKsMax];
  const unsigned long long cm = g_fe_mul, cs = g_fe_sq;  // key-cache build is not per signature
  uint32_t meta[kHostKsMax];
  for (int j = 0; j < nsig; ++j) {
    meta[j] = key_comb(ca[j], A[j]);
    ca[j].memo.clear();
  }
  g_fe_mul = cm;
  g_fe_sq = cs;
  HostLoader<KC> ld{A, S, msgs, lens, meta, ca};
  HostStash st;
  uint64_t bits;
  if ((mode & 0xff) == kMixed) {  // mode = kMixed | strict_mask << 8 (the kernel's key_idx bit 31)
    for (int j = 0; j < nsig; ++j)
      if ((mode >> (8 + j)) & 1) meta[j] |= kKeyWantStrict;
    bits = verify_cached_batch<kMixed, kHostKsMax>(ld, bcomb(), st, nsig);
  } else {
    bits = mode == 0 ? verify_cached_batch<kStrict, kHostKsMax>(ld, bcomb(), st, nsig)
                     : verify_cached_batch<kCofactorless, kHostKsMax>(ld, bcomb(), st, nsig);
  }
  for (int j = 0; j < nsig; ++j) out[j] = (bits >> j) & 1;
  return 0;
}
extern "C" {
int nth_verify_cached_n(int mode, int nsig, const uint8_t* pk, const uint8_t* sig, const uint8_t* const* msgs,
                        const uint64_t* lens, int* out) {
  return verify_cached_impl<HostKeyComb>(mode, nsig, pk, sig, msgs, lens, out);
}
// the same through key combs of `bits`-bit digits (20: 13 positions; 21: reduced scalars, 12 positions)
int nth_verify_cached_nw(int bits, int mode, int nsig, const uint8_t* pk, const uint8_t* sig,
                         const uint8_t* const* msgs, const uint64_t* lens, int* out) {
  if (bits == kKeyCombReduced) return verify_cached_impl<HostKeyCombRed>(mode, nsig, pk, sig, msgs, lens, out);
  if (bits == kKeyCombWide) return verify_cached_impl<HostKeyComb>(mode, nsig, pk, sig, msgs, lens, out);
  return -1;
}
// [k](-A) through the key comb of `bits`-bit digits as the key-cache kernel forms it
// (cached_point: the reduced comb takes k or k - L and adds [L](-A) when it used k - L);
// out = the point's canonical encoding, returns the key's kKey* bits
uint32_t nth_key_comb_sum(int bits, const uint8_t* A32, const uint8_t* k32, uint8_t* out32) {
  uint32_t Aw[8], k[8];
  words(Aw, A32);
  words(k, k32);
  ge_p3 acc;
  uint32_t meta = 0;
  auto finish = [&]() {
    fe zi, x, y;
    fe_invert(zi, acc.Z);
    fe_mul(x, acc.X, zi);
    fe_mul(y, acc.Y, zi);
    uint32_t yw[8], xw[8];
    fe_tobytes_w(yw, y);
    fe_tobytes_w(xw, x);
    yw[7] |= (xw[0] & 1u) << 31;
    std::memcpy(out32, yw, 32);
  };
  if (bits == kKeyCombReduced) {
    static HostKeyCombRed c;
    meta = key_comb(c, Aw);
    c.memo.clear();
    const uint32_t kneg = sc_reduce_half(k);
    wcomb_acc<HostCombRef<HostKeyCombRed>, true>(acc, k, HostCombRef<HostKeyCombRed>{&c}, kneg);
    if (kneg && (meta & kKeyTorsion)) {
      ge_niels q;
      c.load_corr(q);
      ge_cp t;
      ge_add_niels(t, acc, q);
      ge_cp_to_p3(acc, t);
    }
  } else {
    static HostKeyComb c;
    meta = key_comb(c, Aw);
    c.memo.clear();
    wcomb_acc<HostCombRef<HostKeyComb>, true>(acc, k, HostCombRef<HostKeyComb>{&c});
  }
  finish();
  return meta;
}
void nth_verify_cached_pair(int mode, const uint8_t* pk64, const uint8_t* sig128, const uint8_t* m0, uint64_t l0,
                            const uint8_t* m1, uint64_t l1, int* out2) {
  const uint8_t* ms[2] = {m0, m1};
  const uint64_t ls[2] = {l0, l1};
  nth_verify_cached_n(mode, 2, pk64, sig128, ms, ls, out2);
}
void nth_sign(const uint8_t* seed, const uint8_t* msg, uint64_t len, uint8_t* pk, uint8_t* sig) {
  uint32_t sw[8], A[8], R[8], s[8];
  words(sw, seed);
  sign_one(A, R, s, sw, msg, len, bcomb());
  std::memcpy(pk, A, 32);
  std::memcpy(sig, R, 32);
  std::memcpy(sig + 32, s, 32);
}
// The device's wide-comb construction run on the host for one chunk: entries
// j0-1 .. j0+63 (j0 = 1 + 64c; entry j0-1 only written for c = 0) of position
// pos of the comb of P (negate: of -P), as 65 x 32 words.  Returns kKey* bits.
uint32_t nth_wcomb_chunk(int bits, const uint8_t* enc32, int negate, int pos, int c, uint32_t* out) {
  uint32_t w[8];
  words(w, enc32);
  ge_p3 P;
  const uint32_t ok = ge_frombytes_w(P, w);
  const uint32_t meta = (ok ? kKeyDecodes : 0u) | (ge_is_small_order(P) ? kKeySmallOrder : 0u);
  if (!ok) ge_p3_0(P);
  if (negate) {
    fe_neg(P.X, P.X);
    fe_carry(P.X);
    fe_neg(P.T, P.T);
    fe_carry(P.T);
  }
  static uint32_t bases[CombGeom<kKeyCombNarrow>::kPos * 40];
  static uint32_t tmp[kWChunk * 10];
  std::memset(out, 0, 65 * kWStride * 4);
  if (bits == kKeyCombWide) {
    wcomb_bases<kKeyCombWide>(bases, P);
    wcomb_fill<kKeyCombWide>(out + kWStride, tmp, bases + 40 * pos, (uint32_t)c);
  } else if (bits == kKeyCombNarrow) {
    wcomb_bases<kKeyCombNarrow>(bases, P);
    wcomb_fill<kKeyCombNarrow>(out + kWStride, tmp, bases + 40 * pos, (uint32_t)c);
  } else {
    return ~0u;
  }
  return meta;
}
// small-order test of a decodable encoding both ways: [8]P by doublings and
// the torsion-y compare the kernels use; returns decode ok
int nth_small_order(const uint8_t* enc32, int* by_dbl, int* by_y) {
  uint32_t w[8];
  words(w, enc32);
  ge_p3 P;
  const uint32_t ok = ge_frombytes_w(P, w);
  *by_dbl = (int)ge_is_small_order(P);
  *by_y = (int)ge_is_small_order_affine(P);
  return (int)ok;
}
void nth_counts_reset() { bcomb(); g_fe_mul = g_fe_sq = 0; }
unsigned long long nth_count_mul() { return g_fe_mul; }
unsigned long long nth_count_sq() { return g_fe_sq; }
int nth_bcomb_bits() { return kBCombBits; }
// the key-cache launch plan (ks_plan.hpp): out = waves, chunks, base_rows, extra, per_simd, rounds
void nth_ks_plan(unsigned long long n, uint32_t cus, uint32_t cap, int force, uint32_t* out) {
  const KsPlan p = ks_plan(n, cus, cap, force);
  out[0] = p.waves; out[1] = p.chunks; out[2] = p.base_rows; out[3] = p.extra; out[4] = p.per_simd; out[5] = p.rounds;
}
// the stash bound every plan of a launch of <= rows rows fits in (ks_plan.hpp)
unsigned long long nth_ks_stash_rows_bound(unsigned long long rows, uint32_t cus) {
  return ks_stash_rows_bound(rows, cus);
}
// host entry points' chunk plans (pipe_plan.hpp): chunk sizes into out (at most maxn), returns the count
int nth_verify_chunk_targets(unsigned long long total, unsigned long long r1, unsigned long long cap,
                             unsigned long long* out, int maxn) {
  const auto t = verify_chunk_targets(total, r1, cap);
  for (size_t i = 0; i < t.size() && (int)i < maxn; ++i) out[i] = t[i];
  return (int)t.size();
}
int nth_chunk_targets(unsigned long long total, unsigned long long r, unsigned long long cap, int round4,
                      unsigned long long* out, int maxn) {
  const auto t = chunk_targets(total, r, cap, round4 != 0);
  for (size_t i = 0; i < t.size() && (int)i < maxn; ++i) out[i] = t[i];
  return (int)t.size();
}
// certificate-group chunks: groups [0, G) with counts cnt, targets as above; out = chunk ends g1
int nth_plan_group_chunks(unsigned long long G, const uint32_t* cnt, const unsigned long long* targets, int nt,
                          unsigned long long* out, int maxn) {
  const std::vector<uint64_t> tg(targets, targets + nt);
  const auto r = plan_group_chunks(0, G, cnt, tg);
  for (size_t i = 0; i < r.size() && (int)i < maxn; ++i) out[i] = r[i].second;
  return (int)r.size();
}
// streamed rows (ks_stream_plan): out = waves, rows, prow, per_simd
void nth_ks_stream_plan(unsigned long long n, uint32_t cus, uint32_t cap, int force, uint32_t* out) {
  const KsPlan p = ks_stream_plan(n, cus, cap, force);
  out[0] = p.waves; out[1] = p.rows; out[2] = p.prow; out[3] = p.per_simd;
}
// field inversion: Fermat (fe_invert) and the variable-time binary GCD (fe_invert_vt); limbs in, canonical bytes out
void nth_fe_invert(const uint32_t* f, uint8_t* out32, int vt) {
  fe a, r;
  std::memcpy(a.v, f, 40);
  if (vt) fe_invert_vt(r, a);
  else fe_invert(r, a);
  uint32_t w[8];
  fe_tobytes_w(w, r);
  std::memcpy(out32, w, 32);
}
// n pseudo-random inputs (xorshift from seed; 4 in 8 structured: small, near p, powers of two,
// p + s as a non-canonical encoding) within fe_invert's input contract: number whose two inversions differ
unsigned long long nth_fe_invert_cmp(unsigned long long n, unsigned long long seed) {
  unsigned long long bad = 0, x = seed | 1;
  auto rnd = [&x]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
  for (unsigned long long i = 0; i < n; ++i) {
    fe a;
    const uint64_t r0 = rnd();
    const int kind = (int)(r0 & 7);
    for (int l = 0; l < 10; ++l) a.v[l] = (uint32_t)rnd() & ((l & 1) ? NT_M25 : NT_M26);
    if (kind == 1) {  // small: < 2^64
      for (int l = 3; l < 10; ++l) a.v[l] = 0;
      a.v[2] &= 0x3fffu;
    } else if (kind == 2) {  // p - small
      a.v[0] = NT_M26 - 18u - (uint32_t)(rnd() & 0xffff);
      for (int l = 1; l < 10; ++l) a.v[l] = (l & 1) ? NT_M25 : NT_M26;
    } else if (kind == 3) {  // a power of two (or zero)
      for (int l = 0; l < 10; ++l) a.v[l] = 0;
      const int l = (int)(rnd() % 10);
      a.v[l] = 1u << (rnd() % ((l & 1) ? 25 : 26));
    } else if (kind == 4) {  // p + s, s < 19: reduced-size limbs, non-canonical value (= s)
      a.v[0] = NT_M26 - 18u + (uint32_t)(rnd() % 19);
      for (int l = 1; l < 10; ++l) a.v[l] = (l & 1) ? NT_M25 : NT_M26;
    }
    uint8_t o1[32], o2[32];
    nth_fe_invert(a.v, o1, 0);
    nth_fe_invert(a.v, o2, 1);
    bad += std::memcmp(o1, o2, 32) != 0;
  }
  return bad;
}
}

// ---- small-call routing (small_model.hpp) and the key registry's host index (key_table.hpp)
extern "C" {
// 1 = the host lane serves a verify call of nsig signatures on `threads` threads, given the
// model fields m[0..3] = cpu_verify_us, spawn_us, gpu_verify_us, gpu_keyset_us; kind 0 =
// uncached kernel, 1 = key cache
int nth_small_verify_on_host(const double* m, unsigned long long nsig, int threads, int kind) {
  NtSmallModel mm;
  mm.cpu_verify_us = m[0];
  mm.spawn_us = m[1];
  mm.gpu_verify_us = m[2];
  mm.gpu_keyset_us = m[3];
  return nt::small_verify_on_host(mm, nsig, threads, kind) ? 1 : 0;
}

// KeyTable over keys[0 .. nkeys) (seed varies the hash), then find() of each of the nq queries
void nth_key_table_find(const uint8_t* keys, uint32_t nkeys, unsigned long long seed, const uint8_t* q,
                        unsigned long long nq, uint32_t* out) {
  nt::KeyTable t;
  t.build(keys, nkeys, seed);
  for (unsigned long long i = 0; i < nq; ++i) out[i] = t.find(q + 32 * i);
}
}
