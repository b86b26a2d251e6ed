// fe25519.hpp -- GF(2^255-19) for gfx950.
//
// Representation: 10 unsigned 32-bit limbs in radix 2^25.5 (limb i has weight
// 2^ceil(25.5 i); even limbs hold 26 bits, odd limbs 25 bits when reduced).
// Why this radix on CDNA4: the integer ALU microbenchmark
// (tools/microbench/alu_rate.hip, profiles/r01_alu_rate.txt) shows
// v_mad_u64_u32 -- a 32x32->64 multiply with a 64-bit accumulate -- issuing at
// the same rate as v_add_u32's neighbours (~4.5 cycles per wave64 on a SIMD).
// With 25.5-bit limbs every column of the 10x10 schoolbook product fits a u64,
// so each partial product is exactly ONE v_mad_u64_u32 with no carry
// handling (a radix-2^32 product needs a v_addc per partial product).
//
// Bound discipline (all limbs unsigned):
//   "R"  reduced   : output of mul/sq/carry: even limbs < 2^26, odd < 2^25 (+2^18 on limb 1)
//   mul(f, g)      : f limbs < 2^28.6 (odd limbs get x2), g limbs < 2^27.75 (get x19)
//                    => each term < 2^60.4, 10 terms < 2^63.8 < 2^64
//   sq(f)          : f even limbs < 2^26.1, odd < 2^25.1 (13 pre-scaled limbs)
//   sq_wide(f)     : f limbs < 2^27 (4f x 19f terms, <= 6 per column => < 2^62.8)
//   sub(f,g)       : f + 2p - g, needs g "R" (or sub4: f + 4p - g, g < 2^27 even / 2^26 odd)
// Every point formula in ge25519.hpp is annotated with the bound it relies on.
#pragma once
#include "nt_common.hpp"

#if defined(NT_OPCOUNT) && !defined(__HIP_DEVICE_COMPILE__)
// Host-only instrumentation (tools/opcount.cpp): counts field multiplies.
namespace nt { extern unsigned long long g_fe_mul, g_fe_sq; }
#define NT_COUNT_MUL() (++::nt::g_fe_mul)
#define NT_COUNT_SQ() (++::nt::g_fe_sq)
#else
#define NT_COUNT_MUL() ((void)0)
#define NT_COUNT_SQ() ((void)0)
#endif

// Scheduling fence after each multiply: the 10 column chains inside one mul
// are enough ILP for a wave; letting the scheduler overlap several muls only
// multiplies register pressure (spills, lower occupancy).
// -DNT_FENCE_POINT (A/B builds): fence after each point operation instead, so
// the 3-4 independent multiplies of one formula may interleave.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(NT_NO_MUL_FENCE) && !defined(NT_FENCE_POINT)
#define NT_MUL_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define NT_MUL_FENCE() ((void)0)
#endif
#if defined(__HIP_DEVICE_COMPILE__) && defined(NT_FENCE_POINT)
#define NT_POINT_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define NT_POINT_FENCE() ((void)0)
#endif

// Pins a value as a 32-bit VGPR (no instruction emitted).  Without it LLVM
// folds the u64 -> u32 truncation of a carried column into the next multiply
// of a loop (the loop-carried value stays a u64 pair and the squaring/multiply
// of the next iteration does 64x32-bit partial products: measured 130 VALU per
// fe_sq in the exponentiation loops vs 107).
#if defined(__HIP_DEVICE_COMPILE__)
#define NT_OPAQUE32(x) asm("" : "+v"(x))
#else
#define NT_OPAQUE32(x) ((void)0)
#endif

namespace nt {

struct fe {
  uint32_t v[10];
};

#define NT_M26 0x3ffffffu
#define NT_M25 0x1ffffffu

NT_HD NT_INLINE uint32_t fe_mask(int i) { return (i & 1) ? NT_M25 : NT_M26; }
NT_HD NT_INLINE int fe_shift(int i) { return (i & 1) ? 25 : 26; }

NT_HD NT_INLINE void fe_0(fe& h) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = 0;
}
NT_HD NT_INLINE void fe_1(fe& h) {
  fe_0(h);
  h.v[0] = 1;
}

NT_HD NT_INLINE void fe_add(fe& h, const fe& f, const fe& g) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = f.v[i] + g.v[i];
}

// h = f + 2p - g   (g reduced)
NT_HD NT_INLINE void fe_sub(fe& h, const fe& f, const fe& g) {
  h.v[0] = f.v[0] + 0x7ffffdau - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = f.v[i] + ((i & 1) ? 0x3fffffeu : 0x7fffffeu) - g.v[i];
}

// h = f + 4p - g   (g even limbs < 2^28-76, odd < 2^27-4)
NT_HD NT_INLINE void fe_sub4(fe& h, const fe& f, const fe& g) {
  h.v[0] = f.v[0] + 0xfffffb4u - g.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = f.v[i] + ((i & 1) ? 0x7fffffcu : 0xffffffcu) - g.v[i];
}

// h = 2f + 4p - g   (f reduced, g as fe_sub4): one shift-add and one subtract per limb
NT_HD NT_INLINE void fe_dbl_sub4(fe& h, const fe& f, const fe& g) {
  h.v[0] = (f.v[0] << 1) + (0xfffffb4u - g.v[0]);
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = (f.v[i] << 1) + (((i & 1) ? 0x7fffffcu : 0xffffffcu) - g.v[i]);
}

// h = 2p - f  (f reduced)
NT_HD NT_INLINE void fe_neg(fe& h, const fe& f) {
  h.v[0] = 0x7ffffdau - f.v[0];
#pragma unroll
  for (int i = 1; i < 10; ++i) h.v[i] = ((i & 1) ? 0x3fffffeu : 0x7fffffeu) - f.v[i];
}

// conditional move: h = c ? g : h   (c is 0/1)
NT_HD NT_INLINE void fe_cmov(fe& h, const fe& g, uint32_t c) {
#pragma unroll
  for (int i = 0; i < 10; ++i) h.v[i] = c ? g.v[i] : h.v[i];
}

// Weak reduction of 32-bit limbs (inputs < 2^31): output "R".
NT_HD NT_INLINE void fe_carry(fe& h) {
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c = h.v[i] >> fe_shift(i);
    h.v[i] &= fe_mask(i);
    h.v[i + 1] += c;
  }
  c = h.v[9] >> 25;
  h.v[9] &= NT_M25;
  h.v[0] += 19u * c;
  c = h.v[0] >> 26;
  h.v[0] &= NT_M26;
  h.v[1] += c;
}

// Carry a 64-bit column vector into reduced 32-bit limbs.
NT_HD NT_INLINE void fe_carry_wide(fe& out, uint64_t h[10]) {
  uint64_t c;
  // interleaved chains (0->1->2..., 4->5->6...) shorten the dependency path
  c = h[0] >> 26; h[1] += c; h[0] &= NT_M26;
  c = h[4] >> 26; h[5] += c; h[4] &= NT_M26;
  c = h[1] >> 25; h[2] += c; h[1] &= NT_M25;
  c = h[5] >> 25; h[6] += c; h[5] &= NT_M25;
  c = h[2] >> 26; h[3] += c; h[2] &= NT_M26;
  c = h[6] >> 26; h[7] += c; h[6] &= NT_M26;
  c = h[3] >> 25; h[4] += c; h[3] &= NT_M25;
  c = h[7] >> 25; h[8] += c; h[7] &= NT_M25;
  c = h[4] >> 26; h[5] += c; h[4] &= NT_M26;
  c = h[8] >> 26; h[9] += c; h[8] &= NT_M26;
  c = h[9] >> 25; h[0] += c * 19u; h[9] &= NT_M25;
  c = h[0] >> 26; h[1] += c; h[0] &= NT_M26;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    out.v[i] = (uint32_t)h[i];
    NT_OPAQUE32(out.v[i]);
  }
}

#if defined(NT_HOST_FAST_FE) && !defined(__HIP_DEVICE_COMPILE__)
// ---- host lane only (csrc/cpu_lane.cpp, the small-call path) ----------------
// On x86-64 a 64x64->128 multiply costs what a 32x32->64 one does, so the host
// lane multiplies in radix 2^51: limbs 2k and 2k+1 of the radix-2^25.5 form
// are exactly one radix-2^51 limb (weights 2^51k and 2^(51k+26)), giving 25
// (mul) / 15 (sq) products instead of 100 / 55; the result is split back into
// the 10-limb "R" form (even < 2^26, odd <= 2^25) every other function
// expects.  Inputs: anything within the device contracts above (limbs < 2^28.6
// -> radix-2^51 limbs < 2^54.6; every column < 2^115, carried in u128).
typedef unsigned __int128 nt_u128;
NT_HD NT_INLINE void fe51_pack(uint64_t F[5], const fe& f) {
  for (int k = 0; k < 5; ++k) F[k] = (uint64_t)f.v[2 * k] + ((uint64_t)f.v[2 * k + 1] << 26);
}
NT_HD NT_INLINE void fe51_finish(fe& out, nt_u128 t0, nt_u128 t1, nt_u128 t2, nt_u128 t3, nt_u128 t4) {
  const uint64_t M51 = (1ull << 51) - 1;
  t1 += t0 >> 51; t0 &= M51;
  t2 += t1 >> 51; t1 &= M51;
  t3 += t2 >> 51; t2 &= M51;
  t4 += t3 >> 51; t3 &= M51;
  const nt_u128 c = t4 >> 51; t4 &= M51;
  t0 += c * 19;
  t1 += t0 >> 51; t0 &= M51;
  const uint64_t r[5] = {(uint64_t)t0, (uint64_t)t1, (uint64_t)t2, (uint64_t)t3, (uint64_t)t4};
  for (int k = 0; k < 5; ++k) {
    out.v[2 * k] = (uint32_t)(r[k] & NT_M26);
    out.v[2 * k + 1] = (uint32_t)(r[k] >> 26);
  }
}
NT_HD NT_INLINE void fe_mul(fe& out, const fe& f, const fe& g) {
  NT_COUNT_MUL();
  uint64_t F[5], G[5];
  fe51_pack(F, f);
  fe51_pack(G, g);
  const uint64_t g1 = 19 * G[1], g2 = 19 * G[2], g3 = 19 * G[3], g4 = 19 * G[4];
#define NT_W(a, b) ((nt_u128)(a) * (b))
  fe51_finish(out, NT_W(F[0], G[0]) + NT_W(F[1], g4) + NT_W(F[2], g3) + NT_W(F[3], g2) + NT_W(F[4], g1),
              NT_W(F[0], G[1]) + NT_W(F[1], G[0]) + NT_W(F[2], g4) + NT_W(F[3], g3) + NT_W(F[4], g2),
              NT_W(F[0], G[2]) + NT_W(F[1], G[1]) + NT_W(F[2], G[0]) + NT_W(F[3], g4) + NT_W(F[4], g3),
              NT_W(F[0], G[3]) + NT_W(F[1], G[2]) + NT_W(F[2], G[1]) + NT_W(F[3], G[0]) + NT_W(F[4], g4),
              NT_W(F[0], G[4]) + NT_W(F[1], G[3]) + NT_W(F[2], G[2]) + NT_W(F[3], G[1]) + NT_W(F[4], G[0]));
}
NT_HD NT_INLINE void fe51_square(fe& out, const fe& f) {
  uint64_t F[5];
  fe51_pack(F, f);
  const uint64_t f0_2 = 2 * F[0], f1_2 = 2 * F[1], f1_38 = 38 * F[1], f2_38 = 38 * F[2], f3_38 = 38 * F[3];
  const uint64_t f3_19 = 19 * F[3], f4_19 = 19 * F[4];
  fe51_finish(out, NT_W(F[0], F[0]) + NT_W(f1_38, F[4]) + NT_W(f2_38, F[3]),
              NT_W(f0_2, F[1]) + NT_W(f2_38, F[4]) + NT_W(f3_19, F[3]),
              NT_W(f0_2, F[2]) + NT_W(F[1], F[1]) + NT_W(f3_38, F[4]),
              NT_W(f0_2, F[3]) + NT_W(f1_2, F[2]) + NT_W(f4_19, F[4]),
              NT_W(f0_2, F[4]) + NT_W(f1_2, F[3]) + NT_W(F[2], F[2]));
#undef NT_W
}
NT_HD NT_INLINE void fe_sq_wide(fe& out, const fe& f) {
  NT_COUNT_SQ();
  fe51_square(out, f);
}
NT_HD NT_INLINE void fe_sq(fe& out, const fe& f) {
  NT_COUNT_SQ();
  fe51_square(out, f);
}
#else
// h = f * g.  Each partial product is one v_mad_u64_u32.
NT_HD NT_INLINE void fe_mul(fe& out, const fe& f, const fe& g) {
  NT_COUNT_MUL();
  uint32_t g19[10], f2[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    g19[i] = 19u * g.v[i];
    f2[i] = (i & 1) ? 2u * f.v[i] : f.v[i];
  }
  uint64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      const int j = (k - i + 10) % 10;
      const bool wrap = (i + j) >= 10;
      const bool oo = (i & 1) && (j & 1);
      const uint32_t a = oo ? f2[i] : f.v[i];
      const uint32_t b = wrap ? g19[j] : g.v[j];
      acc += (uint64_t)a * b;
    }
    h[k] = acc;
  }
  fe_carry_wide(out, h);
  NT_MUL_FENCE();
}

// h = f^2 for an UNREDUCED f (limbs < 2^27, e.g. X + Y in ge_dbl): symmetric
// products, 55 multiplies, coefficients split as (1|2|4) f_i x (1|19) f_j.
NT_HD NT_INLINE void fe_sq_wide(fe& out, const fe& f) {
  NT_COUNT_SQ();
  uint32_t f2[10], f4[10], f19[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    f2[i] = 2u * f.v[i];
    f4[i] = 4u * f.v[i];
    f19[i] = 19u * f.v[i];
  }
  uint64_t h[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) h[k] = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
#pragma unroll
    for (int j = i; j < 10; ++j) {
      const int k = (i + j) % 10;
      const bool wrap = (i + j) >= 10;
      const bool oo = (i & 1) && (j & 1);
      // coefficient = (i==j ? 1 : 2) * (oo ? 2 : 1) * (wrap ? 19 : 1), split as a(i) * b(j)
      const int ca = (i == j ? 1 : 2) * (oo ? 2 : 1);
      const uint32_t a = ca == 1 ? f.v[i] : (ca == 2 ? f2[i] : f4[i]);
      const uint32_t b = wrap ? f19[j] : f.v[j];
      h[k] += (uint64_t)a * b;
    }
  }
  fe_carry_wide(out, h);
  NT_MUL_FENCE();
}

// h = f^2 for f with reduced-size limbs (even < 2^26.1, odd < 2^25.1: every
// fe_mul / fe_sq / fe_carry output, plus small additions such as d y^2 + 1).
// The odd-odd doubling is folded into 38 = 2 * 19 on the wrapped factor, so
// only 13 limbs are pre-scaled (2 f_0..7, 38 f_5, 19 f_6, 38 f_7, 19 f_8,
// 38 f_9 < 2^30.4); terms < 2^57.5, <= 6 per column.
NT_HD NT_INLINE void fe_sq(fe& out, const fe& f) {
  NT_COUNT_SQ();
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = 2u * f0, f1_2 = 2u * f1, f2_2 = 2u * f2, f3_2 = 2u * f3;
  const uint32_t f4_2 = 2u * f4, f5_2 = 2u * f5, f6_2 = 2u * f6, f7_2 = 2u * f7;
  const uint32_t f5_38 = 38u * f5, f6_19 = 19u * f6, f7_38 = 38u * f7, f8_19 = 19u * f8, f9_38 = 38u * f9;
#define NT_M(a, b) ((uint64_t)(a) * (b))
  uint64_t h[10];
  h[0] = NT_M(f0, f0) + NT_M(f1_2, f9_38) + NT_M(f2_2, f8_19) + NT_M(f3_2, f7_38) + NT_M(f4_2, f6_19) + NT_M(f5, f5_38);
  h[1] = NT_M(f0_2, f1) + NT_M(f2, f9_38) + NT_M(f3_2, f8_19) + NT_M(f4, f7_38) + NT_M(f5_2, f6_19);
  h[2] = NT_M(f0_2, f2) + NT_M(f1_2, f1) + NT_M(f3_2, f9_38) + NT_M(f4_2, f8_19) + NT_M(f5_2, f7_38) + NT_M(f6, f6_19);
  h[3] = NT_M(f0_2, f3) + NT_M(f1_2, f2) + NT_M(f4, f9_38) + NT_M(f5_2, f8_19) + NT_M(f6, f7_38);
  h[4] = NT_M(f0_2, f4) + NT_M(f1_2, f3_2) + NT_M(f2, f2) + NT_M(f5_2, f9_38) + NT_M(f6_2, f8_19) + NT_M(f7, f7_38);
  h[5] = NT_M(f0_2, f5) + NT_M(f1_2, f4) + NT_M(f2_2, f3) + NT_M(f6, f9_38) + NT_M(f7_2, f8_19);
  h[6] = NT_M(f0_2, f6) + NT_M(f1_2, f5_2) + NT_M(f2_2, f4) + NT_M(f3_2, f3) + NT_M(f7_2, f9_38) + NT_M(f8, f8_19);
  h[7] = NT_M(f0_2, f7) + NT_M(f1_2, f6) + NT_M(f2_2, f5) + NT_M(f3_2, f4) + NT_M(f8, f9_38);
  h[8] = NT_M(f0_2, f8) + NT_M(f1_2, f7_2) + NT_M(f2_2, f6) + NT_M(f3_2, f5_2) + NT_M(f4, f4) + NT_M(f9, f9_38);
  h[9] = NT_M(f0_2, f9) + NT_M(f1_2, f8) + NT_M(f2_2, f7) + NT_M(f3_2, f6) + NT_M(f4_2, f5);
#undef NT_M
  fe_carry_wide(out, h);
  NT_MUL_FENCE();
}

#endif  // NT_HOST_FAST_FE

// Repeated squaring; kept as a loop (not unrolled) so the exponentiation chains
// stay small in the instruction cache.
NT_HD NT_INLINE void fe_sqn(fe& out, const fe& f, int n) {
  fe_sq(out, f);
#pragma unroll 1
  for (int i = 1; i < n; ++i) fe_sq(out, out);
}

// Load 255 bits little-endian (bit 255 ignored; value NOT reduced mod p),
// from 8 little-endian 32-bit words.
NT_HD NT_INLINE void fe_frombytes_w(fe& h, const uint32_t w[8]) {
  h.v[0] = w[0] & NT_M26;                                  // bits 0..25
  h.v[1] = ((w[0] >> 26) | (w[1] << 6)) & NT_M25;         // 26..50
  h.v[2] = ((w[1] >> 19) | (w[2] << 13)) & NT_M26;        // 51..76
  h.v[3] = ((w[2] >> 13) | (w[3] << 19)) & NT_M25;        // 77..101
  h.v[4] = (w[3] >> 6) & NT_M26;                          // 102..127
  h.v[5] = w[4] & NT_M25;                                  // 128..152
  h.v[6] = ((w[4] >> 25) | (w[5] << 7)) & NT_M26;         // 153..178
  h.v[7] = ((w[5] >> 19) | (w[6] << 13)) & NT_M25;        // 179..203
  h.v[8] = ((w[6] >> 12) | (w[7] << 20)) & NT_M26;        // 204..229
  h.v[9] = (w[7] >> 6) & NT_M25;                          // 230..254
}

// Fully reduce (canonical, < p) and pack into 8 little-endian words.
NT_HD NT_INLINE void fe_tobytes_w(uint32_t w[8], const fe& f) {
  fe h = f;
  fe_carry(h);  // h < 2^255 + small
  // q = 1 iff h >= p  (h + 19 >= 2^255)
  uint32_t q = (h.v[0] + 19u) >> 26;
#pragma unroll
  for (int i = 1; i < 10; ++i) q = (h.v[i] + q) >> fe_shift(i);
  h.v[0] += 19u * q;
  uint32_t c;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c = h.v[i] >> fe_shift(i);
    h.v[i] &= fe_mask(i);
    h.v[i + 1] += c;
  }
  h.v[9] &= NT_M25;  // drop 2^255 (subtracts p together with +19 q)
  w[0] = h.v[0] | (h.v[1] << 26);
  w[1] = (h.v[1] >> 6) | (h.v[2] << 19);
  w[2] = (h.v[2] >> 13) | (h.v[3] << 13);
  w[3] = (h.v[3] >> 19) | (h.v[4] << 6);
  w[4] = h.v[5] | (h.v[6] << 25);
  w[5] = (h.v[6] >> 7) | (h.v[7] << 19);
  w[6] = (h.v[7] >> 13) | (h.v[8] << 12);
  w[7] = (h.v[8] >> 20) | (h.v[9] << 6);
}

NT_HD NT_INLINE uint32_t fe_iszero(const fe& f) {
  uint32_t w[8];
  fe_tobytes_w(w, f);
  uint32_t a = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) a |= w[i];
  return a == 0;
}

NT_HD NT_INLINE uint32_t fe_isneg(const fe& f) {
  uint32_t w[8];
  fe_tobytes_w(w, f);
  return w[0] & 1;
}

// f == g as field elements (both inputs "R" or sums thereof)
NT_HD NT_INLINE uint32_t fe_eq(const fe& f, const fe& g) {
  fe d;
  fe_sub(d, f, g);
  return fe_iszero(d);
}

// z^(2^252 - 3)
NT_HD NT_INLINE void fe_pow22523(fe& out, const fe& z) {
  fe t0, t1, t2;
  fe_sq(t0, z);           // 2
  fe_sqn(t1, t0, 2);      // 8
  fe_mul(t1, z, t1);      // 9
  fe_mul(t0, t0, t1);     // 11
  fe_sq(t0, t0);          // 22
  fe_mul(t0, t1, t0);     // 2^5 - 1
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);     // 2^10 - 1
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);     // 2^20 - 1
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);     // 2^40 - 1
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);     // 2^50 - 1
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);     // 2^100 - 1
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);     // 2^200 - 1
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);     // 2^250 - 1
  fe_sqn(t0, t0, 2);      // 2^252 - 4
  fe_mul(out, t0, z);     // 2^252 - 3
}

// z^(p-2)
NT_HD NT_INLINE void fe_invert(fe& out, const fe& z) {
  fe t0, t1, t2, t3;
  fe_sq(t0, z);           // 2
  fe_sqn(t1, t0, 2);      // 8
  fe_mul(t1, z, t1);      // 9
  fe_mul(t0, t0, t1);     // 11
  fe_sq(t2, t0);          // 22
  fe_mul(t1, t1, t2);     // 31
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);     // 2^10 - 1
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);     // 2^20 - 1
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);     // 2^40 - 1
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);     // 2^50 - 1
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);     // 2^100 - 1
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);     // 2^200 - 1
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);     // 2^250 - 1
  fe_sqn(t1, t1, 5);      // 2^255 - 32
  fe_mul(out, t1, t0);    // 2^255 - 21
}

// ---- curve constants (radix 2^25.5 limbs), generated by tools/gen_constants.py
// and checked against the oracle-independent golden model in tests/.
struct FeConst {
  uint32_t v[10];
};

}  // namespace nt
