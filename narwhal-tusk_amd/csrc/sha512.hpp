// sha512.hpp -- FIPS 180-4 SHA-512 for one lane per message on gfx950.
//
// 64-bit rotates lower to v_alignbit_b32 pairs, 64-bit adds to v_lshl_add_u64,
// the three-way XORs of the Sigma/sigma functions and Maj to gfx950's
// v_bitop3_b32 (any 3-input boolean function in one instruction: 0x96 = XOR3,
// 0xE8 = MAJ), Ch to v_bitop3/v_bfi; big-endian word loads are byte-swapped
// with v_perm_b32.  The 16-entry circular message schedule keeps the state in
// 8 + 16 64-bit registers (48 VGPRs).
//
// Streams: the hashed byte string is  prefix (PW 32-bit words held in
// registers, 4*PW < 128)  ||  msg[0..len)  (global memory, any alignment).
//   PW = 0  : batch digests        worker/src/processor.rs:38
//   PW = 16 : k = H(R || A || M)    dalek verify_strict / verify_batch
//   PW = 8  : r = H(prefix || M)    RFC 8032 signing (crypto/src/lib.rs:185-191)
#pragma once
#include "nt_common.hpp"

namespace nt {

static constexpr uint64_t kSha512K[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL,
    0x3956c25bf348b538ULL, 0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL,
    0xd807aa98a3030242ULL, 0x12835b0145706fbeULL, 0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL,
    0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL, 0xc19bf174cf692694ULL,
    0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL,
    0x983e5152ee66dfabULL, 0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL,
    0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL, 0x06ca6351e003826fULL, 0x142929670a0e6e70ULL,
    0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL, 0x53380d139d95b3dfULL,
    0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL,
    0xd192e819d6ef5218ULL, 0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL,
    0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL, 0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL,
    0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL, 0x682e6ff3d6b2b8a3ULL,
    0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL,
    0xca273eceea26619cULL, 0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL,
    0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL, 0x113f9804bef90daeULL, 0x1b710b35131c471bULL,
    0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL, 0x431d67c49c100d4cULL,
    0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

NT_HD NT_INLINE uint64_t rotr64_generic(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// 64-bit rotate / shift by a constant as two v_alignbit_b32 (the compiler's own
// lowering used shift/shift/or sequences: ~2x the instructions).
template <int N>
NT_HD NT_INLINE uint64_t rotr64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rlo, rhi;
  if constexpr (N < 32) {
    rlo = __builtin_amdgcn_alignbit(hi, lo, N);
    rhi = __builtin_amdgcn_alignbit(lo, hi, N);
  } else {
    rlo = __builtin_amdgcn_alignbit(lo, hi, N - 32);
    rhi = __builtin_amdgcn_alignbit(hi, lo, N - 32);
  }
  return ((uint64_t)rhi << 32) | rlo;
#else
  return rotr64_generic(x, N);
#endif
}
template <int N>
NT_HD NT_INLINE uint64_t shr64(uint64_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> N) << 32) | __builtin_amdgcn_alignbit(hi, lo, N);
#else
  return x >> N;
#endif
}
// 3-input boolean functions per 32-bit half: one v_bitop3_b32 each
// (truth-table immediate indexed by (x << 2) | (y << 1) | z)
template <int TT>
NT_HD NT_INLINE uint64_t bitop3_64(uint64_t x, uint64_t y, uint64_t z) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = __builtin_amdgcn_bitop3_b32((uint32_t)x, (uint32_t)y, (uint32_t)z, TT);
  const uint32_t hi =
      __builtin_amdgcn_bitop3_b32((uint32_t)(x >> 32), (uint32_t)(y >> 32), (uint32_t)(z >> 32), TT);
  return ((uint64_t)hi << 32) | lo;
#else
  if constexpr (TT == 0x96) return x ^ y ^ z;                       // XOR3
  if constexpr (TT == 0xE8) return (x & y) | (z & (x | y));         // MAJ
  if constexpr (TT == 0xCA) return z ^ (x & (y ^ z));               // CH
  uint64_t r = 0;
  for (int i = 0; i < 8; ++i)
    if ((TT >> i) & 1) {
      const uint64_t mx = (i & 4) ? x : ~x, my = (i & 2) ? y : ~y, mz = (i & 1) ? z : ~z;
      r |= mx & my & mz;
    }
  return r;
#endif
}
// 64-bit add as one v_lshl_add_u64 behind an asm boundary: values rebuilt from
// 32-bit halves (bitop3 / alignbit results) otherwise get their additions split
// into half-width pieces by the optimizer (+25% instructions per block).
NT_HD NT_INLINE uint64_t add64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return a + b;
#endif
}
// a + K with K an SGPR pair
NT_HD NT_INLINE uint64_t add64_s(uint64_t a, uint64_t k) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "s"(k));
  return r;
#else
  return a + k;
#endif
}
NT_HD NT_INLINE uint64_t xor3_64(uint64_t x, uint64_t y, uint64_t z) { return bitop3_64<0x96>(x, y, z); }
NT_HD NT_INLINE uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) { return bitop3_64<0xE8>(a, b, c); }
NT_HD NT_INLINE uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) { return bitop3_64<0xCA>(e, f, g); }

NT_HD NT_INLINE uint32_t bswap32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bswap32(x);
#else
  return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
#endif
}

NT_HD NT_INLINE void sha512_init(uint64_t st[8]) {
  st[0] = 0x6a09e667f3bcc908ULL; st[1] = 0xbb67ae8584caa73bULL;
  st[2] = 0x3c6ef372fe94f82bULL; st[3] = 0xa54ff53a5f1d36f1ULL;
  st[4] = 0x510e527fade682d1ULL; st[5] = 0x9b05688c2b3e6c1fULL;
  st[6] = 0x1f83d9abfb41bd6bULL; st[7] = 0x5be0cd19137e2179ULL;
}

// Round constant K as an SGPR pair materialized at its use.  A plain constant
// is hoisted out of the block loop by LICM into 160 VGPRs (80 x 64-bit),
// which is what drove the first build of this kernel to 256 VGPRs.  The
// volatile asm cannot be hoisted, costs two SALU slots per round and no VGPR.
template <int R>
NT_HD NT_INLINE uint64_t sha_k() {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3"
               : "=s"(lo), "=s"(hi)
               : "i"((uint32_t)kSha512K[R]), "i"((uint32_t)(kSha512K[R] >> 32)));
  return ((uint64_t)hi << 32) | lo;
#else
  return kSha512K[R];
#endif
}

template <int R>
NT_HD NT_INLINE void sha_round(uint64_t v[8], uint64_t W[16]) {
  // working variables rotate by index instead of by moves
  uint64_t& a = v[(8 - R % 8) % 8];
  uint64_t& b = v[(9 - R % 8) % 8];
  uint64_t& c = v[(10 - R % 8) % 8];
  uint64_t& d = v[(11 - R % 8) % 8];
  uint64_t& e = v[(12 - R % 8) % 8];
  uint64_t& f = v[(13 - R % 8) % 8];
  uint64_t& g = v[(14 - R % 8) % 8];
  uint64_t& h = v[(15 - R % 8) % 8];
  if constexpr (R >= 16) {
    constexpr int i = R & 15;
    const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
    const uint64_t s0 = xor3_64(rotr64<1>(w15), rotr64<8>(w15), shr64<7>(w15));
    const uint64_t s1 = xor3_64(rotr64<19>(w2), rotr64<61>(w2), shr64<6>(w2));
    W[i] = add64(add64(W[i], s0), add64(W[(i + 9) & 15], s1));
  }
  const uint64_t kw = add64_s(W[R & 15], sha_k<R>());
  const uint64_t t1 = add64(add64(h, kw), add64(xor3_64(rotr64<14>(e), rotr64<18>(e), rotr64<41>(e)), ch64(e, f, g)));
  const uint64_t t2 = add64(xor3_64(rotr64<28>(a), rotr64<34>(a), rotr64<39>(a)), maj64(a, b, c));
  d = add64(d, t1);
  h = add64(t1, t2);
}

template <int R>
NT_HD NT_INLINE void sha_rounds(uint64_t v[8], uint64_t W[16]) {
  if constexpr (R < 80) {
    sha_round<R>(v, W);
    sha_rounds<R + 1>(v, W);
  }
}

// ---- split form for the producer/consumer kernel (k_sha512_pipe) ----
// Producer: the 80 words K[t] + W[t] of one block, handed out in pairs.
template <int R, class Sink>
NT_HD NT_INLINE void sha_kw_pairs(uint64_t W[16], Sink& sink) {
  if constexpr (R < 80) {
    constexpr int i = R & 15;
    if constexpr (R >= 16) {
      const uint64_t w15 = W[(i + 1) & 15], w2 = W[(i + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64<1>(w15), rotr64<8>(w15), shr64<7>(w15));
      const uint64_t s1 = xor3_64(rotr64<19>(w2), rotr64<61>(w2), shr64<6>(w2));
      W[i] = add64(add64(W[i], s0), add64(W[(i + 9) & 15], s1));
    }
    const uint64_t kw0 = add64_s(W[i], sha_k<R>());
    constexpr int j = (R + 1) & 15;
    if constexpr (R + 1 >= 16) {
      const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
      const uint64_t s0 = xor3_64(rotr64<1>(w15), rotr64<8>(w15), shr64<7>(w15));
      const uint64_t s1 = xor3_64(rotr64<19>(w2), rotr64<61>(w2), shr64<6>(w2));
      W[j] = add64(add64(W[j], s0), add64(W[(j + 9) & 15], s1));
    }
    const uint64_t kw1 = add64_s(W[j], sha_k<R + 1>());
    sink.template put<R / 2>(kw0, kw1);
    sha_kw_pairs<R + 2>(W, sink);
  }
}

// Consumer: one round given kw = K[t] + W[t].
template <int R>
NT_HD NT_INLINE void sha_round_kw(uint64_t v[8], uint64_t kw) {
  uint64_t& a = v[(8 - R % 8) % 8];
  uint64_t& b = v[(9 - R % 8) % 8];
  uint64_t& c = v[(10 - R % 8) % 8];
  uint64_t& d = v[(11 - R % 8) % 8];
  uint64_t& e = v[(12 - R % 8) % 8];
  uint64_t& f = v[(13 - R % 8) % 8];
  uint64_t& g = v[(14 - R % 8) % 8];
  uint64_t& h = v[(15 - R % 8) % 8];
  const uint64_t t1 = add64(add64(h, kw), add64(xor3_64(rotr64<14>(e), rotr64<18>(e), rotr64<41>(e)), ch64(e, f, g)));
  const uint64_t t2 = add64(xor3_64(rotr64<28>(a), rotr64<34>(a), rotr64<39>(a)), maj64(a, b, c));
  d = add64(d, t1);
  h = add64(t1, t2);
}
template <int R, class Source>
NT_HD NT_INLINE void sha_rounds_kw(uint64_t v[8], const Source& src) {
  if constexpr (R < 80) {
    uint64_t kw0, kw1;
    src.template get<R / 2>(kw0, kw1);
    sha_round_kw<R>(v, kw0);
    sha_round_kw<R + 1>(v, kw1);
    sha_rounds_kw<R + 2>(v, src);
  }
}

// big-endian message words of a block
NT_HD NT_INLINE void sha512_block_w(uint64_t W[16], const uint32_t blk[32]) {
#pragma unroll
  for (int t = 0; t < 16; ++t) W[t] = ((uint64_t)bswap32(blk[2 * t]) << 32) | bswap32(blk[2 * t + 1]);
}

// One compression. blk[i] = LE 32-bit words of the 128-byte block as stored in memory.
NT_HD NT_INLINE void sha512_compress_words(uint64_t st[8], const uint32_t blk[32]) {
  uint64_t W[16];
#pragma unroll
  for (int t = 0; t < 16; ++t)
    W[t] = ((uint64_t)bswap32(blk[2 * t]) << 32) | bswap32(blk[2 * t + 1]);
  uint64_t v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = st[i];
  sha_rounds<0>(v, W);
#pragma unroll
  for (int i = 0; i < 8; ++i) st[i] = add64(st[i], v[i]);
}

// Load NW little-endian words starting at byte address p (any alignment) from
// an interval that contains all of [p, p + 4 NW).  Aligned dword loads +
// v_alignbyte_b32; the extra word is only fetched when p is misaligned and it
// then shares a 4-byte granule with the last wanted byte.
template <int NW>
NT_HD NT_INLINE void load_words(uint32_t* w, const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t sh = (uint32_t)(a & 3u);
  const uint32_t* pw = (const uint32_t*)(a & ~(uintptr_t)3);
  if (sh == 0) {
    if ((a & 15u) == 0 && (NW % 4) == 0) {
#pragma unroll
      for (int i = 0; i < NW / 4; ++i) {
        const uint4 q = ((const uint4*)pw)[i];
        w[4 * i] = q.x; w[4 * i + 1] = q.y; w[4 * i + 2] = q.z; w[4 * i + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NW; ++i) w[i] = pw[i];
    }
  } else {
    uint32_t prev = pw[0];
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const uint32_t nxt = pw[i + 1];
#if defined(__HIP_DEVICE_COMPILE__)
      w[i] = __builtin_amdgcn_alignbyte(nxt, prev, sh);
#else
      w[i] = (uint32_t)((((uint64_t)nxt << 32) | prev) >> (8 * sh));
#endif
      prev = nxt;
    }
  }
}

// Tail block b (not made only of message bytes): message bytes, 0x80, zeros
// and -- in the last block -- the 128-bit big-endian bit length.  Only 4-byte
// granules that contain message bytes are read (predicated aligned loads).
template <int PW>
NT_HD NT_INLINE void sha512_tail_block(uint32_t blk[32], const uint32_t* prefix, const uint8_t* msg,
                                       uint64_t len, uint64_t b, bool last) {
  const uint64_t total = (uint64_t)(4 * PW) + len;
  const uintptr_t base = (uintptr_t)msg;
  const uint32_t sh = (uint32_t)(base & 3u);
  const uint32_t* pw = (const uint32_t*)(base & ~(uintptr_t)3);
  const uint64_t mend = (uint64_t)sh + len;  // message end relative to pw (bytes)
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const uint64_t pos = 128 * b + 4 * i;  // stream position of this word
    if (i < PW && b == 0) {
      blk[i] = prefix[i < PW ? i : 0];
      continue;
    }
    // message-relative byte offset of the word (pos >= 4*PW here)
    const uint64_t r = pos - 4 * PW;
    const uint64_t g0 = (r + sh) >> 2;  // aligned granule holding the first byte
    const uint32_t lo = (4 * g0 < mend) ? pw[g0] : 0u;
    const uint32_t hi = (sh != 0 && 4 * (g0 + 1) < mend) ? pw[g0 + 1] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, sh);
#else
    uint32_t w = (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
#endif
    // keep bytes < len, put 0x80 at byte len, zero the rest
    const uint64_t have = (len > r) ? (len - r) : 0;  // message bytes in this word
    const uint32_t keep = have >= 4 ? 0xffffffffu : ((1u << (8 * (uint32_t)have)) - 1u);
    const uint32_t pad = (pos <= total && total < pos + 4) ? (0x80u << (8 * (uint32_t)(total - pos))) : 0u;
    blk[i] = (w & keep) | pad;
  }
  if (last) {
    const uint64_t bits = total << 3;
    blk[28] = 0;
    blk[29] = bswap32((uint32_t)(total >> 61));
    blk[30] = bswap32((uint32_t)(bits >> 32));
    blk[31] = bswap32((uint32_t)bits);
  }
}

// Hash  prefix[0..PW) || msg[0..len)  and return the 8 state words.
template <int PW>
NT_HD NT_INLINE void sha512_prefixed(uint64_t st[8], const uint32_t* prefix, const uint8_t* msg,
                                     uint64_t len) {
  sha512_init(st);
  const uint64_t total = (uint64_t)(4 * PW) + len;
  const uint64_t nblocks = (total + 17 + 127) / 128;
  const uint64_t nfull = total / 128;  // blocks made only of prefix/message bytes
  uint32_t blk[32];
  uint64_t b = 0;
  if (PW > 0 && nfull > 0) {
#pragma unroll
    for (int i = 0; i < PW; ++i) blk[i] = prefix[i];
    load_words<32 - PW>(blk + PW, msg);
    sha512_compress_words(st, blk);
    b = 1;
  }
#pragma unroll 1
  for (; b < nfull; ++b) {
    load_words<32>(blk, msg + (128 * b - 4 * PW));
    sha512_compress_words(st, blk);
  }
#pragma unroll 1
  for (; b < nblocks; ++b) {
    sha512_tail_block<PW>(blk, prefix, msg, len, b, b == nblocks - 1);
    sha512_compress_words(st, blk);
  }
}

// The same with one compression site (full and tail blocks chosen per block):
// about half the code of sha512_prefixed, for kernels built on a tight register
// budget (k_sha512_trunc32 at 80 VGPRs).
template <int PW>
NT_HD NT_INLINE void sha512_prefixed_1site(uint64_t st[8], const uint32_t* prefix, const uint8_t* msg,
                                           uint64_t len) {
  sha512_init(st);
  const uint64_t total = (uint64_t)(4 * PW) + len;
  const uint64_t nblocks = (total + 17 + 127) / 128;
  const uint64_t nfull = total / 128;
#pragma unroll 1
  for (uint64_t b = 0; b < nblocks; ++b) {
    uint32_t blk[32];
    if (b < nfull && (PW == 0 || b > 0)) load_words<32>(blk, msg + (128 * b - 4 * PW));
    else sha512_tail_block<PW>(blk, prefix, msg, len, b, b == nblocks - 1);
    sha512_compress_words(st, blk);
  }
}

// k = H(R || A || M) for a 32-byte M (every key-cache signature: headers, votes and
// certificates sign a 32-byte digest, crypto/src/lib.rs:185-204): the 96 bytes
// are one block built straight from registers -- no byte-granular tail assembly
// (679 VALU in the key-cache kernel's ISA for the general path).
NT_HD NT_INLINE void sha512_96(uint64_t st[8], const uint32_t prefix[16], const uint32_t m[8]) {
  sha512_init(st);
  uint32_t blk[32];
#pragma unroll
  for (int i = 0; i < 16; ++i) blk[i] = prefix[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) blk[16 + i] = m[i];
  blk[24] = 0x80u;  // the padding bit right after byte 95
#pragma unroll
  for (int i = 25; i < 31; ++i) blk[i] = 0u;
  blk[31] = bswap32(96u * 8u);  // 128-bit big-endian bit length 768
  sha512_compress_words(st, blk);
}

// First 32 bytes / all 64 bytes of the digest as little-endian memory words.
NT_HD NT_INLINE void sha512_out_words(uint32_t* out, const uint64_t st[8], int nwords) {
  for (int i = 0; i < nwords / 2; ++i) {
    out[2 * i] = bswap32((uint32_t)(st[i] >> 32));
    out[2 * i + 1] = bswap32((uint32_t)st[i]);
  }
}

}  // namespace nt
