/*
 * chacha20_ref.c -- ChaCha20 keystream with a 64-bit block counter (words
 * 12..13) and 64-bit stream id (words 14..15), the layout of rand_chacha 0.2's
 * ChaCha20Rng, which is rand 0.7's StdRng.  TEST INFRASTRUCTURE ONLY.
 *
 * Used to reproduce the reference's key fixture exactly:
 *   keys() = StdRng::from_seed([0;32]) -> 4 x dalek Keypair::generate, each
 *   drawing 32 bytes with fill_bytes      crypto/src/tests/crypto_tests.rs:26-29
 *                                         primary/src/tests/common.rs:29-32
 * so secret i = keystream bytes [32 i, 32 i + 32) for key 0^32, stream 0.
 */
#include "ntoracle.h"
#include <string.h>

#define QR(a, b, c, d)                 \
  a += b; d ^= a; d = (d << 16) | (d >> 16); \
  c += d; b ^= c; b = (b << 12) | (b >> 20); \
  a += b; d ^= a; d = (d << 8) | (d >> 24);  \
  c += d; b ^= c; b = (b << 7) | (b >> 25);

static void chacha_block(const uint32_t in[16], uint8_t out[64]) {
  uint32_t x[16];
  memcpy(x, in, sizeof x);
  for (int r = 0; r < 10; ++r) {
    QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13])
    QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
    QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12])
    QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
  }
  for (int i = 0; i < 16; ++i) {
    uint32_t v = x[i] + in[i];
    out[4 * i + 0] = (uint8_t)v; out[4 * i + 1] = (uint8_t)(v >> 8);
    out[4 * i + 2] = (uint8_t)(v >> 16); out[4 * i + 3] = (uint8_t)(v >> 24);
  }
}

void ntor_chacha20_keystream(const uint8_t key32[32], uint64_t stream_id, uint64_t counter,
                             uint8_t *out, uint64_t len) {
  uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
  for (int i = 0; i < 8; ++i)
    st[4 + i] = (uint32_t)key32[4 * i] | ((uint32_t)key32[4 * i + 1] << 8) |
                ((uint32_t)key32[4 * i + 2] << 16) | ((uint32_t)key32[4 * i + 3] << 24);
  st[14] = (uint32_t)stream_id;
  st[15] = (uint32_t)(stream_id >> 32);
  uint8_t blk[64];
  while (len) {
    st[12] = (uint32_t)counter;
    st[13] = (uint32_t)(counter >> 32);
    chacha_block(st, blk);
    uint64_t take = len < 64 ? len : 64;
    memcpy(out, blk, take);
    out += take;
    len -= take;
    ++counter;
  }
}
