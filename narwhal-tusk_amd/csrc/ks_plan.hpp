// ks_plan.hpp -- launch plan of the key-cache verification kernel (host-only
// arithmetic, shared by k_misc.hip and the host test harness).
//
// A launch of n signatures is R = ceil(n / 64) rows (one signature per lane of
// a wave).  A lane verifies the rows of a chunk with ONE field inversion
// (Montgomery's trick), so a chunk of p rows costs about A p + B multiply-
// accumulates per lane (A = 16.66 k: the comb additions, SHA-512, compare;
// B = 15.07 k: the inversion; profiles/opcount.json).  The plan launches a
// persistent grid of `waves` waves (2 or 3 per SIMD) and cuts the rows into
// chunks = k x waves chunks of `base_rows` or `base_rows + 1` rows (at most
// `cap`), so every wave runs k chunks of (nearly) equal size: no SIMD ends with
// a lone tail wave, which the fixed 8-rows-per-wave grid of round 2 left at
// 4.32, 2.16, 1.08 and 0.54 rounds per launch for config 3 on 1, 2, 4 and 8
// GPUs.  Candidates: 2 or 3 waves per SIMD, and k = the fewest
// rounds at <= cap rows per chunk or, when that is one round, also two; the
// plan takes the cheapest of
//   k (A pmax + B) x (waves per SIMD) / T(waves per SIMD) x (k == 1 ? L : 1)
// with T(2) = 0.97, T(3) = 1 (issue rate of 2 vs 3 resident waves,
// profiles/r01/ab_occ_v9) and L = 1.07: with one claim per wave nothing
// rebalances waves that run at different speeds, and a one-round plan measured
// ~7 % slower than the model's relative cost predicts (config 3, 2 waves per
// SIMD: 52 rows in one chunk 11.07 vs 2 x 26 rows 11.71 M certificates/s;
// profiles/r03/ab_ks_plan2/).
#pragma once
#include <stdint.h>

namespace nt {

struct KsPlan {
  uint32_t waves;      // persistent waves launched (<= per_simd x 4 x cus)
  uint32_t chunks;     // chunk indices claimed from the launch's counter
  uint32_t base_rows;  // rows of a chunk; the first `extra` chunks have one more
  uint32_t extra;
  uint32_t per_simd;   // resident waves per SIMD the launch is sized for (2 or 3)
  uint32_t rounds;     // k: chunks per wave
  // streamed rows (ks_stream_plan): rows claimed one at a time, up to `prow`
  // rows per inversion (the stash rows of a wave); chunks / base / extra unused
  uint32_t stream = 0;
  uint32_t rows = 0;
  uint32_t prow = 0;
  // stash rows of one wave either way
  uint32_t stash_rows() const { return stream ? prow : base_rows + (extra ? 1u : 0u); }
};

// Streamed rows: a persistent grid of per_simd x 4 x cus waves (fewer when the
// launch has fewer rows) in which every wave claims ONE row at a time from the
// launch's counter and inverts once when the rows run out -- so waves that run
// at different speeds take different row counts (the one-claim plans above lose
// ~7 % to exactly that), the inversion is shared by all of a wave's rows instead
// of a chunk's, and at any moment the grid works on ~`waves` consecutive rows of
// the key-grouped order (a few committee keys' combs instead of all of them).
// prow = the average rows per wave + 2 (<= cap): a wave that fills its stash
// inverts and starts another batch.  Waves per SIMD: 3 when that still leaves
// >= 16 rows per wave, else 2 (interleaved A/B, profiles/r03/ab_inv_sort: 3
// waves +0.7 % on config 3's one-GPU launch (35 rows per wave) and +0.3 % on
// the 2-GPU shard, -0.5 / -1.3 % on the 4- and 8-GPU shards, where a third
// wave's inversion is shared by only 9 / 4 rows).
inline KsPlan ks_stream_plan(uint64_t n, uint32_t cus, uint32_t cap, int force_per_simd) {
  const uint64_t rows = (n + 63) / 64;
  const uint32_t per = force_per_simd ? (uint32_t)force_per_simd
                                      : (rows >= (uint64_t)16 * 3 * 4 * (cus ? cus : 1) ? 3u : 2u);
  const uint64_t slots = (uint64_t)per * 4 * (cus ? cus : 1);
  const uint64_t W = rows < slots ? rows : slots;
  KsPlan p{(uint32_t)W, 0, 0, 0, per, 1};
  p.stream = 1;
  p.rows = (uint32_t)rows;
  if (W == 0) return p;
  uint64_t pr = (rows + W - 1) / W + 2;
  if (cap == 0) cap = 1;
  p.prow = (uint32_t)(pr < cap ? pr : cap);
  return p;
}

// Stash rows (waves x rows per wave) any plan of either kind needs for a launch
// of at most `rows` rows: streamed, W (ceil(rows / W) + 2) <= rows + 3 W;
// chunked, W (base + 1) <= rows + W, with W <= 3 x 4 x cus resident waves.
// Monotone in rows, so a caller that sizes the stash once for its largest
// launch may run every smaller one into it (the chunked plan's own
// waves x stash_rows is NOT monotone -- 36,864 rows on 256 CUs plan 18,432
// stash rows, 30,720 rows plan 30,720).
inline uint64_t ks_stash_rows_bound(uint64_t rows, uint32_t cus) {
  return rows + 3ull * 3 * 4 * (cus ? cus : 1) + 1;
}

// force_per_simd: 0 = cheaper of 2 and 3, else 2 or 3; cap: most rows per chunk (1..64)
inline KsPlan ks_plan(uint64_t n, uint32_t cus, uint32_t cap, int force_per_simd) {
  const double A = 16.66, B = 15.07, kLone = 1.07;
  const uint64_t rows = (n + 63) / 64;
  if (cap == 0) cap = 1;
  KsPlan best{0, 0, 0, 0, 2, 0};
  double best_t = -1.0;
  for (uint32_t w = 2; w <= 3; ++w) {
    if (force_per_simd && (int)w != force_per_simd) continue;
    const uint64_t slots = (uint64_t)w * 4 * (cus ? cus : 1);
    const uint64_t W = rows < slots ? rows : slots;
    if (W == 0) return KsPlan{0, 0, 0, 0, w, 0};
    const uint64_t kmin = (rows + cap * W - 1) / (cap * W);
    for (uint64_t k = kmin; k <= (kmin > 2 ? kmin : 2); ++k) {
      const uint64_t C = k * W < rows ? k * W : rows;  // cap 1: one row per chunk
      if (k > kmin && C == rows) break;                 // a second round of empty chunks
      const uint64_t base = rows / C, extra = rows % C;
      const uint64_t pmax = base + (extra ? 1 : 0);
      // waves per SIMD actually resident (a launch smaller than the slots fills fewer)
      const uint64_t per = (W + 4 * (uint64_t)cus - 1) / (4 * (uint64_t)(cus ? cus : 1));
      const double T = w == 2 ? 0.97 : 1.0;
      const double t = (double)k * (A * (double)pmax + B) * (double)per / T * (k == 1 ? kLone : 1.0);
      if (best_t < 0 || t < best_t - 1e-9) {
        best_t = t;
        best = KsPlan{(uint32_t)W, (uint32_t)C, (uint32_t)base, (uint32_t)extra, w, (uint32_t)k};
      }
    }
  }
  return best;
}

}  // namespace nt
