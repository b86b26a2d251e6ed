// pipe_plan.hpp -- chunk plans of the host entry points' copy / kernel
// pipeline (host-only arithmetic, shared by ntcrypto.cpp and the host test
// harness).  Every boundary but the end is a multiple of 64
// items, so each chunk owns whole 64-bit verdict words.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

namespace nt {

constexpr int kMaxChunks = 16;  // chunk events per execution slot (runtime.hpp cev)

// Chunks of a host verify call (one round R1 = the signatures one wave of
// resident waves covers at ONE signature per lane).  The call is PCIe-bound --
// 608 B per verify over ~50 GB/s against ~95 verifies per us of kernel -- and
// its copies run back to back, so it ends one kernel latency after the last
// copy; a launch's latency is its lanes' serial signatures.  So: a quarter
// round first (the first kernel starts after a short copy), whole rounds at
// one signature per lane in the middle (a round's copy ~ its kernel), and a
// last chunk of at most half a round (one wave per SIMD: the shortest tail).
// More than kMaxChunks - 2 middle chunks grow by whole rounds.
inline std::vector<uint64_t> verify_chunk_targets(uint64_t total, uint64_t R1, uint64_t cap) {
  const uint64_t half = std::max<uint64_t>(64, R1 / 2 / 64 * 64), quarter = std::max<uint64_t>(64, R1 / 4 / 64 * 64);
  if (cap < 3 || total <= half + quarter) return {total};
  std::vector<uint64_t> t{quarter};
  // the last chunk starts on a multiple of 64 (every chunk owns whole verdict words)
  const uint64_t last_start = std::max(quarter, (total - half + 63) / 64 * 64);
  uint64_t mid = last_start - quarter;
  const uint64_t per = std::max<uint64_t>(R1, ((mid + cap - 3) / (cap - 2) + R1 - 1) / R1 * R1);
  while (mid > 0) {
    const uint64_t c = std::min(per, mid);
    t.push_back(c);
    mid -= c;
  }
  t.push_back(total - last_start);
  return t;
}

// Item counts per chunk (the key-cache, group and digest calls).  A host call's
// copies run back to back on the copy stream, so it takes about the whole copy
// plus the kernels that can only start after the LAST copy.  Calls of at least
// two rounds R ramp at both ends (below); shorter ones take a quarter-round
// first chunk (the first kernel starts after a short copy), whole rounds R in
// the middle and at most a quarter round last.  NT_PIPE_PLAN=round restores
// round 4's plan (one-round first chunk, equal whole-round chunks, the rest
// last) for A/B (round4).
inline std::vector<uint64_t> chunk_targets(uint64_t total, uint64_t R, uint64_t cap, bool round4 = false) {
  if (cap <= 1 || total <= R) return {total};
  if (!round4 && cap >= 6 && total >= 2 * R) {
    // A ramp at both ends (R/8, R/4, R/2 ... R/2, R/4, <= R/8).  When a chunk's
    // copy takes about as long as its kernels (the key-cache kernel verifies
    // ~0.85 M signatures/ms, PCIe moves ~0.85 M of its 68-B items/ms), chunk c+1
    // must be no bigger than about chunk c, or the GPU idles while it copies;
    // and what runs after the last copy lands is one short launch.
    auto w = [](uint64_t x) { return std::max<uint64_t>(64, x / 64 * 64); };
    const uint64_t e = w(R / 8), q = w(R / 4), h = w(R / 2);
    std::vector<uint64_t> t{e, q, h};
    const uint64_t head = e + q + h;
    const uint64_t s3 = std::max(head + q, (total - std::min(e, total) + 63) / 64 * 64);  // the last chunk
    const uint64_t s2 = s3 - q;                                                          // R/4 before it
    const uint64_t mid = s2 - head;
    if (mid) {
      const uint64_t n = std::min(cap - 5, (mid + h - 1) / h);
      const uint64_t per = (mid + n - 1) / n + 63;
      uint64_t left = mid;
      while (left > 0) {
        const uint64_t c = std::min(per / 64 * 64, left);
        t.push_back(c);
        left -= c;
      }
    }
    t.push_back(q);
    if (total > s3) t.push_back(total - s3);
    return t;
  }
  if (!round4 && cap >= 3) {
    const uint64_t q = std::max<uint64_t>(64, R / 4 / 64 * 64);
    std::vector<uint64_t> t{q};
    // the last chunk starts on a multiple of 64 (every chunk owns whole verdict words)
    const uint64_t tail = std::max<uint64_t>(q, (total - std::min<uint64_t>(q, total - q)) / 64 * 64);
    const uint64_t last = total - tail;
    uint64_t mid_total = tail - q;
    // whole rounds, grown to whole multiples of R when cap - 2 chunks would not cover it
    const uint64_t per = std::max<uint64_t>(R, (mid_total + cap - 3) / (cap - 2) + R - 1) / R * R;
    while (mid_total > 0) {
      const uint64_t c = std::min(per, mid_total);
      t.push_back(c);
      mid_total -= c;
    }
    if (last) t.push_back(last);
    return t;
  }
  const uint64_t k = std::min<uint64_t>(cap, (total + R - 1) / R);
  const uint64_t mid = ((total - R + k - 2) / (k - 1) + R - 1) / R * R;
  std::vector<uint64_t> t{R};
  uint64_t left = total - R;
  while (left > mid) {
    t.push_back(mid);
    left -= mid;
  }
  t.push_back(left);
  return t;
}

// Certificate groups [glo, ghi) -> chunks [g0, g1) holding about targets[c]
// signatures each (at most that many when a boundary allows), every g0 - glo
// a multiple of 64 (whole group-verdict words).
inline std::vector<std::pair<uint64_t, uint64_t>> plan_group_chunks(uint64_t glo, uint64_t ghi, const uint32_t* cnt,
                                                             const std::vector<uint64_t>& targets) {
  std::vector<std::pair<uint64_t, uint64_t>> r;
  uint64_t g0 = glo, acc = 0, cut = 0, acc_cut = 0;
  size_t ti = 0;
  for (uint64_t g = glo; g < ghi && ti + 1 < targets.size(); ++g) {
    acc += cnt[g];
    const uint64_t next = g + 1;
    if ((next - glo) % 64 != 0 || next >= ghi) continue;
    if (acc <= targets[ti]) {
      cut = next;
      acc_cut = acc;
      if (acc < targets[ti]) continue;
    } else if (cut == 0) {
      cut = next;
      acc_cut = acc;
    }
    r.emplace_back(g0, cut);
    g0 = cut;
    acc -= acc_cut;
    cut = acc_cut = 0;
    ++ti;
  }
  r.emplace_back(g0, ghi);
  return r;
}

}  // namespace nt
