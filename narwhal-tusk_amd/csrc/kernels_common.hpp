// kernels_common.hpp -- definitions shared by the gfx950 kernel translation
// units (k_misc.hip, k_verify_*.hip, k_keyset_*.hip): block size, workspace
// layout, table accessors, and the occupancy-variant switch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "ed25519_ops.hpp"
#include "kernels.hpp"

namespace nt {

constexpr int kBlock = 256;

// Short kernels that run beside a long key-cache or verify launch of another
// stream (digests, key sort, verdict packing, group AND, wire parsing) raise
// their waves' issue priority on entry.  The SIMD arbiter otherwise prefers
// the older waves of the long launch, which is VALU-issue-bound: a 15 us
// certificate-digest launch on the next pipeline step then waits ~0.8 ms, for
// the other launch's tail (rocprofv3 trace).  -DNT_AUX_PRIO=0
// keeps the default priority (A/B).
#ifndef NT_AUX_PRIO
#define NT_AUX_PRIO 2
#endif
NT_D NT_INLINE void aux_priority() {
#if NT_AUX_PRIO
  __builtin_amdgcn_s_setprio(NT_AUX_PRIO);
#endif
}
#ifndef NT_VERIFY_PER_LANE
#define NT_VERIFY_PER_LANE 2
#endif
// signatures per lane per block iteration of k_ed25519_verify (1 or 2; A/B builds)
constexpr int kVPer = NT_VERIFY_PER_LANE;
constexpr int kAEntries = 18;         // j*(+-A) and j*(-R), |digit| in 0..8
// Signed entries (NT_ATAB_SIGNED=1): each cached coordinate in its own 3-quad
// slot -- Y+X, Y-X, 2Z, 2dT and -2dT -- so a lookup of digit -j reads the slots
// of +j in swapped order (per-lane addresses) instead of negating the entry
// with 10 subtracts and 30 selects (ge_cached_cneg) on every ladder addition.
#ifndef NT_ATAB_SIGNED
#define NT_ATAB_SIGNED 0
#endif
constexpr int kAQuads = NT_ATAB_SIGNED ? 15 : 10;  // uint4 per entry

// --------------------------------------------------------------------------
// Table accessors
// --------------------------------------------------------------------------
// Wide comb of one point with digit width W, layout [pos][entry][32 words];
// 8 x 16-byte loads.
#ifndef NT_COMB_NT
#define NT_COMB_NT 0
#endif
template <int W>
struct WideComb {
  static constexpr int kBits = W;
  const uint32_t* base;
  NT_D NT_INLINE void load(uint32_t pos, uint32_t idx, ge_niels& q) const {
#ifdef NT_EXPERIMENT_CACHED_COMB
    idx &= 7;  // timing experiment only (wrong results): every lookup hits in cache
#endif
#ifdef NT_EXPERIMENT_BHALF
    if (W == kBCombBits) idx >>= 1;  // timing experiment only (wrong results): half of each position's table
#endif
#ifdef NT_EXPERIMENT_KHALF
    if (W == kKeyCombWide) idx >>= 1;  // timing experiment only (wrong results): half of each key position's table
#endif
    const uint4* e = (const uint4*)(base + ((size_t)pos * CombGeom<W>::kEntries + idx) * kWStride);
    uint32_t w[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#if NT_COMB_NT
      // A/B build (-DNT_COMB_NT=1): non-temporal loads -- a random comb line is read once
      typedef unsigned int u4v __attribute__((ext_vector_type(4)));
      const u4v t = __builtin_nontemporal_load((const u4v*)e + i);
      const uint4 v = make_uint4(t.x, t.y, t.z, t.w);
#else
      const uint4 v = e[i];
#endif
      w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      q.ypx.v[i] = w[i];
      q.ymx.v[i] = w[10 + i];
      q.xy2d.v[i] = w[20 + i];
    }
  }
  // the point's [L]P entry after the positions (reduced-scalar combs, CombGeom::kCorrWord)
  NT_D NT_INLINE void load_corr(ge_niels& q) const {
    const uint4* e = (const uint4*)(base + CombGeom<W>::kCorrWord);
    uint32_t w[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 v = e[i];
      w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      q.ypx.v[i] = w[i];
      q.ymx.v[i] = w[10 + i];
      q.xy2d.v[i] = w[20 + i];
    }
  }
};

// Per-lane point tables in the global workspace, uint4 granules.  Lane-major
// ([slot][lane][entry][quad], NT_ATAB_LANE_MAJOR=1): an entry is 160 contiguous
// bytes of one lane, so the 10 loads of a table lookup use every byte of the
// ~1.5 lines they fetch.  Lane-minor ([slot][entry][quad][lane]): a lookup's
// loads coalesce only among lanes that picked the same entry -- with 9 entry
// magnitudes per 8-lane line that fetched ~5x the bytes used (PMC v7: 63 GB per
// 1M-verify launch, 5.5 TB/s).  Measured (same box, interleaved): lane-major
// 95.5 vs lane-minor 88.1 M verifies/s.
#ifndef NT_ATAB_LANE_MAJOR
#define NT_ATAB_LANE_MAJOR 1
#endif
struct WsATab {
  uint4* ws;
  uint32_t slot;
#if NT_ATAB_LANE_MAJOR
  static constexpr size_t kQuadStride = 1;
  NT_D NT_INLINE uint4* at(uint32_t entry) const {
    return ws + ((size_t)(slot * kBlock + threadIdx.x) * kAEntries + entry) * kAQuads;
  }
#else
  static constexpr size_t kQuadStride = kBlock;
  NT_D NT_INLINE uint4* at(uint32_t entry) const {
    return ws + ((size_t)(slot * kAEntries + entry) * kAQuads) * kBlock + threadIdx.x;
  }
#endif
#if NT_ATAB_SIGNED
  // slot k of an entry: 3 quads, words 0..9 used
  NT_D NT_INLINE void store_fe(uint4* q, const fe& f) const {
    q[0 * kQuadStride] = make_uint4(f.v[0], f.v[1], f.v[2], f.v[3]);
    q[1 * kQuadStride] = make_uint4(f.v[4], f.v[5], f.v[6], f.v[7]);
    q[2 * kQuadStride] = make_uint4(f.v[8], f.v[9], 0u, 0u);
  }
  NT_D NT_INLINE void load_fe(const uint4* q, fe& f) const {
    const uint4 a = q[0 * kQuadStride], b = q[1 * kQuadStride], c = q[2 * kQuadStride];
    f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w;
    f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
    f.v[8] = c.x; f.v[9] = c.y;
  }
  NT_D NT_INLINE void store(uint32_t entry, const ge_cached& c) const {
    uint4* base = at(entry);
    fe n;
    fe_neg(n, c.T2d);  // T2d is a multiply output (reduced): 2p - T2d < 2^27
    store_fe(base, c.YpX);
    store_fe(base + 3 * kQuadStride, c.YmX);
    store_fe(base + 6 * kQuadStride, c.Z2);
    store_fe(base + 9 * kQuadStride, c.T2d);
    store_fe(base + 12 * kQuadStride, n);
  }
  // entry e0 + |d| negated when d < 0: -(Y+X, Y-X, 2Z, 2dT) = (Y-X, Y+X, 2Z, -2dT)
  NT_D NT_INLINE void load_signed(uint32_t e0, int32_t d, ge_cached& c) const {
    const uint32_t neg = d < 0 ? 1u : 0u;
    uint32_t entry = e0 + (uint32_t)(d < 0 ? -d : d);
#ifdef NT_EXPERIMENT_CACHED_ATAB
    entry = entry >= kTabR ? kTabR + 1 : 1;  // timing experiment only (wrong results): lookups hit one entry
#endif
    const uint4* base = at(entry);
    load_fe(base + (neg ? 3 : 0) * kQuadStride, c.YpX);
    load_fe(base + (neg ? 0 : 3) * kQuadStride, c.YmX);
    load_fe(base + 6 * kQuadStride, c.Z2);
    load_fe(base + (neg ? 12 : 9) * kQuadStride, c.T2d);
  }
  NT_D NT_INLINE void load(uint32_t entry, ge_cached& c) const { load_signed(entry, 0, c); }
#else
  NT_D NT_INLINE void load_signed(uint32_t e0, int32_t d, ge_cached& c) const {
    load(e0 + (uint32_t)(d < 0 ? -d : d), c);
    ge_cached_cneg(c, d < 0);
  }
  NT_D NT_INLINE void store(uint32_t entry, const ge_cached& c) const {
    uint32_t w[40];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      w[i] = c.YpX.v[i]; w[10 + i] = c.YmX.v[i]; w[20 + i] = c.Z2.v[i]; w[30 + i] = c.T2d.v[i];
    }
    uint4* base = at(entry);
#pragma unroll
    for (int q = 0; q < kAQuads; ++q)
      base[q * kQuadStride] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  NT_D NT_INLINE void load(uint32_t entry, ge_cached& c) const {
#ifdef NT_EXPERIMENT_CACHED_ATAB
    entry = entry >= kTabR ? kTabR + 1 : 1;  // timing experiment only (wrong results): lookups hit one entry
#endif
    uint32_t w[40];
    const uint4* base = at(entry);
#pragma unroll
    for (int q = 0; q < kAQuads; ++q) {
      const uint4 v = base[q * kQuadStride];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c.YpX.v[i] = w[i]; c.YmX.v[i] = w[10 + i]; c.Z2.v[i] = w[20 + i]; c.T2d.v[i] = w[30 + i];
    }
  }
#endif
};

// ---- key-cache verification: up to 64 signatures per lane, one inversion ----
#ifndef NT_KS_PER_LANE
#define NT_KS_PER_LANE 64
#endif
// most signatures per lane sharing one inversion; a launch runs
// keyset_per_lane() <= kKsPerLane of them (a kernel argument)
constexpr int kKsPerLane = NT_KS_PER_LANE;
constexpr int kKsQuads = 10;  // X, Y, Z, prefix: 40 words per (signature, lane)

// Per-lane stash in global memory, layout [wave][j][quad][lane] of uint4
// (lane-minor: a wave's 16-byte accesses are contiguous); a wave's region is
// (most rows of a chunk) * kKsQuads * 64 quads.
struct KsStash {
  uint4* base;  // this wave's region
  NT_D NT_INLINE uint4* at(int j, int q) const {
    return base + ((size_t)(j * kKsQuads + q) * 64 + (threadIdx.x & 63u));
  }
  NT_D NT_INLINE void put(int j, const ge_p2& P, const fe& a) const {
    uint32_t w[40];
#pragma unroll
    for (int i = 0; i < 10; ++i) { w[i] = P.X.v[i]; w[10 + i] = P.Y.v[i]; w[20 + i] = P.Z.v[i]; w[30 + i] = a.v[i]; }
#pragma unroll
    for (int q = 0; q < kKsQuads; ++q) *at(j, q) = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  NT_D NT_INLINE void get_point(int j, ge_p2& P) const {
    uint32_t w[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint4 v = *at(j, q);
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) { P.X.v[i] = w[i]; P.Y.v[i] = w[10 + i]; P.Z.v[i] = w[20 + i]; }
  }
  NT_D NT_INLINE void get_prefix(int j, fe& a) const {
    uint32_t w[12];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint4 v = *at(j, 7 + q);
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) a.v[i] = w[2 + i];
  }
};

// The launch's verdict epilogue (round 6): each signature's
// verdict goes straight into the caller's 64-bit words -- a ballot store when a
// row is one word (input order), an atomic OR of its bit when the launch runs
// in key-grouped order (no verdict bytes, no k_pack_bytes launch) -- and a
// rejected signature that lies in a certificate group clears that group's bit
// (the launch's init kernel set every group word to ones), so no k_group_and
// launch follows.  Groups: G ranges [gfirst[g], gfirst[g] + gcnt[g]) of the
// launch's signature indices (offset by ibase), gfirst non-decreasing; a
// signature in no group (a header signature of a mixed launch) only gets its bit.
struct KsVerdict {
  unsigned long long* bits;   // the launch's verdict words
  uint8_t* bytes;             // key-grouped order with the separate pack launch (NT_KEYSET_PACK=1), else null
  const uint64_t* gfirst;
  const uint32_t* gcnt;
  uint64_t G;
  unsigned long long* gwords;
  uint64_t ibase;             // index of the launch's signature 0 among the groups' indices

  NT_D NT_INLINE void group_fail(uint64_t i) const {
    const uint64_t x = ibase + i;
    if (G == 0 || gfirst[0] > x) return;
    uint64_t lo = 0, hi = G;  // the last group whose first index is <= x
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (gfirst[mid] <= x) lo = mid;
      else hi = mid;
    }
    if (x < gfirst[lo] + gcnt[lo]) atomicAnd(&gwords[lo >> 6], ~(1ull << (lo & 63)));
  }
  // signature i of the launch (key-grouped order: its own index), verdict ok
  NT_D NT_INLINE void scattered(uint64_t i, uint32_t ok) const {
    if (bytes) {
      bytes[i] = (uint8_t)ok;
    } else if (ok) {
      atomicOr(&bits[i >> 6], 1ull << (i & 63));
    }
    if (!ok) group_fail(i);
  }
  // row `row` of the launch in input order (lane = its signature), this lane's verdict ok
  NT_D NT_INLINE void row(uint64_t row, uint32_t lane, uint32_t ok, uint64_t n) const {
    const uint64_t gi = 64 * row + lane;
    const unsigned long long bal = __ballot(ok & (gi < n));
    if (lane == 0) bits[row] = bal;
    if (!ok && gi < n) group_fail(gi);
  }
};

// Per-mode launchers, explicitly instantiated in k_verify_<mode>.hip and
// k_keyset_<mode>.hip (one translation unit per kernel family and mode, so
// the build compiles them in parallel); dispatched by launch_verify /
// launch_verify_keyset in k_misc.hip.
// WB = digit width of the comb of B (kBCombBits or kBCombFallback), WA = the
// committee keys' comb width.
template <int MODE, int WB>
hipError_t launch_verify_m(uint64_t blocks, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                           uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                           const uint32_t* d_combB, void* d_ws, uint64_t* d_out_words, hipStream_t s, int per_lane);
template <int MODE, int WA, int WB>
hipError_t launch_keyset_m(const KsPlan& plan, const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                           uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n, const uint32_t* d_meta,
                           const uint32_t* d_enc, const uint32_t* d_combA, uint32_t nkeys,
                           const uint32_t* d_combB, void* d_stash, const uint32_t* d_perm, const KsVerdict& vd,
                           uint32_t* d_chunk_ctr, hipStream_t s);
int keyset_occupancy();

// Occupancy variants (waves per SIMD the register allocator targets), chosen
// at run time for A/B measurement: NT_VERIFY_OCC in {1, 2, 3} (default 2),
// NT_KEYSET_OCC in {2, 3} (default 3).
inline int env_occ(const char* name, int dflt, int lo, int hi) {
  const char* e = std::getenv(name);
  const int v = e ? std::atoi(e) : dflt;
  return v < lo || v > hi ? dflt : v;
}

}  // namespace nt
