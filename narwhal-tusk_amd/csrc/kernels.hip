// kernels.hip -- gfx950 kernels of the Narwhal/Tusk crypto hot path.
//
//   k_sha512_trunc32      one lane per message, Digest = SHA-512[..32]
//                         (worker/src/processor.rs:38; primary/src/messages.rs:70-84,145-153,226-234)
//   k_ed25519_verify<M>   one lane per signature; M = strict (crypto/src/lib.rs:200-204 ->
//                         dalek verify_strict) or cofactorless (per-entry rule of
//                         crypto/src/lib.rs:206-219 -> dalek verify_batch);
//                         writes one verdict bit per signature (64-bit ballot words)
//   k_group_and           AND of per-signature bits over each certificate's vote range
//   k_ed25519_sign        keygen + RFC 8032 signing (corpus generation / SignatureService
//                         batch form; crypto/src/lib.rs:163-191) -- not constant time
//   k_btab_init           [j]B, j = 0..128, affine-niels table (built once per device)
//
// SIMT design: every lane runs the same window schedule (fixed signed windows,
// never per-lane sliding windows), so lanes of a wave never diverge inside the
// double-scalar ladder.  [s]B uses 8-bit windows over a 129-entry affine table
// staged in LDS (16.5 KiB per workgroup); [k](-A) uses 4-bit windows over a
// per-lane 9-entry cached table in a global workspace laid out lane-minor so
// each lane's 16-byte accesses coalesce across the workgroup.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "ed25519_ops.hpp"
#include "kernels.hpp"

namespace nt {

constexpr int kBlock = 256;
constexpr int kBEntries = 129;        // |digit| in 0..128
constexpr int kBStride = 32;          // words per niels entry (30 used)
constexpr int kAEntries = 9;          // |digit| in 0..8
constexpr int kAQuads = 10;           // uint4 per cached entry (40 words)

// --------------------------------------------------------------------------
// SHA-512 digests
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sha512_trunc32(const uint8_t* __restrict__ data,
                                                          const uint64_t* __restrict__ off,
                                                          const uint64_t* __restrict__ len,
                                                          uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  uint64_t st[8];
  sha512_prefixed<0>(st, nullptr, data + off[i], len[i]);
  uint32_t w[8];
  sha512_out_words(w, st, 8);
  uint4* o = (uint4*)(out + 8 * i);
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// --------------------------------------------------------------------------
// Base-point table: one thread per entry j = 0..128
// --------------------------------------------------------------------------
__global__ void k_btab_init(uint32_t* __restrict__ tab) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= kBEntries) return;
  ge_niels q;
  btab_entry(q, (uint32_t)j);
  uint32_t* dst = tab + (size_t)j * kBStride;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    dst[i] = q.ypx.v[i];
    dst[10 + i] = q.ymx.v[i];
    dst[20 + i] = q.xy2d.v[i];
  }
  dst[30] = 0;
  dst[31] = 0;
}

// --------------------------------------------------------------------------
// Table accessors
// --------------------------------------------------------------------------
// [j]B entries staged in LDS, 32 words per entry (8 x ds_read_b128).
struct LdsBTab {
  const uint32_t* lds;
  NT_D NT_INLINE void load(uint32_t idx, ge_niels& q) const {
    const uint4* e = (const uint4*)(lds + idx * kBStride);
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

// j*(-A) entries in the global workspace, layout [slot][entry][quad][lane] of
// uint4: a lane's 16-byte accesses are adjacent to its neighbours'.
struct WsATab {
  uint4* ws;
  uint32_t slot;
  NT_D NT_INLINE uint4* at(uint32_t entry) const {
    return ws + ((size_t)(slot * kAEntries + entry) * kAQuads) * kBlock + threadIdx.x;
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
      base[(size_t)q * kBlock] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  NT_D NT_INLINE void load(uint32_t entry, ge_cached& c) const {
    uint32_t w[40];
    const uint4* base = at(entry);
#pragma unroll
    for (int q = 0; q < kAQuads; ++q) {
      const uint4 v = base[(size_t)q * kBlock];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c.YpX.v[i] = w[i]; c.YmX.v[i] = w[10 + i]; c.Z2.v[i] = w[20 + i]; c.T2d.v[i] = w[30 + i];
    }
  }
};

NT_D NT_INLINE void load_btab_lds(uint32_t* lds, const uint32_t* __restrict__ btab_g) {
  const uint4* src = (const uint4*)btab_g;
  uint4* dst = (uint4*)lds;
  for (int i = threadIdx.x; i < kBEntries * kBStride / 4; i += kBlock) dst[i] = src[i];
  __syncthreads();
}

NT_D NT_INLINE void load8(uint32_t w[8], const uint32_t* __restrict__ p) {
  const uint4* q = (const uint4*)p;
  const uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

// --------------------------------------------------------------------------
// Verification: one lane per signature, grid-stride over workspace slots
// --------------------------------------------------------------------------
template <int MODE, int OCC>
__global__ __launch_bounds__(kBlock, OCC) void k_ed25519_verify(
    const uint32_t* __restrict__ pk, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint64_t n,
    const uint32_t* __restrict__ btab_g, uint4* __restrict__ ws,
    unsigned long long* __restrict__ out_bits) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[kBEntries * kBStride];
  load_btab_lds(btab, btab_g);
  const LdsBTab bt{btab};
  WsATab at{ws, blockIdx.x};
  for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += (uint64_t)gridDim.x * kBlock) {
    const uint64_t gi = base + threadIdx.x;
    const uint32_t active = gi < n;
    const uint64_t i = active ? gi : n - 1;
    uint32_t Aw[8], Rw[8], Sw[8];
    load8(Aw, pk + 8 * i);
    load8(Rw, sig + 16 * i);
    load8(Sw, sig + 16 * i + 8);
    const uint32_t ok = active & verify_one<MODE>(Aw, Rw, Sw, msg + off[i], len[i], at, bt);
    const unsigned long long bal = __ballot(ok);
    const uint64_t wbase = base + (threadIdx.x & ~63u);
    if ((threadIdx.x & 63u) == 0 && wbase < n) out_bits[wbase >> 6] = bal;
  }
}

// --------------------------------------------------------------------------
// Committee key cache: comb tables  [pos][key][entry][32 words]
// --------------------------------------------------------------------------
// One thread per (key, pos, entry).  sign_neg = 1 builds the comb of -P (keys),
// 0 the comb of P itself (the base point).  meta[key] gets kKey* bits.
__global__ void k_comb_build(const uint32_t* __restrict__ enc, uint32_t nkeys, int negate,
                             uint32_t* __restrict__ comb, uint32_t* __restrict__ meta) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t per_key = (uint64_t)kCombPos * kCombEntries;
  if (t >= per_key * nkeys) return;
  const uint32_t key = (uint32_t)(t / per_key);
  const uint32_t pos = (uint32_t)((t % per_key) / kCombEntries);
  const uint32_t j = (uint32_t)(t % kCombEntries);
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = enc[8 * key + i];
  ge_p3 P;
  const uint32_t ok = ge_frombytes_w(P, w);
  if (pos == 0 && j == 0 && meta) meta[key] = (ok ? kKeyDecodes : 0u) | (ge_is_small_order(P) ? kKeySmallOrder : 0u);
  if (negate) {
    fe_neg(P.X, P.X);
    fe_carry(P.X);
    fe_neg(P.T, P.T);
    fe_carry(P.T);
  }
  ge_niels q;
  if (ok) comb_entry(q, P, pos, j);
  else ge_niels_0(q);
  uint32_t* dst = comb + (((uint64_t)pos * nkeys + key) * kCombEntries + j) * kBStride;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    dst[i] = q.ypx.v[i];
    dst[10 + i] = q.ymx.v[i];
    dst[20 + i] = q.xy2d.v[i];
  }
  dst[30] = 0;
  dst[31] = 0;
}

struct GlobalComb {
  const uint32_t* comb;
  uint32_t nkeys, key;
  NT_D NT_INLINE void load(uint32_t pos, uint32_t idx, ge_niels& q) const {
    const uint4* e = (const uint4*)(comb + (((uint64_t)pos * nkeys + key) * kCombEntries + idx) * kBStride);
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

// Verification against a cached committee: each lane verifies TWO signatures
// (wave w, lane l: signatures 128w + l and 128w + 64 + l) sharing one field
// inversion; key_idx[i] selects the key (>= nkeys -> unknown key -> reject).
template <int MODE>
__global__ __launch_bounds__(kBlock, 2) void k_ed25519_verify_keyset(
    const uint32_t* __restrict__ key_idx, const uint32_t* __restrict__ sig, const uint8_t* __restrict__ msg,
    const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint64_t n,
    const uint32_t* __restrict__ meta, const uint32_t* __restrict__ enc, const uint32_t* __restrict__ combA,
    uint32_t nkeys, const uint32_t* __restrict__ combB, unsigned long long* __restrict__ out_bits) {
  const uint64_t wave = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t act[2], m[2], Aw[2][8], Rw[2][8], Sw[2][8];
  const uint8_t* mp[2];
  uint64_t ml[2];
  GlobalComb ca[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const uint64_t gi = 128 * wave + 64 * j + lane;
    act[j] = gi < n;
    const uint64_t i = act[j] ? gi : n - 1;
    const uint32_t kraw = key_idx[i];
    const uint32_t known = kraw < nkeys;
    const uint32_t key = known ? kraw : 0u;
    load8(Aw[j], enc + 8 * key);
    load8(Rw[j], sig + 16 * i);
    load8(Sw[j], sig + 16 * i + 8);
    m[j] = known ? meta[key] : 0u;
    mp[j] = msg + off[i];
    ml[j] = len[i];
    ca[j] = GlobalComb{combA, nkeys, key};
  }
  const GlobalComb cb{combB, 1u, 0u};
  uint32_t ok[2];
  verify_two_cached<MODE>(ok, m, Aw, Rw, Sw, mp, ml, ca, cb);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const unsigned long long bal = __ballot(ok[j] & act[j]);
    const uint64_t wbase = 128 * wave + 64 * j;
    if (lane == 0 && wbase < n) out_bits[wbase >> 6] = bal;
  }
}

// --------------------------------------------------------------------------
// Certificate groups: AND of the per-signature bits in [first, first + cnt)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_group_and(const uint64_t* __restrict__ first,
                                                     const uint32_t* __restrict__ cnt, uint64_t G,
                                                     const unsigned long long* __restrict__ sig_bits,
                                                     unsigned long long* __restrict__ out_bits) {
  const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint32_t ok = 0;
  if (g < G) {
    ok = 1;
    const uint64_t f = first[g];
    const uint64_t e = f + cnt[g];
    for (uint64_t x = f; x < e;) {
      const uint64_t w = x >> 6, sh = x & 63;
      const uint64_t take = (64 - sh) < (e - x) ? (64 - sh) : (e - x);
      const unsigned long long m = (take == 64 ? ~0ull : ((1ull << take) - 1)) << sh;
      ok &= ((sig_bits[w] & m) == m);
      x += take;
    }
  }
  const unsigned long long bal = __ballot(ok);
  const uint64_t wbase = (uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u);
  if ((threadIdx.x & 63u) == 0 && wbase < G) out_bits[wbase >> 6] = bal;
}

// --------------------------------------------------------------------------
// Keygen + signing (RFC 8032 / dalek Keypair::sign)
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_ed25519_sign(const uint32_t* __restrict__ seed,
                                                        const uint8_t* __restrict__ msg,
                                                        const uint64_t* __restrict__ off,
                                                        const uint64_t* __restrict__ len, uint64_t n,
                                                        const uint32_t* __restrict__ btab_g,
                                                        uint32_t* __restrict__ out_pk,
                                                        uint32_t* __restrict__ out_sig) {
  __shared__ __attribute__((aligned(16))) uint32_t btab[kBEntries * kBStride];
  load_btab_lds(btab, btab_g);
  const LdsBTab bt{btab};
  for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += (uint64_t)gridDim.x * kBlock) {
    const uint64_t gi = base + threadIdx.x;
    const uint32_t active = gi < n;
    const uint64_t i = active ? gi : n - 1;
    uint32_t sw[8];
    load8(sw, seed + 8 * i);
    uint32_t Aw[8], Rw[8], s[8];
    const uint8_t* m = msg ? msg + off[i] : nullptr;
    const uint64_t ml = msg ? len[i] : 0;
    sign_one(Aw, Rw, s, sw, m, ml, bt);
    if (active) {
      uint4* po = (uint4*)(out_pk + 8 * i);
      po[0] = make_uint4(Aw[0], Aw[1], Aw[2], Aw[3]);
      po[1] = make_uint4(Aw[4], Aw[5], Aw[6], Aw[7]);
      if (out_sig) {
        uint4* so = (uint4*)(out_sig + 16 * i);
        so[0] = make_uint4(Rw[0], Rw[1], Rw[2], Rw[3]);
        so[1] = make_uint4(Rw[4], Rw[5], Rw[6], Rw[7]);
        so[2] = make_uint4(s[0], s[1], s[2], s[3]);
        so[3] = make_uint4(s[4], s[5], s[6], s[7]);
      }
    }
  }
}

// --------------------------------------------------------------------------
// Launchers (host)
// --------------------------------------------------------------------------
hipError_t launch_btab_init(uint32_t* d_tab, hipStream_t s) {
  hipLaunchKernelGGL(k_btab_init, dim3((kBEntries + 63) / 64), dim3(64), 0, s, d_tab);
  return hipGetLastError();
}

hipError_t launch_sha512_trunc32(const uint8_t* d_data, const uint64_t* d_off, const uint64_t* d_len,
                                 uint64_t n, uint8_t* d_out32, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_sha512_trunc32, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_data, d_off,
                     d_len, n, (uint32_t*)d_out32);
  return hipGetLastError();
}

// Occupancy variant of the verify kernel (waves per SIMD the register
// allocator targets): 1 = no spills, 2 = twice the latency hiding with some
// scratch.  NT_VERIFY_OCC selects at run time (A/B measurement); default 2.
static int verify_occ() {
  static int occ = [] {
    const char* e = std::getenv("NT_VERIFY_OCC");
    return (e && std::atoi(e) == 1) ? 1 : 2;
  }();
  return occ;
}

template <int MODE>
static void launch_verify_mode(uint64_t blocks, const uint8_t* d_pk, const uint8_t* d_sig,
                               const uint8_t* d_msg, const uint64_t* d_off, const uint64_t* d_len,
                               uint64_t n, const uint32_t* d_btab, void* d_ws, uint64_t* d_out_words,
                               hipStream_t s) {
  if (verify_occ() == 1)
    hipLaunchKernelGGL((k_ed25519_verify<MODE, 1>), dim3((uint32_t)blocks), dim3(kBlock), 0, s,
                       (const uint32_t*)d_pk, (const uint32_t*)d_sig, d_msg, d_off, d_len, n, d_btab,
                       (uint4*)d_ws, (unsigned long long*)d_out_words);
  else
    hipLaunchKernelGGL((k_ed25519_verify<MODE, 2>), dim3((uint32_t)blocks), dim3(kBlock), 0, s,
                       (const uint32_t*)d_pk, (const uint32_t*)d_sig, d_msg, d_off, d_len, n, d_btab,
                       (uint4*)d_ws, (unsigned long long*)d_out_words);
}

hipError_t launch_verify(int mode, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                         const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                         const uint32_t* d_btab, void* d_ws, uint32_t ws_slots, uint64_t* d_out_words,
                         hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > ws_slots) blocks = ws_slots;
  if (mode == kStrict)
    launch_verify_mode<kStrict>(blocks, d_pk, d_sig, d_msg, d_off, d_len, n, d_btab, d_ws, d_out_words, s);
  else
    launch_verify_mode<kCofactorless>(blocks, d_pk, d_sig, d_msg, d_off, d_len, n, d_btab, d_ws,
                                      d_out_words, s);
  return hipGetLastError();
}

hipError_t launch_group_and(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G,
                            const uint64_t* d_sig_words, uint64_t* d_group_words, hipStream_t s) {
  if (G == 0) return hipSuccess;
  const uint64_t blocks = (G + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_group_and, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_first, d_cnt, G,
                     (const unsigned long long*)d_sig_words, (unsigned long long*)d_group_words);
  return hipGetLastError();
}

hipError_t launch_sign(const uint8_t* d_seed, const uint8_t* d_msg, const uint64_t* d_off,
                       const uint64_t* d_len, uint64_t n, const uint32_t* d_btab, uint8_t* d_pk,
                       uint8_t* d_sig, uint32_t max_blocks, hipStream_t s) {
  if (n == 0) return hipSuccess;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > max_blocks) blocks = max_blocks;
  hipLaunchKernelGGL(k_ed25519_sign, dim3((uint32_t)blocks), dim3(kBlock), 0, s,
                     (const uint32_t*)d_seed, d_msg, d_off, d_len, n, d_btab, (uint32_t*)d_pk,
                     (uint32_t*)d_sig);
  return hipGetLastError();
}

hipError_t launch_comb_build(const uint32_t* d_enc, uint32_t nkeys, int negate, uint32_t* d_comb,
                             uint32_t* d_meta, hipStream_t s) {
  const uint64_t threads = (uint64_t)nkeys * kCombPos * kCombEntries;
  if (!threads) return hipSuccess;
  hipLaunchKernelGGL(k_comb_build, dim3((uint32_t)((threads + 127) / 128)), dim3(128), 0, s, d_enc, nkeys, negate,
                     d_comb, d_meta);
  return hipGetLastError();
}

hipError_t launch_verify_keyset(int mode, const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                                const uint64_t* d_off, const uint64_t* d_len, uint64_t n, const uint32_t* d_meta,
                                const uint32_t* d_enc, const uint32_t* d_combA, uint32_t nkeys,
                                const uint32_t* d_combB, uint64_t* d_out_words, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t blocks = (n + 2 * kBlock - 1) / (2 * kBlock);  // two signatures per lane
  if (mode == kStrict)
    hipLaunchKernelGGL(k_ed25519_verify_keyset<kStrict>, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_key_idx,
                       (const uint32_t*)d_sig, d_msg, d_off, d_len, n, d_meta, d_enc, d_combA, nkeys, d_combB,
                       (unsigned long long*)d_out_words);
  else
    hipLaunchKernelGGL(k_ed25519_verify_keyset<kCofactorless>, dim3((uint32_t)blocks), dim3(kBlock), 0, s,
                       d_key_idx, (const uint32_t*)d_sig, d_msg, d_off, d_len, n, d_meta, d_enc, d_combA, nkeys,
                       d_combB, (unsigned long long*)d_out_words);
  return hipGetLastError();
}

size_t comb_bytes_per_key() { return (size_t)kCombPos * kCombEntries * kBStride * 4; }

size_t btab_bytes() { return (size_t)kBEntries * kBStride * 4; }
size_t ws_bytes_per_slot() { return (size_t)kAEntries * kAQuads * kBlock * 16; }

}  // namespace nt
