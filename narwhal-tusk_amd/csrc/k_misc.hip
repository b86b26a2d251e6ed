// k_misc.hip -- gfx950 kernels of the Narwhal/Tusk crypto hot path other than
// verification (which lives in k_verify_*.hip / k_keyset_*.hip), plus every
// host launcher.  Kernel map of the library:
//
//   k_sha512_pipe         few long messages: producer wave (K+W into LDS) + consumer wave (rounds)
//   k_sha512_trunc32      many messages: one lane per message, Digest = SHA-512[..32]
//                         (worker/src/processor.rs:38; primary/src/messages.rs:70-84,145-153,226-234)
//   k_ed25519_verify<M>   two signatures per lane, half-size scalars; M = strict
//                         (crypto/src/lib.rs:200-204 -> dalek verify_strict) or cofactorless
//                         (per-entry rule of crypto/src/lib.rs:206-219 -> dalek verify_batch,
//                         SURVEY.md A.3); one verdict bit per signature (64-bit ballot words)
//   k_ed25519_verify_keyset<M>  the same against a committee key cache (wide combs of -A),
//                         persistent waves streaming rows, one (binary-GCD) inversion per wave batch
//   k_group_and           AND of per-signature bits over each certificate's vote range
//   k_group_msgs          per-signature message offset/length of certificate groups
//   k_ed25519_sign        keygen + RFC 8032 signing (corpus generation / SignatureService
//                         batch form; crypto/src/lib.rs:163-191) -- not constant time
//   k_wcomb_bases/fill    wide-comb construction (B once per device, committee keys)
//   k_clock_probe         diagnostics: the shader clock under a fixed multiply load (bench.py)
//
// SIMT design: every lane runs the same window schedule (fixed signed windows,
// a wave-uniform window count, never per-lane sliding windows), so lanes of a
// wave never diverge inside the scalar multiplications.  [v s]B is 11 mixed
// additions from the 11.8 GB 24-bit wide comb of B (random 128-byte lines, the
// next one prefetched during the current addition); [u](+-A) + [v](-R) use
// joint 4-bit windows over per-lane 9-entry cached tables in a global
// workspace laid out lane-major, so a lookup's loads use whole lines.
#include <algorithm>

#include "kernels_common.hpp"

namespace nt {

// --------------------------------------------------------------------------
// SHA-512 digests
// --------------------------------------------------------------------------
// digest of an out-of-bounds item (msg_slice): 32 zero bytes, counted in *bad
// (when the caller passed a counter) -- the message is never read
NT_D NT_INLINE void sha512_put(uint32_t* __restrict__ out, uint64_t i, const uint64_t st[8], uint32_t ok,
                               uint32_t* __restrict__ bad) {
  uint32_t w[8];
  sha512_out_words(w, st, 8);
#pragma unroll
  for (int q = 0; q < 8; ++q) w[q] = ok ? w[q] : 0u;
  uint4* o = (uint4*)(out + 8 * i);
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
  if (!ok && bad) atomicAdd(bad, 1u);
}
template <bool kOneSite>
NT_D NT_INLINE void sha512_trunc32_one(const uint8_t* __restrict__ data, uint64_t data_bytes,
                                       const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint64_t n,
                                       uint32_t* __restrict__ out, uint32_t* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const MsgSlice ms = msg_slice(off[i], len[i], data_bytes);
  uint64_t st[8];
  if (kOneSite) sha512_prefixed_1site<0>(st, nullptr, data + ms.off, ms.len);
  else sha512_prefixed<0>(st, nullptr, data + ms.off, ms.len);
  sha512_put(out, i, st, ms.ok, bad);
}
__global__ __launch_bounds__(kBlock) void k_sha512_trunc32(const uint8_t* __restrict__ data, uint64_t data_bytes,
                                                          const uint64_t* __restrict__ off,
                                                          const uint64_t* __restrict__ len,
                                                          uint64_t n, uint32_t* __restrict__ out,
                                                          uint32_t* __restrict__ bad) {
  aux_priority();
  sha512_trunc32_one<false>(data, data_bytes, off, len, n, out, bad);
}
// The same in at most 80 VGPRs (6 waves per SIMD; one compression site, ~184 B
// of spills per lane) against the general kernel's 165, for launches of at most
// kLeanMaxMsgs messages (one wave per SIMD of a 256-CU device): such a launch is
// latency-bound, and beside a key-cache launch of two waves per SIMD (2 x 216 of
// a SIMD's 512 VGPRs) the 80-VGPR kernel is placed at once instead of after that
// launch's waves exit -- config 3's shards run the header-id digests (12.5k -
// 50k x 3.3 KB, side streams) beside the other stream's key-cache launch.
// Larger launches keep the general kernel: the full config-3 step's 100k header
// digests ran ~1 % slower spilling (profiles/r05/ab_sha_lean_r05.txt).
// NT_SHA_LEAN_MSGS overrides the bound (0: never); -DNT_SHA_LEAN_MAX=0 builds it out.
#ifndef NT_SHA_LEAN_MAX
#define NT_SHA_LEAN_MAX 1
#endif
#if NT_SHA_LEAN_MAX > 0
__global__ __launch_bounds__(kBlock, 6) void k_sha512_trunc32_lean(const uint8_t* __restrict__ data,
                                                                   uint64_t data_bytes,
                                                                   const uint64_t* __restrict__ off,
                                                                   const uint64_t* __restrict__ len,
                                                                   uint64_t n, uint32_t* __restrict__ out,
                                                                   uint32_t* __restrict__ bad) {
  aux_priority();
  sha512_trunc32_one<true>(data, data_bytes, off, len, n, out, bad);
}
#endif

// Few long messages (n <= kPipeMaxMsgs, e.g. config 4: 16,384 x 500 kB): one
// lane per message is latency-bound (the per-block instruction stream of a
// wave alone on its SIMD), so the work of a block is split over two waves of
// a 128-thread workgroup that hold the same 64 messages.  Wave 0 (producer)
// loads block b and expands K[t] + W[t], t < 80, into an LDS ring slot; wave 1
// (consumer) runs the 80 rounds of block b-1 from the other slot.  One
// s_barrier per block; the consumer's stream is ~2/3 of the one-wave stream.
constexpr int kPipeMaxMsgs = 32768;  // 80 KB LDS per workgroup: 2 per CU
// ... and only for long messages: when every message is known to be shorter
// (headers, votes and certificate digests: 72 B - 3.3 KB) the one-lane kernel
// (no LDS) runs -- a pipe launch's 80 KB workgroups can hold a CU's LDS while a
// key-cache launch of another stream runs there, and a short digest launch
// queued behind them then waits for that launch's tail (rocprofv3 trace,
// DESIGN.md §10).
constexpr uint64_t kPipeMinLen = 16384;
struct KwLdsSink {
  uint4* slot;  // [40][64]
  uint32_t lane;
  template <int P>
  NT_D NT_INLINE void put(uint64_t kw0, uint64_t kw1) {
    slot[P * 64 + lane] = make_uint4((uint32_t)kw0, (uint32_t)(kw0 >> 32), (uint32_t)kw1, (uint32_t)(kw1 >> 32));
  }
};
// The consumer keeps kKwAhead LDS reads in flight: consuming pair P issues the
// read of pair P + kKwAhead, so each read has ~2 kKwAhead rounds of work to
// land in and the wait before a round is (almost) never a stall.  (Reading a
// pair only when its rounds start left ~100 cycles of LDS latency per 4
// rounds; reading all 40 up front makes one wait for 40 KB per block.)
constexpr int kKwAhead = 12;  // <= 15: the lgkmcnt counter tracks every read in flight
struct KwPrefetchSource {
  const uint4* lds;  // this lane's pair 0 in the ring slot (pairs 64 uint4 apart)
  uint4* q;          // [40] registers
  template <int P>
  NT_D NT_INLINE void get(uint64_t& kw0, uint64_t& kw1) const {
    if constexpr (P + kKwAhead < 40) q[P + kKwAhead] = lds[(P + kKwAhead) * 64];
    kw0 = ((uint64_t)q[P].y << 32) | q[P].x;
    kw1 = ((uint64_t)q[P].w << 32) | q[P].z;
  }
};

__global__ __launch_bounds__(128) void k_sha512_pipe(const uint8_t* __restrict__ data, uint64_t data_bytes,
                                                     const uint64_t* __restrict__ off,
                                                     const uint64_t* __restrict__ len, uint64_t n,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ bad) {
  aux_priority();
  __shared__ uint4 ring[2][40 * 64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  const uint64_t gi = (uint64_t)blockIdx.x * 64 + lane;
  const bool act = gi < n;
  const uint64_t i = act ? gi : n - 1;
  const MsgSlice ms = msg_slice(off[i], len[i], data_bytes);
  const uint8_t* msg = data + ms.off;
  const uint64_t ln = ms.len;
  const uint64_t nblocks = (ln + 17 + 127) / 128;
  const uint64_t nfull = ln / 128;
  // trip count shared by both waves (same 64 messages): max over the lanes
  uint32_t nb = (uint32_t)nblocks;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t y = __shfl_xor(nb, o);
    nb = nb > y ? nb : y;
  }
  nb = __builtin_amdgcn_readfirstlane(nb);
  if (wave == 0) {
    // full blocks are prefetched one block ahead (HBM latency ~ half a block's work)
    uint32_t pre[32];
    if (nfull > 0) load_words<32>(pre, msg);
#pragma unroll 1
    for (uint32_t it = 0; it <= nb; ++it) {
      if (it < nb) {
        uint32_t blk[32];
        if (it < nfull) {
#pragma unroll
          for (int q = 0; q < 32; ++q) blk[q] = pre[q];
          if (it + 1 < nfull) load_words<32>(pre, msg + 128 * (uint64_t)(it + 1));
        } else {
          sha512_tail_block<0>(blk, nullptr, msg, ln, it, it + 1 == nblocks);
        }
        uint64_t W[16];
        sha512_block_w(W, blk);
        KwLdsSink sink{ring[it & 1], lane};
        sha_kw_pairs<0>(W, sink);
      }
      __syncthreads();
    }
  } else {
    uint64_t st[8];
    sha512_init(st);
#pragma unroll 1
    for (uint32_t it = 0; it <= nb; ++it) {
      if (it > 0) {
        const uint32_t b = it - 1;
        uint64_t v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = st[q];
        uint4 q[40];
        const uint4* lds = ring[b & 1] + lane;
#pragma unroll
        for (int p = 0; p < kKwAhead; ++p) q[p] = lds[p * 64];
        const KwPrefetchSource src{lds, q};
        sha_rounds_kw<0>(v, src);
        const bool upd = b < nblocks;
#pragma unroll
        for (int q = 0; q < 8; ++q) st[q] = upd ? add64(st[q], v[q]) : st[q];
      }
      __syncthreads();
    }
    if (act) sha512_put(out, gi, st, ms.ok, bad);
  }
}

// --------------------------------------------------------------------------
// Wide-comb construction
// --------------------------------------------------------------------------
// One thread per point: decode (or take B), optionally negate, write the
// kPos bases 2^(W i) P.  meta[key] gets the kKey* bits.  Keys that do not decode get
// identity bases (every entry the identity; such keys always reject via meta).
// Reduced-scalar combs (CombGeom::kReduced) also get the point's [L]P entry
// after their positions and, in meta, kKeyTorsion when it is not the identity.
template <int W>
__global__ void k_wcomb_bases(const uint32_t* __restrict__ enc, uint32_t nkeys, int negate,
                              uint32_t* __restrict__ bases, uint32_t* __restrict__ meta, uint32_t* __restrict__ comb) {
  const uint32_t key = blockIdx.x * blockDim.x + threadIdx.x;
  if (key >= nkeys) return;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = enc[8 * key + i];
  ge_p3 P;
  const uint32_t ok = ge_frombytes_w(P, w);
  uint32_t m = (ok ? kKeyDecodes : 0u) | (ge_is_small_order(P) ? kKeySmallOrder : 0u);
  if (!ok) ge_p3_0(P);
  if (negate) {
    fe_neg(P.X, P.X);
    fe_carry(P.X);
    fe_neg(P.T, P.T);
    fe_carry(P.T);
  }
  if (CombGeom<W>::kReduced) {
    ge_niels q;
    m |= wcomb_corr(q, P) ? kKeyTorsion : 0u;
    uint32_t* o = comb + (size_t)key * CombGeom<W>::kWordsPerPoint + CombGeom<W>::kCorrWord;
#pragma unroll
    for (int l = 0; l < 10; ++l) { o[l] = q.ypx.v[l]; o[10 + l] = q.ymx.v[l]; o[20 + l] = q.xy2d.v[l]; }
    o[30] = 0;
    o[31] = 0;
  }
  if (meta) meta[key] = m;
  wcomb_bases<W>(bases + (size_t)key * CombGeom<W>::kPos * 40, P);
}

// One thread per (key, position, chunk of 64 entries).
template <int W>
__global__ void k_wcomb_fill(const uint32_t* __restrict__ bases, uint32_t nkeys, uint32_t* __restrict__ comb,
                             uint32_t* __restrict__ tmp) {
  using G = CombGeom<W>;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t per_key = (uint64_t)G::kPos * G::kChunks;
  if (t >= per_key * nkeys) return;
  const uint32_t key = (uint32_t)(t / per_key);
  const uint32_t pos = (uint32_t)((t % per_key) / G::kChunks);
  const uint32_t c = (uint32_t)(t % G::kChunks);
  uint32_t* dst = comb + key * G::kWordsPerPoint + ((size_t)pos * G::kEntries + 1 + (size_t)kWChunk * c) * kWStride;
  wcomb_fill<W>(dst, tmp + t * (kWChunk * 10), bases + ((size_t)key * G::kPos + pos) * 40, c);
}

// --------------------------------------------------------------------------
// Certificate groups: AND of the per-signature bits in [first, first + cnt)
// --------------------------------------------------------------------------
// Per-signature message slices of certificate groups (message g = 32 bytes at
// 32 g): the host entry points send first/cnt per group instead of 16 bytes of
// offset/length per signature over PCIe.
// One wave per group: the lanes write the group's consecutive entries, so
// the stores of a wave are contiguous (a thread per group strided them by
// cnt x 8 bytes: one cache line per lane per store).
__global__ __launch_bounds__(kBlock) void k_group_msgs(const uint64_t* __restrict__ first,
                                                      const uint32_t* __restrict__ cnt, uint64_t G,
                                                      uint64_t* __restrict__ off, uint64_t* __restrict__ len) {
  aux_priority();
  const uint64_t g = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  if (g >= G) return;
  const uint64_t f = first[g], c = cnt[g];
  for (uint64_t q = lane; q < c; q += 64) {
    off[f + q] = 32 * g;
    len[f + q] = 32;
  }
}

__global__ __launch_bounds__(kBlock) void k_group_and(const uint64_t* __restrict__ first,
                                                     const uint32_t* __restrict__ cnt, uint64_t G,
                                                     const unsigned long long* __restrict__ sig_bits,
                                                     unsigned long long* __restrict__ out_bits) {
  aux_priority();
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
template <int WB>
__global__ __launch_bounds__(kBlock) void k_ed25519_sign(const uint32_t* __restrict__ seed,
                                                        const uint8_t* __restrict__ msg, uint64_t msg_bytes,
                                                        const uint64_t* __restrict__ off,
                                                        const uint64_t* __restrict__ len, uint64_t n,
                                                        const uint32_t* __restrict__ combB,
                                                        uint32_t* __restrict__ out_pk,
                                                        uint32_t* __restrict__ out_sig) {
  const WideComb<WB> wb{combB};
  for (uint64_t base = (uint64_t)blockIdx.x * kBlock; base < n; base += (uint64_t)gridDim.x * kBlock) {
    const uint64_t gi = base + threadIdx.x;
    const uint32_t active = gi < n;
    const uint64_t i = active ? gi : n - 1;
    uint32_t sw[8];
    ld8(sw, seed + 8 * i);
    uint32_t Aw[8], Rw[8], s[8];
    // an out-of-bounds message (msg_slice): nothing read, an all-zero signature
    const MsgSlice ms = msg ? msg_slice(off[i], len[i], msg_bytes) : MsgSlice{0, 0, 1};
    sign_one(Aw, Rw, s, sw, msg ? msg + ms.off : nullptr, ms.len, wb);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      Rw[q] = ms.ok ? Rw[q] : 0u;
      s[q] = ms.ok ? s[q] : 0u;
    }
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
// Clock probe (nt_dev_clock_probe): the verify kernels' instruction mix --
// v_mad_u64_u32 partial products with 64-bit carry shifts and adds -- on every
// SIMD at two waves per SIMD for `iters` x 16 steps of 4 independent chains;
// each wave stamps the shader-clock counter (one tick per shader cycle) and the
// 100 MHz wall-clock counter around its loop and adds the differences to out[0]
// / out[1] (zeroed by the launcher).  Their ratio is the clock the chip holds
// under this load (MI355X_MICROARCH.md "DVFS give-back" item 6).
// --------------------------------------------------------------------------
NT_D NT_INLINE uint64_t stamp_cycles() {
  uint64_t t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
NT_D NT_INLINE uint64_t stamp_wall() {
  uint64_t t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ __launch_bounds__(kBlock, 2) void k_clock_probe(uint32_t iters, uint32_t seed,
                                                          unsigned long long* __restrict__ out) {
  const uint32_t x0 = seed ^ (threadIdx.x * 0x9e3779b9u), x1 = x0 * 3u + 1u, x2 = x0 * 5u + 7u, x3 = x0 * 9u + 3u;
  uint64_t a0 = x0, a1 = x1, a2 = x2, a3 = x3;
  const uint64_t c0 = stamp_cycles(), w0 = stamp_wall();
#pragma unroll 1
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a0 = (uint64_t)(uint32_t)a0 * x1 + (a0 >> 26);
      a1 = (uint64_t)(uint32_t)a1 * x2 + (a1 >> 26);
      a2 = (uint64_t)(uint32_t)a2 * x3 + (a2 >> 26);
      a3 = (uint64_t)(uint32_t)a3 * x0 + (a3 >> 26);
    }
  }
  const uint64_t c1 = stamp_cycles(), w1 = stamp_wall();
  if ((threadIdx.x & 63u) == 0) {
    atomicAdd(&out[0], (unsigned long long)(c1 - c0));
    atomicAdd(&out[1], (unsigned long long)(w1 - w0));
  }
  if ((a0 ^ a1 ^ a2 ^ a3) == 0x5a5a5a5a5a5a5a5aull) atomicAdd(&out[0], 1ull);  // keeps the chains live
}

hipError_t launch_clock_probe(uint32_t iters, uint32_t cus, uint64_t* d_out2, hipStream_t s) {
  hipError_t e = hipMemsetAsync(d_out2, 0, 16, s);
  if (e != hipSuccess) return e;
  const uint32_t blocks = cus * 4 * 2 * 64 / kBlock;  // two waves per SIMD
  hipLaunchKernelGGL(k_clock_probe, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, iters, 0x2545f491u,
                     (unsigned long long*)d_out2);
  return hipGetLastError();
}

// --------------------------------------------------------------------------
// Launchers (host)
// --------------------------------------------------------------------------
hipError_t launch_sha512_trunc32(const uint8_t* d_data, uint64_t data_bytes, const uint64_t* d_off,
                                 const uint64_t* d_len, uint64_t n, uint8_t* d_out32, hipStream_t s, uint64_t max_len,
                                 uint32_t* d_bad) {
  if (n == 0) return hipSuccess;
  if (n <= (uint64_t)kPipeMaxMsgs && max_len >= kPipeMinLen && !std::getenv("NT_SHA_NO_PIPE")) {
    hipLaunchKernelGGL(k_sha512_pipe, dim3((uint32_t)((n + 63) / 64)), dim3(128), 0, s, d_data, data_bytes, d_off,
                       d_len, n, (uint32_t*)d_out32, d_bad);
    return hipGetLastError();
  }
  const uint64_t blocks = (n + kBlock - 1) / kBlock;
#if NT_SHA_LEAN_MAX > 0
  static const uint64_t lean_max = (uint64_t)env_occ("NT_SHA_LEAN_MSGS", 65536, 0, 1 << 30);
  if (n <= lean_max) {
    hipLaunchKernelGGL(k_sha512_trunc32_lean, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_data, data_bytes, d_off,
                       d_len, n, (uint32_t*)d_out32, d_bad);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL(k_sha512_trunc32, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_data, data_bytes, d_off, d_len, n,
                     (uint32_t*)d_out32, d_bad);
  return hipGetLastError();
}

static int verify_occ() {
  static const int occ = env_occ("NT_VERIFY_OCC", 2, 1, 3);
  return occ;
}
static int keyset_occ() {
  static const int occ = env_occ("NT_KEYSET_OCC", 3, 2, 3);
  return occ;
}
int verify_occupancy() { return verify_occ(); }
int keyset_occupancy() { return keyset_occ(); }

hipError_t launch_verify(int mode, const uint8_t* d_pk, const uint8_t* d_sig, const uint8_t* d_msg,
                         uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n,
                         const uint32_t* d_combB, int bbits, void* d_ws, uint32_t ws_slots, uint64_t* d_out_words,
                         hipStream_t s, int per_lane) {
  if (n == 0) return hipSuccess;
  if (!d_combB || !d_ws) return hipErrorInvalidValue;
  const int pl = verify_per_lane_for(per_lane);
  const uint64_t blocks = verify_grid(n, ws_slots, pl);
#define NT_V_ARGS blocks, d_pk, d_sig, d_msg, msg_bytes, d_off, d_len, n, d_combB, d_ws, d_out_words, s, pl
  if (bbits == kBCombBits)
    return mode == kStrict ? launch_verify_m<kStrict, kBCombBits>(NT_V_ARGS)
                           : launch_verify_m<kCofactorless, kBCombBits>(NT_V_ARGS);
  if (bbits == kBCombFallback)
    return mode == kStrict ? launch_verify_m<kStrict, kBCombFallback>(NT_V_ARGS)
                           : launch_verify_m<kCofactorless, kBCombFallback>(NT_V_ARGS);
#undef NT_V_ARGS
  return hipErrorInvalidValue;
}

hipError_t launch_group_and(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G,
                            const uint64_t* d_sig_words, uint64_t* d_group_words, hipStream_t s) {
  if (G == 0) return hipSuccess;
  const uint64_t blocks = (G + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_group_and, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_first, d_cnt, G,
                     (const unsigned long long*)d_sig_words, (unsigned long long*)d_group_words);
  return hipGetLastError();
}

hipError_t launch_group_msgs(const uint64_t* d_first, const uint32_t* d_cnt, uint64_t G, uint64_t* d_off,
                             uint64_t* d_len, hipStream_t s) {
  if (G == 0) return hipSuccess;
  const uint64_t groups_per_block = kBlock / 64;
  const uint64_t blocks = (G + groups_per_block - 1) / groups_per_block;
  hipLaunchKernelGGL(k_group_msgs, dim3((uint32_t)blocks), dim3(kBlock), 0, s, d_first, d_cnt, G, d_off, d_len);
  return hipGetLastError();
}

hipError_t launch_sign(const uint8_t* d_seed, const uint8_t* d_msg, uint64_t msg_bytes, const uint64_t* d_off,
                       const uint64_t* d_len, uint64_t n, const uint32_t* d_combB, int bbits, uint8_t* d_pk,
                       uint8_t* d_sig, uint32_t max_blocks, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (!d_combB) return hipErrorInvalidValue;
  uint64_t blocks = (n + kBlock - 1) / kBlock;
  if (blocks > max_blocks) blocks = max_blocks;
#define NT_SIGN_LAUNCH(WB)                                                                              \
  hipLaunchKernelGGL(k_ed25519_sign<WB>, dim3((uint32_t)blocks), dim3(kBlock), 0, s,                   \
                     (const uint32_t*)d_seed, d_msg, msg_bytes, d_off, d_len, n, d_combB, (uint32_t*)d_pk, (uint32_t*)d_sig)
  if (bbits == kBCombBits) NT_SIGN_LAUNCH(kBCombBits);
  else if (bbits == kBCombFallback) NT_SIGN_LAUNCH(kBCombFallback);
  else return hipErrorInvalidValue;
#undef NT_SIGN_LAUNCH
  return hipGetLastError();
}

// Builds the W-bit wide combs of nkeys points, `batch` keys per fill launch (tmp
// must hold wcomb_fill_tmp_bytes_per_key(W) * batch bytes; bases nkeys *
// wcomb_bases_bytes_per_key(W)).
template <int W>
static hipError_t wcomb_build(const uint32_t* d_enc, uint32_t nkeys, int negate, uint32_t* d_comb,
                              uint32_t* d_meta, uint32_t* d_bases, uint32_t* d_tmp, uint32_t batch, hipStream_t s) {
  using G = CombGeom<W>;
  hipLaunchKernelGGL(k_wcomb_bases<W>, dim3((nkeys + 63) / 64), dim3(64), 0, s, d_enc, nkeys, negate, d_bases,
                     d_meta, d_comb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  for (uint32_t k0 = 0; k0 < nkeys; k0 += batch) {
    const uint32_t nk = nkeys - k0 < batch ? nkeys - k0 : batch;
    const uint64_t threads = (uint64_t)nk * G::kPos * G::kChunks;
    hipLaunchKernelGGL(k_wcomb_fill<W>, dim3((uint32_t)((threads + 63) / 64)), dim3(64), 0, s,
                       d_bases + (size_t)k0 * G::kPos * 40, nk, d_comb + (size_t)k0 * G::kWordsPerPoint, d_tmp);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_wcomb_build(int bits, const uint32_t* d_enc, uint32_t nkeys, int negate, uint32_t* d_comb,
                              uint32_t* d_meta, uint32_t* d_bases, uint32_t* d_tmp, uint32_t batch,
                              hipStream_t s) {
  if (nkeys == 0) return hipSuccess;
  if (batch == 0) return hipErrorInvalidValue;
  switch (bits) {
    case kKeyCombReduced:
      return wcomb_build<kKeyCombReduced>(d_enc, nkeys, negate, d_comb, d_meta, d_bases, d_tmp, batch, s);
    case kKeyCombWide: return wcomb_build<kKeyCombWide>(d_enc, nkeys, negate, d_comb, d_meta, d_bases, d_tmp, batch, s);
    case kKeyCombMid: return wcomb_build<kKeyCombMid>(d_enc, nkeys, negate, d_comb, d_meta, d_bases, d_tmp, batch, s);
    case kBCombBits: return wcomb_build<kBCombBits>(d_enc, nkeys, negate, d_comb, d_meta, d_bases, d_tmp, batch, s);  // B only
    case kKeyCombNarrow:
      return wcomb_build<kKeyCombNarrow>(d_enc, nkeys, negate, d_comb, d_meta, d_bases, d_tmp, batch, s);
    default: return hipErrorInvalidValue;
  }
}

// signatures per key-cache launch (a multiple of 64: verdict words stay aligned)
constexpr uint64_t kKsMaxPerLaunch = 8ull << 20;

// --------------------------------------------------------------------------
// Key-grouped order for key-cache launches.  A wave's 256 signatures verified
// against 64+ different committee keys make every comb lookup a random 128-B
// line in a random 2 MB page of an 87 GB table set (translation misses on
// most of them); grouped by key, a wave walks one key's 872 MB comb.  Measured
// on config 3 (profiles/r02/ab_keysort): 12.02 -> 9.79 ms per 6.8M-signature
// launch.  A counting sort by committee index (block-local LDS ranks, one
// global reservation per bucket per block) gives slot -> signature; the
// kernel writes one verdict byte at the signature's own index and
// k_pack_bytes turns them into the caller's 64-bit ballot words.
// --------------------------------------------------------------------------
constexpr uint32_t kSortBuckets = 4096;  // committee keys + 1 "unknown" bucket
constexpr uint64_t kSortMin = 65536;     // smaller launches keep the input order
constexpr int kSortTile = 16;            // items per thread of k_key_scatter
constexpr int kHistTile = 16;            // independent key loads in flight per thread of k_key_hist
// Global bucket counters one 128-B line apart: every block's flush / reservation
// is one device-scope atomic per bucket, and with the counters packed 32 to a
// line those atomics serialize per LINE (rocprof r03b: k_key_scatter 66 us at
// 1,661 blocks, ~1.6 ns per atomic on one of 4 lines; k_key_hist 43 us whatever
// the size, one dependent load + LDS atomic per loop iteration).
constexpr uint32_t kCtrStride = 32;

NT_D NT_INLINE uint32_t sort_bucket(uint32_t k, int mixed, uint32_t nkeys) {
  if (mixed) k &= ~kKeyWantStrict;
  return k < nkeys ? k : nkeys;
}

__global__ __launch_bounds__(kBlock) void k_key_hist(const uint32_t* __restrict__ key, uint64_t n, int mixed,
                                                    uint32_t nkeys, uint32_t* __restrict__ hist) {
  aux_priority();
  extern __shared__ uint32_t sort_lds[];  // nkeys + 1 counters (launch_verify_keyset sizes it)
  uint32_t* h = sort_lds;
  for (uint32_t b = threadIdx.x; b <= nkeys; b += kBlock) h[b] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * kHistTile;
  for (uint64_t t0 = (uint64_t)blockIdx.x * kBlock * kHistTile; t0 < n; t0 += stride) {
    uint32_t k[kHistTile];
#pragma unroll
    for (int r = 0; r < kHistTile; ++r) {  // all loads issued before the first is used
      const uint64_t i = t0 + (uint64_t)r * kBlock + threadIdx.x;
      k[r] = i < n ? key[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kHistTile; ++r)
      if (t0 + (uint64_t)r * kBlock + threadIdx.x < n) atomicAdd(&h[sort_bucket(k[r], mixed, nkeys)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b <= nkeys; b += kBlock)
    if (h[b]) atomicAdd(&hist[b * kCtrStride], h[b]);
}

// Each block computes the exclusive prefix of the global histogram itself (the
// counts are final: k_key_hist ran before on the stream) and reserves its
// ranges with one atomic per bucket on the bucket line's second word (zeroed
// with the histogram by one memset): no separate scan launch.
__global__ __launch_bounds__(kBlock) void k_key_scatter(const uint32_t* __restrict__ key, uint64_t n, int mixed,
                                                       uint32_t nkeys, uint32_t* __restrict__ lines,
                                                       uint32_t* __restrict__ perm) {
  aux_priority();
  extern __shared__ uint32_t sort_lds[];  // cnt[nkeys + 1], base[nkeys + 1], part[kBlock]
  const uint32_t nb = nkeys + 1;
  uint32_t* cnt = sort_lds;
  uint32_t* base = sort_lds + nb;
  uint32_t* part = sort_lds + 2 * nb;
  const uint32_t per = (nb + kBlock - 1) / kBlock, b0 = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) sum += lines[b * kCtrStride];
  part[threadIdx.x] = sum;
  for (uint32_t b = threadIdx.x; b <= nkeys; b += kBlock) cnt[b] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int t = 0; t < kBlock; ++t) {
      const uint32_t v = part[t];
      part[t] = acc;
      acc += v;
    }
  }
  __syncthreads();
  {
    uint32_t acc = part[threadIdx.x];
    for (uint32_t b = b0; b < b0 + per && b < nb; ++b) {
      base[b] = acc;
      acc += lines[b * kCtrStride];
    }
  }
  const uint64_t t0 = (uint64_t)blockIdx.x * kBlock * kSortTile;
  uint32_t bk[kSortTile], rk[kSortTile];
#pragma unroll
  for (int r = 0; r < kSortTile; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kBlock + threadIdx.x;
    bk[r] = i < n ? sort_bucket(key[i], mixed, nkeys) : 0u;
    rk[r] = i < n ? atomicAdd(&cnt[bk[r]], 1u) : 0u;
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b <= nkeys; b += kBlock)
    if (cnt[b]) base[b] += atomicAdd(&lines[b * kCtrStride + 1], cnt[b]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSortTile; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kBlock + threadIdx.x;
    if (i < n) perm[base[bk[r]] + rk[r]] = (uint32_t)i;
  }
}

// verdict bytes -> 64-bit ballot words
__global__ __launch_bounds__(kBlock) void k_pack_bytes(const uint8_t* __restrict__ b, uint64_t n,
                                                      unsigned long long* __restrict__ out) {
  aux_priority();
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  const unsigned long long bal = __ballot(i < n && b[i] != 0);
  const uint64_t wbase = i & ~(uint64_t)63;
  if ((threadIdx.x & 63u) == 0 && wbase < n) out[wbase >> 6] = bal;
}

static bool keyset_sort_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NT_KEYSET_SORT");
    return !(e && *e == '0');
  }();
  return on;
}

// d_sort layout: [16 words: row / chunk counter][4096 bucket lines of 32 words: word 0 the
// histogram count, word 1 the scatter's reservation counter][perm m][verdict bytes m]
constexpr size_t kSortHdr = 64;
size_t keyset_sort_bytes(uint64_t n) {
  const uint64_t m = n < kKsMaxPerLaunch ? n : kKsMaxPerLaunch;
  return kSortHdr + (size_t)kSortBuckets * kCtrStride * 4 + (size_t)m * 5 + 64;
}

// NT_KEYSET_STREAM=0 selects the chunked plan (ks_plan) instead of streamed rows
static bool keyset_stream_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NT_KEYSET_STREAM");
    return !(e && *e == '0');
  }();
  return on;
}

KsPlan keyset_plan(uint64_t n, uint32_t cus) {
  // 1 (streamed plan only): one wave per SIMD per launch, for launches that
  // overlap another stream's on the same SIMDs (A/B)
  static const int force = env_occ("NT_KEYSET_WAVES", 0, 1, 3);
  return keyset_stream_enabled() ? ks_stream_plan(n, cus, keyset_per_lane(), force)
                                 : ks_plan(n, cus, keyset_per_lane(), force == 1 ? 2 : force);
}

// A key-cache launch's first kernel: the row counter and, for a key-grouped
// launch, the bucket lines (count + reservation) zeroed; the verdict words of a
// key-grouped launch zeroed (its kernel ORs the accepted bits in); each group
// word set to ones for its groups (the kernel clears a group's bit when one of
// its signatures rejects; a group reaching past the call's n signatures starts
// rejected, as k_group_and would find its missing bits clear).  One launch, as
// the memset it replaces.
__global__ __launch_bounds__(kBlock) void k_ks_init(uint32_t* __restrict__ ctr, uint32_t nctr,
                                                   unsigned long long* __restrict__ sw, uint64_t nsw,
                                                   const uint64_t* __restrict__ gfirst,
                                                   const uint32_t* __restrict__ gcnt, uint64_t G, uint64_t n,
                                                   unsigned long long* __restrict__ gw) {
  aux_priority();
  const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x, stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t i = t; i < nctr; i += stride) ctr[i] = 0u;
  for (uint64_t i = t; i < nsw; i += stride) sw[i] = 0ull;
  // one lane per group, one ballot per word (a wave's 64 lanes are one word:
  // kBlock and the stride are multiples of 64, so the loop is wave-uniform).
  // Round 6's first version looped over a word's 64 groups in one lane: 64
  // loads in a row, 60-80 us per launch beside a key-cache launch (r06p trace).
  const uint64_t ng = (G + 63) / 64 * 64;
  for (uint64_t g = t; g < ng; g += stride) {
    const bool ok = g < G && gfirst[g] + gcnt[g] <= n;
    const unsigned long long bal = __ballot(ok);
    if ((threadIdx.x & 63u) == 0) gw[g >> 6] = bal;
  }
}

// NT_KEYSET_FUSE=0 (A/B): round 5's epilogue -- verdict bytes + k_pack_bytes for a
// key-grouped launch and a k_group_and launch for groups
static bool keyset_fuse() {
  static const bool on = [] {
    const char* e = std::getenv("NT_KEYSET_FUSE");
    return !(e && *e == '0');
  }();
  return on;
}

hipError_t launch_verify_keyset(int mode, int key_bits, const uint32_t* d_key_idx, const uint8_t* d_sig, const uint8_t* d_msg,
                                uint64_t msg_bytes, const uint64_t* d_off, const uint64_t* d_len, uint64_t n, const uint32_t* d_meta,
                                const uint32_t* d_enc, const uint32_t* d_combA, uint32_t nkeys,
                                const uint32_t* d_combB, int bbits, void* d_stash, void* d_sort, uint64_t* d_out_words,
                                uint32_t cus, hipStream_t s, const uint64_t* d_gfirst, const uint32_t* d_gcnt, uint64_t G,
                                uint64_t* d_group_words) {
  if (!d_sort || !d_stash || !d_combB) return hipErrorInvalidValue;
  if (bbits != kBCombBits && bbits != kBCombFallback) return hipErrorInvalidValue;
  if (G && (!d_gfirst || !d_gcnt || !d_group_words)) return hipErrorInvalidValue;
  const bool fuse = keyset_fuse();
  uint32_t* ctr = (uint32_t*)d_sort;
  uint32_t* hist = ctr + kSortHdr / 4;
  uint32_t* p = hist + kSortBuckets * kCtrStride;
  // launches of at most kKsMaxPerLaunch signatures reuse one stash (stream-ordered)
  for (uint64_t lo = 0; lo < n; lo += kKsMaxPerLaunch) {
    const uint64_t m = n - lo < kKsMaxPerLaunch ? n - lo : kKsMaxPerLaunch;
    const KsPlan pl = keyset_plan(m, cus);
    const uint32_t* perm = nullptr;
    const bool sorted = keyset_sort_enabled() && m >= kSortMin && nkeys + 1 <= kSortBuckets;
    const uint64_t gi = fuse && lo == 0 ? G : 0;  // group words: set once, by the first launch's init
    const uint32_t nctr = sorted ? (uint32_t)((kSortHdr + 4ull * kCtrStride * (nkeys + 1)) / 4) : 1u;
    const uint64_t nsw = sorted && fuse ? (m + 63) / 64 : 0;
    const uint64_t most = std::max<uint64_t>(std::max<uint64_t>(nctr, nsw), (gi + 63) / 64 * 64);
    const uint32_t ib = (uint32_t)std::min<uint64_t>(1024, (most + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_ks_init, dim3(ib ? ib : 1), dim3(kBlock), 0, s, ctr, nctr,
                       (unsigned long long*)(d_out_words + lo / 64), nsw, d_gfirst, d_gcnt, gi, n,
                       (unsigned long long*)d_group_words);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (sorted) {
      const int mixed = mode == kMixed;
      // one tile of kHistTile keys per thread and at most 512 blocks (each flushes its
      // LDS histogram with one global atomic per bucket)
      const uint64_t hw = (m + (uint64_t)kBlock * kHistTile - 1) / ((uint64_t)kBlock * kHistTile);
      const uint32_t hb = (uint32_t)(hw < 512 ? hw : 512);
      // LDS sized to the committee (nkeys + 1 buckets), not to kSortBuckets: a
      // 101-key committee's scatter block takes 1.8 KB instead of 33 KB, so it
      // finds room on a CU beside the other stream's key-cache launch
      // (profiles/r06/shard8_trace_r06p.txt: the 33 KB blocks waited ~0.7 ms)
      const size_t hist_lds = 4ull * (nkeys + 1), scat_lds = 4ull * (2ull * (nkeys + 1) + kBlock);
      hipLaunchKernelGGL(k_key_hist, dim3(hb), dim3(kBlock), hist_lds, s, d_key_idx + lo, m, mixed, nkeys, hist);
      const uint64_t sb = (m + (uint64_t)kBlock * kSortTile - 1) / ((uint64_t)kBlock * kSortTile);
      hipLaunchKernelGGL(k_key_scatter, dim3((uint32_t)sb), dim3(kBlock), scat_lds, s, d_key_idx + lo, m, mixed, nkeys,
                         hist, p);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      perm = p;
    }
    const KsVerdict vd{(unsigned long long*)(d_out_words + lo / 64), sorted && !fuse ? (uint8_t*)(p + m) : nullptr,
                       fuse ? d_gfirst : nullptr, fuse ? d_gcnt : nullptr, fuse ? G : 0,
                       (unsigned long long*)d_group_words, lo};
#define NT_KS_ARGS                                                                                           \
  pl, d_key_idx + lo, d_sig + 64 * lo, d_msg, msg_bytes, d_off + lo, d_len + lo, m, d_meta, d_enc, d_combA, nkeys,     \
      d_combB, d_stash, perm, vd, ctr, s
#define NT_KS_MODES(WA, WB)                                                  \
  (mode == kStrict  ? launch_keyset_m<kStrict, WA, WB>(NT_KS_ARGS)            \
   : mode == kMixed ? launch_keyset_m<kMixed, WA, WB>(NT_KS_ARGS)             \
                    : launch_keyset_m<kCofactorless, WA, WB>(NT_KS_ARGS))
#define NT_KS_WIDTHS(WB)                                                     \
  (key_bits == kKeyCombReduced  ? NT_KS_MODES(kKeyCombReduced, WB)           \
   : key_bits == kKeyCombWide   ? NT_KS_MODES(kKeyCombWide, WB)              \
   : key_bits == kKeyCombMid    ? NT_KS_MODES(kKeyCombMid, WB)               \
   : key_bits == kKeyCombNarrow ? NT_KS_MODES(kKeyCombNarrow, WB)            \
                                : hipErrorInvalidValue)
    e = bbits == kBCombBits ? NT_KS_WIDTHS(kBCombBits) : NT_KS_WIDTHS(kBCombFallback);
#undef NT_KS_WIDTHS
#undef NT_KS_MODES
#undef NT_KS_ARGS
    if (e != hipSuccess) return e;
    if (vd.bytes) {
      hipLaunchKernelGGL(k_pack_bytes, dim3((uint32_t)((m + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                         (const uint8_t*)vd.bytes, m, (unsigned long long*)(d_out_words + lo / 64));
      if ((e = hipGetLastError()) != hipSuccess) return e;
    }
  }
  if (G && !fuse) return launch_group_and(d_gfirst, d_gcnt, G, d_out_words, d_group_words, s);
  return hipSuccess;
}

template <int W>
static size_t comb_size(int what) {
  using G = CombGeom<W>;
  switch (what) {
    case 0: return G::kWordsPerPoint * 4;
    case 1: return (size_t)G::kPos * 40 * 4;
    case 2: return (size_t)G::kPos * G::kChunks * kWChunk * 10 * 4;
    default: return (size_t)std::max<uint64_t>(1, (128u << 10) / ((uint64_t)G::kPos * G::kChunks));
  }
}
static size_t comb_size(int bits, int what) {
  return bits == kKeyCombReduced  ? comb_size<kKeyCombReduced>(what)
         : bits == kKeyCombWide   ? comb_size<kKeyCombWide>(what)
         : bits == kKeyCombMid    ? comb_size<kKeyCombMid>(what)
         : bits == kKeyCombNarrow ? comb_size<kKeyCombNarrow>(what)
         : bits == kBCombBits     ? comb_size<kBCombBits>(what)
                                  : 0;
}
size_t wcomb_bytes_per_key(int bits) { return comb_size(bits, 0); }
size_t wcomb_bases_bytes_per_key(int bits) { return comb_size(bits, 1); }
size_t wcomb_fill_tmp_bytes_per_key(int bits) { return comb_size(bits, 2); }
// keys per fill launch: >= 128k threads per launch (16 keys at W = 16, 2 at W = 20)
uint32_t wcomb_fill_batch(int bits) { return (uint32_t)comb_size(bits, 3); }
// verify grid: one 512-signature block per workspace slot, at most ws_slots
int verify_per_lane_for(int per_lane) {
  // NT_VERIFY_NPER=1 (A/B): one signature per lane for every launch that does not ask
  static const int dflt = env_occ("NT_VERIFY_NPER", kVPer, 1, 2);
  const int p = per_lane ? per_lane : dflt;
  return p == 1 && verify_occupancy() == 2 ? 1 : kVPer;
}
uint64_t verify_grid(uint64_t n, uint32_t ws_slots, int per_lane) {
  const uint64_t per = (uint64_t)verify_per_lane_for(per_lane) * kBlock;  // signatures per block iteration
  const uint64_t blocks = (n + per - 1) / per;
  return blocks < ws_slots ? blocks : ws_slots;
}

// signatures one wave of resident workgroups covers (every CU full at the
// kernel's occupancy): launches sized in whole rounds leave no partial last wave
// host-side chunk sizing of the pipelined entry points: 8 rows per wave (round 2's
// grid; the launch plan itself is ks_plan's, whatever the chunk)
uint64_t keyset_round_sigs(uint32_t cus) {
  return (uint64_t)cus * 4 * keyset_occ() * 64 * std::min<uint32_t>(keyset_per_lane(), 8);
}
uint64_t verify_round_sigs(uint32_t cus, int per_lane) {
  return (uint64_t)cus * verify_occupancy() * verify_per_lane_for(per_lane) * kBlock;
}
// most rows (signatures per lane) of a key-cache chunk, one inversion each: 64,
// the plan picks the chunk size (ks_plan.hpp; round-3 A/B in DESIGN.md §5.2);
// NT_KEYSET_PER_LANE in [1, kKsPerLane] caps it for A/B runs
uint32_t keyset_per_lane() {
  static const uint32_t m = (uint32_t)env_occ("NT_KEYSET_PER_LANE", kKsPerLane, 1, kKsPerLane);
  return m;
}
// stash of any launch of at most n signatures (each <= kKsMaxPerLaunch):
// ks_stash_rows_bound rows x 64 lanes x 160 B, an upper bound of every plan's
// waves x stash rows that grows with n (ks_plan.hpp)
size_t keyset_stash_bytes(uint64_t n, uint32_t cus) {
  const uint64_t m = n < kKsMaxPerLaunch ? n : kKsMaxPerLaunch;
  return (size_t)ks_stash_rows_bound((m + 63) / 64, cus) * 64 * kKsQuads * 16;
}
size_t ws_bytes_per_slot() { return (size_t)kAEntries * kAQuads * kBlock * 16; }

}  // namespace nt
