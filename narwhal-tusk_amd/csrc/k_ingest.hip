// k_ingest.hip -- the primary's certificate ingestion on the device (SURVEY
// §8(f).2): bincode PrimaryMessage::Certificate bytes, copied to HBM as they
// arrived from the network (primary/src/primary.rs:225-244), are parsed,
// checked in Certificate::verify's order (primary/src/messages.rs:189-215,
// with Core::sanitize_certificate's round filter, core.rs:339-346) and turned
// into the key-cache launch buffers without a host decode.
//
//   k_cert_parse    one wave per message: layout, base64 key strings -> committee
//                   indices, canonical (strictly increasing) payload / parents,
//                   payload workers; anything irregular -> "host" (the host
//                   decoder decides those messages)
//   k_cert_scan     exclusive scans of the vote counts and preimage lengths
//   k_cert_scatter  one wave per message: the header signature and every vote
//                   (key index, signature, message) into the dense arrays of ONE
//                   NT_MODE_MIXED key-cache launch, the header digest preimage
//                   (author || round || payload || parents) and the certificate
//                   digest preimage, the votes' first reuse / unknown error and
//                   the stake they carry
//   k_cert_verdict  one thread per message: the DagError of the first failing
//                   check, in the reference order
// Message bytes are read with aligned dword loads joined by v_alignbyte (the
// wire buffer keeps 64 bytes of slack on both sides), so messages may start
// at any byte.
#include "kernels_common.hpp"

namespace nt {

namespace {

constexpr uint32_t kMiss = 0xffffffffu;
constexpr uint32_t kCertHost = 1u, kCertWorkersBad = 2u;
constexpr uint32_t kMaxVotes = 1024;        // larger certificates go to the host decoder
constexpr uint64_t kMaxEntries = 1u << 20;  // payload / parents entries (ditto)
constexpr int kWavesPerBlock = kBlock / 64;

// primary::DagError (host/narwhal.hpp; the reference's error.rs variants)
enum : uint32_t {
  kDagOk = 0, kDagInvalidSignature = 1, kDagInvalidHeaderId = 2, kDagMalformedHeader = 3,
  kDagUnknownAuthority = 4, kDagAuthorityReuse = 5, kDagRequiresQuorum = 6, kDagTooOld = 7,
};

NT_D NT_INLINE uint32_t ldu32(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}
NT_D NT_INLINE uint64_t ldu64(const uint8_t* p) { return ldu32(p) | ((uint64_t)ldu32(p + 4) << 32); }
template <int N>
NT_D NT_INLINE void ldwords(const uint8_t* p, uint32_t w[N]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t d[N + 1];
#pragma unroll
  for (int k = 0; k <= N; ++k) d[k] = q[k];
#pragma unroll
  for (int k = 0; k < N; ++k) w[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// committee index of a 44-character key string, kMiss unless it is exactly a
// committee key's canonical base64 text (ingest.cpp's KeyIndex::find_b64:
// first 8 characters hashed, the rest compared)
NT_D uint32_t key_lookup(const CertCommittee& c, const uint8_t* s) {
  uint32_t w[11];
  ldwords<11>(s, w);
  const uint64_t head = w[0] | ((uint64_t)w[1] << 32);
  const uint64_t mask = (1ull << c.sbits) - 1;
  uint64_t i = (head * 0x9E3779B97F4A7C15ull) >> (64 - c.sbits);
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    const uint32_t k = c.slot_idx[i];
    if (k == kMiss) return kMiss;
    if (c.slot_head[i] == head) {
      const uint32_t* e = c.enc + 12 * (size_t)k;
      uint32_t eq = 1;
#pragma unroll
      for (int j = 2; j < 11; ++j) eq &= e[j] == w[j];
      if (eq) return k;
    }
    i = (i + 1) & mask;
  }
  return kMiss;
}

// memcmp order of the 32-byte digests at a and b: < 0, 0, > 0
NT_D int cmp32(const uint8_t* a, const uint8_t* b) {
  uint32_t x[8], y[8];
  ldwords<8>(a, x);
  ldwords<8>(b, y);
  for (int j = 0; j < 8; ++j)
    if (x[j] != y[j]) return __builtin_bswap32(x[j]) < __builtin_bswap32(y[j]) ? -1 : 1;
  return 0;
}

NT_D NT_INLINE bool in_sorted(const uint32_t* v, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) / 2;
    if (v[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && v[lo] == x;
}

NT_D NT_INLINE bool wave_any(bool x) { return __ballot(x) != 0; }

}  // namespace

// Wire layout of PrimaryMessage::Certificate (bincode 1.x, fixint, little
// endian; host/wire.cpp): u32 tag = 2 | u64 44 | author base64 (44) | u64
// round | u64 np | np x (digest 32, worker u32) | u64 nq | nq x digest 32 |
// id 32 | signature 64 | u64 nv | nv x (u64 44 | key base64 (44) | signature 64)
__global__ __launch_bounds__(kBlock) void k_cert_parse(CertCommittee c, CertBufs b) {
  aux_priority();
  const uint64_t i = (uint64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (i >= b.n) return;  // whole waves
  const uint8_t* p = b.wire + b.moff[i];
  const uint64_t L = b.mlen[i];
  bool host = false, wbad = false;
  uint32_t author = 0;
  uint64_t round = 0, np = 0, nq = 0, nv = 0, off_par = 0, off_votes = 0;
  // every value below is the same in all lanes (wave-uniform control flow)
  if (L < 72 || ldu32(p) != 2u || ldu64(p + 4) != 44u) host = true;
  if (!host) {
    author = key_lookup(c, p + 12);
    round = ldu64(p + 56);
    np = ldu64(p + 64);
    uint64_t pos = 72;
    if (author == kMiss || np > (L - pos) / 36 || np > kMaxEntries) {
      host = true;
    } else {
      pos += 36 * np;
      if (L - pos < 8) {
        host = true;
      } else {
        nq = ldu64(p + pos);
        pos += 8;
        if (nq > (L - pos) / 32 || nq > kMaxEntries) {
          host = true;
        } else {
          off_par = pos;
          pos += 32 * nq;
          if (L - pos < 104) {
            host = true;
          } else {
            pos += 96;
            nv = ldu64(p + pos);
            pos += 8;
            if (nv > (L - pos) / 116 || nv > kMaxVotes) host = true;
            off_votes = pos;
          }
        }
      }
    }
  }
  if (!host) {
    bool bad = false;
    for (uint64_t v = lane; v < nv; v += 64) {
      const uint8_t* q = p + off_votes + 116 * v;
      if (ldu64(q) != 44u || key_lookup(c, q + 8) == kMiss) bad = true;
    }
    const uint32_t w0 = c.wfirst[author], wn = c.wfirst[author + 1] - w0;
    for (uint64_t k = lane; k < np; k += 64) {
      const uint8_t* e = p + 72 + 36 * k;
      if (k && cmp32(e - 36, e) >= 0) bad = true;  // BTreeMap order, no repeats
      if (!in_sorted(c.wids + w0, wn, ldu32(e + 32))) wbad = true;
    }
    for (uint64_t k = lane + 1; k < nq; k += 64) {
      const uint8_t* e = p + off_par + 32 * k;
      if (cmp32(e - 32, e) >= 0) bad = true;  // BTreeSet order, no repeats
    }
    host = wave_any(bad);
    wbad = wave_any(wbad);
  }
  if (lane == 0) {
    b.round[i] = round;
    b.author[i] = author;
    b.np[i] = host ? 0u : (uint32_t)np;
    b.nq[i] = host ? 0u : (uint32_t)nq;
    b.nv[i] = host ? 0u : (uint32_t)nv;
    b.flags[i] = (host ? kCertHost : 0u) | (wbad ? kCertWorkersBad : 0u);
    b.plen[i] = host ? 0u : (uint32_t)(40 + 36 * np + 32 * nq);
  }
}

// exclusive scans (one workgroup): vbase[i] = sum nv[< i], pbase[i] = sum of
// the 16-byte-rounded preimage lengths; [n] = the totals
__global__ __launch_bounds__(1024) void k_cert_scan(CertBufs b) {
  aux_priority();
  __shared__ uint64_t ta[1024], tb[1024];
  const uint32_t t = threadIdx.x;
  const uint64_t n = b.n, per = (n + 1023) / 1024;
  const uint64_t lo = t * per < n ? t * per : n, hi = lo + per < n ? lo + per : n;
  uint64_t x = 0, y = 0;
  for (uint64_t i = lo; i < hi; ++i) {
    x += b.nv[i];
    y += (b.plen[i] + 15u) & ~15u;
  }
  ta[t] = x;
  tb[t] = y;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint64_t u = t >= o ? ta[t - o] : 0, v = t >= o ? tb[t - o] : 0;
    __syncthreads();
    ta[t] += u;
    tb[t] += v;
    __syncthreads();
  }
  uint64_t ex = ta[t] - x, ey = tb[t] - y;
  for (uint64_t i = lo; i < hi; ++i) {
    b.vbase[i] = ex;
    b.pbase[i] = ey;
    ex += b.nv[i];
    ey += (b.plen[i] + 15u) & ~15u;
  }
  if (t == 1023) {
    b.vbase[n] = ta[1023];
    b.pbase[n] = tb[1023];
  }
}

// Launch-buffer entries of message i: signature index i = the header's
// (strict: key | NT_KEY_STRICT_BIT, message = the claimed id), n + vbase[i] +
// v = vote v (cofactorless, message = the certificate digest computed by the
// SHA-512 launch); SHA-512 inputs i (header preimage) and n + i (certificate
// preimage id || round || origin, messages.rs:226-234).
__global__ __launch_bounds__(kBlock) void k_cert_scatter(CertCommittee c, CertBufs b) {
  aux_priority();
  __shared__ uint32_t vkey[kWavesPerBlock][kMaxVotes];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint64_t i = (uint64_t)blockIdx.x * kWavesPerBlock + w;
  if (i >= b.n) return;
  const uint64_t n = b.n;
  const uint32_t fl = b.flags[i];
  const uint8_t* p = b.wire + b.moff[i];
  const uint64_t hid_off = 32 * i, dig_cert = 32 * n + 32 * (n + i), cpre_off = 96 * n + 72 * i;
  uint32_t* sw = (uint32_t*)b.sigs;
  uint32_t* mw = (uint32_t*)b.mbase;
  const uint64_t vb = b.vbase[i];
  if (fl & kCertHost) {  // the host decoder decides this message: inert entries
    if (lane < 16) sw[16 * i + lane] = 0;
    if (lane < 8) mw[hid_off / 4 + lane] = 0;
    if (lane < 18) mw[cpre_off / 4 + lane] = 0;
    if (lane == 0) {
      b.keys[i] = 0x7fffffffu;  // not a committee index: rejects, verdict unused
      b.smoff[i] = hid_off;
      b.smlen[i] = 32;
      b.soff[i] = b.pre_off;
      b.slen[i] = 0;
      b.soff[n + i] = cpre_off;
      b.slen[n + i] = 72;
      b.gfirst[i] = n + vb;
      b.gcnt[i] = 0;
      b.verr[i] = 0;
      b.weight[i] = 0;
    }
    return;
  }
  const uint64_t np = b.np[i], nq = b.nq[i], nv = b.nv[i];
  const uint64_t off_par = 80 + 36 * np, off_id = off_par + 32 * nq, off_sig = off_id + 32, off_votes = off_id + 104;
  const uint32_t a = b.author[i];
  const uint64_t round = b.round[i];
  const uint32_t* raw = c.raw + 8 * (size_t)a;
  if (lane < 16) sw[16 * i + lane] = ldu32(p + off_sig + 4 * lane);
  if (lane < 8) mw[hid_off / 4 + lane] = ldu32(p + off_id + 4 * lane);
  if (lane < 18) {  // id || round_le || origin
    const uint32_t o = 4 * lane;
    mw[cpre_off / 4 + lane] = o < 32 ? ldu32(p + off_id + o)
                              : o < 40 ? (uint32_t)(round >> (o == 32 ? 0 : 32))
                                       : raw[(o - 40) / 4];
  }
  // Header::digest preimage: author || round_le || (digest || worker_le)* || parent*
  // (messages.rs:70-84) -- the canonical wire order is already the map / set order
  const uint64_t plen = 40 + 36 * np + 32 * nq, pay_end = 40 + 36 * np;
  uint32_t* pre = (uint32_t*)(b.mbase + b.pre_off + b.pbase[i]);
  for (uint64_t t = lane; t < plen / 4; t += 64) {
    const uint64_t o = 4 * t;
    pre[t] = o < 32 ? raw[o / 4]
             : o < 40 ? (uint32_t)(round >> (o == 32 ? 0 : 32))
             : o < pay_end ? ldu32(p + 72 + (o - 40))
                           : ldu32(p + off_par + (o - pay_end));
  }
  // votes: key index, signature, message
  for (uint64_t v = lane; v < nv; v += 64) {
    const uint8_t* q = p + off_votes + 116 * v;
    const uint32_t k = key_lookup(c, q + 8);  // found (k_cert_parse)
    vkey[w][v] = k;
    const uint64_t e = n + vb + v;
    b.keys[e] = k;
    b.smoff[e] = dig_cert;
    b.smlen[e] = 32;
    uint32_t s[16];
    ldwords<16>(q + 52, s);
    uint4* d = b.sigs + 4 * e;
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = make_uint4(s[4 * r], s[4 * r + 1], s[4 * r + 2], s[4 * r + 3]);
  }
  __threadfence_block();
  __builtin_amdgcn_wave_barrier();
  // the quorum loop of Certificate::verify (messages.rs:198-211): the first vote
  // whose key was already used (AuthorityReuse) or has no stake (UnknownAuthority)
  uint32_t first = kMiss, wsum = 0;
  for (uint64_t v = lane; v < nv; v += 64) {
    const uint32_t k = vkey[w][v];
    bool reused = false;
    for (uint64_t u = 0; u < v; ++u) reused |= vkey[w][u] == k;
    const uint32_t st = c.stake[k];
    const uint32_t code = reused ? kDagAuthorityReuse : (st == 0 ? kDagUnknownAuthority : 0u);
    if (code && first == kMiss) first = ((uint32_t)v << 8) | code;
    wsum += st;  // Stake is u32 (the mirror's and the reference's type)
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t f2 = __shfl_xor(first, o);
    first = f2 < first ? f2 : first;
    wsum += __shfl_xor(wsum, o);
  }
  if (lane == 0) {
    b.verr[i] = first == kMiss ? 0u : (first & 0xffu);
    b.weight[i] = wsum;
    b.keys[i] = a | kKeyWantStrict;
    b.smoff[i] = hid_off;
    b.smlen[i] = 32;
    b.soff[i] = b.pre_off + b.pbase[i];
    b.slen[i] = plen;
    b.soff[n + i] = cpre_off;
    b.slen[n + i] = 72;
    b.gfirst[i] = n + vb;
    b.gcnt[i] = (uint32_t)nv;
  }
}

NT_D NT_INLINE bool word_bit(const uint64_t* w, uint64_t i) { return (w[i >> 6] >> (i & 63)) & 1u; }

// DagError of message i, first failing check in the reference order: the round
// filter (core.rs:339-342), genesis (messages.rs:190-193), Header::verify's id,
// author, workers and signature (:48-67), the quorum loop (:198-211), the votes'
// verify_batch (:213); 0xff = decided by the host decoder
__global__ __launch_bounds__(kBlock) void k_cert_verdict(CertCommittee c, CertBufs b, uint64_t gc_round) {
  aux_priority();
  const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= b.n) return;
  const uint32_t fl = b.flags[i];
  uint32_t code = kDagOk;
  if (fl & kCertHost) {
    code = 0xffu;
  } else if (b.round[i] < gc_round) {
    code = kDagTooOld;
  } else {
    const uint32_t* hid = (const uint32_t*)(b.mbase + 32 * i);
    const uint32_t* dig = (const uint32_t*)(b.mbase + 32 * b.n + 32 * i);
    uint32_t zero = 1, same = 1;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      zero &= hid[j] == 0u;
      same &= hid[j] == dig[j];
    }
    if (zero && b.round[i] == 0) code = kDagOk;  // a committee member's genesis certificate
    else if (!same) code = kDagInvalidHeaderId;
    else if (c.stake[b.author[i]] == 0) code = kDagUnknownAuthority;
    else if (fl & kCertWorkersBad) code = kDagMalformedHeader;
    else if (!word_bit(b.sig_words, i)) code = kDagInvalidSignature;
    else if (b.verr[i]) code = b.verr[i];
    else if (b.weight[i] < c.quorum) code = kDagRequiresQuorum;
    else if (!word_bit(b.grp_words, i)) code = kDagInvalidSignature;
  }
  b.code[i] = (uint8_t)code;
}

hipError_t launch_cert_parse(const CertCommittee& c, const CertBufs& b, hipStream_t s) {
  if (b.n == 0) return hipSuccess;
  const uint64_t blocks = (b.n + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_cert_parse, dim3((uint32_t)blocks), dim3(kBlock), 0, s, c, b);
  return hipGetLastError();
}
hipError_t launch_cert_scan(const CertBufs& b, hipStream_t s) {
  if (b.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_cert_scan, dim3(1), dim3(1024), 0, s, b);
  return hipGetLastError();
}
hipError_t launch_cert_scatter(const CertCommittee& c, const CertBufs& b, hipStream_t s) {
  if (b.n == 0) return hipSuccess;
  const uint64_t blocks = (b.n + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_cert_scatter, dim3((uint32_t)blocks), dim3(kBlock), 0, s, c, b);
  return hipGetLastError();
}
hipError_t launch_cert_verdict(const CertCommittee& c, const CertBufs& b, uint64_t gc_round, hipStream_t s) {
  if (b.n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_cert_verdict, dim3((uint32_t)((b.n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, c, b,
                     gc_round);
  return hipGetLastError();
}

}  // namespace nt
