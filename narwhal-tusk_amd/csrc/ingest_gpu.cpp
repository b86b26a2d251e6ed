// ingest_gpu.cpp -- C ABI of the certificate ingestion from wire bytes
// (include/ntcrypto.h: nt_committee_*, nt_certificates_ingest; kernels in
// k_ingest.hip).
//
// Per device shard the messages are cut into chunks that alternate between
// the slot's two compute streams.  A chunk is two halves:
//   front: copy the chunk's wire bytes and rebased offsets, parse (one wave per
//          message), scan the vote counts / preimage lengths, copy the two
//          totals back (pinned) and record an event;
//   back:  (needs the vote total V to size the launch) scatter into the launch
//          buffers, one SHA-512 launch (header ids + certificate digests), one
//          NT_MODE_MIXED key-cache launch over n + V signatures, group AND,
//          verdicts, codes back to pinned host memory.
// The host issues front(c) before waiting for front(c - 1)'s totals and
// issuing back(c - 1), so chunk c's PCIe copy and parse run under chunk
// c - 1's signature launch on the other stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "../../include/ntcrypto.h"
#include "kernels.hpp"
#include "runtime.hpp"

using namespace ntrt;

struct nt_committee {
  nt_ctx* ctx = nullptr;
  std::shared_ptr<KsTables> kt;  // the key set's device tables, kept alive by the committee
  uint32_t nkeys = 0, sbits = 0, quorum = 0;
  struct PerDev {
    int ordinal = -1;
    nt::CertCommittee c{};
    void* mem = nullptr;  // one allocation holding every table
  };
  std::vector<PerDev> dev;
  ~nt_committee() {
    for (auto& d : dev) {
      if (d.ordinal < 0 || !d.mem) continue;
      (void)hipSetDevice(d.ordinal);
      (void)hipFree(d.mem);
    }
  }
};

namespace {

// base64 0.13 STANDARD (padded) of 32 bytes: the 44-character text the
// reference's PublicKey serde writes (crypto/src/lib.rs:73-79)
std::string b64_32(const uint8_t* k) {
  static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string s;
  for (int i = 0; i < 32; i += 3) {
    const uint32_t v = ((uint32_t)k[i] << 16) | (i + 1 < 32 ? (uint32_t)k[i + 1] << 8 : 0u) |
                       (i + 2 < 32 ? (uint32_t)k[i + 2] : 0u);
    s += A[(v >> 18) & 63];
    s += A[(v >> 12) & 63];
    s += i + 1 < 32 ? A[(v >> 6) & 63] : '=';
    s += i + 2 < 32 ? A[v & 63] : '=';
  }
  return s;
}

constexpr uint64_t kSlack = 64;  // readable bytes before / after the wire bytes (k_ingest.hip)

struct Side {  // device buffers of one chunk parity, grow-only
  DevBuf wire, moff, mlen, round, u32s, scans, mbase, keys, sigs, smsg, sha, grp, words, code;
  HostBuf tot;
  hipEvent_t ev = nullptr;
};

struct IngestState {
  int ordinal = -1;
  Side side[2];
  HostBuf hoff, hlen, hcode;
  ~IngestState() {
    if (ordinal < 0) return;
    (void)hipSetDevice(ordinal);
    for (auto& s : side) {
      for (DevBuf* b : {&s.wire, &s.moff, &s.mlen, &s.round, &s.u32s, &s.scans, &s.mbase, &s.keys, &s.sigs, &s.smsg,
                        &s.sha, &s.grp, &s.words, &s.code})
        if (b->p) (void)hipFree(b->p);
      if (s.tot.p) (void)hipHostFree(s.tot.p);
      if (s.ev) (void)hipEventDestroy(s.ev);
    }
    for (HostBuf* b : {&hoff, &hlen, &hcode})
      if (b->p) (void)hipHostFree(b->p);
  }
};

// grow a buffer the stream's earlier work may still use: wait for it first
int grow(DevBuf& b, size_t bytes, hipStream_t s) {
  if (bytes <= b.cap) return NT_OK;
  if (b.p && hipStreamSynchronize(s) != hipSuccess) return NT_EHIP;
  return b.ensure(bytes);
}

uint64_t chunk_msgs() {
  const char* e = std::getenv("NT_INGEST_CHUNK");
  const long long v = e ? std::atoll(e) : 6250;
  return (uint64_t)std::max(64ll, v);
}

struct Chunk {
  uint64_t a = 0, b = 0;     // messages [a, b) of the shard
  uint64_t base = 0, span = 0;  // host bytes [base, base + span)
  uint64_t vmax = 0;
  uint64_t lmax = 0;  // longest message (bounds its header preimage)
  nt::CertBufs cb{};
};

}  // namespace

extern "C" {

int nt_committee_create(nt_ctx* ctx, const nt_keyset* ks, const uint32_t* stake, const uint64_t* worker_first,
                        const uint32_t* worker_ids, uint32_t quorum, nt_committee** out) {
  if (!ctx || !ks || ks->ctx != ctx || !out || (!stake && ks->nkeys) || !worker_first) return NT_EINVAL;
  *out = nullptr;
  const uint32_t nk = ks->nkeys;
  auto cm = std::make_unique<nt_committee>();
  cm->ctx = ctx;
  cm->kt = ks->t;
  cm->nkeys = nk;
  cm->quorum = quorum;
  // host tables
  std::vector<uint32_t> enc(12ull * std::max<uint32_t>(nk, 1), 0);
  for (uint32_t k = 0; k < nk; ++k) std::memcpy(&enc[12ull * k], b64_32(&ks->enc[32ull * k]).data(), 44);
  uint32_t sbits = 4;
  while ((1ull << sbits) < 4ull * nk) ++sbits;
  const uint64_t S = 1ull << sbits;
  std::vector<uint64_t> head(S, 0);
  std::vector<uint32_t> sidx(S, 0xffffffffu);
  for (uint32_t k = 0; k < nk; ++k) {
    uint64_t h;
    std::memcpy(&h, &enc[12ull * k], 8);
    uint64_t i = (h * 0x9E3779B97F4A7C15ull) >> (64 - sbits);
    while (sidx[i] != 0xffffffffu) i = (i + 1) & (S - 1);
    head[i] = h;
    sidx[i] = k;
  }
  cm->sbits = sbits;
  std::vector<uint32_t> wfirst(nk + 1, 0), wids;
  for (uint32_t k = 0; k < nk; ++k) {
    if (worker_first[k + 1] < worker_first[k]) return NT_EINVAL;
    std::vector<uint32_t> w(worker_ids + worker_first[k], worker_ids + worker_first[k + 1]);
    std::sort(w.begin(), w.end());
    w.erase(std::unique(w.begin(), w.end()), w.end());
    wids.insert(wids.end(), w.begin(), w.end());
    wfirst[k + 1] = (uint32_t)wids.size();
  }
  std::vector<uint32_t> st(stake, stake + nk);
  // one allocation per device entry: [enc][head][sidx][stake][wfirst][wids]
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_enc = 0, o_head = al(o_enc + enc.size() * 4), o_sidx = al(o_head + S * 8),
               o_st = al(o_sidx + S * 4), o_wf = al(o_st + std::max<size_t>(nk, 1) * 4),
               o_wid = al(o_wf + wfirst.size() * 4), total = al(o_wid + std::max<size_t>(wids.size(), 1) * 4);
  for (size_t d = 0; d < ctx->devs.size(); ++d) {
    Device& dv = *ctx->devs[d];
    nt_committee::PerDev pd;
    pd.ordinal = dv.ordinal;
    if (hipSetDevice(dv.ordinal) != hipSuccess) return NT_EHIP;
    if (hipMalloc(&pd.mem, total) != hipSuccess) return NT_ENOMEM;
    cm->dev.push_back(pd);
    uint8_t* m = (uint8_t*)pd.mem;
    if (hipMemcpy(m + o_enc, enc.data(), enc.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(m + o_head, head.data(), S * 8, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(m + o_sidx, sidx.data(), S * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (nk && hipMemcpy(m + o_st, st.data(), nk * 4ull, hipMemcpyHostToDevice) != hipSuccess) ||
        hipMemcpy(m + o_wf, wfirst.data(), wfirst.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (!wids.empty() && hipMemcpy(m + o_wid, wids.data(), wids.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
      return NT_EHIP;
    nt::CertCommittee& c = cm->dev.back().c;
    c.enc = (const uint32_t*)(m + o_enc);
    c.slot_head = (const uint64_t*)(m + o_head);
    c.slot_idx = (const uint32_t*)(m + o_sidx);
    c.stake = (const uint32_t*)(m + o_st);
    c.wfirst = (const uint32_t*)(m + o_wf);
    c.wids = (const uint32_t*)(m + o_wid);
    c.raw = ks->t->dev[d].d_enc;
    c.nkeys = nk;
    c.sbits = sbits;
    c.quorum = quorum;
  }
  *out = cm.release();
  return NT_OK;
}

void nt_committee_free(nt_committee* cm) { delete cm; }

}  // extern "C"

namespace {

// front half of chunk ch on stream s (see the file comment)
int ingest_front(Device& dv, IngestState& S, Side& sd, Chunk& ch, const nt_committee::PerDev& pd,
                 const uint8_t* data, const uint64_t* off, const uint64_t* len, hipStream_t s) {
  const uint64_t m = ch.b - ch.a;
  uint64_t* ho = S.hoff.as<uint64_t>() + ch.a;
  uint64_t* hl = S.hlen.as<uint64_t>() + ch.a;
  uint64_t mn = UINT64_MAX, mx = 0;
  for (uint64_t i = ch.a; i < ch.b; ++i) {
    if (len[i] == 0) continue;
    mn = std::min(mn, off[i]);
    mx = std::max(mx, off[i] + len[i]);
  }
  if (mn == UINT64_MAX) mn = mx = 0;
  ch.base = mn & ~(uint64_t)15;
  ch.span = mx - ch.base;
  ch.vmax = 0;
  ch.lmax = 0;
  for (uint64_t i = ch.a; i < ch.b; ++i) {
    ho[i - ch.a] = len[i] ? kSlack + off[i] - ch.base : kSlack;
    hl[i - ch.a] = len[i];
    ch.vmax += len[i] / 116;
    ch.lmax = std::max(ch.lmax, len[i]);
  }
  NT_CHK0(grow(sd.wire, ch.span + 2 * kSlack, s));
  NT_CHK0(grow(sd.moff, m * 8, s));
  NT_CHK0(grow(sd.mlen, m * 8, s));
  NT_CHK0(grow(sd.round, m * 8, s));
  NT_CHK0(grow(sd.u32s, m * 4 * 10, s));
  NT_CHK0(grow(sd.scans, (m + 1) * 16, s));
  NT_CHK0(grow(sd.sha, m * 32, s));
  NT_CHK0(grow(sd.grp, m * 8 + (m / 64 + 2) * 8, s));
  NT_CHK0(grow(sd.code, m, s));
  NT_CHK0(sd.tot.ensure(16));
  uint8_t* wire = sd.wire.as<uint8_t>();
  if (ch.span) NT_TRY(hipMemcpyAsync(wire + kSlack, data + ch.base, ch.span, hipMemcpyHostToDevice, s));
  NT_TRY(hipMemcpyAsync(sd.moff.p, ho, m * 8, hipMemcpyHostToDevice, s));
  NT_TRY(hipMemcpyAsync(sd.mlen.p, hl, m * 8, hipMemcpyHostToDevice, s));
  nt::CertBufs& b = ch.cb;
  b = nt::CertBufs{};
  b.wire = wire;
  b.moff = sd.moff.as<uint64_t>();
  b.mlen = sd.mlen.as<uint64_t>();
  b.n = m;
  b.round = sd.round.as<uint64_t>();
  uint32_t* u = sd.u32s.as<uint32_t>();
  b.author = u;
  b.np = u + m;
  b.nq = u + 2 * m;
  b.nv = u + 3 * m;
  b.flags = u + 4 * m;
  b.plen = u + 5 * m;
  b.verr = u + 6 * m;
  b.weight = u + 7 * m;
  b.gcnt = u + 8 * m;
  b.vbase = sd.scans.as<uint64_t>();
  b.pbase = b.vbase + (m + 1);
  b.soff = sd.sha.as<uint64_t>();
  b.slen = b.soff + 2 * m;
  b.gfirst = sd.grp.as<uint64_t>();
  b.grp_words = b.gfirst + m;
  b.code = sd.code.as<uint8_t>();
  NT_TRY(nt::launch_cert_parse(pd.c, b, s));
  NT_TRY(nt::launch_cert_scan(b, s));
  // the totals: vbase[m], pbase[m]
  NT_TRY(hipMemcpyAsync(sd.tot.as<uint64_t>(), b.vbase + m, 8, hipMemcpyDeviceToHost, s));
  NT_TRY(hipMemcpyAsync(sd.tot.as<uint64_t>() + 1, b.pbase + m, 8, hipMemcpyDeviceToHost, s));
  NT_TRY(hipEventRecord(sd.ev, s));
  return NT_OK;
}

int ingest_back(Device& dv, IngestState& S, Side& sd, int parity, Chunk& ch, const nt_committee& cm,
                const nt_committee::PerDev& pd, uint64_t gc_round, hipStream_t s) {
  const uint64_t m = ch.b - ch.a;
  NT_TRY(hipEventSynchronize(sd.ev));
  const uint64_t V = sd.tot.as<uint64_t>()[0], P = sd.tot.as<uint64_t>()[1];
  if (V > ch.vmax) return NT_EHIP;  // k_cert_parse bounds every count by the message length
  const uint64_t nsig = m + V;
  // the event above follows every earlier use of this side's buffers on s
  NT_CHK0(sd.mbase.ensure(168 * m + 16 + P + 64));
  NT_CHK0(sd.keys.ensure(nsig * 4 + 64));
  NT_CHK0(sd.sigs.ensure(nsig * 64 + 64));
  NT_CHK0(sd.smsg.ensure(nsig * 16 + 64));
  NT_CHK0(sd.words.ensure(((nsig + 63) / 64 + 1) * 8));
  nt::CertBufs& b = ch.cb;
  b.mbase = sd.mbase.as<uint8_t>();
  b.pre_off = (168 * m + 15) & ~(uint64_t)15;
  b.keys = sd.keys.as<uint32_t>();
  b.sigs = sd.sigs.as<uint4>();
  b.smoff = sd.smsg.as<uint64_t>();
  b.smlen = b.smoff + nsig;
  b.sig_words = sd.words.as<uint64_t>();
  NT_TRY(nt::launch_cert_scatter(pd.c, b, s));
  const uint64_t mbytes = 168 * m + 16 + P;  // the preimages and digests k_cert_scatter wrote
  NT_TRY(nt::launch_sha512_trunc32(b.mbase, mbytes, b.soff, b.slen, 2 * m, b.mbase + 32 * m, s,
                                   std::max<uint64_t>(ch.lmax, 72)));
  NT_CHK0(dv.ensure_stash(parity, nsig));
  void* st = parity ? dv.stash2.p : dv.d[B_STASH].p;
  void* so = parity ? dv.sort2.p : dv.d[B_SORT].p;
  const auto& kd = cm.kt->dev[dv.group];
  NT_CHK0(dv.keyset_launch(s, st, [&] {
    return nt::launch_verify_keyset(NT_MODE_MIXED, cm.kt->bits, b.keys, (const uint8_t*)b.sigs, b.mbase, mbytes, b.smoff,
                                    b.smlen, nsig, kd.d_meta, kd.d_enc, kd.d_comb, cm.kt->nkeys, dv.d_combB, dv.bbits,
                                    st, so, sd.words.as<uint64_t>(), dv.cus, s, b.gfirst, b.gcnt, m,
                                    (uint64_t*)b.grp_words);  // the vote groups' AND in the kernel's epilogue
  }));
  NT_TRY(nt::launch_cert_verdict(pd.c, b, gc_round, s));
  NT_TRY(hipMemcpyAsync(S.hcode.as<uint8_t>() + ch.a, b.code, m, hipMemcpyDeviceToHost, s));
  return NT_OK;
}

int ingest_shard(Device& dv, const nt_committee& cm, const uint8_t* data, const uint64_t* off, const uint64_t* len,
                 uint64_t lo, uint64_t hi, uint64_t gc_round, uint8_t* out) {
  const uint64_t n = hi - lo;
  if (!n) return NT_OK;
  NT_CHK0(comb_b_for(dv));
  if (!dv.ingest) {
    auto st = std::make_shared<IngestState>();
    st->ordinal = dv.ordinal;
    for (auto& sd : st->side) NT_TRY(hipEventCreateWithFlags(&sd.ev, hipEventDisableTiming));
    dv.ingest = st;
  }
  IngestState& S = *(IngestState*)dv.ingest.get();
  // both compute streams must be idle before the shared host staging is rewritten
  NT_TRY(hipStreamSynchronize(dv.stream));
  NT_TRY(hipStreamSynchronize(dv.stream2));
  NT_CHK0(S.hoff.ensure(n * 8));
  NT_CHK0(S.hlen.ensure(n * 8));
  NT_CHK0(S.hcode.ensure(n));
  const nt_committee::PerDev& pd = cm.dev[dv.group];
  const uint64_t C = chunk_msgs();
  std::vector<Chunk> ch;
  for (uint64_t a = 0; a < n; a += C) {
    Chunk c;
    c.a = a;
    c.b = std::min(n, a + C);
    ch.push_back(c);
  }
  const uint8_t* d = data;
  const uint64_t* o = off + lo;
  const uint64_t* l = len + lo;
  for (size_t k = 0; k <= ch.size(); ++k) {
    if (k < ch.size()) NT_CHK0(ingest_front(dv, S, S.side[k & 1], ch[k], pd, d, o, l, dv.cstr((int)k)));
    if (k >= 1) NT_CHK0(ingest_back(dv, S, S.side[(k - 1) & 1], (int)((k - 1) & 1), ch[k - 1], cm, pd, gc_round,
                                    dv.cstr((int)(k - 1))));
  }
  NT_TRY(hipStreamSynchronize(dv.stream));
  NT_TRY(hipStreamSynchronize(dv.stream2));
  std::memcpy(out + lo, S.hcode.p, n);
  return NT_OK;
}

}  // namespace

extern "C" {

int nt_certificates_ingest(nt_ctx* ctx, const nt_committee* cm, const uint8_t* data, const uint64_t* off,
                           const uint64_t* len, uint64_t n, uint64_t gc_round, uint8_t* out_code) {
  if (!ctx || !cm || cm->ctx != ctx || (n && (!data || !off || !len || !out_code))) return NT_EINVAL;
  if (n == 0) return NT_OK;
  ctx->calls_gpu++;
  return run_sharded(ctx, n, 1, [&](Device& dv, uint64_t lo, uint64_t hi) {
    return ingest_shard(dv, *cm, data, off, len, lo, hi, gc_round, out_code);
  });
}

}  // extern "C"
