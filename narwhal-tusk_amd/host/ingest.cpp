// ingest.cpp -- wire ingestion straight into SoA buffers.
//
// Core::ingest decodes bincode PrimaryMessages on host threads WITHOUT building
// the reference's object graph (no BTreeMap/BTreeSet/Vec per message): each
// message becomes a flat record, the header digest preimage is copied out of
// the wire bytes (a canonical BTreeMap/BTreeSet serialization is already the
// preimage's order: author || round || (digest || worker)* || parent*), public
// keys map to committee indices by their base64 text, and the signatures land
// in the arrays the GPU launches take.  Then Core's checks run in the reference
// order (core.rs:306-346, messages.rs:48-67,131-142,189-215) with one SHA-512
// launch, one verify_strict launch and one verify_batch launch for the batch.
// Messages whose payload / parents are not in canonical order (possible only
// for hand-made bytes) take the general decoder + sanitize_batch; results are
// identical either way (tests/test_wire.py compares both paths).
#include <algorithm>
#include <chrono>
#include <exception>
#include <cstring>
#include <string_view>
#include <thread>
#include <unordered_map>

#include "../../include/ntcrypto.h"
#include "narwhal.hpp"
#include "wire.hpp"

namespace primary {

namespace {

constexpr uint32_t kNoKey = 0xffffffffu;  // not a committee key (stake 0)

struct KeyIndex {
  std::vector<PublicKey> keys;        // committee order (BTreeMap = byte order)
  std::vector<Stake> stake;
  std::vector<std::vector<WorkerId>> workers;
  std::vector<std::string> b64;                          // canonical encodings
  std::unordered_map<std::string_view, uint32_t> by_b64;  // views into b64
  explicit KeyIndex(const Committee& c) {
    b64.reserve(c.authorities.size());
    for (const auto& kv : c.authorities) {
      b64.push_back(kv.first.encode_base64());
      by_b64.emplace(std::string_view(b64.back()), (uint32_t)keys.size());
      keys.push_back(kv.first);
      stake.push_back(kv.second.stake);
      workers.emplace_back(kv.second.workers.begin(), kv.second.workers.end());
    }
  }
  uint32_t of_bytes(const PublicKey& pk) const {
    auto it = std::lower_bound(keys.begin(), keys.end(), pk);
    return (it != keys.end() && *it == pk) ? (uint32_t)(it - keys.begin()) : kNoKey;
  }
};

enum Status : uint8_t { kRecOk = 0, kRecBad = 1, kRecGeneral = 2 };

struct Rec {
  uint8_t kind = 0, status = kRecOk, workers_ok = 1;
  uint64_t round = 0;
  uint32_t author = kNoKey, origin = kNoKey;  // committee indices
  PublicKey author_pk, origin_pk;             // raw keys (preimages, vote target check)
  std::array<uint8_t, 32> id{};
  std::array<uint8_t, 64> sig{};
  uint64_t pre_off = 0, pre_len = 0;          // header preimage in the thread arena
  uint64_t vote_off = 0, vote_cnt = 0;        // certificate votes in the thread arena
};

struct Arena {
  std::vector<uint8_t> pre;       // header preimages
  std::vector<uint32_t> vkey;     // certificate vote key indices
  std::vector<const uint8_t*> vsig;  // certificate vote signatures (64 B each, in the wire buffer)
};

}  // namespace

// Buffers kept across Core::ingest calls: the first call pays the page faults
// of ~1.5 GB of staging for a config-3 batch, later calls reuse the capacity.
struct IngestWorkspace {
  std::vector<Rec> recs;
  std::vector<Arena> arenas;
  std::vector<uint8_t> need, pre, dig, gsig, gpk;
  std::vector<uint64_t> dig_at, poff, plen;
  std::vector<uint32_t> gkey;
  std::vector<DagError> res;
};

namespace {

struct Fast {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  const KeyIndex& ki;
  bool need(size_t k) { return ok = ok && n - pos >= k; }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t x;
    std::memcpy(&x, p + pos, 4);
    pos += 4;
    return x;
  }
  uint64_t u64() {
    if (!need(8)) return 0;
    uint64_t x;
    std::memcpy(&x, p + pos, 8);
    pos += 8;
    return x;
  }
  const uint8_t* take(size_t k) {
    if (!need(k)) return nullptr;
    const uint8_t* q = p + pos;
    pos += k;
    return q;
  }
  uint64_t count(size_t min_elem) {
    const uint64_t c = u64();
    if (ok && c > (n - pos) / min_elem) ok = false;
    return ok ? c : 0;
  }
  // PublicKey string -> committee index (kNoKey if valid but unknown); raw key out
  uint32_t key(PublicKey& raw) {
    const uint64_t len = count(1);
    const uint8_t* s = take(len);
    if (!ok) return kNoKey;
    auto it = ki.by_b64.find(std::string_view((const char*)s, (size_t)len));
    if (it != ki.by_b64.end()) {
      raw = ki.keys[it->second];
      return it->second;
    }
    // not a canonical committee encoding: full serde String + base64 decode
    if (!decode_public_key(s, (size_t)len, raw)) {
      ok = false;
      return kNoKey;
    }
    return ki.of_bytes(raw);
  }
  // header fields into rec + preimage into the arena; canonical order checked
  void header(Rec& r, Arena& a) {
    r.author = key(r.author_pk);
    r.round = u64();
    if (!ok) return;
    const size_t p0 = a.pre.size();
    a.pre.insert(a.pre.end(), r.author_pk.bytes.begin(), r.author_pk.bytes.end());
    const uint8_t* rb = p + pos - 8;
    a.pre.insert(a.pre.end(), rb, rb + 8);
    const uint64_t np = count(36);
    const uint8_t* pay = take(36 * np);
    if (!ok) return;
    for (uint64_t i = 0; i < np; ++i) {
      if (i && std::memcmp(pay + 36 * (i - 1), pay + 36 * i, 32) >= 0) r.status = kRecGeneral;
      uint32_t w;
      std::memcpy(&w, pay + 36 * i + 32, 4);
      if (r.author != kNoKey) {
        const auto& ws = ki.workers[r.author];
        if (!std::binary_search(ws.begin(), ws.end(), w)) r.workers_ok = 0;
      }
    }
    a.pre.insert(a.pre.end(), pay, pay + 36 * np);
    const uint64_t nq = count(32);
    const uint8_t* par = take(32 * nq);
    if (!ok) return;
    for (uint64_t i = 1; i < nq; ++i)
      if (std::memcmp(par + 32 * (i - 1), par + 32 * i, 32) >= 0) r.status = kRecGeneral;
    a.pre.insert(a.pre.end(), par, par + 32 * nq);
    const uint8_t* id = take(32);
    const uint8_t* sg = take(64);
    if (!ok) return;
    std::memcpy(r.id.data(), id, 32);
    std::memcpy(r.sig.data(), sg, 64);
    r.pre_off = p0;
    r.pre_len = a.pre.size() - p0;
  }
  void message(Rec& r, Arena& a) {
    const uint32_t tag = u32();
    if (!ok || tag > 3) {
      ok = false;
      return;
    }
    r.kind = (uint8_t)tag;
    if (tag == 0) {
      header(r, a);
    } else if (tag == 1) {
      const uint8_t* id = take(32);
      r.round = u64();
      r.origin = key(r.origin_pk);
      r.author = key(r.author_pk);
      const uint8_t* sg = take(64);
      if (!ok) return;
      std::memcpy(r.id.data(), id, 32);
      std::memcpy(r.sig.data(), sg, 64);
    } else if (tag == 2) {
      header(r, a);
      const uint64_t nv = count(8 + 64);
      r.vote_off = a.vkey.size();
      r.vote_cnt = nv;
      for (uint64_t i = 0; ok && i < nv; ++i) {
        PublicKey raw;
        const uint32_t k = key(raw);
        const uint8_t* sg = take(64);
        if (!ok) return;
        a.vkey.push_back(k);
        a.vsig.push_back(sg);
      }
    } else {
      const uint64_t nd = count(32);
      take(32 * nd);
      PublicKey raw;
      key(raw);
    }
  }
};

double since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
}

void check(int rc, const char* what) {
  if (rc != 0) throw crypto::BackendError(std::string(what) + ": " + nt_strerror(rc));
}

}  // namespace

IngestStats& last_ingest_stats() {
  static thread_local IngestStats st;
  return st;
}

template <class F>
void parallel_for(int threads, F&& f) {
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(f, t);
  f(0);
  for (auto& th : pool) th.join();
}

std::vector<DagError> Core::ingest_soa(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                       int threads, double* decode_seconds) const {
  const auto t0 = std::chrono::steady_clock::now();
  const Committee& cm = *committee;
  const KeyIndex ki(cm);
  if (threads < 1) threads = 1;
  if ((size_t)threads > n) threads = n ? (int)n : 1;
  const int T = threads;
  auto lo = [&](int t) { return n * t / T; };
  auto hi = [&](int t) { return n * (t + 1) / T; };
  if (!ws) ws = std::make_shared<IngestWorkspace>();
  IngestWorkspace& W = *ws;
  // ---- phase A: parallel flat decode (thread t owns messages [lo(t), hi(t)))
  std::vector<Rec>& recs = W.recs;
  recs.assign(n, Rec{});
  std::vector<Arena>& arenas = W.arenas;
  arenas.resize(T);
  for (auto& a : arenas) {
    a.pre.clear();
    a.vkey.clear();
    a.vsig.clear();
  }
  parallel_for(T, [&](int t) {
    for (size_t i = lo(t); i < hi(t); ++i) {
      Fast f{data + off[i], (size_t)len[i], 0, true, ki};
      Arena& a = arenas[t];
      const size_t npre = a.pre.size(), nvote = a.vkey.size();
      f.message(recs[i], a);
      if (!f.ok) {
        // drop whatever the failed message appended: vkey[k] and vsig[k] must
        // stay the same vote for every later certificate of this thread
        recs[i].status = kRecBad;
        a.pre.resize(npre);
        a.vkey.resize(nvote);
        a.vsig.resize(nvote);
      }
    }
  });
  if (decode_seconds) *decode_seconds = since(t0);
  IngestStats& st = last_ingest_stats();
  st = IngestStats{};
  st.decode = since(t0);
  auto tp = std::chrono::steady_clock::now();

  std::vector<DagError>& res = W.res;
  res.assign(n, DagError::Ok);
  // ---- non-canonical messages: general decoder + sanitize_batch
  {
    std::vector<PrimaryMessage> gen;
    std::vector<size_t> gidx;
    for (size_t i = 0; i < n; ++i)
      if (recs[i].status == kRecGeneral) {
        PrimaryMessage m;
        if (decode(data + off[i], (size_t)len[i], m)) {
          gen.push_back(std::move(m));
          gidx.push_back(i);
        } else {
          recs[i].status = kRecBad;
        }
      }
    if (!gen.empty()) {
      const auto r = sanitize_batch(gen);
      for (size_t k = 0; k < gidx.size(); ++k) res[gidx[k]] = r[k];
    }
  }
  // ---- phase B: round filters + digest preimages, per thread, then concatenated
  enum Need : uint8_t { kNone, kHeader, kVote, kCert };
  std::vector<uint8_t>& need = W.need;
  need.assign(n, kNone);
  std::vector<uint64_t>& dig_at = W.dig_at;  // thread-local digest index, made global below
  dig_at.assign(n, 0);
  static const std::array<uint8_t, 32> zero{};
  struct PreBuf {
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> off, len;
  };
  std::vector<PreBuf> pb(T);
  parallel_for(T, [&](int t) {
    PreBuf& b = pb[t];
    const Arena& a = arenas[t];
    size_t bytes = 0;
    for (size_t i = lo(t); i < hi(t); ++i) bytes += recs[i].pre_len + 72;
    b.bytes.reserve(bytes);
    auto add = [&](const uint8_t* q, size_t k) {
      b.off.push_back(b.bytes.size());
      b.len.push_back(k);
      b.bytes.insert(b.bytes.end(), q, q + k);
    };
    auto add_short = [&](const std::array<uint8_t, 32>& id, uint64_t round, const PublicKey& pk) {
      uint8_t v[72];  // id || round_le || key (messages.rs:145-153, 226-234)
      std::memcpy(v, id.data(), 32);
      std::memcpy(v + 32, &round, 8);
      std::memcpy(v + 40, pk.bytes.data(), 32);
      add(v, 72);
    };
    for (size_t i = lo(t); i < hi(t); ++i) {
      const Rec& r = recs[i];
      if (r.status == kRecBad) { res[i] = DagError::SerializationError; continue; }
      if (r.status == kRecGeneral) continue;
      switch (r.kind) {
        case 0:
          if (r.round < gc_round) { res[i] = DagError::TooOld; break; }
          need[i] = kHeader;
          dig_at[i] = b.off.size();
          add(a.pre.data() + r.pre_off, r.pre_len);
          break;
        case 1:
          if (r.round < current_header.round) { res[i] = DagError::TooOld; break; }
          if (!(r.id == current_header.id.bytes && r.origin_pk == current_header.author &&
                r.round == current_header.round)) {
            res[i] = DagError::UnexpectedVote;
            break;
          }
          need[i] = kVote;
          dig_at[i] = b.off.size();
          add_short(r.id, r.round, r.origin_pk);
          break;
        case 2:
          if (r.round < gc_round) { res[i] = DagError::TooOld; break; }
          if (r.id == zero && r.round == 0 && r.author != kNoKey) break;  // genesis
          need[i] = kCert;
          dig_at[i] = b.off.size();
          add(a.pre.data() + r.pre_off, r.pre_len);
          add_short(r.id, r.round, r.author_pk);
          break;
        default: res[i] = DagError::UnexpectedMessage; break;
      }
    }
  });
  std::vector<uint64_t> pre_base(T + 1, 0), dig_base(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    pre_base[t + 1] = pre_base[t] + pb[t].bytes.size();
    dig_base[t + 1] = dig_base[t] + pb[t].off.size();
  }
  const size_t nd = dig_base[T];
  std::vector<uint8_t>& pre = W.pre;
  pre.resize(std::max<uint64_t>(pre_base[T], 1));
  std::vector<uint64_t>& poff = W.poff;
  std::vector<uint64_t>& plen = W.plen;
  poff.resize(std::max<size_t>(nd, 1));
  plen.resize(std::max<size_t>(nd, 1));
  parallel_for(T, [&](int t) {
    std::memcpy(pre.data() + pre_base[t], pb[t].bytes.data(), pb[t].bytes.size());
    for (size_t k = 0; k < pb[t].off.size(); ++k) {
      poff[dig_base[t] + k] = pre_base[t] + pb[t].off[k];
      plen[dig_base[t] + k] = pb[t].len[k];
    }
    for (size_t i = lo(t); i < hi(t); ++i) dig_at[i] += dig_base[t];
    std::vector<uint8_t>().swap(pb[t].bytes);
  });
  nt_ctx* ctx = crypto::Backend::global().ctx();
  st.prep += since(tp);
  tp = std::chrono::steady_clock::now();
  std::vector<uint8_t>& dig = W.dig;
  dig.resize(32 * std::max<size_t>(nd, 1));
  if (nd) check(nt_sha512_trunc32(ctx, pre.data(), poff.data(), plen.data(), nd, dig.data()), "nt_sha512_trunc32");
  st.digest = since(tp);
  tp = std::chrono::steady_clock::now();

  // ---- phase C: prechecks in the reference order, per thread; the vote arrays
  // of all arenas are concatenated once and certificate groups point into them
  std::vector<uint64_t> vbase(T + 1, 0);
  for (int t = 0; t < T; ++t) vbase[t + 1] = vbase[t] + arenas[t].vkey.size();
  const uint64_t nv = vbase[T];
  std::vector<uint32_t>& gkey = W.gkey;
  std::vector<uint8_t>& gsig = W.gsig;
  std::vector<uint8_t>& gpk = W.gpk;
  gkey.resize(std::max<uint64_t>(nv, 1));
  gsig.resize(64 * std::max<uint64_t>(nv, 1));
  gpk.resize(cache ? 0 : 32 * std::max<uint64_t>(nv, 1));
  struct SigOut {
    std::vector<uint32_t> key;
    std::vector<uint8_t> pk, sig, msg;
    std::vector<size_t> who;                 // message index per strict entry
    std::vector<uint64_t> first;             // groups: global vote offset
    std::vector<uint32_t> cnt;
    std::vector<uint8_t> gmsg;
    std::vector<size_t> gwho;
  };
  std::vector<SigOut> so(T);
  const Stake quorum = cm.quorum_threshold();
  parallel_for(T, [&](int t) {
    const Arena& a = arenas[t];
    std::memcpy(gkey.data() + vbase[t], a.vkey.data(), 4 * a.vkey.size());
    for (size_t k = 0; k < a.vsig.size(); ++k) std::memcpy(&gsig[64 * (vbase[t] + k)], a.vsig[k], 64);
    if (!cache)
      for (size_t k = 0; k < a.vkey.size(); ++k)
        if (a.vkey[k] != kNoKey) std::memcpy(&gpk[32 * (vbase[t] + k)], ki.keys[a.vkey[k]].bytes.data(), 32);
    SigOut& o = so[t];
    std::vector<uint32_t> stamp(ki.keys.size(), 0);
    uint32_t stamp_id = 0;
    auto add_sig = [&](size_t i, uint32_t key, const std::array<uint8_t, 64>& sg, const uint8_t* msg) {
      o.who.push_back(i);
      o.key.push_back(key);
      if (!cache) o.pk.insert(o.pk.end(), ki.keys[key].bytes.begin(), ki.keys[key].bytes.end());
      o.sig.insert(o.sig.end(), sg.begin(), sg.end());
      o.msg.insert(o.msg.end(), msg, msg + 32);
    };
    for (size_t i = lo(t); i < hi(t); ++i) {
      const Rec& r = recs[i];
      const uint8_t* d = &dig[32 * dig_at[i]];
      if (need[i] == kHeader || need[i] == kCert) {
        if (std::memcmp(d, r.id.data(), 32) != 0) { res[i] = DagError::InvalidHeaderId; continue; }
        if (r.author == kNoKey || ki.stake[r.author] == 0) { res[i] = DagError::UnknownAuthority; continue; }
        if (!r.workers_ok) { res[i] = DagError::MalformedHeader; continue; }
        if (need[i] == kCert) {
          ++stamp_id;
          Stake weight = 0;
          DagError e = DagError::Ok;
          for (uint64_t v = 0; v < r.vote_cnt; ++v) {
            const uint32_t k = a.vkey[r.vote_off + v];
            if (k != kNoKey && stamp[k] == stamp_id) { e = DagError::AuthorityReuse; break; }
            if (k == kNoKey || ki.stake[k] == 0) { e = DagError::UnknownAuthority; break; }
            stamp[k] = stamp_id;
            weight += ki.stake[k];
          }
          if (e == DagError::Ok && weight < quorum) e = DagError::CertificateRequiresQuorum;
          if (e != DagError::Ok) { res[i] = e; continue; }
          o.gwho.push_back(i);
          o.first.push_back(vbase[t] + r.vote_off);
          o.cnt.push_back((uint32_t)r.vote_cnt);
          o.gmsg.insert(o.gmsg.end(), d + 32, d + 64);
        }
        add_sig(i, r.author, r.sig, r.id.data());
      } else if (need[i] == kVote) {
        if (r.author == kNoKey || ki.stake[r.author] == 0) { res[i] = DagError::UnknownAuthority; continue; }
        add_sig(i, r.author, r.sig, d);
      }
    }
  });
  // strict entries and groups are a few per message: concatenate serially
  SigOut all;
  for (auto& o : so) {
    all.who.insert(all.who.end(), o.who.begin(), o.who.end());
    all.key.insert(all.key.end(), o.key.begin(), o.key.end());
    all.pk.insert(all.pk.end(), o.pk.begin(), o.pk.end());
    all.sig.insert(all.sig.end(), o.sig.begin(), o.sig.end());
    all.msg.insert(all.msg.end(), o.msg.begin(), o.msg.end());
    all.gwho.insert(all.gwho.end(), o.gwho.begin(), o.gwho.end());
    all.first.insert(all.first.end(), o.first.begin(), o.first.end());
    all.cnt.insert(all.cnt.end(), o.cnt.begin(), o.cnt.end());
    all.gmsg.insert(all.gmsg.end(), o.gmsg.begin(), o.gmsg.end());
  }
  st.prep += since(tp);
  tp = std::chrono::steady_clock::now();
  // ---- phase D: one verify_strict launch, one verify_batch launch
  const size_t ns = all.key.size(), G = all.cnt.size();
  std::vector<uint8_t> sbm((ns + 7) / 8 + 1), gbm((G + 7) / 8 + 1);
  if (ns) {
    std::vector<uint64_t> mo(ns), ml(ns, 32);
    for (size_t k = 0; k < ns; ++k) mo[k] = 32 * k;
    if (cache)
      check(nt_ed25519_verify_keyset(ctx, cache->handle(), NT_MODE_STRICT, all.key.data(), all.sig.data(),
                                     all.msg.data(), mo.data(), ml.data(), ns, sbm.data()),
            "nt_ed25519_verify_keyset");
    else
      check(nt_ed25519_verify_strict(ctx, all.pk.data(), all.sig.data(), all.msg.data(), mo.data(), ml.data(), ns,
                                     sbm.data()),
            "nt_ed25519_verify_strict");
  }
  st.strict = since(tp);
  tp = std::chrono::steady_clock::now();
  if (G) {
    if (cache)
      check(nt_ed25519_verify_batch_groups_keyset(ctx, cache->handle(), gkey.data(), gsig.data(), all.first.data(),
                                                  all.cnt.data(), all.gmsg.data(), G, gbm.data(), nullptr),
            "nt_ed25519_verify_batch_groups_keyset");
    else
      check(nt_ed25519_verify_batch_groups(ctx, gpk.data(), gsig.data(), all.first.data(), all.cnt.data(),
                                           all.gmsg.data(), G, gbm.data(), nullptr),
            "nt_ed25519_verify_batch_groups");
  }
  st.batch = since(tp);
  for (size_t k = 0; k < ns; ++k)
    if (!((sbm[k / 8] >> (k % 8)) & 1)) res[all.who[k]] = DagError::InvalidSignature;
  for (size_t g = 0; g < G; ++g)
    if (!((gbm[g / 8] >> (g % 8)) & 1)) res[all.gwho[g]] = DagError::InvalidSignature;
  st.total = since(t0);
  return res;  // a copy: the workspace keeps its buffers
}

std::vector<DagError> Core::ingest_pipelined(const uint8_t* data, const uint64_t* off, const uint64_t* len,
                                             size_t n, int threads, size_t chunk) const {
  if (chunk == 0 || chunk >= n) return ingest_soa(data, off, len, n, threads);
  if (!ws) ws = std::make_shared<IngestWorkspace>();
  if (!ws_alt) ws_alt = std::make_shared<IngestWorkspace>();
  Core a = *this, b = *this;
  b.ws = ws_alt;
  std::vector<DagError> res(n);
  const size_t K = (n + chunk - 1) / chunk;
  auto run = [&](const Core& c, size_t k) {
    const size_t lo = k * chunk, hi = std::min(n, lo + chunk);
    const auto r = c.ingest_soa(data, off + lo, len + lo, hi - lo, threads);
    std::copy(r.begin(), r.end(), res.begin() + lo);
  };
  std::exception_ptr err;
  std::thread tb([&] {
    try {
      for (size_t k = 1; k < K; k += 2) run(b, k);
    } catch (...) {
      err = std::current_exception();
    }
  });
  try {
    for (size_t k = 0; k < K; k += 2) run(a, k);
  } catch (...) {
    tb.join();
    throw;
  }
  tb.join();
  if (err) std::rethrow_exception(err);
  return res;
}

}  // namespace primary
