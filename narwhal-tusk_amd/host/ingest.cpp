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
  std::vector<std::string> b64;       // canonical encodings
  explicit KeyIndex(const Committee& c) {
    for (const auto& kv : c.authorities) {
      b64.push_back(kv.first.encode_base64());
      keys.push_back(kv.first);
      stake.push_back(kv.second.stake);
      workers.emplace_back(kv.second.workers.begin(), kv.second.workers.end());
    }
    build_slots();
  }
  // Canonical encodings by their first 8 characters (open addressing; the other
  // 36 are compared): one multiply, one probe and a 36-byte compare per key
  // string instead of hashing all 44 bytes into an unordered_map.
  static constexpr uint32_t kEmpty = 0xffffffffu;
  std::vector<uint64_t> slot_head;
  std::vector<uint32_t> slot_idx;
  int slot_bits = 0;
  static uint64_t head_of(const uint8_t* s) {
    uint64_t h;
    std::memcpy(&h, s, 8);
    return h;
  }
  size_t slot_of(uint64_t h) const { return (size_t)((h * 0x9E3779B97F4A7C15ull) >> (64 - slot_bits)); }
  void build_slots() {
    slot_bits = 4;
    while ((1ull << slot_bits) < 4 * b64.size()) ++slot_bits;
    slot_head.assign(1ull << slot_bits, 0);
    slot_idx.assign(1ull << slot_bits, kEmpty);
    const size_t mask = (1ull << slot_bits) - 1;
    for (uint32_t k = 0; k < b64.size(); ++k) {
      const uint64_t h = head_of((const uint8_t*)b64[k].data());
      size_t i = slot_of(h);
      while (slot_idx[i] != kEmpty) i = (i + 1) & mask;
      slot_head[i] = h;
      slot_idx[i] = k;
    }
  }
  // committee index of a canonical 44-character encoding, kEmpty otherwise
  uint32_t find_b64(const uint8_t* s, size_t len) const {
    if (len != 44) return kEmpty;
    const uint64_t h = head_of(s);
    const size_t mask = (1ull << slot_bits) - 1;
    for (size_t i = slot_of(h); slot_idx[i] != kEmpty; i = (i + 1) & mask)
      if (slot_head[i] == h && std::memcmp(b64[slot_idx[i]].data() + 8, s + 8, 36) == 0) return slot_idx[i];
    return kEmpty;
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
  const uint8_t* pay = nullptr;               // header payload entries (36 B each) in the wire
  const uint8_t* par = nullptr;               // header parents (32 B each) in the wire
  uint64_t np = 0, nq = 0;
  uint64_t vote_off = 0, vote_cnt = 0;        // certificate votes in the thread arena
  // Header::digest preimage: author || round_le || (digest || worker_le)* || parent*
  // (messages.rs:70-84) -- the canonical map/set wire order is already sorted
  uint64_t pre_len() const { return 40 + 36 * np + 32 * nq; }
  void write_pre(uint8_t* o) const {
    std::memcpy(o, author_pk.bytes.data(), 32);
    std::memcpy(o + 32, &round, 8);
    std::memcpy(o + 40, pay, 36 * np);
    std::memcpy(o + 40 + 36 * np, par, 32 * nq);
  }
};

struct Arena {
  std::vector<uint32_t> vkey;     // certificate vote key indices
  std::vector<const uint8_t*> vsig;  // certificate vote signatures (64 B each, in the wire buffer)
};

// Grow-only page-locked buffer (nt_host_alloc): the host entry points DMA
// straight from it instead of staging a copy.
struct PinnedBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf&) = delete;
  PinnedBuf& operator=(const PinnedBuf&) = delete;
  ~PinnedBuf() { nt_host_free(p); }
  template <class T = uint8_t>
  T* ensure(size_t bytes) {
    if (bytes > cap || !p) {
      nt_host_free(p);
      p = nullptr;
      cap = 0;
      const size_t want = std::max<size_t>(bytes + bytes / 4, 1 << 20);
      p = (uint8_t*)nt_host_alloc(want);
      if (!p) throw crypto::BackendError("nt_host_alloc: no pinned host memory");
      cap = want;
    }
    return (T*)p;
  }
};

}  // namespace

// Buffers kept across Core::ingest calls: the first call pays the page faults
// of ~1.5 GB of staging for a config-3 batch, later calls reuse the capacity.
struct IngestWorkspace {
  std::vector<Rec> recs;
  std::vector<Arena> arenas;
  std::vector<uint8_t> need, dig, gpk;
  std::vector<uint64_t> dig_at, poff, plen;
  PinnedBuf pre, gkey, gsig;  // digest preimages; dense group keys and signatures
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
  // PublicKey string -> committee index (kNoKey if valid but unknown); raw key
  // out unless `raw` is null (vote keys: only the index is used)
  uint32_t key(PublicKey* raw) {
    const uint64_t len = count(1);
    const uint8_t* s = take(len);
    if (!ok) return kNoKey;
    const uint32_t k = ki.find_b64(s, (size_t)len);
    if (k != KeyIndex::kEmpty) {
      if (raw) *raw = ki.keys[k];
      return k;
    }
    PublicKey tmp;
    if (!raw) raw = &tmp;
    // not a canonical committee encoding: full serde String + base64 decode
    if (!decode_public_key(s, (size_t)len, *raw)) {
      ok = false;
      return kNoKey;
    }
    return ki.of_bytes(*raw);
  }
  // header fields into rec + preimage into the arena; canonical order checked
  void header(Rec& r) {
    r.author = key(&r.author_pk);
    r.round = u64();
    if (!ok) return;
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
    const uint64_t nq = count(32);
    const uint8_t* par = take(32 * nq);
    if (!ok) return;
    for (uint64_t i = 1; i < nq; ++i)
      if (std::memcmp(par + 32 * (i - 1), par + 32 * i, 32) >= 0) r.status = kRecGeneral;
    const uint8_t* id = take(32);
    const uint8_t* sg = take(64);
    if (!ok) return;
    std::memcpy(r.id.data(), id, 32);
    std::memcpy(r.sig.data(), sg, 64);
    r.pay = pay;
    r.np = np;
    r.par = par;
    r.nq = nq;
  }
  void message(Rec& r, Arena& a) {
    const uint32_t tag = u32();
    if (!ok || tag > 3) {
      ok = false;
      return;
    }
    r.kind = (uint8_t)tag;
    if (tag == 0) {
      header(r);
    } else if (tag == 1) {
      const uint8_t* id = take(32);
      r.round = u64();
      r.origin = key(&r.origin_pk);
      r.author = key(&r.author_pk);
      const uint8_t* sg = take(64);
      if (!ok) return;
      std::memcpy(r.id.data(), id, 32);
      std::memcpy(r.sig.data(), sg, 64);
    } else if (tag == 2) {
      header(r);
      const uint64_t nv = count(8 + 64);
      r.vote_off = a.vkey.size();
      r.vote_cnt = nv;
      for (uint64_t i = 0; ok && i < nv; ++i) {
        const uint32_t k = key(nullptr);
        const uint8_t* sg = take(64);
        if (!ok) return;
        a.vkey.push_back(k);
        a.vsig.push_back(sg);
      }
    } else {
      const uint64_t nd = count(32);
      take(32 * nd);
      key(nullptr);
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
    a.vkey.clear();
    a.vsig.clear();
  }
  parallel_for(T, [&](int t) {
    for (size_t i = lo(t); i < hi(t); ++i) {
      Fast f{data + off[i], (size_t)len[i], 0, true, ki};
      Arena& a = arenas[t];
      const size_t nvote = a.vkey.size();
      f.message(recs[i], a);
      if (!f.ok) {
        // drop whatever the failed message appended: vkey[k] and vsig[k] must
        // stay the same vote for every later certificate of this thread
        recs[i].status = kRecBad;
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
  // ---- phase B: round filters, then every digest preimage written once,
  // straight into the pinned launch buffer (sizes first, then the copies)
  enum Need : uint8_t { kNone, kHeader, kVote, kCert };
  std::vector<uint8_t>& need = W.need;
  need.assign(n, kNone);
  std::vector<uint64_t>& dig_at = W.dig_at;  // thread-local digest index, made global below
  dig_at.assign(n, 0);
  static const std::array<uint8_t, 32> zero{};
  std::vector<uint64_t> pre_base(T + 1, 0), dig_base(T + 1, 0);
  parallel_for(T, [&](int t) {
    uint64_t bytes = 0, nd = 0;
    for (size_t i = lo(t); i < hi(t); ++i) {
      const Rec& r = recs[i];
      if (r.status == kRecBad) { res[i] = DagError::SerializationError; continue; }
      if (r.status == kRecGeneral) continue;
      switch (r.kind) {
        case 0:
          if (r.round < gc_round) { res[i] = DagError::TooOld; break; }
          need[i] = kHeader;
          bytes += r.pre_len();
          nd += 1;
          break;
        case 1:
          if (r.round < current_header.round) { res[i] = DagError::TooOld; break; }
          if (!(r.id == current_header.id.bytes && r.origin_pk == current_header.author &&
                r.round == current_header.round)) {
            res[i] = DagError::UnexpectedVote;
            break;
          }
          need[i] = kVote;
          bytes += 72;
          nd += 1;
          break;
        case 2:
          if (r.round < gc_round) { res[i] = DagError::TooOld; break; }
          if (r.id == zero && r.round == 0 && r.author != kNoKey) break;  // genesis
          need[i] = kCert;
          bytes += r.pre_len() + 72;
          nd += 2;
          break;
        default: res[i] = DagError::UnexpectedMessage; break;
      }
    }
    pre_base[t + 1] = bytes;
    dig_base[t + 1] = nd;
  });
  for (int t = 0; t < T; ++t) {
    pre_base[t + 1] += pre_base[t];
    dig_base[t + 1] += dig_base[t];
  }
  const size_t nd = dig_base[T];
  uint8_t* pre = W.pre.ensure(std::max<uint64_t>(pre_base[T], 1));
  std::vector<uint64_t>& poff = W.poff;
  std::vector<uint64_t>& plen = W.plen;
  poff.resize(std::max<size_t>(nd, 1));
  plen.resize(std::max<size_t>(nd, 1));
  parallel_for(T, [&](int t) {
    uint64_t o = pre_base[t], d = dig_base[t];
    auto add_short = [&](const std::array<uint8_t, 32>& id, uint64_t round, const PublicKey& pk) {
      // id || round_le || key (messages.rs:145-153, 226-234)
      std::memcpy(pre + o, id.data(), 32);
      std::memcpy(pre + o + 32, &round, 8);
      std::memcpy(pre + o + 40, pk.bytes.data(), 32);
      poff[d] = o;
      plen[d] = 72;
      o += 72;
      ++d;
    };
    for (size_t i = lo(t); i < hi(t); ++i) {
      const Rec& r = recs[i];
      if (need[i] == kNone) continue;
      dig_at[i] = d;
      if (need[i] == kVote) {
        add_short(r.id, r.round, r.origin_pk);
        continue;
      }
      r.write_pre(pre + o);
      poff[d] = o;
      plen[d] = r.pre_len();
      o += r.pre_len();
      ++d;
      if (need[i] == kCert) add_short(r.id, r.round, r.author_pk);
    }
  });
  nt_ctx* ctx = crypto::Backend::global().ctx();
  st.prep += since(tp);
  tp = std::chrono::steady_clock::now();
  std::vector<uint8_t>& dig = W.dig;
  dig.resize(32 * std::max<size_t>(nd, 1));
  if (nd) check(nt_sha512_trunc32(ctx, pre, poff.data(), plen.data(), nd, dig.data()), "nt_sha512_trunc32");
  st.digest = since(tp);
  tp = std::chrono::steady_clock::now();

  // ---- phase C: prechecks in the reference order, per thread; then the votes
  // of the certificates that passed are packed densely, in group order, into
  // the pinned key / signature buffers the verify_batch launch reads directly
  struct SigOut {
    std::vector<uint32_t> key;
    std::vector<uint8_t> pk, sig, msg;
    std::vector<size_t> who;                 // message index per strict entry
    std::vector<uint64_t> first;             // groups: thread-local dense vote offset
    std::vector<uint32_t> cnt;
    std::vector<uint8_t> gmsg;
    std::vector<size_t> gwho;
  };
  std::vector<SigOut> so(T);
  const Stake quorum = cm.quorum_threshold();
  std::vector<uint64_t> vbase(T + 1, 0);
  parallel_for(T, [&](int t) {
    const Arena& a = arenas[t];
    SigOut& o = so[t];
    std::vector<uint32_t> stamp(ki.keys.size(), 0);
    uint32_t stamp_id = 0;
    uint64_t dense = 0;
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
          if (e != DagError::Ok) {
            // Header::verify (signature included) precedes the quorum loop
            // (messages.rs:194-211): the header signature still goes to the strict
            // launch, whose failure overrides this error below
            res[i] = e;
            add_sig(i, r.author, r.sig, r.id.data());
            continue;
          }
          o.gwho.push_back(i);
          o.first.push_back(dense);
          o.cnt.push_back((uint32_t)r.vote_cnt);
          o.gmsg.insert(o.gmsg.end(), d + 32, d + 64);
          dense += r.vote_cnt;
        }
        add_sig(i, r.author, r.sig, r.id.data());
      } else if (need[i] == kVote) {
        if (r.author == kNoKey || ki.stake[r.author] == 0) { res[i] = DagError::UnknownAuthority; continue; }
        add_sig(i, r.author, r.sig, d);
      }
    }
    vbase[t + 1] = dense;
  });
  for (int t = 0; t < T; ++t) vbase[t + 1] += vbase[t];
  const uint64_t nv = vbase[T];
  uint32_t* gkey = W.gkey.ensure<uint32_t>(4 * std::max<uint64_t>(nv, 1));
  uint8_t* gsig = W.gsig.ensure(64 * std::max<uint64_t>(nv, 1));
  std::vector<uint8_t>& gpk = W.gpk;
  gpk.resize(cache ? 0 : 32 * std::max<uint64_t>(nv, 1));
  parallel_for(T, [&](int t) {
    const Arena& a = arenas[t];
    SigOut& o = so[t];
    for (size_t k = 0; k < o.gwho.size(); ++k) {
      const Rec& r = recs[o.gwho[k]];
      const uint64_t dst = vbase[t] + o.first[k];
      o.first[k] = dst;
      for (uint64_t v = 0; v < r.vote_cnt; ++v) {
        const uint32_t key = a.vkey[r.vote_off + v];
        gkey[dst + v] = key;
        std::memcpy(gsig + 64 * (dst + v), a.vsig[r.vote_off + v], 64);
        if (!cache) std::memcpy(&gpk[32 * (dst + v)], ki.keys[key].bytes.data(), 32);
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
      check(nt_ed25519_verify_batch_groups_keyset(ctx, cache->handle(), gkey, gsig, all.first.data(),
                                                  all.cnt.data(), all.gmsg.data(), G, gbm.data(), nullptr),
            "nt_ed25519_verify_batch_groups_keyset");
    else
      check(nt_ed25519_verify_batch_groups(ctx, gpk.data(), gsig, all.first.data(), all.cnt.data(),
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

// The committee on the device (nt_committee) for ingest_device: built once per
// Core from its committee and key cache (same key order: the committee map's).
struct DeviceCommittee {
  nt_committee* cm = nullptr;
  ~DeviceCommittee() { nt_committee_free(cm); }
};

std::vector<DagError> Core::ingest_device(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                          int threads, size_t* host_decided) const {
  if (!cache) throw crypto::BackendError("Core::ingest_device needs the committee key cache");
  nt_ctx* ctx = crypto::Backend::global().ctx();
  if (!dev_committee) {
    const Committee& cm = *committee;
    std::vector<uint32_t> stake, wids;
    std::vector<uint64_t> wfirst{0};
    for (const auto& kv : cm.authorities) {
      stake.push_back(kv.second.stake);
      wids.insert(wids.end(), kv.second.workers.begin(), kv.second.workers.end());
      wfirst.push_back(wids.size());
    }
    auto d = std::make_shared<DeviceCommittee>();
    check(nt_committee_create(ctx, cache->handle(), stake.data(), wfirst.data(), wids.data(), cm.quorum_threshold(),
                              &d->cm),
          "nt_committee_create");
    dev_committee = d;
  }
  std::vector<uint8_t> code(std::max<size_t>(n, 1));
  if (n) check(nt_certificates_ingest(ctx, dev_committee->cm, data, off, len, n, gc_round, code.data()),
               "nt_certificates_ingest");
  std::vector<DagError> res(n, DagError::Ok);
  std::vector<uint64_t> hoff, hlen;
  std::vector<size_t> hidx;
  for (size_t i = 0; i < n; ++i) {
    if (code[i] == NT_DAG_HOST) {
      hidx.push_back(i);
      hoff.push_back(off[i]);
      hlen.push_back(len[i]);
    } else {
      res[i] = (DagError)code[i];
    }
  }
  if (host_decided) *host_decided = hidx.size();
  if (!hidx.empty()) {
    const auto r = ingest_soa(data, hoff.data(), hlen.data(), hidx.size(), threads);
    for (size_t k = 0; k < hidx.size(); ++k) res[hidx[k]] = r[k];
  }
  return res;
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
