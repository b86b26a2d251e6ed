// narwhal.cpp -- primary/worker caller mirrors over the crypto mirror.
#include "narwhal.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "../../include/ntcrypto.h"
#include "wire.hpp"

namespace primary {

const char* to_string(DagError e) {
  switch (e) {
    case DagError::Ok: return "Ok";
    case DagError::InvalidSignature: return "InvalidSignature";
    case DagError::InvalidHeaderId: return "InvalidHeaderId";
    case DagError::MalformedHeader: return "MalformedHeader";
    case DagError::UnknownAuthority: return "UnknownAuthority";
    case DagError::AuthorityReuse: return "AuthorityReuse";
    case DagError::CertificateRequiresQuorum: return "CertificateRequiresQuorum";
    case DagError::TooOld: return "TooOld";
    case DagError::UnexpectedVote: return "UnexpectedVote";
    case DagError::SerializationError: return "SerializationError";
    case DagError::UnexpectedMessage: return "UnexpectedMessage";
  }
  return "?";
}

Stake Committee::stake(const PublicKey& name) const {
  auto it = authorities.find(name);
  return it == authorities.end() ? 0 : it->second.stake;
}

Stake Committee::quorum_threshold() const {
  Stake total = 0;
  for (const auto& kv : authorities) total += kv.second.stake;
  return 2 * total / 3 + 1;
}

bool Committee::has_worker(const PublicKey& name, WorkerId id) const {
  auto it = authorities.find(name);
  return it != authorities.end() && it->second.workers.count(id);
}

namespace {
void put(std::vector<uint8_t>& v, const uint8_t* p, size_t n) { v.insert(v.end(), p, p + n); }
void put_u64(std::vector<uint8_t>& v, uint64_t x) {
  for (int i = 0; i < 8; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}
void put_u32(std::vector<uint8_t>& v, uint32_t x) {
  for (int i = 0; i < 4; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}
}  // namespace

// messages.rs:70-84: author || round_le || (digest || worker_id_le)* || parent*
std::vector<uint8_t> Header::digest_preimage() const {
  std::vector<uint8_t> v;
  put(v, author.bytes.data(), 32);
  put_u64(v, round);
  for (const auto& kv : payload) {
    put(v, kv.first.bytes.data(), 32);
    put_u32(v, kv.second);
  }
  for (const auto& p : parents) put(v, p.bytes.data(), 32);
  return v;
}
Digest Header::digest() const { return crypto::sha512_digest(digest_preimage()); }

// messages.rs:145-153: id || round_le || origin
std::vector<uint8_t> Vote::digest_preimage() const {
  std::vector<uint8_t> v;
  put(v, id.bytes.data(), 32);
  put_u64(v, round);
  put(v, origin.bytes.data(), 32);
  return v;
}
Digest Vote::digest() const { return crypto::sha512_digest(digest_preimage()); }

// messages.rs:226-234: header.id || round_le || origin (same layout as Vote)
std::vector<uint8_t> Certificate::digest_preimage() const {
  std::vector<uint8_t> v;
  put(v, header.id.bytes.data(), 32);
  put_u64(v, round());
  put(v, origin().bytes.data(), 32);
  return v;
}
Digest Certificate::digest() const { return crypto::sha512_digest(digest_preimage()); }

bool Certificate::operator==(const Certificate& o) const {
  return header.id == o.header.id && round() == o.round() && origin() == o.origin();
}

std::vector<Certificate> Certificate::genesis(const Committee& committee) {
  std::vector<Certificate> out;
  for (const auto& kv : committee.authorities) {
    Certificate c;
    c.header.author = kv.first;
    out.push_back(c);
  }
  return out;
}

namespace {
// Header checks before the signature (messages.rs:48-61); id digest given.
DagError header_precheck(const Header& h, const Digest& computed, const Committee& committee) {
  if (computed != h.id) return DagError::InvalidHeaderId;
  if (committee.stake(h.author) == 0) return DagError::UnknownAuthority;
  for (const auto& kv : h.payload)
    if (!committee.has_worker(h.author, kv.second)) return DagError::MalformedHeader;
  return DagError::Ok;
}

// Quorum accounting (messages.rs:196-211)
DagError quorum_check(const Certificate& c, const Committee& committee) {
  Stake weight = 0;
  std::set<PublicKey> used;
  for (const auto& kv : c.votes) {
    if (used.count(kv.first)) return DagError::AuthorityReuse;
    const Stake s = committee.stake(kv.first);
    if (s == 0) return DagError::UnknownAuthority;
    used.insert(kv.first);
    weight += s;
  }
  if (weight < committee.quorum_threshold()) return DagError::CertificateRequiresQuorum;
  return DagError::Ok;
}
}  // namespace

DagError Header::verify(const Committee& committee) const {
  const DagError e = header_precheck(*this, digest(), committee);
  if (e != DagError::Ok) return e;
  try {
    signature.verify(id, author);
  } catch (const crypto::CryptoError&) {
    return DagError::InvalidSignature;
  }
  return DagError::Ok;
}

DagError Vote::verify(const Committee& committee) const {
  if (committee.stake(author) == 0) return DagError::UnknownAuthority;
  try {
    signature.verify(digest(), author);
  } catch (const crypto::CryptoError&) {
    return DagError::InvalidSignature;
  }
  return DagError::Ok;
}

DagError Certificate::verify(const Committee& committee) const {
  for (const auto& g : genesis(committee))
    if (g == *this) return DagError::Ok;
  DagError e = header.verify(committee);
  if (e != DagError::Ok) return e;
  e = quorum_check(*this, committee);
  if (e != DagError::Ok) return e;
  try {
    Signature::verify_batch(digest(), votes);
  } catch (const crypto::CryptoError&) {
    return DagError::InvalidSignature;
  }
  return DagError::Ok;
}

std::unique_ptr<crypto::KeySet> committee_keyset(const Committee& committee) {
  std::vector<PublicKey> keys;
  for (const auto& kv : committee.authorities) keys.push_back(kv.first);
  return std::make_unique<crypto::KeySet>(keys);
}

std::vector<DagError> verify_certificates(const Committee& committee, const std::vector<Certificate>& certs,
                                          const crypto::KeySet* cache) {
  const size_t n = certs.size();
  std::vector<DagError> res(n, DagError::Ok);
  if (!n) return res;
  const auto genesis = Certificate::genesis(committee);
  // 1) all header digests and certificate digests in one SHA launch
  std::vector<std::vector<uint8_t>> pre;
  pre.reserve(2 * n);
  for (const auto& c : certs) pre.push_back(c.header.digest_preimage());
  for (const auto& c : certs) pre.push_back(c.digest_preimage());
  const auto dig = crypto::sha512_digest_batch(pre);
  // 2) host checks in the reference order; collect GPU work
  std::vector<size_t> todo;
  std::vector<bool> is_genesis(n, false);
  for (size_t i = 0; i < n; ++i) {
    for (const auto& g : genesis)
      if (g == certs[i]) is_genesis[i] = true;
    if (is_genesis[i]) continue;
    DagError e = header_precheck(certs[i].header, dig[i], committee);
    if (e == DagError::Ok) todo.push_back(i);
    res[i] = e;
  }
  // 3) header signatures: one verify_strict launch
  std::vector<Digest> hd;
  std::vector<PublicKey> hk;
  std::vector<Signature> hs;
  for (size_t i : todo) {
    hd.push_back(certs[i].header.id);
    hk.push_back(certs[i].header.author);
    hs.push_back(certs[i].header.signature);
  }
  const auto hv = cache ? cache->verify_many(hd, hk, hs) : crypto::verify_many(hd, hk, hs);
  // 4) quorum, then every remaining certificate's votes in one verify_batch launch
  std::vector<size_t> grp_idx;
  std::vector<Digest> gd;
  std::vector<const std::vector<std::pair<PublicKey, Signature>>*> groups;
  for (size_t t = 0; t < todo.size(); ++t) {
    const size_t i = todo[t];
    if (!hv[t]) {
      res[i] = DagError::InvalidSignature;
      continue;
    }
    const DagError e = quorum_check(certs[i], committee);
    if (e != DagError::Ok) {
      res[i] = e;
      continue;
    }
    grp_idx.push_back(i);
    gd.push_back(dig[n + i]);
    groups.push_back(&certs[i].votes);
  }
  const auto gv = cache ? cache->verify_batch_many(gd, groups) : crypto::verify_batch_many(gd, groups);
  for (size_t t = 0; t < grp_idx.size(); ++t)
    if (!gv[t]) res[grp_idx[t]] = DagError::InvalidSignature;
  return res;
}

namespace {
bool is_genesis(const Certificate& c, const Committee& committee) {
  // Certificate::genesis(committee).contains(c): default header (zero id,
  // round 0) of a committee member, compared by (id, round, origin)
  static const Digest zero{};
  return c.header.id == zero && c.round() == 0 && committee.authorities.count(c.origin());
}
}  // namespace

std::vector<DagError> Core::sanitize_batch(const std::vector<PrimaryMessage>& msgs) const {
  const Committee& cm = *committee;
  const size_t n = msgs.size();
  std::vector<DagError> res(n, DagError::Ok);
  // 1) round filters (core.rs:307-310, 317-329, 339-342); collect digest preimages
  enum Need : uint8_t { kNone, kHeader, kVote, kCert };
  std::vector<Need> need(n, kNone);
  std::vector<std::vector<uint8_t>> pre;
  std::vector<size_t> pre_at(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const auto& m = msgs[i];
    switch (m.kind) {
      case MsgKind::Header:
        if (m.header.round < gc_round) { res[i] = DagError::TooOld; break; }
        need[i] = kHeader;
        pre_at[i] = pre.size();
        pre.push_back(m.header.digest_preimage());
        break;
      case MsgKind::Vote: {
        const Vote& v = m.vote;
        if (v.round < current_header.round) { res[i] = DagError::TooOld; break; }
        if (!(v.id == current_header.id && v.origin == current_header.author && v.round == current_header.round)) {
          res[i] = DagError::UnexpectedVote;
          break;
        }
        need[i] = kVote;
        pre_at[i] = pre.size();
        pre.push_back(v.digest_preimage());
        break;
      }
      case MsgKind::Certificate: {
        const Certificate& c = m.certificate;
        if (c.round() < gc_round) { res[i] = DagError::TooOld; break; }
        if (is_genesis(c, cm)) break;
        need[i] = kCert;
        pre_at[i] = pre.size();
        pre.push_back(c.header.digest_preimage());
        pre.push_back(c.digest_preimage());
        break;
      }
      case MsgKind::CertificatesRequest: res[i] = DagError::UnexpectedMessage; break;
    }
  }
  const auto dig = crypto::sha512_digest_batch(pre);  // launch 1
  // 2) host prechecks in the reference order; collect the signature work
  std::vector<Digest> sd;
  std::vector<PublicKey> sk;
  std::vector<Signature> ss;
  std::vector<size_t> s_of(n, SIZE_MAX);
  std::vector<Digest> gd;
  std::vector<const std::vector<std::pair<PublicKey, Signature>>*> groups;
  std::vector<size_t> g_of(n, SIZE_MAX);
  for (size_t i = 0; i < n; ++i) {
    const auto& m = msgs[i];
    if (need[i] == kHeader || need[i] == kCert) {
      const Header& h = need[i] == kHeader ? m.header : m.certificate.header;
      const DagError e = header_precheck(h, dig[pre_at[i]], cm);
      if (e != DagError::Ok) { res[i] = e; continue; }
      s_of[i] = sd.size();
      sd.push_back(h.id);
      sk.push_back(h.author);
      ss.push_back(h.signature);
      if (need[i] == kCert) {
        // Certificate::verify runs Header::verify -- signature included -- before
        // the quorum loop (messages.rs:194-211): a failed quorum is reported only
        // if the header signature passes, so the header stays in the strict launch
        const DagError q = quorum_check(m.certificate, cm);
        if (q != DagError::Ok) { res[i] = q; continue; }
        g_of[i] = gd.size();
        gd.push_back(dig[pre_at[i] + 1]);
        groups.push_back(&m.certificate.votes);
      }
    } else if (need[i] == kVote) {
      if (cm.stake(m.vote.author) == 0) { res[i] = DagError::UnknownAuthority; continue; }
      s_of[i] = sd.size();
      sd.push_back(dig[pre_at[i]]);
      sk.push_back(m.vote.author);
      ss.push_back(m.vote.signature);
    }
  }
  // 3) launch 2 (every header/vote signature) and launch 3 (every certificate's votes).
  // A certificate whose header signature fails reports InvalidSignature whatever
  // its quorum or votes, so its vote group may be checked in the same pass; one
  // that failed the quorum check keeps that error unless its header signature fails.
  const auto sv = cache ? cache->verify_many(sd, sk, ss) : crypto::verify_many(sd, sk, ss);
  const auto gv = groups.empty() ? std::vector<bool>{}
                  : cache ? cache->verify_batch_many(gd, groups) : crypto::verify_batch_many(gd, groups);
  for (size_t i = 0; i < n; ++i) {
    if (s_of[i] != SIZE_MAX && !sv[s_of[i]]) res[i] = DagError::InvalidSignature;
    else if (g_of[i] != SIZE_MAX && !gv[g_of[i]]) res[i] = DagError::InvalidSignature;
  }
  return res;
}

std::vector<DagError> Core::ingest_general(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                   int threads, double* decode_seconds) const {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<PrimaryMessage> msgs(n);
  std::vector<uint8_t> ok(n, 0);
  if (threads < 1) threads = 1;
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (size_t i = n * t / threads; i < n * (t + 1) / threads; ++i)
        ok[i] = decode(data + off[i], (size_t)len[i], msgs[i]);
    });
  for (auto& th : pool) th.join();
  if (decode_seconds)
    *decode_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::vector<PrimaryMessage> good;
  std::vector<size_t> idx;
  good.reserve(n);
  for (size_t i = 0; i < n; ++i)
    if (ok[i]) {
      idx.push_back(i);
      good.push_back(std::move(msgs[i]));
    }
  std::vector<DagError> res(n, DagError::SerializationError);
  const auto r = sanitize_batch(good);
  for (size_t k = 0; k < idx.size(); ++k) res[idx[k]] = r[k];
  return res;
}

}  // namespace primary

namespace worker {

namespace {
// processor.rs:40-48: bincode WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, worker id)
std::vector<uint8_t> processor_message(const Processor& p, const crypto::Digest& d) {
  std::vector<uint8_t> msg;
  const uint32_t tag = p.own_digest ? 0 : 1;
  for (int i = 0; i < 4; ++i) msg.push_back((uint8_t)(tag >> (8 * i)));
  msg.insert(msg.end(), d.bytes.begin(), d.bytes.end());
  for (int i = 0; i < 4; ++i) msg.push_back((uint8_t)(p.id >> (8 * i)));
  return msg;
}
}  // namespace

// One side of the double buffer: the batches' bytes back to back in pinned
// memory (nt_host_alloc; ordinary memory if pinning fails -- the flush then
// goes through the library's staging copy), their offsets / lengths, and the
// waiting Processors.
struct DigestBatcher::Queue {
  uint8_t* arena = nullptr;
  bool pinned = false;
  size_t cap = 0, used = 0;
  std::vector<uint64_t> off, len;
  std::vector<Processor> procs;
  std::vector<std::promise<Output>> waiters;
  std::chrono::steady_clock::time_point oldest;
  ~Queue() { release(arena, pinned); }
  static void release(uint8_t* a, bool pin) {
    if (!a) return;
    if (pin) nt_host_free(a);
    else std::free(a);
  }
  void reserve(size_t need) {
    if (need <= cap) return;
    size_t c = std::max<size_t>(need, std::max<size_t>(2 * cap, 1u << 20));
    bool pin = true;
    auto* a = (uint8_t*)nt_host_alloc(c);
    if (!a) {
      pin = false;
      a = (uint8_t*)std::malloc(c);
    }
    if (!a) throw std::bad_alloc();
    if (used) std::memcpy(a, arena, used);
    release(arena, pinned);
    arena = a;
    pinned = pin;
    cap = c;
  }
  void clear() {
    used = 0;
    off.clear();
    len.clear();
    procs.clear();
    waiters.clear();
  }
};

DigestBatcher::DigestBatcher() : DigestBatcher(Policy()) {}

DigestBatcher::DigestBatcher(Policy policy)
    : policy_(policy), front_(std::make_unique<Queue>()), back_(std::make_unique<Queue>()) {
  th_ = std::thread([this] { run(); });
}

DigestBatcher::~DigestBatcher() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

std::future<DigestBatcher::Output> DigestBatcher::submit(const Processor& p, const uint8_t* data, size_t len) {
  std::promise<Output> pr;
  auto fut = pr.get_future();
  {
    std::lock_guard<std::mutex> lk(mu_);
    Queue& q = *front_;
    if (q.off.empty()) q.oldest = std::chrono::steady_clock::now();
    q.reserve(q.used + len + 1);
    if (len) std::memcpy(q.arena + q.used, data, len);
    q.off.push_back(q.used);
    q.len.push_back(len);
    q.used += len;
    q.procs.push_back(p);
    q.waiters.push_back(std::move(pr));
  }
  cv_.notify_all();
  return fut;
}

void DigestBatcher::flush() {
  std::unique_lock<std::mutex> lk(mu_);
  const uint64_t ticket = ++flush_req_;
  force_ = true;
  cv_.notify_all();
  done_cv_.wait(lk, [&] { return flush_done_ >= ticket; });
}

size_t DigestBatcher::pending() const {
  std::lock_guard<std::mutex> lk(mu_);
  return front_->off.size();
}

DigestBatcher::Stats DigestBatcher::stats() const {
  std::lock_guard<std::mutex> lk(mu_);
  return stats_;
}

// Flusher: wait until a flush rule fires (bytes, batch count, age of the
// oldest batch, an explicit flush or shutdown), swap the queues, hash the
// taken queue with one C-ABI call while submitters fill the other one.
void DigestBatcher::run() {
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    auto due = [&] {
      const Queue& q = *front_;
      return stop_ || force_ || q.used >= policy_.max_bytes || q.off.size() >= policy_.max_batches;
    };
    if (!stop_ && !force_ && front_->off.empty()) {
      cv_.wait(lk, [&] { return stop_ || force_ || !front_->off.empty(); });
      continue;  // the first batch starts the age clock: re-evaluate the rules
    }
    // returns when a rule fires or at the oldest batch's deadline (age rule)
    if (!due()) cv_.wait_until(lk, front_->oldest + std::chrono::microseconds(policy_.max_delay_us), due);
    const bool stopping = stop_;
    const uint64_t req = flush_req_;  // every flush() so far is served by this swap
    force_ = false;
    std::swap(front_, back_);
    lk.unlock();
    if (!back_->off.empty()) hash(*back_);
    back_->clear();
    lk.lock();
    flush_done_ = std::max(flush_done_, req);
    done_cv_.notify_all();
    if (stopping && front_->off.empty()) return;
  }
}

// Runs on the flusher thread: every waiter of the taken queue is resolved,
// with a digest or with an exception -- an exception that escaped here would
// end the thread and with it the process (std::terminate), e.g. the
// BackendError of a first nt_init that fails or a std::bad_alloc.
void DigestBatcher::hash(Queue& q) {
  const size_t n = q.off.size();
  size_t done = 0;  // waiters resolved so far
  try {
    std::vector<crypto::Digest> dig(n);
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = nt_sha512_trunc32(crypto::Backend::global().ctx(), q.arena, q.off.data(), q.len.data(), n,
                                     dig[0].bytes.data());
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    {
      std::lock_guard<std::mutex> lk(mu_);
      stats_.flushes += 1;
      stats_.batches += n;
      stats_.bytes += q.used;
      stats_.hash_seconds += dt;
    }
    for (; done < n; ++done) {
      if (rc != NT_OK) {  // a backend failure is an error for every waiter, never a digest
        q.waiters[done].set_exception(std::make_exception_ptr(
            crypto::BackendError(std::string("nt_sha512_trunc32 failed: ") + nt_strerror(rc))));
        continue;
      }
      q.waiters[done].set_value(Output{dig[done], processor_message(q.procs[done], dig[done])});
    }
  } catch (...) {
    const std::exception_ptr ex = std::current_exception();
    for (; done < n; ++done) {
      try {
        q.waiters[done].set_exception(ex);
      } catch (...) {  // already satisfied: nothing left to tell this waiter
      }
    }
  }
}

std::vector<uint8_t> serialize_batch(const Batch& batch) {
  std::vector<uint8_t> v;
  auto u32 = [&](uint32_t x) { for (int i = 0; i < 4; ++i) v.push_back((uint8_t)(x >> (8 * i))); };
  auto u64 = [&](uint64_t x) { for (int i = 0; i < 8; ++i) v.push_back((uint8_t)(x >> (8 * i))); };
  u32(0);  // WorkerMessage::Batch
  u64(batch.size());
  for (const auto& tx : batch) {
    u64(tx.size());
    v.insert(v.end(), tx.begin(), tx.end());
  }
  return v;
}

crypto::Digest batch_digest(const std::vector<uint8_t>& serialized) { return crypto::sha512_digest(serialized); }

std::vector<crypto::Digest> batch_digests(const std::vector<std::vector<uint8_t>>& serialized) {
  return crypto::sha512_digest_batch(serialized);
}

std::vector<uint8_t> Processor::process(const std::vector<uint8_t>& serialized_batch, crypto::Digest* digest_out) const {
  const crypto::Digest d = batch_digest(serialized_batch);
  if (digest_out) *digest_out = d;
  return processor_message(*this, d);
}

}  // namespace worker
