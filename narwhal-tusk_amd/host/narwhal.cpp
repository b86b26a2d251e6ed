// narwhal.cpp -- primary/worker caller mirrors over the crypto mirror.
#include "narwhal.hpp"

#include <cstring>

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

}  // namespace primary

namespace worker {

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
  std::vector<uint8_t> msg;
  const uint32_t tag = own_digest ? 0 : 1;  // OurBatch / OthersBatch
  for (int i = 0; i < 4; ++i) msg.push_back((uint8_t)(tag >> (8 * i)));
  msg.insert(msg.end(), d.bytes.begin(), d.bytes.end());
  for (int i = 0; i < 4; ++i) msg.push_back((uint8_t)(id >> (8 * i)));
  return msg;
}

}  // namespace worker
