// narwhal.hpp -- C++ mirror of the reference callers of the crypto hot path.
//
//   primary::Header / Vote / Certificate   primary/src/messages.rs:13-264
//     digest layouts                        :70-84, :145-153, :226-234
//     verify (check order, error kinds)     :48-67, :131-142, :189-215
//   primary::Committee (stake, quorum)      config/src/lib.rs:140-173
//   primary::verify_certificates            caller-level batching of Core::sanitize_certificate
//                                           (primary/src/core.rs:338-346):
//                                           one GPU launch for every header signature and
//                                           one for every certificate's votes
//   worker::serialize_batch / batch_digest / Processor
//                                           worker/src/batch_maker.rs:117-119,
//                                           worker/src/processor.rs:35-55
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "crypto.hpp"

namespace primary {

using crypto::Digest;
using crypto::PublicKey;
using crypto::Signature;
using Round = uint64_t;
using WorkerId = uint32_t;
using Stake = uint32_t;

// DagError variants reachable from the verify paths (primary/src/error.rs)
enum class DagError {
  Ok = 0,
  InvalidSignature,
  InvalidHeaderId,
  MalformedHeader,
  UnknownAuthority,
  AuthorityReuse,
  CertificateRequiresQuorum,
};
const char* to_string(DagError e);

struct Authority {
  Stake stake = 0;
  std::set<WorkerId> workers;
};

struct Committee {
  std::map<PublicKey, Authority> authorities;
  Stake stake(const PublicKey& name) const;
  Stake quorum_threshold() const;  // 2 * total / 3 + 1
  bool has_worker(const PublicKey& name, WorkerId id) const;
};

struct Header {
  PublicKey author;
  Round round = 0;
  std::map<Digest, WorkerId> payload;
  std::set<Digest> parents;
  Digest id;
  Signature signature;

  std::vector<uint8_t> digest_preimage() const;
  Digest digest() const;
  DagError verify(const Committee& committee) const;
};

struct Vote {
  Digest id;
  Round round = 0;
  PublicKey origin;
  PublicKey author;
  Signature signature;

  std::vector<uint8_t> digest_preimage() const;
  Digest digest() const;
  DagError verify(const Committee& committee) const;
};

struct Certificate {
  Header header;
  std::vector<std::pair<PublicKey, Signature>> votes;

  static std::vector<Certificate> genesis(const Committee& committee);
  Round round() const { return header.round; }
  PublicKey origin() const { return header.author; }
  std::vector<uint8_t> digest_preimage() const;
  Digest digest() const;
  DagError verify(const Committee& committee) const;
  // PartialEq (messages.rs:256-264): id, round and origin
  bool operator==(const Certificate& o) const;
};

// Verify many certificates with two GPU launches (header signatures, vote
// groups) plus one digest launch; same verdicts as Certificate::verify each.
// With `cache` (the committee's KeySet) both launches use the
// per-key comb tables instead of decompressing every public key.
std::vector<DagError> verify_certificates(const Committee& committee, const std::vector<Certificate>& certs,
                                          const crypto::KeySet* cache = nullptr);
// KeySet over the committee's authorities (BTreeMap order).
std::unique_ptr<crypto::KeySet> committee_keyset(const Committee& committee);

}  // namespace primary

namespace worker {

using Transaction = std::vector<uint8_t>;
using Batch = std::vector<Transaction>;
// bincode WorkerMessage::Batch(batch)
std::vector<uint8_t> serialize_batch(const Batch& batch);
// Digest(Sha512::digest(&serialized)[..32])  (processor.rs:38)
crypto::Digest batch_digest(const std::vector<uint8_t>& serialized);
std::vector<crypto::Digest> batch_digests(const std::vector<std::vector<uint8_t>>& serialized);

// Processor (processor.rs:35-55) minus the store: hash the batch and return the
// bincode WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, id).
struct Processor {
  uint32_t id;
  bool own_digest;
  std::vector<uint8_t> process(const std::vector<uint8_t>& serialized_batch, crypto::Digest* digest_out = nullptr) const;
};

}  // namespace worker
