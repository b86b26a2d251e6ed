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
//   primary::Core::sanitize_batch / ingest  core.rs:306-411 batched (SURVEY §8(f).1, (f).2;
//                                           bincode codec in wire.hpp)
//   worker::serialize_batch / batch_digest / Processor / DigestBatcher
//                                           worker/src/batch_maker.rs:117-119,
//                                           worker/src/processor.rs:35-55 (§8(f).3)
#pragma once
#include <condition_variable>
#include <cstdint>
#include <future>
#include <map>
#include <mutex>
#include <thread>
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
  TooOld,               // core.rs:307-310, 317-320, 339-342
  UnexpectedVote,       // core.rs:323-329
  SerializationError,   // primary.rs:230 (bincode decode failure)
  UnexpectedMessage,    // core.rs:384 (CertificatesRequest is not a Core message)
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

struct PrimaryMessage;  // wire.hpp
struct IngestWorkspace;  // ingest.cpp
struct DeviceCommittee;  // ingest.cpp: the nt_committee of a Core's committee + key cache

// Phase times (seconds) of this thread's last Core::ingest (SoA path).
struct IngestStats {
  double decode = 0, prep = 0, digest = 0, strict = 0, batch = 0, total = 0;
};
IngestStats& last_ingest_stats();

// Caller-level batching of primary::Core (core.rs:306-411): the
// Core's sanitize_header / sanitize_vote / sanitize_certificate over a whole
// drained batch of messages, with the same verdict per message as calling them
// one at a time, but every digest in ONE SHA-512 launch, every header and vote
// signature in ONE verify_strict launch and every certificate's votes in ONE
// verify_batch launch.  (The reference's only state these checks read is the
// GC round and the header currently being voted on.)
struct Core {
  const Committee* committee = nullptr;
  Round gc_round = 0;
  Header current_header;
  const crypto::KeySet* cache = nullptr;  // committee key cache (§8(f).4), optional
  // staging reused across ingest calls (one ingest at a time per Core, like the
  // reference's single Core task)
  mutable std::shared_ptr<IngestWorkspace> ws, ws_alt;
  mutable std::shared_ptr<DeviceCommittee> dev_committee;

  std::vector<DagError> sanitize_batch(const std::vector<PrimaryMessage>& msgs) const;
  // wire ingestion (§8(f).2): bincode bytes of n PrimaryMessages (packed, off/len).
  // ingest: flat decode straight into SoA launch buffers on `threads` host threads
  // (ingest.cpp; failure: SerializationError), reference-order checks, 3 launches.
  // ingest_general: decode into the object model (wire.cpp) + sanitize_batch --
  // the same verdicts, kept as the cross-check.  decode_seconds (optional) gets
  // the host decode time.
  std::vector<DagError> ingest(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                               int threads = 1, double* decode_seconds = nullptr) const {
    return ingest_soa(data, off, len, n, threads, decode_seconds);
  }
  std::vector<DagError> ingest_soa(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                   int threads = 1, double* decode_seconds = nullptr) const;
  std::vector<DagError> ingest_general(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                       int threads = 1, double* decode_seconds = nullptr) const;
  // ingest_device: certificates parsed and checked on the GPU from the wire
  // bytes (nt_certificates_ingest; needs the key cache); the messages that path
  // leaves to the host (NT_DAG_HOST: other kinds, non-canonical or malformed
  // bytes) go through ingest_soa.  Same verdicts as ingest.
  std::vector<DagError> ingest_device(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                      int threads = 1, size_t* host_decided = nullptr) const;
  // the batch in chunks of `chunk` messages, two chunks in flight on two
  // workspaces: one chunk's host decode and checks overlap the other's GPU
  // launches.  Same verdicts as ingest (messages are independent).
  std::vector<DagError> ingest_pipelined(const uint8_t* data, const uint64_t* off, const uint64_t* len, size_t n,
                                         int threads, size_t chunk) const;
};

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

// Worker digest batching.  The two Processor tasks of a
// worker (worker.rs:182-188 own batches, :227-233 others' batches) submit into
// one batcher from their own threads; a flusher thread hashes everything queued
// in ONE nt_sha512_trunc32 call when the queued bytes reach max_bytes, the
// queue reaches max_batches, or the oldest queued batch is max_delay_us old.
// submit() copies the batch once into a pinned arena (so the call DMAs it
// without a staging copy) and returns a future of the Processor's output
// (processor.rs:38-48: the digest and the bincode WorkerPrimaryMessage).  A
// Processor that keeps several batches in flight awaits its futures in
// submission order, so its outputs keep the reference's order.  Whether a flush
// runs on the GPU or on the host lane is the C ABI's small-call decision
// (nt_set_small_call_path on the shared context).
class DigestBatcher {
 public:
  struct Policy {
    size_t max_bytes = 256u << 20;
    size_t max_batches = 4096;
    uint32_t max_delay_us = 1000;
  };
  struct Output {
    crypto::Digest digest;
    std::vector<uint8_t> message;  // bincode WorkerPrimaryMessage::{OurBatch, OthersBatch}(digest, id)
  };
  struct Stats {
    uint64_t flushes = 0, batches = 0, bytes = 0;
    double hash_seconds = 0;  // inside nt_sha512_trunc32
  };
  DigestBatcher();
  explicit DigestBatcher(Policy policy);
  ~DigestBatcher();  // hashes what is still queued, then stops the flusher
  DigestBatcher(const DigestBatcher&) = delete;
  DigestBatcher& operator=(const DigestBatcher&) = delete;

  std::future<Output> submit(const Processor& p, const uint8_t* data, size_t len);
  std::future<Output> submit(const Processor& p, const std::vector<uint8_t>& serialized) {
    return submit(p, serialized.data(), serialized.size());
  }
  // Processor::process through the batcher: submit and wait
  Output process(const Processor& p, const std::vector<uint8_t>& serialized) { return submit(p, serialized).get(); }
  void flush();  // hash everything queued now
  size_t pending() const;
  Stats stats() const;

 private:
  struct Queue;
  void run();
  void hash(Queue& q);
  Policy policy_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::unique_ptr<Queue> front_, back_;  // submit into front_, the flusher hashes back_
  bool stop_ = false, force_ = false;
  uint64_t flush_req_ = 0, flush_done_ = 0;
  std::condition_variable done_cv_;
  Stats stats_;
  std::thread th_;
};

}  // namespace worker
