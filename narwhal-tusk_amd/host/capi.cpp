// capi.cpp -- C entry points of libntnarwhal.so for the Python tests and bench.py
// (ctypes): the wire codec (CPU only) and the batched primary::Core ingestion
// path of SURVEY §8(f).1/(f).2 (GPU through libntcrypto).  Not part of the
// crypto crate's boundary (include/ntcrypto.h is).
#include <algorithm>
#include <cstring>
#include <future>
#include <exception>
#include <memory>

#include "../../include/ntcrypto.h"
#include "narwhal.hpp"
#include "wire.hpp"

namespace {
struct CoreHandle {
  primary::Committee committee;
  std::unique_ptr<crypto::KeySet> keyset;
  primary::Core core;
};
}  // namespace

extern "C" {

// Decode one bincode PrimaryMessage and encode it again.  Returns the encoded
// length (<= cap written to out), -1 on a decode error, -2 if cap is too small.
// `used` receives the number of input bytes the decoder consumed.
int64_t ntn_wire_reencode(const uint8_t* data, uint64_t len, uint8_t* out, uint64_t cap, uint64_t* used) {
  primary::PrimaryMessage m;
  size_t u = 0;
  if (!primary::decode(data, (size_t)len, m, &u)) return -1;
  if (used) *used = u;
  const auto v = primary::encode(m);
  if (v.size() > cap) return -2;
  std::memcpy(out, v.data(), v.size());
  return (int64_t)v.size();
}

// Header digest (messages.rs:70-84) of a decoded bincode PrimaryMessage::Header
// or ::Certificate, computed on the host preimage (CPU check of the layout);
// returns the preimage length or -1.
int64_t ntn_wire_header_preimage(const uint8_t* data, uint64_t len, uint8_t* out, uint64_t cap) {
  primary::PrimaryMessage m;
  if (!primary::decode(data, (size_t)len, m)) return -1;
  const primary::Header& h = m.kind == primary::MsgKind::Certificate ? m.certificate.header : m.header;
  const auto v = h.digest_preimage();
  if (v.size() > cap) return -2;
  std::memcpy(out, v.data(), v.size());
  return (int64_t)v.size();
}

// Committee of n authorities (keys32[n][32], stake[n], workers 0..nworkers[i]-1),
// Core state (gc_round, current header as bincode of a PrimaryMessage::Header,
// may be null), optional committee key cache.  Returns null on failure.
void* ntn_core_new(const uint8_t* keys32, const uint32_t* stakes, const uint32_t* nworkers, uint32_t n,
                   uint64_t gc_round, const uint8_t* cur_header, uint64_t cur_len, int use_keyset) {
  try {
    auto h = std::make_unique<CoreHandle>();
    for (uint32_t i = 0; i < n; ++i) {
      crypto::PublicKey pk;
      std::memcpy(pk.bytes.data(), keys32 + 32 * (size_t)i, 32);
      primary::Authority a;
      a.stake = stakes[i];
      for (uint32_t w = 0; w < nworkers[i]; ++w) a.workers.insert(w);
      h->committee.authorities[pk] = a;
    }
    if (cur_header) {
      primary::PrimaryMessage m;
      if (!primary::decode(cur_header, (size_t)cur_len, m) || m.kind != primary::MsgKind::Header) return nullptr;
      h->core.current_header = m.header;
    }
    if (use_keyset) h->keyset = primary::committee_keyset(h->committee);
    h->core.committee = &h->committee;
    h->core.gc_round = gc_round;
    h->core.cache = h->keyset.get();
    return h.release();
  } catch (const std::exception&) {
    return nullptr;
  }
}

void ntn_core_free(void* p) { delete (CoreHandle*)p; }

// Core::ingest over n packed wire messages: out_codes[i] = primary::DagError.
// Returns 0, or -2 on a backend failure (never reported as a verdict).
// general = 1: the object-model decoder + sanitize_batch (cross-check path);
// general = 2: Core::ingest_device (certificates parsed on the GPU), and
// decode_seconds then returns the count of messages left to the host decoder.
int ntn_core_ingest(void* p, const uint8_t* data, const uint64_t* off, const uint64_t* len, uint64_t n,
                    int threads, int32_t* out_codes, double* decode_seconds, int general) {
  try {
    const auto& core = ((CoreHandle*)p)->core;
    std::vector<primary::DagError> r;
    if (general == 2) {
      size_t host = 0;
      r = core.ingest_device(data, off, len, (size_t)n, threads, &host);
      if (decode_seconds) *decode_seconds = (double)host;  // mode 2: messages left to the host decoder
    } else {
      r = general ? core.ingest_general(data, off, len, (size_t)n, threads, decode_seconds)
                  : core.ingest(data, off, len, (size_t)n, threads, decode_seconds);
    }
    for (uint64_t i = 0; i < n; ++i) out_codes[i] = (int32_t)r[i];
    return 0;
  } catch (const std::exception&) {
    return -2;
  }
}

// Core::ingest_pipelined: chunks of `chunk` messages, two in flight.
int ntn_core_ingest_pipelined(void* p, const uint8_t* data, const uint64_t* off, const uint64_t* len, uint64_t n,
                              int threads, uint64_t chunk, int32_t* out_codes) {
  try {
    const auto r = ((CoreHandle*)p)->core.ingest_pipelined(data, off, len, (size_t)n, threads, (size_t)chunk);
    for (uint64_t i = 0; i < n; ++i) out_codes[i] = (int32_t)r[i];
    return 0;
  } catch (const std::exception&) {
    return -2;
  }
}

// phase times of the calling thread's last ingest: decode, prep, digest,
// verify_strict, verify_batch, total (seconds)
void ntn_last_ingest_stats(double out[6]) {
  const auto& s = primary::last_ingest_stats();
  out[0] = s.decode;
  out[1] = s.prep;
  out[2] = s.digest;
  out[3] = s.strict;
  out[4] = s.batch;
  out[5] = s.total;
}

// ---- worker::DigestBatcher -------------------------------
void* ntn_batcher_new(uint64_t max_bytes, uint64_t max_batches, uint32_t max_delay_us) {
  try {
    worker::DigestBatcher::Policy p;
    p.max_bytes = (size_t)max_bytes;
    p.max_batches = (size_t)max_batches;
    p.max_delay_us = max_delay_us;
    return new worker::DigestBatcher(p);
  } catch (const std::exception&) {
    return nullptr;
  }
}
void ntn_batcher_free(void* b) { delete (worker::DigestBatcher*)b; }

// queue one serialized batch of Processor (worker_id, own); returns a ticket
// for ntn_batcher_wait (NULL on failure)
void* ntn_batcher_submit(void* b, uint32_t worker_id, int own, const uint8_t* data, uint64_t len) {
  try {
    worker::Processor p{worker_id, own != 0};
    return new std::future<worker::DigestBatcher::Output>(
        ((worker::DigestBatcher*)b)->submit(p, data, (size_t)len));
  } catch (const std::exception&) {
    return nullptr;
  }
}

// wait for a ticket (and free it): digest32 (32 bytes) and the Processor's
// 40-byte output message; 0, or -2 if the backend failed
int ntn_batcher_wait(void* ticket, uint8_t* digest32, uint8_t* msg40) {
  auto* f = (std::future<worker::DigestBatcher::Output>*)ticket;
  int rc = 0;
  try {
    const auto o = f->get();
    std::memcpy(digest32, o.digest.bytes.data(), 32);
    std::memcpy(msg40, o.message.data(), std::min<size_t>(40, o.message.size()));
  } catch (const std::exception&) {
    rc = -2;
  }
  delete f;
  return rc;
}

void ntn_batcher_flush(void* b) { ((worker::DigestBatcher*)b)->flush(); }

// flushes, batches, bytes, seconds inside nt_sha512_trunc32
void ntn_batcher_stats(void* b, double out[4]) {
  const auto s = ((worker::DigestBatcher*)b)->stats();
  out[0] = (double)s.flushes;
  out[1] = (double)s.batches;
  out[2] = (double)s.bytes;
  out[3] = s.hash_seconds;
}

// the small-call path of the mirror's shared context (include/ntcrypto.h)
int ntn_set_small_call_path(int mode, int threads) {
  try {
    return nt_set_small_call_path(crypto::Backend::global().ctx(), mode, threads);
  } catch (const std::exception&) {
    return -2;
  }
}

}  // extern "C"
