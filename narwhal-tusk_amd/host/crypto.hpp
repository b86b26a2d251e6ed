// crypto.hpp -- C++ mirror of the reference `crypto` crate (crypto/src/lib.rs)
// over the gfx950 C ABI (include/ntcrypto.h).  Same names, argument meaning and
// error behaviour as the Rust API so that callers (primary/worker mirrors in
// narwhal.hpp) and tests read like the reference:
//
//   Digest            crypto/src/lib.rs:21-58
//   Hash              crypto/src/lib.rs:60-62
//   PublicKey         crypto/src/lib.rs:65-119   (base64 serde form)
//   SecretKey         crypto/src/lib.rs:121-161  (seed || pk, zeroized on drop)
//   generate_keypair  crypto/src/lib.rs:163-175
//   Signature         crypto/src/lib.rs:177-219  (new / verify / verify_batch)
//   SignatureService  crypto/src/lib.rs:222-249
//   CryptoError       crypto/src/lib.rs:18       (opaque ed25519::Error)
//
// Every cryptographic operation runs on the GPU; a device/library failure
// throws BackendError (never reported as a rejected signature).
#pragma once
#include <array>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <future>
#include <mutex>
#include <queue>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

struct nt_ctx;
struct nt_keyset;

namespace crypto {

class CryptoError : public std::runtime_error {
 public:
  CryptoError() : std::runtime_error("signature error") {}
};

// A failure of the GPU backend itself (maps the C ABI's negative returns).
class BackendError : public std::runtime_error {
 public:
  explicit BackendError(const std::string& m) : std::runtime_error(m) {}
};

std::string base64_encode(const uint8_t* p, size_t n);
// Standard alphabet with padding (base64 0.13); throws std::invalid_argument.
std::vector<uint8_t> base64_decode(const std::string& s);

struct Digest {
  std::array<uint8_t, 32> bytes{};
  Digest() = default;
  explicit Digest(const std::array<uint8_t, 32>& b) : bytes(b) {}
  static Digest from_slice(const uint8_t* p, size_t n);  // TryFrom<&[u8]>
  std::vector<uint8_t> to_vec() const { return {bytes.begin(), bytes.end()}; }
  size_t size() const { return 32; }
  std::string debug() const;    // full base64 (fmt::Debug)
  std::string display() const;  // first 16 base64 chars (fmt::Display)
  bool operator==(const Digest& o) const { return bytes == o.bytes; }
  bool operator!=(const Digest& o) const { return bytes != o.bytes; }
  bool operator<(const Digest& o) const { return bytes < o.bytes; }
};

struct PublicKey {
  std::array<uint8_t, 32> bytes{};
  std::string encode_base64() const;
  static PublicKey decode_base64(const std::string& s);
  std::string display() const { return encode_base64().substr(0, 16); }
  bool operator==(const PublicKey& o) const { return bytes == o.bytes; }
  bool operator!=(const PublicKey& o) const { return bytes != o.bytes; }
  bool operator<(const PublicKey& o) const { return bytes < o.bytes; }
};

class SecretKey {
 public:
  SecretKey() = default;
  explicit SecretKey(const std::array<uint8_t, 64>& b) : bytes_(b) {}
  SecretKey(const SecretKey&) = default;
  SecretKey& operator=(const SecretKey&) = default;
  ~SecretKey() { bytes_.fill(0); }
  std::string encode_base64() const;
  static SecretKey decode_base64(const std::string& s);
  const std::array<uint8_t, 64>& raw() const { return bytes_; }
  bool operator==(const SecretKey& o) const { return bytes_ == o.bytes_; }

 private:
  std::array<uint8_t, 64> bytes_{};
};

// The GPU context shared by the mirror (nt_init over all visible devices).
class Backend {
 public:
  static Backend& global();
  nt_ctx* ctx() const { return ctx_; }
  ~Backend();

 private:
  Backend();
  nt_ctx* ctx_ = nullptr;
};

// Digest(Sha512::digest(data)[..32]) -- worker/src/processor.rs:38
Digest sha512_digest(const uint8_t* data, size_t n);
inline Digest sha512_digest(const std::vector<uint8_t>& v) { return sha512_digest(v.data(), v.size()); }
// Many messages in one launch.
std::vector<Digest> sha512_digest_batch(const std::vector<std::vector<uint8_t>>& msgs);

// RngCore: fills a buffer with random bytes.
using Rng = std::function<void(uint8_t*, size_t)>;
std::pair<PublicKey, SecretKey> generate_keypair(const Rng& rng);
std::pair<PublicKey, SecretKey> generate_production_keypair();

struct Signature {
  std::array<uint8_t, 32> part1{};  // R
  std::array<uint8_t, 32> part2{};  // s
  static Signature new_(const Digest& digest, const SecretKey& secret);
  std::array<uint8_t, 64> flatten() const;
  // throws CryptoError on reject (dalek verify_strict)
  void verify(const Digest& digest, const PublicKey& public_key) const;
  // throws CryptoError on reject (dalek verify_batch, deterministic rule A.3)
  static void verify_batch(const Digest& digest,
                           const std::vector<std::pair<PublicKey, Signature>>& votes);
};

// Batched forms used by the callers (one GPU launch for many items).
// verdicts[i] = true iff item i verifies (verify_strict).
std::vector<bool> verify_many(const std::vector<Digest>& digests, const std::vector<PublicKey>& keys,
                              const std::vector<Signature>& sigs);
// One verdict per group (certificate): all of groups[g] over digests[g].
std::vector<bool> verify_batch_many(
    const std::vector<Digest>& digests,
    const std::vector<const std::vector<std::pair<PublicKey, Signature>>*>& groups);

// Committee key cache (nt_keyset): per-key comb tables on every device.  Keys
// are addressed by their index in `keys`; verification against a key that is
// not in the set rejects (as an unknown PublicKey would fail later checks).
class KeySet {
 public:
  explicit KeySet(const std::vector<PublicKey>& keys);
  ~KeySet();
  KeySet(const KeySet&) = delete;
  KeySet& operator=(const KeySet&) = delete;
  // index of `pk`, or UINT32_MAX if absent
  uint32_t index_of(const PublicKey& pk) const;
  ::nt_keyset* handle() const { return ks_; }
  size_t size() const { return keys_.size(); }
  // verify_strict of (digest_i, key_i, sig_i) for keys in the set
  std::vector<bool> verify_many(const std::vector<Digest>& digests, const std::vector<PublicKey>& keys,
                                const std::vector<Signature>& sigs) const;
  // verify_batch per group, all signers looked up in the set
  std::vector<bool> verify_batch_many(
      const std::vector<Digest>& digests,
      const std::vector<const std::vector<std::pair<PublicKey, Signature>>*>& groups) const;

 private:
  std::vector<PublicKey> keys_;
  std::vector<std::pair<PublicKey, uint32_t>> sorted_;
  ::nt_keyset* ks_ = nullptr;
};

class SignatureService {
 public:
  explicit SignatureService(SecretKey secret);
  ~SignatureService();
  SignatureService(const SignatureService&) = delete;
  std::future<Signature> request_signature(const Digest& digest);

 private:
  void run();
  SecretKey secret_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::queue<std::pair<Digest, std::promise<Signature>>> q_;
  bool stop_ = false;
  std::thread th_;
};

}  // namespace crypto
