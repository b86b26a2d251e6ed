// crypto.cpp -- implementation of the crypto crate mirror over include/ntcrypto.h.
#include "crypto.hpp"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../include/ntcrypto.h"

namespace crypto {

namespace {
const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

void check(int rc, const char* what) {
  if (rc != NT_OK) throw BackendError(std::string(what) + ": " + nt_strerror(rc));
}
}  // namespace

std::string base64_encode(const uint8_t* p, size_t n) {
  std::string out;
  out.reserve((n + 2) / 3 * 4);
  for (size_t i = 0; i < n; i += 3) {
    uint32_t v = (uint32_t)p[i] << 16;
    if (i + 1 < n) v |= (uint32_t)p[i + 1] << 8;
    if (i + 2 < n) v |= p[i + 2];
    out.push_back(kB64[(v >> 18) & 63]);
    out.push_back(kB64[(v >> 12) & 63]);
    out.push_back(i + 1 < n ? kB64[(v >> 6) & 63] : '=');
    out.push_back(i + 2 < n ? kB64[v & 63] : '=');
  }
  return out;
}

std::vector<uint8_t> base64_decode(const std::string& s) {
  auto val = [](char c) -> int {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    return -1;
  };
  if (s.size() % 4) throw std::invalid_argument("InvalidLength");
  std::vector<uint8_t> out;
  for (size_t i = 0; i < s.size(); i += 4) {
    int v[4];
    int pad = 0;
    for (int j = 0; j < 4; ++j) {
      const char c = s[i + j];
      if (c == '=' && i + 4 == s.size() && j >= 2) {
        v[j] = 0;
        ++pad;
      } else {
        if (pad) throw std::invalid_argument("InvalidByte");
        v[j] = val(c);
        if (v[j] < 0) throw std::invalid_argument("InvalidByte");
      }
    }
    // base64 0.13 rejects non-zero unused bits in the last data symbol (InvalidLastSymbol)
    if ((pad == 1 && (v[2] & 3)) || (pad == 2 && (v[1] & 15))) throw std::invalid_argument("InvalidLastSymbol");
    const uint32_t w = ((uint32_t)v[0] << 18) | ((uint32_t)v[1] << 12) | ((uint32_t)v[2] << 6) | (uint32_t)v[3];
    out.push_back((uint8_t)(w >> 16));
    if (pad < 2) out.push_back((uint8_t)(w >> 8));
    if (pad < 1) out.push_back((uint8_t)w);
  }
  return out;
}

Digest Digest::from_slice(const uint8_t* p, size_t n) {
  if (n != 32) throw std::invalid_argument("TryFromSliceError");
  Digest d;
  std::memcpy(d.bytes.data(), p, 32);
  return d;
}
std::string Digest::debug() const { return base64_encode(bytes.data(), 32); }
std::string Digest::display() const { return debug().substr(0, 16); }

std::string PublicKey::encode_base64() const { return base64_encode(bytes.data(), 32); }
PublicKey PublicKey::decode_base64(const std::string& s) {
  const auto b = base64_decode(s);
  if (b.size() < 32) throw std::invalid_argument("InvalidLength");
  PublicKey pk;
  std::memcpy(pk.bytes.data(), b.data(), 32);
  return pk;
}
std::string SecretKey::encode_base64() const { return base64_encode(bytes_.data(), 64); }
SecretKey SecretKey::decode_base64(const std::string& s) {
  const auto b = base64_decode(s);
  if (b.size() < 64) throw std::invalid_argument("InvalidLength");
  std::array<uint8_t, 64> a;
  std::memcpy(a.data(), b.data(), 64);
  return SecretKey(a);
}

// every visible device, or only ordinal $NT_DEVICE (one process per GPU)
Backend::Backend() {
  const char* d = std::getenv("NT_DEVICE");
  if (d && *d) check(nt_init_device(&ctx_, std::atoi(d)), "nt_init_device");
  else check(nt_init(&ctx_, 0), "nt_init");
}
Backend::~Backend() {
  if (ctx_) nt_free(ctx_);
}
Backend& Backend::global() {
  static Backend b;
  return b;
}

Digest sha512_digest(const uint8_t* data, size_t n) {
  const uint64_t off = 0, len = n;
  Digest d;
  static const uint8_t empty = 0;
  check(nt_sha512_trunc32(Backend::global().ctx(), n ? data : &empty, &off, &len, 1, d.bytes.data()),
        "nt_sha512_trunc32");
  return d;
}

std::vector<Digest> sha512_digest_batch(const std::vector<std::vector<uint8_t>>& msgs) {
  std::vector<uint8_t> data;
  std::vector<uint64_t> off, len;
  for (const auto& m : msgs) {
    off.push_back(data.size());
    len.push_back(m.size());
    data.insert(data.end(), m.begin(), m.end());
  }
  data.push_back(0);
  std::vector<Digest> out(msgs.size());
  if (msgs.empty()) return out;
  check(nt_sha512_trunc32(Backend::global().ctx(), data.data(), off.data(), len.data(), msgs.size(),
                          out[0].bytes.data()),
        "nt_sha512_trunc32");
  return out;
}

std::pair<PublicKey, SecretKey> generate_keypair(const Rng& rng) {
  uint8_t seed[32];
  rng(seed, 32);  // dalek Keypair::generate draws the 32-byte secret from the RNG
  PublicKey pk;
  check(nt_ed25519_keypair_batch(Backend::global().ctx(), seed, 1, pk.bytes.data()), "nt_ed25519_keypair_batch");
  std::array<uint8_t, 64> sk;
  std::memcpy(sk.data(), seed, 32);
  std::memcpy(sk.data() + 32, pk.bytes.data(), 32);
  std::memset(seed, 0, sizeof seed);
  return {pk, SecretKey(sk)};
}

std::pair<PublicKey, SecretKey> generate_production_keypair() {
  std::random_device rd;
  return generate_keypair([&](uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) p[i] = (uint8_t)rd();
  });
}

Signature Signature::new_(const Digest& digest, const SecretKey& secret) {
  const uint64_t off = 0, len = 32;
  uint8_t pk[32], sig[64];
  check(nt_ed25519_sign_batch(Backend::global().ctx(), secret.raw().data(), digest.bytes.data(), &off, &len, 1,
                              pk, sig),
        "nt_ed25519_sign_batch");
  // dalek Keypair::from_bytes(...).expect("Unable to load secret key")
  if (std::memcmp(pk, secret.raw().data() + 32, 32) != 0) throw std::invalid_argument("Unable to load secret key");
  Signature s;
  std::memcpy(s.part1.data(), sig, 32);
  std::memcpy(s.part2.data(), sig + 32, 32);
  return s;
}

std::array<uint8_t, 64> Signature::flatten() const {
  std::array<uint8_t, 64> out;
  std::memcpy(out.data(), part1.data(), 32);
  std::memcpy(out.data() + 32, part2.data(), 32);
  return out;
}

std::vector<bool> verify_many(const std::vector<Digest>& digests, const std::vector<PublicKey>& keys,
                              const std::vector<Signature>& sigs) {
  const size_t n = digests.size();
  if (keys.size() != n || sigs.size() != n) throw std::invalid_argument("length mismatch");
  std::vector<bool> out(n, false);
  if (!n) return out;
  std::vector<uint8_t> pk(32 * n), sg(64 * n), msg(32 * n);
  std::vector<uint64_t> off(n), len(n, 32);
  for (size_t i = 0; i < n; ++i) {
    std::memcpy(&pk[32 * i], keys[i].bytes.data(), 32);
    const auto f = sigs[i].flatten();
    std::memcpy(&sg[64 * i], f.data(), 64);
    std::memcpy(&msg[32 * i], digests[i].bytes.data(), 32);
    off[i] = 32 * i;
  }
  std::vector<uint8_t> bm((n + 7) / 8);
  check(nt_ed25519_verify_strict(Backend::global().ctx(), pk.data(), sg.data(), msg.data(), off.data(),
                                 len.data(), n, bm.data()),
        "nt_ed25519_verify_strict");
  for (size_t i = 0; i < n; ++i) out[i] = (bm[i / 8] >> (i % 8)) & 1;
  return out;
}

void Signature::verify(const Digest& digest, const PublicKey& public_key) const {
  if (!verify_many({digest}, {public_key}, {*this})[0]) throw CryptoError();
}

std::vector<bool> verify_batch_many(
    const std::vector<Digest>& digests,
    const std::vector<const std::vector<std::pair<PublicKey, Signature>>*>& groups) {
  const size_t G = groups.size();
  if (digests.size() != G) throw std::invalid_argument("length mismatch");
  std::vector<bool> out(G, true);
  if (!G) return out;
  std::vector<uint8_t> pk, sg, msg(32 * G);
  std::vector<uint64_t> first(G);
  std::vector<uint32_t> cnt(G);
  for (size_t g = 0; g < G; ++g) {
    first[g] = pk.size() / 32;
    cnt[g] = (uint32_t)groups[g]->size();
    std::memcpy(&msg[32 * g], digests[g].bytes.data(), 32);
    for (const auto& kv : *groups[g]) {
      pk.insert(pk.end(), kv.first.bytes.begin(), kv.first.bytes.end());
      const auto f = kv.second.flatten();
      sg.insert(sg.end(), f.begin(), f.end());
    }
  }
  pk.resize(std::max<size_t>(pk.size(), 32));
  sg.resize(std::max<size_t>(sg.size(), 64));
  std::vector<uint8_t> bm((G + 7) / 8);
  check(nt_ed25519_verify_batch_groups(Backend::global().ctx(), pk.data(), sg.data(), first.data(), cnt.data(),
                                       msg.data(), G, bm.data(), nullptr),
        "nt_ed25519_verify_batch_groups");
  for (size_t g = 0; g < G; ++g) out[g] = (bm[g / 8] >> (g % 8)) & 1;
  return out;
}

void Signature::verify_batch(const Digest& digest, const std::vector<std::pair<PublicKey, Signature>>& votes) {
  if (!verify_batch_many({digest}, {&votes})[0]) throw CryptoError();
}

KeySet::KeySet(const std::vector<PublicKey>& keys) : keys_(keys) {
  std::vector<uint8_t> pk(32 * std::max<size_t>(keys.size(), 1));
  for (size_t i = 0; i < keys.size(); ++i) {
    std::memcpy(&pk[32 * i], keys[i].bytes.data(), 32);
    sorted_.emplace_back(keys[i], (uint32_t)i);
  }
  std::sort(sorted_.begin(), sorted_.end(),
            [](const std::pair<PublicKey, uint32_t>& a, const std::pair<PublicKey, uint32_t>& b) { return a.first < b.first; });
  check(nt_keyset_create(Backend::global().ctx(), pk.data(), (uint32_t)keys.size(), &ks_), "nt_keyset_create");
}

KeySet::~KeySet() {
  if (ks_) nt_keyset_free(ks_);
}

uint32_t KeySet::index_of(const PublicKey& pk) const {
  auto it = std::lower_bound(sorted_.begin(), sorted_.end(), pk,
                             [](const std::pair<PublicKey, uint32_t>& a, const PublicKey& b) { return a.first < b; });
  return (it != sorted_.end() && it->first == pk) ? it->second : UINT32_MAX;
}

std::vector<bool> KeySet::verify_many(const std::vector<Digest>& digests, const std::vector<PublicKey>& keys,
                                      const std::vector<Signature>& sigs) const {
  const size_t n = digests.size();
  if (keys.size() != n || sigs.size() != n) throw std::invalid_argument("length mismatch");
  std::vector<bool> out(n, false);
  if (!n) return out;
  std::vector<uint32_t> idx(n);
  std::vector<uint8_t> sg(64 * n), msg(32 * n);
  std::vector<uint64_t> off(n), len(n, 32);
  for (size_t i = 0; i < n; ++i) {
    idx[i] = index_of(keys[i]);
    const auto f = sigs[i].flatten();
    std::memcpy(&sg[64 * i], f.data(), 64);
    std::memcpy(&msg[32 * i], digests[i].bytes.data(), 32);
    off[i] = 32 * i;
  }
  std::vector<uint8_t> bm((n + 7) / 8);
  check(nt_ed25519_verify_keyset(Backend::global().ctx(), ks_, NT_MODE_STRICT, idx.data(), sg.data(), msg.data(),
                                 off.data(), len.data(), n, bm.data()),
        "nt_ed25519_verify_keyset");
  for (size_t i = 0; i < n; ++i) out[i] = (bm[i / 8] >> (i % 8)) & 1;
  return out;
}

std::vector<bool> KeySet::verify_batch_many(
    const std::vector<Digest>& digests,
    const std::vector<const std::vector<std::pair<PublicKey, Signature>>*>& groups) const {
  const size_t G = groups.size();
  if (digests.size() != G) throw std::invalid_argument("length mismatch");
  std::vector<bool> out(G, true);
  if (!G) return out;
  std::vector<uint32_t> idx;
  std::vector<uint8_t> sg, msg(32 * G);
  std::vector<uint64_t> first(G);
  std::vector<uint32_t> cnt(G);
  for (size_t g = 0; g < G; ++g) {
    first[g] = idx.size();
    cnt[g] = (uint32_t)groups[g]->size();
    std::memcpy(&msg[32 * g], digests[g].bytes.data(), 32);
    for (const auto& kv : *groups[g]) {
      idx.push_back(index_of(kv.first));
      const auto f = kv.second.flatten();
      sg.insert(sg.end(), f.begin(), f.end());
    }
  }
  idx.resize(std::max<size_t>(idx.size(), 1));
  sg.resize(std::max<size_t>(sg.size(), 64));
  std::vector<uint8_t> bm((G + 7) / 8);
  check(nt_ed25519_verify_batch_groups_keyset(Backend::global().ctx(), ks_, idx.data(), sg.data(), first.data(),
                                              cnt.data(), msg.data(), G, bm.data(), nullptr),
        "nt_ed25519_verify_batch_groups_keyset");
  for (size_t g = 0; g < G; ++g) out[g] = (bm[g / 8] >> (g % 8)) & 1;
  return out;
}

SignatureService::SignatureService(SecretKey secret) : secret_(std::move(secret)) {
  th_ = std::thread([this] { run(); });
}

SignatureService::~SignatureService() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  th_.join();
}

std::future<Signature> SignatureService::request_signature(const Digest& digest) {
  std::promise<Signature> p;
  auto f = p.get_future();
  {
    std::lock_guard<std::mutex> lk(mu_);
    q_.emplace(digest, std::move(p));
  }
  cv_.notify_one();
  return f;
}

void SignatureService::run() {
  for (;;) {
    std::pair<Digest, std::promise<Signature>> item;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      item = std::move(q_.front());
      q_.pop();
    }
    try {
      item.second.set_value(Signature::new_(item.first, secret_));
    } catch (...) {
      item.second.set_exception(std::current_exception());
    }
  }
}

}  // namespace crypto
