// test_narwhal.cpp -- the reference's own hot-path tests, re-expressed against
// the C++ mirror (narwhal-tusk_amd/host/) running on the GPU:
//   crypto/src/tests/crypto_tests.rs         (keys(), verify, batch, service)
//   worker/src/tests/processor_tests.rs:9-46 (hash_and_store, digest part)
//   primary/src/tests/core_tests.rs, common.rs (header / votes / certificates)
// plus negative cases for every DagError the verify paths can return.
// Usage: test_narwhal <pk0_hex> <pk1_hex> <pk2_hex> <pk3_hex>   (golden keys())
#include <climits>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../narwhal-tusk_amd/host/narwhal.hpp"

using namespace crypto;
using primary::Certificate;
using primary::Committee;
using primary::DagError;
using primary::Header;
using primary::Vote;

static int g_fail = 0, g_pass = 0;
#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::printf("  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);        \
      ++g_fail;                                                            \
      return;                                                              \
    }                                                                      \
  } while (0)
#define TEST(name) static void name()
#define RUN(name)                           \
  do {                                      \
    const int f0 = g_fail;                  \
    name();                                 \
    if (g_fail == f0) ++g_pass;             \
    std::printf("%s %s\n", g_fail == f0 ? "ok  " : "FAIL", #name); \
  } while (0)

// ---- rand 0.7 StdRng (ChaCha20, key = seed, stream 0) for keys() ----
struct ChaCha20Rng {
  uint32_t key[8];
  uint64_t counter = 0;
  uint8_t buf[64];
  int pos = 64;
  explicit ChaCha20Rng(const uint8_t seed[32]) { std::memcpy(key, seed, 32); }
  static uint32_t rotl(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
  void block() {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    std::memcpy(st + 4, key, 32);
    st[12] = (uint32_t)counter;
    st[13] = (uint32_t)(counter >> 32);
    st[14] = st[15] = 0;
    uint32_t x[16];
    std::memcpy(x, st, sizeof x);
    auto qr = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 10; ++r) {
      qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
      qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) {
      const uint32_t v = x[i] + st[i];
      std::memcpy(buf + 4 * i, &v, 4);
    }
    ++counter;
    pos = 0;
  }
  void fill(uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
      if (pos == 64) block();
      p[i] = buf[pos++];
    }
  }
};

static std::vector<std::pair<PublicKey, SecretKey>> keys() {  // crypto_tests.rs:26-29
  uint8_t seed[32] = {0};
  ChaCha20Rng rng(seed);
  std::vector<std::pair<PublicKey, SecretKey>> out;
  for (int i = 0; i < 4; ++i) out.push_back(generate_keypair([&](uint8_t* p, size_t n) { rng.fill(p, n); }));
  return out;
}

static Digest digest_of(const std::string& s) { return sha512_digest((const uint8_t*)s.data(), s.size()); }

static std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}

static std::vector<std::string> g_golden_pk;

// ------------------------------------------------------------- crypto_tests.rs
TEST(keys_fixture_matches_golden) {
  const auto k = keys();
  for (int i = 0; i < 4; ++i) CHECK(hex(k[i].first.bytes.data(), 32) == g_golden_pk[i]);
}

TEST(import_export_public_key) {
  const auto pk = keys().back().first;
  const auto exp = pk.encode_base64();
  CHECK(PublicKey::decode_base64(exp) == pk);
}

TEST(import_export_secret_key) {
  const auto sk = keys().back().second;
  CHECK(SecretKey::decode_base64(sk.encode_base64()) == sk);
}

TEST(verify_valid_signature) {
  const auto kp = keys().back();
  const Digest d = digest_of("Hello, world!");
  const Signature s = Signature::new_(d, kp.second);
  bool ok = true;
  try { s.verify(d, kp.first); } catch (const CryptoError&) { ok = false; }
  CHECK(ok);
}

TEST(verify_invalid_signature) {
  const auto kp = keys().back();
  const Signature s = Signature::new_(digest_of("Hello, world!"), kp.second);
  bool rejected = false;
  try { s.verify(digest_of("Bad message!"), kp.first); } catch (const CryptoError&) { rejected = true; }
  CHECK(rejected);
}

TEST(verify_valid_batch) {
  const Digest d = digest_of("Hello, world!");
  auto k = keys();
  std::vector<std::pair<PublicKey, Signature>> sigs;
  for (int i = 0; i < 3; ++i) {
    auto kp = k.back();
    k.pop_back();
    sigs.emplace_back(kp.first, Signature::new_(d, kp.second));
  }
  bool ok = true;
  try { Signature::verify_batch(d, sigs); } catch (const CryptoError&) { ok = false; }
  CHECK(ok);
}

TEST(verify_invalid_batch) {
  const Digest d = digest_of("Hello, world!");
  auto k = keys();
  std::vector<std::pair<PublicKey, Signature>> sigs;
  for (int i = 0; i < 2; ++i) {
    auto kp = k.back();
    k.pop_back();
    sigs.emplace_back(kp.first, Signature::new_(d, kp.second));
  }
  sigs.emplace_back(k.back().first, Signature{});  // Signature::default()
  bool rejected = false;
  try { Signature::verify_batch(d, sigs); } catch (const CryptoError&) { rejected = true; }
  CHECK(rejected);
}

TEST(verify_batch_empty_is_ok) {
  bool ok = true;
  try { Signature::verify_batch(Digest{}, {}); } catch (const CryptoError&) { ok = false; }
  CHECK(ok);
}

TEST(signature_service) {
  const auto kp = keys().back();
  SignatureService service(kp.second);
  const Digest d = digest_of("Hello, world!");
  const Signature s = service.request_signature(d).get();
  bool ok = true;
  try { s.verify(d, kp.first); } catch (const CryptoError&) { ok = false; }
  CHECK(ok);
}

TEST(digest_display_debug) {
  const Digest d = digest_of("Hello, world!");
  CHECK(d.debug().size() == 44);
  CHECK(d.display() == d.debug().substr(0, 16));
}

// ------------------------------------------------------------- processor_tests.rs
TEST(processor_hash_and_store_digest) {
  const worker::Batch batch = {worker::Transaction(100, 0), worker::Transaction(100, 0)};
  const auto ser = worker::serialize_batch(batch);
  CHECK(ser.size() == 228);
  worker::Processor p{0, true};
  Digest d;
  const auto msg = p.process(ser, &d);
  CHECK(hex(d.bytes.data(), 32) == "24d00f74a0767e74808c8546630902972853fa200e079e582b8b7bdecd7331d8");
  CHECK(msg.size() == 4 + 32 + 4);
  CHECK(msg[0] == 0 && std::memcmp(msg.data() + 4, d.bytes.data(), 32) == 0);
  worker::Processor q{7, false};
  const auto m2 = q.process(ser);
  CHECK(m2[0] == 1 && m2[36] == 7);
}

// ------------------------------------------------------------- primary fixtures
static Committee committee() {  // primary/src/tests/common.rs:35-66
  Committee c;
  for (const auto& kp : keys()) c.authorities[kp.first] = primary::Authority{1, {0}};
  return c;
}

static Header make_header(const std::pair<PublicKey, SecretKey>& kp, const Committee& c) {
  Header h;
  h.author = kp.first;
  h.round = 1;
  for (const auto& g : Certificate::genesis(c)) h.parents.insert(g.digest());
  h.id = h.digest();
  h.signature = Signature::new_(h.id, kp.second);
  return h;
}

static std::vector<Vote> votes(const Header& h) {
  std::vector<Vote> out;
  for (const auto& kp : keys()) {
    Vote v;
    v.id = h.id;
    v.round = h.round;
    v.origin = h.author;
    v.author = kp.first;
    v.signature = Signature::new_(v.digest(), kp.second);
    out.push_back(v);
  }
  return out;
}

static Certificate certificate(const Header& h) {
  Certificate c;
  c.header = h;
  for (const auto& v : votes(h)) c.votes.emplace_back(v.author, v.signature);
  return c;
}

TEST(process_header_verifies) {
  const Committee c = committee();
  const Header h = make_header(keys().back(), c);
  CHECK(h.verify(c) == DagError::Ok);
}

TEST(process_votes_verify) {
  const Committee c = committee();
  const Header h = make_header(keys().back(), c);
  for (const auto& v : votes(h)) CHECK(v.verify(c) == DagError::Ok);
}

TEST(process_certificates_verify) {
  const Committee c = committee();
  const auto k = keys();
  std::vector<Certificate> certs;
  for (int i = 0; i < 3; ++i) certs.push_back(certificate(make_header(k[i], c)));
  for (const auto& x : certs) CHECK(x.verify(c) == DagError::Ok);
  const auto batched = primary::verify_certificates(c, certs);
  for (auto e : batched) CHECK(e == DagError::Ok);
}

TEST(genesis_certificate_is_valid) {
  const Committee c = committee();
  for (const auto& g : Certificate::genesis(c)) CHECK(g.verify(c) == DagError::Ok);
}

TEST(header_errors) {
  const Committee c = committee();
  Header h = make_header(keys().back(), c);
  Header bad_id = h;
  bad_id.round = 2;
  CHECK(bad_id.verify(c) == DagError::InvalidHeaderId);
  Header bad_worker = h;
  Digest pd = digest_of("payload");
  bad_worker.payload[pd] = 5;  // worker 5 does not exist
  bad_worker.id = bad_worker.digest();
  CHECK(bad_worker.verify(c) == DagError::MalformedHeader);
  Header bad_sig = h;
  bad_sig.signature.part2[3] ^= 1;
  CHECK(bad_sig.verify(c) == DagError::InvalidSignature);
  Committee c3 = c;
  c3.authorities.erase(h.author);
  CHECK(h.verify(c3) == DagError::UnknownAuthority);
}

TEST(vote_errors) {
  const Committee c = committee();
  const Header h = make_header(keys().back(), c);
  auto vs = votes(h);
  Vote v = vs[0];
  v.round = 9;  // digest changes -> signature no longer matches
  CHECK(v.verify(c) == DagError::InvalidSignature);
  Committee c3 = c;
  c3.authorities.erase(vs[1].author);
  CHECK(vs[1].verify(c3) == DagError::UnknownAuthority);
}

TEST(certificate_errors_and_batched_agreement) {
  const Committee c = committee();
  const auto k = keys();
  std::vector<Certificate> certs;
  Certificate good = certificate(make_header(k[0], c));
  certs.push_back(good);
  Certificate reuse = good;
  reuse.votes[1] = reuse.votes[0];
  certs.push_back(reuse);
  Certificate noq = good;
  noq.votes.resize(2);  // quorum is 3 of 4
  certs.push_back(noq);
  Certificate badvote = good;
  badvote.votes[2].second.part1[0] ^= 0x40;
  certs.push_back(badvote);
  Certificate zero = good;
  zero.votes[3].second = Signature{};
  certs.push_back(zero);
  Certificate badhdr = good;
  badhdr.header.signature.part2[0] ^= 1;
  certs.push_back(badhdr);
  Certificate unknown = good;
  unknown.votes[0].first.bytes[0] ^= 1;
  certs.push_back(unknown);
  const DagError want[] = {DagError::Ok, DagError::AuthorityReuse, DagError::CertificateRequiresQuorum,
                           DagError::InvalidSignature, DagError::InvalidSignature, DagError::InvalidSignature,
                           DagError::UnknownAuthority};
  const auto batched = primary::verify_certificates(c, certs);
  const auto cache = primary::committee_keyset(c);
  const auto cached = primary::verify_certificates(c, certs, cache.get());
  for (size_t i = 0; i < certs.size(); ++i) {
    CHECK(certs[i].verify(c) == want[i]);
    CHECK(batched[i] == want[i]);
    CHECK(cached[i] == want[i]);
  }
}

TEST(committee_keyset_index_and_verify) {
  const Committee c = committee();
  const auto cache = primary::committee_keyset(c);
  CHECK(cache->size() == 4);
  PublicKey stranger;
  stranger.bytes[5] = 7;
  CHECK(cache->index_of(stranger) == UINT32_MAX);
  const auto k = keys();
  const Digest d = digest_of("Hello, world!");
  std::vector<Digest> ds;
  std::vector<PublicKey> ks;
  std::vector<Signature> ss;
  for (const auto& kp : k) {
    ds.push_back(d);
    ks.push_back(kp.first);
    ss.push_back(Signature::new_(d, kp.second));
  }
  ds.push_back(d);
  ks.push_back(stranger);  // not a committee key -> reject
  ss.push_back(ss[0]);
  const auto v = cache->verify_many(ds, ks, ss);
  for (int i = 0; i < 4; ++i) CHECK(v[i]);
  CHECK(!v[4]);
}

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);  // one line per test, also into a file
  for (int i = 1; i < argc; ++i) g_golden_pk.push_back(argv[i]);
  if (g_golden_pk.size() != 4) {
    std::printf("usage: test_narwhal pk0 pk1 pk2 pk3\n");
    return 2;
  }
  try {
    RUN(keys_fixture_matches_golden);
    RUN(import_export_public_key);
    RUN(import_export_secret_key);
    RUN(verify_valid_signature);
    RUN(verify_invalid_signature);
    RUN(verify_valid_batch);
    RUN(verify_invalid_batch);
    RUN(verify_batch_empty_is_ok);
    RUN(signature_service);
    RUN(digest_display_debug);
    RUN(processor_hash_and_store_digest);
    RUN(process_header_verifies);
    RUN(process_votes_verify);
    RUN(process_certificates_verify);
    RUN(genesis_certificate_is_valid);
    RUN(header_errors);
    RUN(vote_errors);
    RUN(certificate_errors_and_batched_agreement);
    RUN(committee_keyset_index_and_verify);
  } catch (const std::exception& e) {
    std::printf("exception: %s\n", e.what());
    return 3;
  }
  std::printf("%d passed, %d failed\n", g_pass, g_fail);
  return g_fail ? 1 : 0;
}
