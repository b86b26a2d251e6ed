// wire.cpp -- bincode codec of PrimaryMessage (see wire.hpp for the format rules).
#include "wire.hpp"

#include <cstring>

namespace primary {

namespace {

struct Writer {
  std::vector<uint8_t> v;
  void raw(const uint8_t* p, size_t n) { v.insert(v.end(), p, p + n); }
  void u32(uint32_t x) {
    for (int i = 0; i < 4; ++i) v.push_back((uint8_t)(x >> (8 * i)));
  }
  void u64(uint64_t x) {
    for (int i = 0; i < 8; ++i) v.push_back((uint8_t)(x >> (8 * i)));
  }
  void str(const std::string& s) {
    u64(s.size());
    raw((const uint8_t*)s.data(), s.size());
  }
  void key(const PublicKey& k) { str(k.encode_base64()); }
  void d32(const std::array<uint8_t, 32>& a) { raw(a.data(), 32); }
  void sig(const Signature& s) {
    d32(s.part1);
    d32(s.part2);
  }
  void header(const Header& h) {
    key(h.author);
    u64(h.round);
    u64(h.payload.size());
    for (const auto& kv : h.payload) {
      d32(kv.first.bytes);
      u32(kv.second);
    }
    u64(h.parents.size());
    for (const auto& p : h.parents) d32(p.bytes);
    d32(h.id.bytes);
    sig(h.signature);
  }
};

struct Reader {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  bool need(size_t k) {
    if (!ok || n - pos < k) ok = false;
    return ok;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i) x |= (uint32_t)p[pos + i] << (8 * i);
    pos += 4;
    return x;
  }
  uint64_t u64() {
    if (!need(8)) return 0;
    uint64_t x = 0;
    for (int i = 0; i < 8; ++i) x |= (uint64_t)p[pos + i] << (8 * i);
    pos += 8;
    return x;
  }
  void d32(std::array<uint8_t, 32>& a) {
    if (!need(32)) return;
    std::memcpy(a.data(), p + pos, 32);
    pos += 32;
  }
  // element count of a sequence whose elements take at least `min_elem` bytes
  uint64_t count(size_t min_elem) {
    const uint64_t c = u64();
    if (ok && min_elem && c > (n - pos) / min_elem) ok = false;
    return ok ? c : 0;
  }
  bool key(PublicKey& k) {
    const uint64_t len = count(1);
    if (!need(len)) return false;
    const std::string s((const char*)p + pos, (size_t)len);
    pos += len;
    return ok = ok && decode_key(s, k);
  }
  void sig(Signature& s) {
    d32(s.part1);
    d32(s.part2);
  }
  void header(Header& h) {
    key(h.author);
    h.round = u64();
    const uint64_t np = count(36);
    for (uint64_t i = 0; ok && i < np; ++i) {
      Digest d;
      d32(d.bytes);
      h.payload[d] = u32();  // BTreeMap::insert: a repeated key keeps the last value
    }
    const uint64_t nq = count(32);
    for (uint64_t i = 0; ok && i < nq; ++i) {
      Digest d;
      d32(d.bytes);
      h.parents.insert(d);
    }
    d32(h.id.bytes);
    sig(h.signature);
  }
  // serde String (UTF-8) -> base64 0.13 STANDARD decode -> bytes[..32]
  static bool decode_key(const std::string& s, PublicKey& k) {
    if (!utf8_ok(s)) return false;
    std::vector<uint8_t> b;
    try {
      b = crypto::base64_decode(s);
    } catch (const std::exception&) {
      return false;
    }
    if (b.size() < 32 || !canonical_tail(s)) return false;
    std::memcpy(k.bytes.data(), b.data(), 32);
    return true;
  }
  static bool utf8_ok(const std::string& s) {
    size_t i = 0;
    while (i < s.size()) {
      const uint8_t c = (uint8_t)s[i];
      const int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
      if (!len || i + len > s.size()) return false;
      for (int j = 1; j < len; ++j)
        if (((uint8_t)s[i + j] >> 6) != 2) return false;
      i += len;
    }
    return true;
  }
  // the last data symbol of a padded group may not carry non-zero unused bits
  static bool canonical_tail(const std::string& s) {
    if (s.size() < 4) return true;
    const size_t pad = (s[s.size() - 1] == '=') + (s[s.size() - 2] == '=');
    if (!pad) return true;
    const char c = s[s.size() - 1 - pad];
    const int v = (c >= 'A' && c <= 'Z') ? c - 'A' : (c >= 'a' && c <= 'z') ? c - 'a' + 26
                : (c >= '0' && c <= '9') ? c - '0' + 52 : c == '+' ? 62 : 63;
    return (v & (pad == 1 ? 3 : 15)) == 0;
  }
};

}  // namespace

bool decode_public_key(const uint8_t* s, size_t len, PublicKey& out) {
  return Reader::decode_key(std::string((const char*)s, len), out);
}

std::vector<uint8_t> encode_header(const Header& h) {
  Writer w;
  w.header(h);
  return std::move(w.v);
}

std::vector<uint8_t> encode(const PrimaryMessage& m) {
  Writer w;
  w.u32((uint32_t)m.kind);
  switch (m.kind) {
    case MsgKind::Header: w.header(m.header); break;
    case MsgKind::Vote:
      w.d32(m.vote.id.bytes);
      w.u64(m.vote.round);
      w.key(m.vote.origin);
      w.key(m.vote.author);
      w.sig(m.vote.signature);
      break;
    case MsgKind::Certificate:
      w.header(m.certificate.header);
      w.u64(m.certificate.votes.size());
      for (const auto& kv : m.certificate.votes) {
        w.key(kv.first);
        w.sig(kv.second);
      }
      break;
    case MsgKind::CertificatesRequest:
      w.u64(m.request_digests.size());
      for (const auto& d : m.request_digests) w.d32(d.bytes);
      w.key(m.requestor);
      break;
  }
  return std::move(w.v);
}

bool decode(const uint8_t* p, size_t n, PrimaryMessage& out, size_t* used) {
  Reader r{p, n};
  out = PrimaryMessage{};
  const uint32_t tag = r.u32();
  if (!r.ok || tag > 3) return false;
  out.kind = (MsgKind)tag;
  switch (out.kind) {
    case MsgKind::Header: r.header(out.header); break;
    case MsgKind::Vote:
      r.d32(out.vote.id.bytes);
      out.vote.round = r.u64();
      r.key(out.vote.origin);
      r.key(out.vote.author);
      r.sig(out.vote.signature);
      break;
    case MsgKind::Certificate: {
      r.header(out.certificate.header);
      const uint64_t nv = r.count(8 + 64);
      out.certificate.votes.reserve(nv);
      for (uint64_t i = 0; r.ok && i < nv; ++i) {
        std::pair<PublicKey, Signature> v;
        r.key(v.first);
        r.sig(v.second);
        out.certificate.votes.push_back(v);
      }
      break;
    }
    case MsgKind::CertificatesRequest: {
      const uint64_t nd = r.count(32);
      for (uint64_t i = 0; r.ok && i < nd; ++i) {
        Digest d;
        r.d32(d.bytes);
        out.request_digests.push_back(d);
      }
      r.key(out.requestor);
      break;
    }
  }
  if (used) *used = r.pos;
  return r.ok;
}

}  // namespace primary
