// wire.hpp -- bincode 1.x codec of the primary's network messages.
//
//   PrimaryMessage  primary/src/primary.rs:32-38   (Header | Vote | Certificate | CertificatesRequest)
//   Header / Vote / Certificate field order         primary/src/messages.rs:14-21, 106-112, 169-172
//   PublicKey serde = base64 string                 crypto/src/lib.rs:94-112
//   Signature serde = {part1: [u8;32], part2: [u8;32]} (64 raw bytes)   crypto/src/lib.rs:177-181
//   deserialize site                                primary/src/primary.rs:230 (bincode::deserialize,
//                                                   errors -> DagError::SerializationError)
//
// bincode 1.x defaults (bincode::serialize / bincode::deserialize): little-endian,
// fixed-width integers, u32 enum variant index, u64 sequence/map/string lengths,
// [u8; 32] as 32 raw bytes, trailing bytes allowed on decode.  Strings must be
// UTF-8; a PublicKey string must be canonical padded standard base64 (base64
// 0.13 rejects non-zero trailing bits) of >= 32 bytes (the reference's
// decode_base64 takes bytes[..32]; a shorter decode panics there -- the mirror
// reports a decode error instead).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "narwhal.hpp"

namespace primary {

enum class MsgKind : uint32_t { Header = 0, Vote = 1, Certificate = 2, CertificatesRequest = 3 };

struct PrimaryMessage {
  MsgKind kind = MsgKind::Header;
  Header header;                        // kind == Header
  Vote vote;                            // kind == Vote
  Certificate certificate;              // kind == Certificate
  std::vector<Digest> request_digests;  // kind == CertificatesRequest
  PublicKey requestor;                  // kind == CertificatesRequest
};

std::vector<uint8_t> encode(const PrimaryMessage& m);
std::vector<uint8_t> encode_header(const Header& h);  // bincode of a bare Header
// serde String + PublicKey::decode_base64 of the len bytes at s (false = error)
bool decode_public_key(const uint8_t* s, size_t len, PublicKey& out);
// false = bincode error (DagError::SerializationError); `used` = bytes consumed
bool decode(const uint8_t* p, size_t n, PrimaryMessage& out, size_t* used = nullptr);

}  // namespace primary
