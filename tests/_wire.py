"""TEST INFRASTRUCTURE: an independent Python model of the primary's wire format
and Core checks, used to pin the C++ mirror (narwhal-tusk_amd/host/wire.cpp,
narwhal.cpp Core::sanitize_batch) and by bench.py's ingest leg.

  bincode 1.x of PrimaryMessage       primary/src/primary.rs:32-38, messages.rs:14-21,106-112,169-172
  PublicKey serde (base64 string)     crypto/src/lib.rs:94-112
  Header / Vote / Certificate digests messages.rs:70-84, 145-153, 226-234
  Core::sanitize_*                    core.rs:306-346
  Header / Vote / Certificate verify  messages.rs:48-67, 131-142, 189-215
Signature verdicts come from the CPU oracle (oracle/, pinned separately).
"""
import base64
import hashlib
import struct

# DagError codes of narwhal.hpp
OK, INVALID_SIGNATURE, INVALID_HEADER_ID, MALFORMED_HEADER, UNKNOWN_AUTHORITY, AUTHORITY_REUSE, \
    REQUIRES_QUORUM, TOO_OLD, UNEXPECTED_VOTE, SERIALIZATION_ERROR, UNEXPECTED_MESSAGE = range(11)


def b64(pk: bytes) -> bytes:
    return base64.b64encode(pk)


def _str(s: bytes) -> bytes:
    return struct.pack("<Q", len(s)) + s


class Header:
    def __init__(self, author, round_, payload, parents, id_=None, sig=b"\0" * 64):
        self.author, self.round, self.payload, self.parents, self.sig = author, round_, dict(payload), set(parents), sig
        self.id = id_ if id_ is not None else self.digest()

    def preimage(self) -> bytes:
        out = self.author + struct.pack("<Q", self.round)
        for d in sorted(self.payload):
            out += d + struct.pack("<I", self.payload[d])
        for p in sorted(self.parents):
            out += p
        return out

    def digest(self) -> bytes:
        return hashlib.sha512(self.preimage()).digest()[:32]

    def encode(self) -> bytes:
        out = _str(b64(self.author)) + struct.pack("<Q", self.round)
        out += struct.pack("<Q", len(self.payload))
        for d in sorted(self.payload):
            out += d + struct.pack("<I", self.payload[d])
        out += struct.pack("<Q", len(self.parents)) + b"".join(sorted(self.parents))
        return out + self.id + self.sig


class Vote:
    def __init__(self, id_, round_, origin, author, sig=b"\0" * 64):
        self.id, self.round, self.origin, self.author, self.sig = id_, round_, origin, author, sig

    def digest(self) -> bytes:
        return hashlib.sha512(self.id + struct.pack("<Q", self.round) + self.origin).digest()[:32]

    def encode(self) -> bytes:
        return self.id + struct.pack("<Q", self.round) + _str(b64(self.origin)) + _str(b64(self.author)) + self.sig


class Certificate:
    def __init__(self, header, votes):
        self.header, self.votes = header, list(votes)

    def digest(self) -> bytes:
        h = self.header
        return hashlib.sha512(h.id + struct.pack("<Q", h.round) + h.author).digest()[:32]

    def encode(self) -> bytes:
        out = self.header.encode() + struct.pack("<Q", len(self.votes))
        for pk, sig in self.votes:
            out += _str(b64(pk)) + sig
        return out


def message(obj) -> bytes:
    """bincode of PrimaryMessage::{Header, Vote, Certificate}(obj) or a
    CertificatesRequest given as (digests, requestor)."""
    if isinstance(obj, Header):
        return struct.pack("<I", 0) + obj.encode()
    if isinstance(obj, Vote):
        return struct.pack("<I", 1) + obj.encode()
    if isinstance(obj, Certificate):
        return struct.pack("<I", 2) + obj.encode()
    digests, requestor = obj
    return struct.pack("<I", 3) + struct.pack("<Q", len(digests)) + b"".join(digests) + _str(b64(requestor))


class Committee:
    def __init__(self, keys, stakes, nworkers):
        self.auth = {k: (s, w) for k, s, w in zip(keys, stakes, nworkers)}

    def stake(self, k):
        return self.auth.get(k, (0, 0))[0]

    def quorum(self):
        return 2 * sum(s for s, _ in self.auth.values()) // 3 + 1

    def has_worker(self, k, w):
        return k in self.auth and w < self.auth[k][1]


def model_sanitize(committee, gc_round, cur, obj, strict, batch):
    """Expected DagError of Core::sanitize_* for one message; strict(digest, pk, sig)
    and batch(digest, [(pk, sig)]) give signature verdicts (the CPU oracle)."""
    def header_verify(h):
        if h.digest() != h.id:
            return INVALID_HEADER_ID
        if committee.stake(h.author) == 0:
            return UNKNOWN_AUTHORITY
        if any(not committee.has_worker(h.author, w) for w in h.payload.values()):
            return MALFORMED_HEADER
        return OK if strict(h.id, h.author, h.sig) else INVALID_SIGNATURE

    if isinstance(obj, Header):
        return TOO_OLD if obj.round < gc_round else header_verify(obj)
    if isinstance(obj, Vote):
        if obj.round < cur.round:
            return TOO_OLD
        if not (obj.id == cur.id and obj.origin == cur.author and obj.round == cur.round):
            return UNEXPECTED_VOTE
        if committee.stake(obj.author) == 0:
            return UNKNOWN_AUTHORITY
        return OK if strict(obj.digest(), obj.author, obj.sig) else INVALID_SIGNATURE
    if isinstance(obj, Certificate):
        h = obj.header
        if h.round < gc_round:
            return TOO_OLD
        if h.id == b"\0" * 32 and h.round == 0 and h.author in committee.auth:
            return OK  # genesis
        e = header_verify(h)
        if e != OK:
            return e
        used, weight = set(), 0
        for pk, _ in obj.votes:
            if pk in used:
                return AUTHORITY_REUSE
            if committee.stake(pk) == 0:
                return UNKNOWN_AUTHORITY
            used.add(pk)
            weight += committee.stake(pk)
        if weight < committee.quorum():
            return REQUIRES_QUORUM
        return OK if batch(obj.digest(), obj.votes) else INVALID_SIGNATURE
    return UNEXPECTED_MESSAGE
