"""Mirror of the reference `crypto` crate surface (crypto/src/lib.rs) over the
gfx950 backend.  Names, argument meaning and error behaviour follow the Rust
API so the parity tests read like crypto/src/tests/crypto_tests.rs.

  Digest            crypto/src/lib.rs:21-58   (32 bytes; Display = first 16 base64 chars)
  Hash              crypto/src/lib.rs:60-62
  PublicKey         crypto/src/lib.rs:65-119  (base64 serde form)
  SecretKey         crypto/src/lib.rs:121-161 (seed || pk, 64 bytes, zeroized)
  generate_keypair  crypto/src/lib.rs:163-175
  Signature         crypto/src/lib.rs:177-219 (new / verify / verify_batch)
  SignatureService  crypto/src/lib.rs:222-249 (thread + queue instead of a tokio task)
  CryptoError       crypto/src/lib.rs:18      (= ed25519::Error, opaque)
"""
import base64
import os
import queue
import threading
from concurrent.futures import Future

import numpy as np

from ._lib import default_backend


class CryptoError(Exception):
    """Opaque signature error (ed25519::Error)."""


class Digest:
    __slots__ = ("_b",)

    def __init__(self, b: bytes = bytes(32)):
        b = bytes(b)
        if len(b) != 32:
            raise ValueError("Digest is 32 bytes")
        self._b = b

    def to_vec(self) -> bytes:
        return self._b

    def size(self) -> int:
        return 32

    def __bytes__(self):
        return self._b

    def __eq__(self, o):
        return isinstance(o, Digest) and o._b == self._b

    def __lt__(self, o):
        return self._b < o._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):
        return base64.b64encode(self._b).decode()

    def __str__(self):
        return base64.b64encode(self._b).decode()[:16]


def b64decode_strict(s: str) -> bytes:
    """base64 0.13 STANDARD decode as the reference's serde path uses it
    (crypto/src/lib.rs:94-112, 152-160): standard alphabet, length a multiple of
    4, '=' only as the last one or two symbols, and no non-zero unused bits in
    the last data symbol (InvalidLastSymbol) -- the same rules as the C++
    mirror's crypto::base64_decode.  Raises ValueError."""
    if isinstance(s, str):
        try:
            s = s.encode("ascii")
        except UnicodeEncodeError:
            raise ValueError("InvalidByte") from None
    if len(s) % 4:
        raise ValueError("InvalidLength")
    try:
        b = base64.b64decode(s, validate=True)
    except Exception:
        raise ValueError("InvalidByte") from None
    pad = len(s) - len(s.rstrip(b"="))
    if pad:
        last = base64.b64decode(s[-4:-pad] + b"A" * pad, validate=True)  # the unused bits land in the tail bytes
        if last[-pad:] != bytes(pad):
            raise ValueError("InvalidLastSymbol")
    return b


def sha512_digest(data: bytes) -> Digest:
    """Digest(Sha512::digest(data)[..32]) on the GPU (worker/src/processor.rs:38)."""
    return Digest(default_backend().digest_many([bytes(data)])[0].tobytes())


def sha512_digest_batch(messages) -> list:
    out = default_backend().digest_many([bytes(m) for m in messages])
    return [Digest(r.tobytes()) for r in out]


class PublicKey:
    __slots__ = ("_b",)

    def __init__(self, b: bytes = bytes(32)):
        b = bytes(b)
        if len(b) != 32:
            raise ValueError("PublicKey is 32 bytes")
        self._b = b

    def __bytes__(self):
        return self._b

    def encode_base64(self) -> str:
        return base64.b64encode(self._b).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "PublicKey":
        b = b64decode_strict(s)
        if len(b) < 32:
            raise ValueError("InvalidLength")
        return cls(b[:32])

    def __eq__(self, o):
        return isinstance(o, PublicKey) and o._b == self._b

    def __lt__(self, o):
        return self._b < o._b

    def __hash__(self):
        return hash(self._b)

    def __repr__(self):
        return self.encode_base64()

    def __str__(self):
        return self.encode_base64()[:16]


class SecretKey:
    __slots__ = ("_b",)

    def __init__(self, b: bytes):
        b = bytearray(b)
        if len(b) != 64:
            raise ValueError("SecretKey is 64 bytes")
        self._b = b

    def encode_base64(self) -> str:
        return base64.b64encode(bytes(self._b)).decode()

    @classmethod
    def decode_base64(cls, s: str) -> "SecretKey":
        b = b64decode_strict(s)
        if len(b) < 64:
            raise ValueError("InvalidLength")
        return cls(b[:64])

    def seed(self) -> bytes:
        return bytes(self._b[:32])

    def __eq__(self, o):
        return isinstance(o, SecretKey) and bytes(o._b) == bytes(self._b)

    def __del__(self):
        for i in range(len(self._b)):
            self._b[i] = 0


def generate_keypair(rng_bytes=None):
    """(PublicKey, SecretKey) from 32 random bytes drawn from `rng_bytes(32)`."""
    seed = (rng_bytes or os.urandom)(32)
    pk = default_backend().sign_batch(np.frombuffer(seed, np.uint8).reshape(1, 32))[0].tobytes()
    return PublicKey(pk), SecretKey(seed + pk)


def generate_production_keypair():
    return generate_keypair(os.urandom)


class Signature:
    __slots__ = ("part1", "part2")

    def __init__(self, part1: bytes = bytes(32), part2: bytes = bytes(32)):
        self.part1 = bytes(part1)
        self.part2 = bytes(part2)

    @classmethod
    def default(cls):
        return cls()

    @classmethod
    def new(cls, digest: Digest, secret: SecretKey) -> "Signature":
        """crypto/src/lib.rs:185-191 (dalek Keypair::sign over the 32-byte digest).

        TEST / CORPUS USE ONLY: this runs the library's batch signer
        (nt_ed25519_sign_batch), which is NOT constant time, with the secret
        key in device memory.  The product binding leaves
        Signature::new / SignatureService on the reference's CPU path
        (SURVEY §3.4); nothing in the hot path signs.
        Deliberate divergence for malformed secrets: dalek's Keypair::from_bytes
        only checks that the public half decompresses and then signs with those
        bytes in H(R || A || M) (an invalid signature when they do not belong to
        the seed); here a public half that is not the seed's key raises
        ValueError instead.  No reference fixture covers that case."""
        seed = np.frombuffer(secret.seed(), np.uint8).reshape(1, 32)
        m = np.frombuffer(bytes(digest), np.uint8)
        pk, sig = default_backend().sign_batch(seed, m, np.array([0], np.uint64), np.array([32], np.uint64))
        if pk[0].tobytes() != bytes(secret._b[32:]):
            raise ValueError("Unable to load secret key")
        s = sig[0].tobytes()
        return cls(s[:32], s[32:])

    def flatten(self) -> bytes:
        return self.part1 + self.part2

    def verify(self, digest: Digest, public_key: PublicKey) -> None:
        """crypto/src/lib.rs:200-204: raises CryptoError on reject."""
        ok = default_backend().verify_strict(
            np.frombuffer(bytes(public_key), np.uint8), np.frombuffer(self.flatten(), np.uint8),
            np.frombuffer(bytes(digest), np.uint8), np.array([0], np.uint64), np.array([32], np.uint64))
        if not ok[0]:
            raise CryptoError("signature verification failed")

    @staticmethod
    def verify_batch(digest: Digest, votes) -> None:
        """crypto/src/lib.rs:206-219 over (PublicKey, Signature) pairs; raises CryptoError."""
        votes = list(votes)
        if not votes:
            return
        pk = np.frombuffer(b"".join(bytes(k) for k, _ in votes), np.uint8)
        sg = np.frombuffer(b"".join(s.flatten() for _, s in votes), np.uint8)
        ok = default_backend().verify_batch_groups(pk, sg, np.array([0], np.uint64),
                                                   np.array([len(votes)], np.uint32),
                                                   np.frombuffer(bytes(digest), np.uint8))
        if not ok[0]:
            raise CryptoError("batch verification failed")

    def __eq__(self, o):
        return isinstance(o, Signature) and o.flatten() == self.flatten()


class SignatureService:
    """crypto/src/lib.rs:222-249: holds the secret key; returns signatures over
    digests.  TEST / CORPUS USE ONLY (see Signature.new: non-constant-time GPU
    signer); the product keeps the reference's CPU SignatureService."""

    def __init__(self, secret: SecretKey):
        self._q = queue.Queue(100)
        self._secret = secret
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while True:
            item = self._q.get()
            if item is None:
                return
            digest, fut = item
            try:
                fut.set_result(Signature.new(digest, self._secret))
            except Exception as e:  # pragma: no cover
                fut.set_exception(e)

    def request_signature(self, digest: Digest) -> Signature:
        fut = Future()
        self._q.put((digest, fut))
        return fut.result()

    def close(self):
        self._q.put(None)
