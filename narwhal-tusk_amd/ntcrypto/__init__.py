"""ntcrypto -- MI355X (gfx950) backend for Narwhal/Tusk's crypto hot path.

Bulk API: `Backend` (numpy in/out over the C ABI, include/ntcrypto.h).
Crate mirror: `Digest, PublicKey, SecretKey, Signature, SignatureService,
CryptoError, generate_keypair` (crypto/src/lib.rs) and the primary/worker
callers in `ntcrypto.narwhal` (primary/src/messages.rs, worker/src/processor.rs).
"""
from ._lib import (EXPORTED, LIB_PATH, NT_KEY_STRICT_BIT, NT_MODE_COFACTORLESS, NT_MODE_MIXED, NT_MODE_STRICT,
                   NT_SMALL_ALWAYS, NT_SMALL_AUTO, NT_SMALL_OFF, Backend, Committee, Keyset, NtError, default_backend,
                   load_library, nbytes)
from .crypto import (CryptoError, Digest, PublicKey, SecretKey, Signature, SignatureService,
                     generate_keypair, generate_production_keypair, sha512_digest, sha512_digest_batch)

__all__ = [
    "Backend", "Committee", "Keyset", "NtError", "default_backend", "load_library", "EXPORTED", "LIB_PATH",
    "NT_MODE_STRICT", "NT_MODE_COFACTORLESS", "NT_MODE_MIXED", "NT_KEY_STRICT_BIT", "NT_SMALL_OFF", "NT_SMALL_AUTO",
    "NT_SMALL_ALWAYS", "CryptoError", "Digest", "nbytes",
    "PublicKey", "SecretKey",
    "Signature", "SignatureService", "generate_keypair", "generate_production_keypair",
    "sha512_digest", "sha512_digest_batch",
]
