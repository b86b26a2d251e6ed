"""ctypes binding of the CPU oracle (oracle/build/libntoracle.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use this module, and only as the checker / CPU baseline.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "build", "libntoracle.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def _ptr(a, t=_u8p):
    return a.ctypes.data_as(t)


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        lib.ntor_ed25519_verify_strict.restype = ctypes.c_int
        lib.ntor_ed25519_verify_batch.restype = ctypes.c_int
        lib.ntor_ed25519_verify_cofactorless.restype = ctypes.c_int
        lib.ntor_ed25519_batch_class.restype = ctypes.c_int
        lib.ntor_sc_is_canonical.restype = ctypes.c_int
        lib.ntor_point_decodes.restype = ctypes.c_int
        lib.ntor_point_is_small_order.restype = ctypes.c_int
        lib.ntor_point_has_torsion.restype = ctypes.c_int
        for f in ("ntor_sha512", "ntor_ed25519_verify_strict", "ntor_ed25519_verify_batch",
                  "ntor_ed25519_verify_cofactorless", "ntor_ed25519_batch_class", "ntor_ed25519_sign"):
            pass

    # --- SHA-512 ---
    def sha512(self, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.ntor_sha512(msg, ctypes.c_uint64(len(msg)), out)
        return out.raw

    def digest(self, msg: bytes) -> bytes:
        return self.sha512(msg)[:32]

    def sha512_trunc32_many(self, data: np.ndarray, off: np.ndarray, ln: np.ndarray, nthreads=1):
        n = len(off)
        out = np.zeros((n, 32), np.uint8)
        data = np.ascontiguousarray(data, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        self.lib.ntor_sha512_trunc32_many(_ptr(data), _ptr(off, _u64p), _ptr(ln, _u64p),
                                          ctypes.c_uint64(n), _ptr(out), ctypes.c_int(nthreads))
        return out

    def chacha20(self, key: bytes, n: int, stream=0, counter=0) -> bytes:
        out = ctypes.create_string_buffer(n)
        self.lib.ntor_chacha20_keystream(key, ctypes.c_uint64(stream), ctypes.c_uint64(counter), out,
                                         ctypes.c_uint64(n))
        return out.raw

    # --- Ed25519 ---
    def pubkey(self, seed: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.ntor_ed25519_pubkey(seed, out)
        return out.raw

    def sign(self, seed: bytes, pk: bytes, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.ntor_ed25519_sign(seed, pk, msg, ctypes.c_uint64(len(msg)), out)
        return out.raw

    def verify_strict(self, pk: bytes, sig: bytes, msg: bytes) -> bool:
        return bool(self.lib.ntor_ed25519_verify_strict(pk, sig, msg, ctypes.c_uint64(len(msg))))

    def verify_cofactorless(self, pk: bytes, sig: bytes, msg: bytes) -> bool:
        return bool(self.lib.ntor_ed25519_verify_cofactorless(pk, sig, msg, ctypes.c_uint64(len(msg))))

    def verify_batch(self, pks, sigs, msg: bytes) -> bool:
        pk = b"".join(pks)
        sg = b"".join(sigs)
        return bool(self.lib.ntor_ed25519_verify_batch(pk, sg, ctypes.c_uint64(len(pks)), msg,
                                                       ctypes.c_uint64(len(msg))))

    def verify_batch_dalek(self, pks, sigs, msg: bytes, zkey: bytes = bytes(32)) -> bool:
        """dalek's randomized batch equation (CPU baseline form, see ntoracle.h)."""
        self.lib.ntor_ed25519_verify_batch_dalek.restype = ctypes.c_int
        return bool(self.lib.ntor_ed25519_verify_batch_dalek(b"".join(pks), b"".join(sigs), ctypes.c_uint64(len(pks)),
                                                             msg, ctypes.c_uint64(len(msg)), zkey))

    def certificates_verify_many(self, hdr, hoff, hlen, ids, hpk, hsig, cpre, vpk, vsig, first, cnt, nthreads=1):
        """Certificate::verify signature + digest work per certificate (CPU baseline)."""
        G = len(cnt)
        out = np.zeros(max(G, 1), np.uint8)
        a = [np.ascontiguousarray(x, np.uint8) for x in (hdr, ids, hpk, hsig, cpre, vpk, vsig)]
        hoff = np.ascontiguousarray(hoff, np.uint64)
        hlen = np.ascontiguousarray(hlen, np.uint64)
        first = np.ascontiguousarray(first, np.uint64)
        cnt = np.ascontiguousarray(cnt, np.uint32)
        self.lib.ntor_certificates_verify_many(_ptr(a[0]), _ptr(hoff, _u64p), _ptr(hlen, _u64p), _ptr(a[1]),
                                               _ptr(a[2]), _ptr(a[3]), _ptr(a[4]), _ptr(a[5]), _ptr(a[6]),
                                               _ptr(first, _u64p), _ptr(cnt, _u32p), ctypes.c_uint64(G), _ptr(out),
                                               ctypes.c_int(nthreads))
        return out[:G]

    def batch_class(self, pk, sig, msg) -> int:
        return int(self.lib.ntor_ed25519_batch_class(pk, sig, msg, ctypes.c_uint64(len(msg))))

    def verify_strict_many(self, pk, sig, msg, off, ln, nthreads=1) -> np.ndarray:
        n = len(off)
        bm = np.zeros((n + 7) // 8, np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        msg = np.ascontiguousarray(msg, np.uint8) if len(msg) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        self.lib.ntor_ed25519_verify_strict_many(_ptr(pk), _ptr(sig), _ptr(msg), _ptr(off, _u64p),
                                                 _ptr(ln, _u64p), ctypes.c_uint64(n), _ptr(bm),
                                                 ctypes.c_int(nthreads))
        return np.unpackbits(bm, bitorder="little")[:n]

    def sodium_verify_many(self, libpath, pk, sig, msg, off, ln, nthreads=1):
        """libsodium crypto_sign_verify_detached over n signatures (external CPU
        comparator, bench.py); None when libsodium is absent."""
        n = len(off)
        out = np.zeros(max(n, 1), np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        msg = np.ascontiguousarray(msg, np.uint8) if len(msg) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        self.lib.ntor_sodium_verify_many.restype = ctypes.c_int
        rc = self.lib.ntor_sodium_verify_many(ctypes.c_char_p(libpath.encode()), _ptr(pk), _ptr(sig), _ptr(msg),
                                              _ptr(off, _u64p), _ptr(ln, _u64p), ctypes.c_uint64(n),
                                              ctypes.c_int(nthreads), _ptr(out))
        return None if rc != 0 else out[:n]

    def verify_batch_groups(self, pk, sig, first, cnt, msg32, nthreads=1):
        G = len(cnt)
        nsig = len(pk)
        gb = np.zeros((G + 7) // 8, np.uint8)
        sb = np.zeros((nsig + 7) // 8 + 1, np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8) if nsig else np.zeros((1, 32), np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8) if nsig else np.zeros((1, 64), np.uint8)
        first = np.ascontiguousarray(first, np.uint64)
        cnt = np.ascontiguousarray(cnt, np.uint32)
        msg32 = np.ascontiguousarray(msg32, np.uint8)
        self.lib.ntor_ed25519_verify_batch_groups(_ptr(pk), _ptr(sig), _ptr(first, _u64p), _ptr(cnt, _u32p),
                                                  _ptr(msg32), ctypes.c_uint64(G), _ptr(gb), _ptr(sb),
                                                  ctypes.c_int(nthreads))
        return (np.unpackbits(gb, bitorder="little")[:G], np.unpackbits(sb, bitorder="little")[:nsig])

    def point_decodes(self, p):
        return bool(self.lib.ntor_point_decodes(p))

    def point_is_small_order(self, p):
        return bool(self.lib.ntor_point_is_small_order(p))

    def point_has_torsion(self, p):
        return bool(self.lib.ntor_point_has_torsion(p))

    def torsion_point(self, i):
        out = ctypes.create_string_buffer(32)
        self.lib.ntor_torsion_point(ctypes.c_int(i), out)
        return out.raw

    def basepoint_mul(self, s: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.ntor_basepoint_mul(s, out)
        return out.raw

    def sc_reduce64(self, b: bytes) -> bytes:
        out = ctypes.create_string_buffer(32)
        self.lib.ntor_sc_reduce64(b, out)
        return out.raw


_cached = None


def load():
    global _cached
    if _cached is None:
        if not os.path.exists(LIB) and os.path.exists(os.path.join(ORACLE_DIR, "Makefile")):
            build()
        _cached = Oracle(ctypes.CDLL(LIB))
    return _cached


def expand(label: bytes, n: int) -> bytes:
    """Deterministic synthetic bytes, identical to tests/golden/make_golden.py."""
    import hashlib
    import struct
    out = bytearray()
    i = 0
    while len(out) < n:
        out += hashlib.sha512(label + struct.pack("<Q", i)).digest()
        i += 1
    return bytes(out[:n])
