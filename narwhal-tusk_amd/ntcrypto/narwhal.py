"""ctypes binding of libntnarwhal.so (narwhal-tusk_amd/host/capi.cpp): the C++
mirror of the primary's callers of the crypto hot path.

  Core            primary::Core batched sanitize over bincode wire messages
                  (core.rs:306-411, SURVEY §8(f).1 + (f).2); verdicts are
                  primary::DagError codes (DAG_ERRORS)
  wire_reencode   decode + re-encode one bincode PrimaryMessage (codec check)

Signature work runs on the GPU through libntcrypto.so; the wire decode runs on
host threads.  A backend failure raises, it is never turned into a verdict.
"""
import ctypes
import os

import numpy as np

from ._lib import PKG_ROOT, NtError

LIB_PATH = os.path.join(PKG_ROOT, "lib", "libntnarwhal.so")
DAG_ERRORS = ["Ok", "InvalidSignature", "InvalidHeaderId", "MalformedHeader", "UnknownAuthority",
              "AuthorityReuse", "CertificateRequiresQuorum", "TooOld", "UnexpectedVote", "SerializationError",
              "UnexpectedMessage"]
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NtError("libntnarwhal.so not built (%s); run `make -C narwhal-tusk_amd`" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        lib.ntn_wire_reencode.argtypes = [_u8p, ctypes.c_uint64, _u8p, ctypes.c_uint64, _u64p]
        lib.ntn_wire_reencode.restype = ctypes.c_int64
        lib.ntn_wire_header_preimage.argtypes = [_u8p, ctypes.c_uint64, _u8p, ctypes.c_uint64]
        lib.ntn_wire_header_preimage.restype = ctypes.c_int64
        lib.ntn_core_new.argtypes = [_u8p, _u32p, _u32p, ctypes.c_uint32, ctypes.c_uint64, _u8p, ctypes.c_uint64,
                                     ctypes.c_int]
        lib.ntn_core_new.restype = ctypes.c_void_p
        lib.ntn_core_free.argtypes = [ctypes.c_void_p]
        lib.ntn_core_free.restype = None
        lib.ntn_core_ingest.argtypes = [ctypes.c_void_p, _u8p, _u64p, _u64p, ctypes.c_uint64, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        lib.ntn_core_ingest.restype = ctypes.c_int
        lib.ntn_core_ingest_pipelined.argtypes = [ctypes.c_void_p, _u8p, _u64p, _u64p, ctypes.c_uint64, ctypes.c_int,
                                                  ctypes.c_uint64, ctypes.POINTER(ctypes.c_int32)]
        lib.ntn_core_ingest_pipelined.restype = ctypes.c_int
        lib.ntn_last_ingest_stats.argtypes = [ctypes.POINTER(ctypes.c_double)]
        lib.ntn_last_ingest_stats.restype = None
        lib.ntn_batcher_new.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32]
        lib.ntn_batcher_new.restype = ctypes.c_void_p
        lib.ntn_batcher_free.argtypes = [ctypes.c_void_p]
        lib.ntn_batcher_free.restype = None
        lib.ntn_batcher_submit.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, _u8p, ctypes.c_uint64]
        lib.ntn_batcher_submit.restype = ctypes.c_void_p
        lib.ntn_batcher_wait.argtypes = [ctypes.c_void_p, _u8p, _u8p]
        lib.ntn_batcher_wait.restype = ctypes.c_int
        lib.ntn_batcher_flush.argtypes = [ctypes.c_void_p]
        lib.ntn_batcher_flush.restype = None
        lib.ntn_batcher_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        lib.ntn_batcher_stats.restype = None
        lib.ntn_set_small_call_path.argtypes = [ctypes.c_int, ctypes.c_int]
        lib.ntn_set_small_call_path.restype = ctypes.c_int
        _lib = lib
    return _lib


def _buf(b):
    a = np.frombuffer(b, np.uint8) if len(b) else np.zeros(1, np.uint8)
    return a, a.ctypes.data_as(_u8p)


def wire_reencode(msg: bytes):
    """(re-encoded bytes, bytes consumed) or None on a bincode decode error"""
    a, p = _buf(msg)
    out = np.zeros(2 * len(msg) + 64, np.uint8)
    used = ctypes.c_uint64(0)
    r = load().ntn_wire_reencode(p, len(msg), out.ctypes.data_as(_u8p), len(out), ctypes.byref(used))
    return None if r < 0 else (out[:r].tobytes(), used.value)


def wire_header_preimage(msg: bytes):
    a, p = _buf(msg)
    out = np.zeros(len(msg) + 64, np.uint8)
    r = load().ntn_wire_header_preimage(p, len(msg), out.ctypes.data_as(_u8p), len(out))
    return None if r < 0 else out[:r].tobytes()


def pack(messages):
    """packed buffer + offsets + lengths of a list of byte strings"""
    ln = np.array([len(m) for m in messages], np.uint64)
    off = np.zeros(len(messages), np.uint64)
    if len(messages) > 1:
        off[1:] = np.cumsum(ln)[:-1]
    data = np.frombuffer(b"".join(messages), np.uint8) if messages else np.zeros(1, np.uint8)
    return data, off, ln


class Core:
    """primary::Core for one committee: keys (n x 32 B), stakes, workers per
    authority, GC round and the header currently being voted on (bincode of a
    PrimaryMessage::Header, or None); use_keyset builds the committee key cache."""

    def __init__(self, keys, stakes, nworkers, gc_round=0, current_header=None, use_keyset=True):
        lib = load()
        keys = np.ascontiguousarray(np.asarray(keys, np.uint8).reshape(-1, 32))
        stakes = np.ascontiguousarray(stakes, np.uint32)
        nworkers = np.ascontiguousarray(nworkers, np.uint32)
        ch, chp = _buf(current_header or b"")
        self._h = lib.ntn_core_new(keys.ctypes.data_as(_u8p), stakes.ctypes.data_as(_u32p),
                                   nworkers.ctypes.data_as(_u32p), len(keys), gc_round,
                                   chp if current_header else None, len(current_header or b""), int(use_keyset))
        if not self._h:
            raise NtError("ntn_core_new failed (no gfx950 device, or a bad current header)")

    def ingest(self, data, off, ln, threads=8, general=False, device=False):
        """DagError codes for n packed wire messages; also returns the host decode
        seconds.  general=True: the object-model decoder (cross-check path).
        device=True: Core::ingest_device -- certificates parsed and checked on the
        GPU from the wire bytes (nt_certificates_ingest), the rest on the host;
        the second value is then the count of messages the host decided."""
        n = len(off)
        codes = np.zeros(max(n, 1), np.int32)
        dec = ctypes.c_double(0)
        data = np.ascontiguousarray(data, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        rc = load().ntn_core_ingest(self._h, data.ctypes.data_as(_u8p), off.ctypes.data_as(_u64p),
                                    ln.ctypes.data_as(_u64p), n, threads,
                                    codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.byref(dec),
                                    2 if device else int(general))
        if rc != 0:
            raise NtError("ntn_core_ingest: backend failure")
        return codes[:n], (int(dec.value) if device else dec.value)

    def ingest_pipelined(self, data, off, ln, threads=8, chunk=25000):
        """Core::ingest_pipelined: chunks of `chunk` messages, two in flight"""
        n = len(off)
        codes = np.zeros(max(n, 1), np.int32)
        data = np.ascontiguousarray(data, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        rc = load().ntn_core_ingest_pipelined(self._h, data.ctypes.data_as(_u8p), off.ctypes.data_as(_u64p),
                                              ln.ctypes.data_as(_u64p), n, threads, chunk,
                                              codes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if rc != 0:
            raise NtError("ntn_core_ingest_pipelined: backend failure")
        return codes[:n]

    @staticmethod
    def last_stats():
        """phase seconds of the last SoA ingest on this thread"""
        a = (ctypes.c_double * 6)()
        load().ntn_last_ingest_stats(a)
        return dict(zip(("decode", "prep", "digest", "verify_strict", "verify_batch", "total"), list(a)))

    def close(self):
        if self._h:
            load().ntn_core_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def set_small_call_path(mode, threads=0):
    """The small-call path of the mirror's shared context (nt_set_small_call_path)."""
    rc = load().ntn_set_small_call_path(int(mode), int(threads))
    if rc != 0:
        raise NtError("ntn_set_small_call_path failed (%d)" % rc)


class DigestBatcher:
    """worker::DigestBatcher (host/narwhal.hpp): both Processor
    tasks of a worker submit serialized batches from their own threads; a
    flusher hashes everything queued in one nt_sha512_trunc32 call when
    max_bytes / max_batches is reached or the oldest batch is max_delay_us old.

    submit() returns a ticket; wait(ticket) -> (digest32 bytes, 40-byte
    WorkerPrimaryMessage).  ctypes releases the GIL in both, so Python threads
    submit and wait concurrently."""

    def __init__(self, max_bytes=256 << 20, max_batches=4096, max_delay_us=1000):
        self._lib = load()
        self._h = self._lib.ntn_batcher_new(max_bytes, max_batches, max_delay_us)
        if not self._h:
            raise NtError("ntn_batcher_new failed")

    def submit(self, worker_id, own, batch):
        a, p = _buf(batch)
        t = self._lib.ntn_batcher_submit(self._h, worker_id, 1 if own else 0, p, len(batch))
        if not t:
            raise NtError("ntn_batcher_submit failed")
        return t

    def wait(self, ticket):
        d = np.zeros(32, np.uint8)
        m = np.zeros(40, np.uint8)
        rc = self._lib.ntn_batcher_wait(ticket, d.ctypes.data_as(_u8p), m.ctypes.data_as(_u8p))
        if rc != 0:
            raise NtError("digest batcher: backend failure")
        return d.tobytes(), m.tobytes()

    def process(self, worker_id, own, batch):
        return self.wait(self.submit(worker_id, own, batch))

    def flush(self):
        self._lib.ntn_batcher_flush(self._h)

    def stats(self):
        out = (ctypes.c_double * 4)()
        self._lib.ntn_batcher_stats(self._h, out)
        return {"flushes": int(out[0]), "batches": int(out[1]), "bytes": int(out[2]), "hash_seconds": out[3]}

    def close(self):
        if self._h:
            self._lib.ntn_batcher_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
