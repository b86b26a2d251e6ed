"""ctypes binding of libntcrypto.so (include/ntcrypto.h).

The product path: every call goes to the gfx950 HIP kernels through the C ABI.
There is no CPU fallback -- if the library or a gfx950 device is missing the
calls raise NtError.
"""
import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("NTCRYPTO_LIB", os.path.join(PKG_ROOT, "lib", "libntcrypto.so"))

NT_MODE_STRICT = 0
NT_MODE_COFACTORLESS = 1
NT_MODE_MIXED = 2             # key-cache only: key_idx bit 31 = strict
NT_KEY_STRICT_BIT = 0x80000000
NT_SMALL_OFF = 0              # small-call path (include/ntcrypto.h): everything on the GPU
NT_SMALL_AUTO = 1             # calls below the host/GPU crossover on host threads
NT_SMALL_ALWAYS = 2           # every host entry point on host threads (tests)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_u64 = ctypes.c_uint64

EXPORTED = [
    "nt_init", "nt_init_device", "nt_init_devices", "nt_free", "nt_num_devices", "nt_strerror", "nt_version",
    "nt_sha512_trunc32", "nt_ed25519_verify_strict", "nt_ed25519_verify_batch_groups",
    "nt_ed25519_sign_batch", "nt_ed25519_keypair_batch", "nt_dev_sha512_trunc32",
    "nt_dev_sha512_trunc32_bounded",
    "nt_dev_ed25519_verify", "nt_dev_group_and", "nt_dev_ed25519_sign", "nt_keyset_create",
    "nt_keyset_free", "nt_keyset_flags", "nt_keyset_info", "nt_ed25519_verify_keyset", "nt_ed25519_verify_batch_groups_keyset",
    "nt_dev_ed25519_verify_keyset", "nt_host_alloc", "nt_host_free", "nt_set_small_call_path", "nt_call_counts",
    "nt_committee_create", "nt_committee_free", "nt_certificates_ingest", "nt_small_call_model",
    "nt_set_hbm_budget", "nt_memory_info", "nt_dev_stream", "nt_set_key_cache", "nt_key_cache_add",
    "nt_key_cache_sync", "nt_key_cache_info", "nt_dev_clock_probe", "nt_dev_ed25519_verify_keyset_groups",
]
KEY_CACHE_INFO_KEYS = ("keys", "max_keys", "comb_bits", "bytes_per_device", "hits", "misses", "admitted", "refused",
                       "pending", "error", "alloc_us", "build_us")
MEMORY_INFO_KEYS = ("comb_b_bits", "comb_b_bytes", "key_comb_bytes", "workspace_bytes", "stash_bytes",
                    "staging_bytes", "budget", "held")


class NtError(RuntimeError):
    pass


_lib = None


def load_library(path=None):
    """Load libntcrypto.so and declare prototypes (no GPU needed)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NtError("libntcrypto.so not built (%s); run `make -C narwhal-tusk_amd`" % p)
    lib = ctypes.CDLL(p)
    lib.nt_init.argtypes = [ctypes.POINTER(_vp), ctypes.c_int]
    lib.nt_init_device.argtypes = [ctypes.POINTER(_vp), ctypes.c_int]
    lib.nt_init_devices.argtypes = [ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.nt_free.argtypes = [_vp]
    lib.nt_free.restype = None
    lib.nt_host_alloc.argtypes = [ctypes.c_uint64]
    lib.nt_host_alloc.restype = _vp
    lib.nt_host_free.argtypes = [_vp]
    lib.nt_host_free.restype = None
    lib.nt_num_devices.argtypes = [_vp]
    lib.nt_strerror.restype = ctypes.c_char_p
    lib.nt_version.restype = ctypes.c_char_p
    lib.nt_sha512_trunc32.argtypes = [_vp, _u8p, _u64p, _u64p, _u64, _u8p]
    lib.nt_ed25519_verify_strict.argtypes = [_vp, _u8p, _u8p, _u8p, _u64p, _u64p, _u64, _u8p]
    lib.nt_ed25519_verify_batch_groups.argtypes = [_vp, _u8p, _u8p, _u64p, _u32p, _u8p, _u64, _u8p, _u8p]
    lib.nt_ed25519_sign_batch.argtypes = [_vp, _u8p, _u8p, _u64p, _u64p, _u64, _u8p, _u8p]
    lib.nt_ed25519_keypair_batch.argtypes = [_vp, _u8p, _u64, _u8p]
    lib.nt_dev_sha512_trunc32.argtypes = [_vp, ctypes.c_int, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp]
    lib.nt_dev_sha512_trunc32_bounded.argtypes = [_vp, ctypes.c_int, _vp, _vp, _u64, _vp, _vp, _u64, _u64, _vp, _vp]
    lib.nt_dev_ed25519_verify.argtypes = [_vp, ctypes.c_int, _vp, ctypes.c_int, _vp, _vp, _vp, _u64, _vp, _vp,
                                          _u64, _vp]
    lib.nt_dev_group_and.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp, _u64, _vp, _vp]
    lib.nt_dev_ed25519_sign.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp]
    lib.nt_keyset_create.argtypes = [_vp, _u8p, ctypes.c_uint32, ctypes.POINTER(_vp)]
    lib.nt_keyset_free.argtypes = [_vp]
    lib.nt_keyset_free.restype = None
    lib.nt_keyset_flags.argtypes = [_vp, ctypes.c_uint32, _u32p]
    lib.nt_keyset_info.argtypes = [_vp, _u32p, _u64p]
    lib.nt_ed25519_verify_keyset.argtypes = [_vp, _vp, ctypes.c_int, _u32p, _u8p, _u8p, _u64p, _u64p, _u64, _u8p]
    lib.nt_ed25519_verify_batch_groups_keyset.argtypes = [_vp, _vp, _u32p, _u8p, _u64p, _u32p, _u8p, _u64, _u8p,
                                                          _u8p]
    lib.nt_dev_ed25519_verify_keyset.argtypes = [_vp, _vp, ctypes.c_int, _vp, ctypes.c_int, _vp, _vp, _vp, _u64,
                                                 _vp, _vp, _u64, _vp]
    lib.nt_set_small_call_path.argtypes = [_vp, ctypes.c_int, ctypes.c_int]
    lib.nt_call_counts.argtypes = [_vp, _u64p, _u64p]
    if hasattr(lib, "nt_small_call_model"):  # absent from older A/B builds (NTCRYPTO_LIB)
        lib.nt_small_call_model.argtypes = [_vp, ctypes.POINTER(ctypes.c_double)]
    lib.nt_committee_create.argtypes = [_vp, _vp, _u32p, _u64p, _u32p, ctypes.c_uint32, ctypes.POINTER(_vp)]
    lib.nt_committee_free.argtypes = [_vp]
    lib.nt_committee_free.restype = None
    lib.nt_certificates_ingest.argtypes = [_vp, _vp, _u8p, _u64p, _u64p, _u64, _u64, _u8p]
    if hasattr(lib, "nt_memory_info"):  # absent from round-3 A/B builds (NTCRYPTO_LIB)
        lib.nt_set_hbm_budget.argtypes = [_vp, ctypes.c_uint64]
        lib.nt_memory_info.argtypes = [_vp, ctypes.c_int, _u64p]
        lib.nt_dev_stream.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]
    if hasattr(lib, "nt_set_key_cache"):  # absent from round-5 A/B builds (NTCRYPTO_LIB)
        lib.nt_set_key_cache.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32]
        lib.nt_key_cache_add.argtypes = [_vp, _u8p, ctypes.c_uint32]
        lib.nt_key_cache_sync.argtypes = [_vp]
        lib.nt_key_cache_info.argtypes = [_vp, _u64p]
        lib.nt_dev_clock_probe.argtypes = [_vp, ctypes.c_int, _vp, ctypes.c_uint32, _vp, _u64p]
        lib.nt_dev_ed25519_verify_keyset_groups.argtypes = [_vp, _vp, ctypes.c_int, _vp, ctypes.c_int, _vp, _vp, _vp,
                                                            _u64, _vp, _vp, _u64, _vp, _vp, _u64, _vp, _vp]
    _lib = lib
    return lib


def _p(a, t=_u8p):
    return a.ctypes.data_as(t)


def _u8(a, shape_tail=None):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a


def _check(rc, what):
    if rc != 0:
        raise NtError("%s failed: %s (%d)" % (what, load_library().nt_strerror(rc).decode(), rc))


def _unpack(bm, n):
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def _torch_first():
    """PyTorch-ROCm wheels bundle their own HIP runtime.  Two runtimes in one
    process work when torch's starts first; torch's first HIP init AFTER
    libntcrypto has mapped its tables fails ("PyTorch in the
    same process").  If this process has imported torch, start its runtime now."""
    import sys
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_available() and not torch.cuda.is_initialized():
        torch.cuda.init()


def nbytes(t):
    """Byte size of a device buffer given as a torch tensor (the msg_bytes /
    data_bytes argument of the device-resident entry points)."""
    return int(t.numel()) * int(t.element_size())


class Backend:
    """A context over one or more gfx950 devices (nt_init / nt_init_device)."""

    def __init__(self, num_gpus=0, device=None, devices=None):
        self.lib = load_library()
        _torch_first()
        ctx = _vp()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            rc = self.lib.nt_init_devices(ctypes.byref(ctx), arr, len(devices))
        elif device is not None:
            rc = self.lib.nt_init_device(ctypes.byref(ctx), int(device))
        else:
            rc = self.lib.nt_init(ctypes.byref(ctx), int(num_gpus))
        _check(rc, "nt_init")
        self.ctx = ctx

    def close(self):
        if self.ctx:
            self.lib.nt_free(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_devices(self):
        return self.lib.nt_num_devices(self.ctx)

    def set_small_call_path(self, mode=NT_SMALL_AUTO, threads=0):
        """Small calls on host threads (include/ntcrypto.h)."""
        _check(self.lib.nt_set_small_call_path(self.ctx, int(mode), int(threads)), "nt_set_small_call_path")

    def pinned(self, shape, dtype=np.uint8):
        """A numpy array in nt_host_alloc memory (pinned, registered with every
        device of the process): inputs placed there are DMA'd by the host entry
        points without the staging copy.  Freed when the array is collected."""
        dt = np.dtype(dtype)
        count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
        nbytes = max(1, count * dt.itemsize)
        p = self.lib.nt_host_alloc(nbytes)
        if not p:
            raise MemoryError("nt_host_alloc(%d)" % nbytes)
        buf = (ctypes.c_uint8 * nbytes).from_address(p)
        arr = np.frombuffer(buf, dtype=np.uint8, count=count * dt.itemsize).view(dt).reshape(shape)
        import weakref
        weakref.finalize(buf, self.lib.nt_host_free, ctypes.c_void_p(p))
        return arr

    def small_call_model(self):
        """The small-call cost model AUTO routes by (nt_small_call_model): the
        host-lane rates and one GPU floor per verify kernel (uncached, key cache)."""
        out = (ctypes.c_double * 10)()
        _check(self.lib.nt_small_call_model(self.ctx, out), "nt_small_call_model")
        keys = ("cpu_verify_us", "gpu_verify_us", "cpu_sha_mbs", "gpu_lane_mbs", "gpu_call_us", "pcie_gbs",
                "spawn_us", "threads", "calibrated", "gpu_keyset_us")
        d = dict(zip(keys, list(out)))
        d["threads"] = int(d["threads"])
        d["calibrated"] = bool(d["calibrated"])
        return d

    def set_hbm_budget(self, nbytes):
        """Cap the tables (comb of B + key combs) this context holds per device
        entry; 0 = no cap (nt_set_hbm_budget)."""
        _check(self.lib.nt_set_hbm_budget(self.ctx, int(nbytes)), "nt_set_hbm_budget")

    def memory_info(self, dev=0):
        """What device entry `dev` of this context holds (nt_memory_info)."""
        out = np.zeros(8, np.uint64)
        _check(self.lib.nt_memory_info(self.ctx, int(dev), _p(out, _u64p)), "nt_memory_info")
        return dict(zip(MEMORY_INFO_KEYS, (int(x) for x in out)))

    def dev_stream(self, dev=0, which=0):
        """Raw hipStream_t of device entry `dev`'s compute stream `which` (0 / 1):
        the streams the host entry points pipeline on (nt_dev_stream)."""
        p = _vp()
        _check(self.lib.nt_dev_stream(self.ctx, int(dev), int(which), ctypes.byref(p)), "nt_dev_stream")
        return int(p.value)

    # ---- the key registry (nt_set_key_cache): the key cache behind the plain entry points ----
    def set_key_cache(self, max_keys, admit_after=1):
        """Enable (max_keys > 0) or disable (0) the context's key registry."""
        _check(self.lib.nt_set_key_cache(self.ctx, int(max_keys), int(admit_after)), "nt_set_key_cache")

    def key_cache_add(self, pks):
        """Admit these 32-byte keys now (waits for their tables)."""
        pks = np.ascontiguousarray(pks, np.uint8).reshape(-1, 32)
        buf = pks if len(pks) else np.zeros((1, 32), np.uint8)
        _check(self.lib.nt_key_cache_add(self.ctx, _p(buf), len(pks)), "nt_key_cache_add")

    def key_cache_sync(self):
        """Wait until queued admissions are published (nt_key_cache_sync)."""
        _check(self.lib.nt_key_cache_sync(self.ctx), "nt_key_cache_sync")

    def key_cache_info(self):
        out = np.zeros(12, np.uint64)
        _check(self.lib.nt_key_cache_info(self.ctx, _p(out, _u64p)), "nt_key_cache_info")
        d = dict(zip(KEY_CACHE_INFO_KEYS, (int(x) for x in out)))
        d["error"] = -d["error"]
        return d

    def dev_clock_probe(self, dev, stream, iters, d_out2):
        """Enqueue the clock probe (nt_dev_clock_probe) on `stream`; returns the
        wall clock's rate in kHz.  d_out2: device uint64[2] (cycles, wall ticks)."""
        khz = np.zeros(1, np.uint64)
        _check(self.lib.nt_dev_clock_probe(self.ctx, int(dev), stream, int(iters), d_out2, _p(khz, _u64p)),
               "nt_dev_clock_probe")
        return int(khz[0])

    def call_counts(self):
        """(host-lane calls, GPU calls) of the host entry points so far."""
        h = np.zeros(1, np.uint64)
        g = np.zeros(1, np.uint64)
        _check(self.lib.nt_call_counts(self.ctx, _p(h, _u64p), _p(g, _u64p)), "nt_call_counts")
        return int(h[0]), int(g[0])

    # ---- SHA-512 ----
    def sha512_trunc32(self, data, off, ln):
        data = _u8(data) if len(data) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        n = len(off)
        out = np.zeros((max(n, 1), 32), np.uint8)
        _check(self.lib.nt_sha512_trunc32(self.ctx, _p(data), _p(off, _u64p), _p(ln, _u64p), n, _p(out)),
               "nt_sha512_trunc32")
        return out[:n]

    def digest_many(self, messages):
        ln = np.array([len(m) for m in messages], np.uint64)
        off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64) if len(messages) else np.zeros(0, np.uint64)
        data = np.frombuffer(b"".join(messages), np.uint8) if messages else np.zeros(0, np.uint8)
        return self.sha512_trunc32(data, off, ln)

    # ---- Ed25519 ----
    def verify_strict(self, pk, sig, msg, off, ln):
        pk = _u8(pk).reshape(-1, 32)
        sig = _u8(sig).reshape(-1, 64)
        n = len(pk)
        msg = _u8(msg) if len(msg) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        bm = np.zeros((n + 7) // 8 + 1, np.uint8)
        _check(self.lib.nt_ed25519_verify_strict(self.ctx, _p(pk), _p(sig), _p(msg), _p(off, _u64p),
                                                  _p(ln, _u64p), n, _p(bm)), "nt_ed25519_verify_strict")
        return _unpack(bm, n)

    def verify_batch_groups(self, pk, sig, first, cnt, msg32, with_sig_bits=False):
        pk = _u8(pk).reshape(-1, 32)
        sig = _u8(sig).reshape(-1, 64)
        if len(pk) == 0:
            pk = np.zeros((1, 32), np.uint8)
            sig = np.zeros((1, 64), np.uint8)
        first = np.ascontiguousarray(first, np.uint64)
        cnt = np.ascontiguousarray(cnt, np.uint32)
        msg32 = _u8(msg32).reshape(-1, 32)
        G = len(cnt)
        nsig = int((first + cnt).max()) if G else 0
        gb = np.zeros((G + 7) // 8 + 1, np.uint8)
        sb = np.zeros((nsig + 7) // 8 + 1, np.uint8)
        _check(self.lib.nt_ed25519_verify_batch_groups(
            self.ctx, _p(pk), _p(sig), _p(first, _u64p), _p(cnt, _u32p), _p(msg32), G, _p(gb),
            _p(sb) if with_sig_bits else None), "nt_ed25519_verify_batch_groups")
        if with_sig_bits:
            return _unpack(gb, G), _unpack(sb, nsig)
        return _unpack(gb, G)

    def sign_batch(self, seeds, msg=None, off=None, ln=None):
        seeds = _u8(seeds).reshape(-1, 32)
        n = len(seeds)
        pk = np.zeros((max(n, 1), 32), np.uint8)
        if msg is None:
            _check(self.lib.nt_ed25519_keypair_batch(self.ctx, _p(seeds), n, _p(pk)), "nt_ed25519_keypair_batch")
            return pk[:n]
        msg = _u8(msg) if len(msg) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        sig = np.zeros((max(n, 1), 64), np.uint8)
        _check(self.lib.nt_ed25519_sign_batch(self.ctx, _p(seeds), _p(msg), _p(off, _u64p), _p(ln, _u64p), n,
                                              _p(pk), _p(sig)), "nt_ed25519_sign_batch")
        return pk[:n], sig[:n]

    # ---- committee key cache ----
    def keyset(self, pks):
        return Keyset(self, pks)

    # ---- device-resident (raw device pointers; stream 0 = HIP's NULL stream) ----
    # Message buffers come with their byte size, as in the C ABI: an item whose
    # slice d_msg[off, off + len) lies outside [0, msg_bytes) is never read.
    def dev_verify(self, dev, stream, mode, d_pk, d_sig, d_msg, msg_bytes, d_off, d_len, n, d_out):
        _check(self.lib.nt_dev_ed25519_verify(self.ctx, dev, stream, mode, d_pk, d_sig, d_msg, int(msg_bytes), d_off,
                                              d_len, n, d_out), "nt_dev_ed25519_verify")

    def dev_sha512(self, dev, stream, d_data, data_bytes, d_off, d_len, n, d_out, max_len=None, d_bad=None):
        """max_len: an upper bound of the message lengths, if known (selects the
        kernel: nt_dev_sha512_trunc32_bounded); d_bad: device uint32 counter of
        out-of-bounds items (zero digests), or None"""
        if max_len is None:
            _check(self.lib.nt_dev_sha512_trunc32(self.ctx, dev, stream, d_data, int(data_bytes), d_off, d_len, n,
                                                  d_bad, d_out), "nt_dev_sha512_trunc32")
        else:
            _check(self.lib.nt_dev_sha512_trunc32_bounded(self.ctx, dev, stream, d_data, int(data_bytes), d_off, d_len,
                                                          n, int(max_len), d_bad, d_out),
                   "nt_dev_sha512_trunc32_bounded")

    def dev_sign(self, dev, stream, d_seed, d_msg, msg_bytes, d_off, d_len, n, d_pk, d_sig):
        _check(self.lib.nt_dev_ed25519_sign(self.ctx, dev, stream, d_seed, d_msg, int(msg_bytes), d_off, d_len, n,
                                            d_pk, d_sig), "nt_dev_ed25519_sign")

    def dev_group_and(self, dev, stream, d_first, d_cnt, G, d_sig_words, d_group_words):
        _check(self.lib.nt_dev_group_and(self.ctx, dev, stream, d_first, d_cnt, G, d_sig_words, d_group_words),
               "nt_dev_group_and")


class Keyset:
    """Per-key comb tables of a static committee on every device (nt_keyset_*)."""

    def __init__(self, backend, pks):
        self.be = backend
        pks = np.ascontiguousarray(pks, np.uint8).reshape(-1, 32)
        self.nkeys = len(pks)
        h = _vp()
        buf = pks if len(pks) else np.zeros((1, 32), np.uint8)
        _check(backend.lib.nt_keyset_create(backend.ctx, _p(buf), self.nkeys, ctypes.byref(h)), "nt_keyset_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.be.lib.nt_keyset_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def flags(self, i):
        f = ctypes.c_uint32()
        _check(self.be.lib.nt_keyset_flags(self.h, i, ctypes.byref(f)), "nt_keyset_flags")
        return int(f.value)

    def info(self):
        """(comb digit width, device bytes per device) -- nt_keyset_info"""
        b, nb = ctypes.c_uint32(), ctypes.c_uint64()
        _check(self.be.lib.nt_keyset_info(self.h, ctypes.byref(b), ctypes.byref(nb)), "nt_keyset_info")
        return int(b.value), int(nb.value)

    def verify(self, mode, key_idx, sig, msg, off, ln):
        key_idx = np.ascontiguousarray(key_idx, np.uint32)
        sig = _u8(sig).reshape(-1, 64)
        n = len(key_idx)
        msg = _u8(msg) if len(msg) else np.zeros(1, np.uint8)
        off = np.ascontiguousarray(off, np.uint64)
        ln = np.ascontiguousarray(ln, np.uint64)
        bm = np.zeros((n + 7) // 8 + 1, np.uint8)
        _check(self.be.lib.nt_ed25519_verify_keyset(self.be.ctx, self.h, mode, _p(key_idx, _u32p), _p(sig), _p(msg),
                                                    _p(off, _u64p), _p(ln, _u64p), n, _p(bm)),
               "nt_ed25519_verify_keyset")
        return _unpack(bm, n)

    def verify_batch_groups(self, key_idx, sig, first, cnt, msg32, with_sig_bits=False):
        key_idx = np.ascontiguousarray(key_idx, np.uint32)
        sig = _u8(sig).reshape(-1, 64)
        if len(key_idx) == 0:
            key_idx = np.zeros(1, np.uint32)
            sig = np.zeros((1, 64), np.uint8)
        first = np.ascontiguousarray(first, np.uint64)
        cnt = np.ascontiguousarray(cnt, np.uint32)
        msg32 = _u8(msg32).reshape(-1, 32)
        G = len(cnt)
        nsig = int((first + cnt).max()) if G else 0
        gb = np.zeros((G + 7) // 8 + 1, np.uint8)
        sb = np.zeros((nsig + 7) // 8 + 1, np.uint8)
        _check(self.be.lib.nt_ed25519_verify_batch_groups_keyset(
            self.be.ctx, self.h, _p(key_idx, _u32p), _p(sig), _p(first, _u64p), _p(cnt, _u32p), _p(msg32), G,
            _p(gb), _p(sb) if with_sig_bits else None), "nt_ed25519_verify_batch_groups_keyset")
        if with_sig_bits:
            return _unpack(gb, G), _unpack(sb, nsig)
        return _unpack(gb, G)

    def dev_verify_groups(self, dev, stream, mode, d_key_idx, d_sig, d_msg, msg_bytes, d_off, d_len, n, d_first,
                          d_cnt, G, d_out, d_group_out):
        """Key-cache verification + the AND per certificate group in one launch chain
        (nt_dev_ed25519_verify_keyset_groups): no verdict-pack / group-AND launch after it."""
        _check(self.be.lib.nt_dev_ed25519_verify_keyset_groups(self.be.ctx, self.h, dev, stream, mode, d_key_idx, d_sig,
                                                               d_msg, int(msg_bytes), d_off, d_len, n, d_first, d_cnt,
                                                               int(G), d_out, d_group_out),
               "nt_dev_ed25519_verify_keyset_groups")

    def dev_verify(self, dev, stream, mode, d_key_idx, d_sig, d_msg, msg_bytes, d_off, d_len, n, d_out):
        _check(self.be.lib.nt_dev_ed25519_verify_keyset(self.be.ctx, self.h, dev, stream, mode, d_key_idx, d_sig,
                                                        d_msg, int(msg_bytes), d_off, d_len, n, d_out),
               "nt_dev_ed25519_verify_keyset")


_default = None


def default_backend():
    """Process-wide backend over all visible devices (created on first use)."""
    global _default
    if _default is None:
        _default = Backend(0)
    return _default


class Committee:
    """A committee over a keyset (nt_committee_*): stake and worker ids per key,
    the quorum threshold; ingest() runs Certificate::verify on wire bytes on the
    device (nt_certificates_ingest).  It keeps the keyset's device tables alive:
    the Keyset may be closed first."""

    def __init__(self, keyset, stakes, workers, quorum):
        self.be = keyset.be
        stakes = np.ascontiguousarray(stakes, np.uint32)
        wfirst = np.zeros(len(workers) + 1, np.uint64)
        wfirst[1:] = np.cumsum([len(w) for w in workers])
        wids = np.ascontiguousarray(np.concatenate([np.asarray(w, np.uint32) for w in workers] + [np.zeros(1, np.uint32)]),
                                    np.uint32)
        h = _vp()
        _check(self.be.lib.nt_committee_create(self.be.ctx, keyset.h, _p(stakes, _u32p), _p(wfirst, _u64p),
                                               _p(wids, _u32p), int(quorum), ctypes.byref(h)), "nt_committee_create")
        self.h = h

    def ingest(self, messages, gc_round=0):
        """primary::DagError code per wire message (NT_DAG_HOST = 0xff: left to the host decoder)."""
        n = len(messages)
        ln = np.array([len(m) for m in messages], np.uint64)
        off = np.zeros(n, np.uint64)
        if n > 1:
            off[1:] = np.cumsum(ln)[:-1]
        data = np.frombuffer(b"".join(messages), np.uint8) if n else np.zeros(1, np.uint8)
        data = data if len(data) else np.zeros(1, np.uint8)
        out = np.zeros(max(n, 1), np.uint8)
        _check(self.be.lib.nt_certificates_ingest(self.be.ctx, self.h, _p(data), _p(off, _u64p), _p(ln, _u64p), n,
                                                  int(gc_round), _p(out)), "nt_certificates_ingest")
        return out[:n]

    def close(self):
        if getattr(self, "h", None):
            self.be.lib.nt_committee_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
