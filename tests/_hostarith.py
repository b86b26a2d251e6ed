"""ctypes binding of tests/cpp/build/libnthost.so -- the device arithmetic compiled
for the host (TEST INFRASTRUCTURE; see tests/cpp/nt_host_harness.cpp)."""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
LIB = os.path.join(CPP, "build", "libnthost.so")
SH = [26, 25] * 5
W = [sum(SH[:i]) for i in range(10)]
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493

_lib = None


def load():
    global _lib
    if _lib is None:
        subprocess.run(["make", "-s", "-C", CPP], check=True)
        _lib = ctypes.CDLL(LIB)
        _lib.nth_verify.restype = ctypes.c_int
        _lib.nth_verify_trivial.restype = ctypes.c_int
        _lib.nth_sc_halfsize.restype = ctypes.c_int
        _lib.nth_wcomb_chunk.restype = ctypes.c_uint32
        _lib.nth_count_mul.restype = ctypes.c_ulonglong
        _lib.nth_count_sq.restype = ctypes.c_ulonglong
        _lib.nth_key_comb_sum.restype = ctypes.c_uint32
    return _lib


def bcomb_bits():
    """digit width of the comb of B the harness (and the product build) uses"""
    return int(load().nth_bcomb_bits())


def arr(limbs):
    return (ctypes.c_uint32 * 10)(*limbs)


def value(limbs):
    return sum(int(l) << w for l, w in zip(limbs, W))


def to_limbs(x):
    out = []
    for s in SH:
        out.append(x & ((1 << s) - 1))
        x >>= s
    return out


def fe_mul(f, g):
    o = (ctypes.c_uint32 * 10)()
    load().nth_fe_mul(arr(f), arr(g), o)
    return list(o)


def fe_sq(f):
    o = (ctypes.c_uint32 * 10)()
    load().nth_fe_sq(arr(f), o)
    return list(o)


def fe_sq_wide(f):
    o = (ctypes.c_uint32 * 10)()
    load().nth_fe_sq_wide(arr(f), o)
    return list(o)


def fe_tobytes(f):
    o = ctypes.create_string_buffer(32)
    load().nth_fe_tobytes(arr(f), o)
    return o.raw


def verify(mode, pk, sig, msg):
    return bool(load().nth_verify(mode, pk, sig, msg, ctypes.c_uint64(len(msg))))


def verify_pair(mode, pk0, sig0, msg0, pk1, sig1, msg1, cached=False):
    """Two signatures through the two-per-lane kernel path (shared inversion);
    cached=True: the committee key-cache path (wide combs of -A)."""
    out = (ctypes.c_int * 2)()
    fn = load().nth_verify_cached_pair if cached else load().nth_verify_pair
    fn(mode, pk0 + pk1, sig0 + sig1, msg0, ctypes.c_uint64(len(msg0)), msg1, ctypes.c_uint64(len(msg1)), out)
    return bool(out[0]), bool(out[1])


def verify_trivial(mode, pk, sig, msg):
    """verify through the trivial lattice vector (k, 1): the 253-bit fallback ladder"""
    return bool(load().nth_verify_trivial(mode, pk, sig, msg, ctypes.c_uint64(len(msg))))


def verify_cached_n(mode, entries, strict_mask=0, bits=20):
    """1..8 (pk, sig, msg) through the key-cache kernel's path: n signatures per
    lane, one inversion (verify_cached_batch, run-time count n).  mode 2 = mixed:
    entry j is checked strictly iff bit j of strict_mask (the kernel's key_idx
    bit 31).  bits: key-comb digit width (20: 13 positions; 21: reduced scalars,
    12 positions)."""
    n = len(entries)
    assert 1 <= n <= 8
    if mode == 2:
        mode = 2 | (strict_mask << 8)
    out = (ctypes.c_int * n)()
    msgs = [e[2] for e in entries]
    mp = (ctypes.c_char_p * n)(*msgs)
    lens = (ctypes.c_uint64 * n)(*[len(m) for m in msgs])
    rc = load().nth_verify_cached_nw(bits, mode, n, b"".join(e[0] for e in entries), b"".join(e[1] for e in entries),
                                     mp, lens, out)
    assert rc == 0
    return tuple(bool(x) for x in out)


KEY_TORSION = 4  # kKeyTorsion (ed25519_ops.hpp)


def key_comb_sum(bits, A: bytes, k: int):
    """[k](-A) as the key-cache kernel forms it from the key's comb of `bits`-bit
    digits (21: k reduced to k or k - L, plus the key's [L](-A) entry when k - L
    was used); returns (encoding, kKey* bits of the key)"""
    out = ctypes.create_string_buffer(32)
    meta = load().nth_key_comb_sum(bits, A, k.to_bytes(32, "little"), out)
    return out.raw, int(meta)


def verify_cached4(mode, entries, strict_mask=0):
    """Four entries (the round-1 kernel's per-lane count)."""
    assert len(entries) == 4
    return verify_cached_n(mode, entries, strict_mask)


def sc_halfsize(k: int):
    """(u, v, bits) from the device lattice reduction for k < 2^256 (u signed)"""
    u = ctypes.create_string_buffer(32)
    v = ctypes.create_string_buffer(32)
    neg = ctypes.c_int(0)
    bits = load().nth_sc_halfsize(k.to_bytes(32, "little"), u, v, ctypes.byref(neg))
    uu = int.from_bytes(u.raw, "little")
    return (-uu if neg.value else uu), int.from_bytes(v.raw, "little"), bits


def halfsize_disagree(ks):
    """number of scalars (ints < 2^256) whose batched (Lehmer) and one-step
    lattice reductions differ in (u, v, sign, bits)"""
    buf = b"".join(k.to_bytes(32, "little") for k in ks)
    return int(load().nth_halfsize_disagree(buf, len(ks)))


def small_order(enc):
    """(decodes, [8]P == 0 by doublings, torsion-y compare) for a 32-byte encoding"""
    a, b = ctypes.c_int(0), ctypes.c_int(0)
    ok = load().nth_small_order(enc, ctypes.byref(a), ctypes.byref(b))
    return bool(ok), bool(a.value), bool(b.value)


def wcomb_chunk(bits, enc, negate, pos, c):
    """Device wide-comb construction on the host: (meta, 65 x 32 words) for
    entries 64c .. 64c+64 of position pos of the `bits`-bit comb (entry 64c only
    filled when c == 0)."""
    import numpy as np
    out = (ctypes.c_uint32 * (65 * 32))()
    meta = load().nth_wcomb_chunk(bits, enc, negate, pos, c, out)
    return meta, np.frombuffer(bytes(out), np.uint32).reshape(65, 32)


def sign(seed, msg):
    pk = ctypes.create_string_buffer(32)
    sig = ctypes.create_string_buffer(64)
    load().nth_sign(seed, msg, ctypes.c_uint64(len(msg)), pk, sig)
    return pk.raw, sig.raw


def sc_reduce512(b):
    o = ctypes.create_string_buffer(32)
    load().nth_sc_reduce512(b, o)
    return o.raw


def sha512(m, one_site=False):
    o = ctypes.create_string_buffer(64)
    load().nth_sha512(m, ctypes.c_uint64(len(m)), o, int(one_site))
    return o.raw


def hram(sig, pk, msg, fast):
    o = ctypes.create_string_buffer(32)
    load().nth_hram(sig, pk, msg, ctypes.c_uint64(len(msg)), int(fast), o)
    return o.raw


def counts_reset():
    load().nth_counts_reset()


def counts():
    return int(load().nth_count_mul()), int(load().nth_count_sq())
