#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Everything here is computed WITHOUT the repo's own oracle (oracle/) or the
product library, so that the fixtures pin both of them:

  * SHA-512 .............. Python hashlib
  * keys() fixture ....... pure-Python ChaCha20 (rand 0.7 StdRng = rand_chacha
                           ChaCha20Rng layout) -> crypto_tests.rs:26-29
  * keygen / signing ..... libsodium 1.0.18 (crypto_sign_seed_keypair /
                           crypto_sign_detached), deterministic RFC 8032 like
                           dalek Keypair::sign (crypto/src/lib.rs:185-191)
  * verify_strict verdict  libsodium crypto_sign_verify_detached AND a
                           pure-Python textbook model of the dalek rules
                           (SURVEY.md Appendix A.2); the generator asserts they
                           agree on every entry (Appendix A.4)
  * verify_batch rule .... the pure-Python model of Appendix A.3 plus the
                           dalek-determinism class of each entry

The reference (Rust, ed25519-dalek 1.0.1) cannot be built here (no cargo, no
crate sources), so these independent implementations are the pin.
Run in the development container (needs /opt/conda/lib/libsodium.so.23):
    python tests/golden/make_golden.py
Outputs: sha512_vectors.json, fixtures_reference.json, ed25519_corpus.npz,
         ed25519_corpus.json, batch_groups.npz
"""
import ctypes
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SODIUM = "/opt/conda/lib/libsodium.so.23"

# --------------------------------------------------------------------------
# Deterministic byte expansion used for synthetic messages (test-reproducible)
# --------------------------------------------------------------------------


def expand(label: bytes, n: int) -> bytes:
    out = bytearray()
    i = 0
    while len(out) < n:
        out += hashlib.sha512(label + struct.pack("<Q", i)).digest()
        i += 1
    return bytes(out[:n])


# --------------------------------------------------------------------------
# ChaCha20 keystream, rand_chacha 0.2 layout (64-bit counter words 12..13,
# 64-bit stream id words 14..15)
# --------------------------------------------------------------------------


def chacha20_keystream(key: bytes, n: int, stream: int = 0, counter: int = 0) -> bytes:
    def rotl(v, c):
        return ((v << c) & 0xFFFFFFFF) | (v >> (32 - c))

    def qr(x, a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF; x[d] = rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF; x[b] = rotl(x[b] ^ x[c], 7)

    kw = list(struct.unpack("<8I", key))
    out = bytearray()
    while len(out) < n:
        st = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + kw + [
            counter & 0xFFFFFFFF, counter >> 32, stream & 0xFFFFFFFF, stream >> 32]
        x = list(st)
        for _ in range(10):
            qr(x, 0, 4, 8, 12); qr(x, 1, 5, 9, 13); qr(x, 2, 6, 10, 14); qr(x, 3, 7, 11, 15)
            qr(x, 0, 5, 10, 15); qr(x, 1, 6, 11, 12); qr(x, 2, 7, 8, 13); qr(x, 3, 4, 9, 14)
        out += struct.pack("<16I", *[(a + b) & 0xFFFFFFFF for a, b in zip(x, st)])
        counter += 1
    return bytes(out[:n])


# --------------------------------------------------------------------------
# Pure-Python textbook Edwards25519 model of the dalek rules
# --------------------------------------------------------------------------
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)
IDENT = (0, 1, 1, 0)


def inv(x):
    return pow(x, P - 2, P)


def padd(p, q):
    X1, Y1, Z1, T1 = p
    X2, Y2, Z2, T2 = q
    A = (Y1 - X1) * (Y2 - X2) % P
    B = (Y1 + X1) * (Y2 + X2) % P
    C = T1 * 2 * D * T2 % P
    DD = Z1 * 2 * Z2 % P
    E, F, G, H = B - A, DD - C, DD + C, B + A
    return (E * F % P, G * H % P, F * G % P, E * H % P)


def pneg(p):
    X, Y, Z, T = p
    return ((-X) % P, Y, Z, (-T) % P)


def pmul(s, p):
    q = IDENT
    while s > 0:
        if s & 1:
            q = padd(q, p)
        p = padd(p, p)
        s >>= 1
    return q


def peq(p, q):
    return (p[0] * q[2] - q[0] * p[2]) % P == 0 and (p[1] * q[2] - q[1] * p[2]) % P == 0


def is_ident(p):
    return peq(p, IDENT)


def decode(b: bytes):
    """curve25519-dalek CompressedEdwardsY::decompress semantics."""
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)  # NOT rejected when >= p
    sign = b[31] >> 7
    y %= P
    u = (y * y - 1) % P
    v = (D * y * y + 1) % P
    x2 = u * inv(v) % P
    x = pow(x2, (P + 3) // 8, P)
    if (x * x - x2) % P:
        x = x * SQRTM1 % P
    if (x * x - x2) % P:
        return None
    if x & 1:
        x = P - x
    if sign:
        x = (P - x) % P  # x = 0 with the sign bit set stays 0 (accepted)
    return (x, y, 1, x * y % P)


def encode(p) -> bytes:
    X, Y, Z, _ = p
    zi = inv(Z)
    x, y = X * zi % P, Y * zi % P
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


BASE = decode((4 * inv(5) % P).to_bytes(32, "little"))


def is_small(p):
    return is_ident(pmul(8, p))


def has_torsion(p):
    return not is_ident(pmul(L, p))


def hram(R: bytes, A: bytes, m: bytes) -> int:
    return int.from_bytes(hashlib.sha512(R + A + m).digest(), "little") % L


def residual(pk, sig, msg):
    """D = R + [k]A - [s]B, or None on a decode failure / s >= L."""
    s = int.from_bytes(sig[32:], "little")
    if s >= L:
        return None
    A, R = decode(pk), decode(sig[:32])
    if A is None or R is None:
        return None
    k = hram(sig[:32], pk, msg)
    return padd(padd(R, pmul(k, A)), pneg(pmul(s, BASE))), A, R


def model_strict(pk, sig, msg) -> bool:
    r = residual(pk, sig, msg)
    if r is None:
        return False
    Dp, A, R = r
    if is_small(A) or is_small(R):
        return False
    return is_ident(Dp)


def model_batch_entry(pk, sig, msg):
    """(rule_accept, dalek_class): class 0 det. reject, 1 det. accept, 2 random."""
    r = residual(pk, sig, msg)
    if r is None:
        return False, 0
    Dp, A, _ = r
    if is_ident(Dp):
        return True, (2 if has_torsion(A) else 1)
    if not is_ident(pmul(8, Dp)):
        return False, 0  # residual has a prime-order part: dalek rejects w.p. ~1
    return False, 2


# torsion generator T8 (order 8)
def _find_t8():
    y = 2
    while True:
        p = decode(y.to_bytes(32, "little"))
        if p is not None:
            t = pmul(L, p)
            if not is_ident(pmul(4, t)):
                return t
        y += 1


T8 = _find_t8()
TORSION = [pmul(i, T8) for i in range(8)]

# --------------------------------------------------------------------------
# libsodium (independent verdicts and signing)
# --------------------------------------------------------------------------
_so = ctypes.CDLL(SODIUM)
assert _so.sodium_init() >= 0


def sodium_keypair(seed: bytes):
    pk = ctypes.create_string_buffer(32)
    sk = ctypes.create_string_buffer(64)
    assert _so.crypto_sign_ed25519_seed_keypair(pk, sk, seed) == 0
    return pk.raw, sk.raw


def sodium_sign(sk: bytes, msg: bytes) -> bytes:
    sig = ctypes.create_string_buffer(64)
    assert _so.crypto_sign_ed25519_detached(sig, None, msg, ctypes.c_ulonglong(len(msg)), sk) == 0
    return sig.raw


def sodium_verify(pk: bytes, sig: bytes, msg: bytes) -> bool:
    return _so.crypto_sign_ed25519_verify_detached(sig, msg, ctypes.c_ulonglong(len(msg)), pk) == 0


# --------------------------------------------------------------------------
# 1) SHA-512 vectors
# --------------------------------------------------------------------------


def sha_vectors():
    lens = [0, 1, 3, 55, 56, 63, 64, 100, 111, 112, 113, 119, 120, 127, 128, 129, 200, 239, 240,
            255, 256, 257, 1000, 4096, 10007]
    vecs = []
    for n in lens:
        m = expand(b"nt-sha-%d" % n, n)
        vecs.append({"label": "nt-sha-%d" % n, "len": n,
                     "digest512": hashlib.sha512(m).hexdigest()})
    # the reference's own fixtures
    ser = struct.pack("<I", 0) + struct.pack("<Q", 2) + (struct.pack("<Q", 100) + bytes(100)) * 2
    hello = b"Hello, world!"
    # a real sealed batch: 977 x 512-B txs, bincode WorkerMessage::Batch
    txs = [expand(b"nt-tx-%d" % i, 512) for i in range(977)]
    real = struct.pack("<I", 0) + struct.pack("<Q", len(txs)) + b"".join(
        struct.pack("<Q", len(t)) + t for t in txs)
    assert len(real) == 508052
    ref = {
        "processor_batch_228B": {
            "hex": ser.hex(), "digest32": hashlib.sha512(ser).hexdigest()[:64],
            "cite": "worker/src/tests/common.rs:86-110, worker/src/tests/processor_tests.rs:9-46"},
        "hello_world": {
            "hex": hello.hex(), "digest32": hashlib.sha512(hello).hexdigest()[:64],
            "cite": "crypto/src/tests/crypto_tests.rs:54-55"},
        "real_batch_977x512": {
            "tx_label": "nt-tx-%d", "ntx": 977, "tx_len": 512, "len": len(real),
            "digest32": hashlib.sha512(real).hexdigest()[:64],
            "cite": "SURVEY.md §8(a) a2: bincode WorkerMessage::Batch sealed at >= 500,000 B"},
        "buffer_500000": {
            "label": "nt-500k", "len": 500000,
            "digest32": hashlib.sha512(expand(b"nt-500k", 500000)).hexdigest()[:64]},
    }
    return {"expand": "sha512(label || u64le(i)) blocks, truncated", "vectors": vecs,
            "reference_fixtures": ref}


# --------------------------------------------------------------------------
# 2) reference fixtures: keys(), signatures, Narwhal header/vote/certificate
# --------------------------------------------------------------------------


def digest32(b: bytes) -> bytes:
    return hashlib.sha512(b).digest()[:32]


def reference_fixtures():
    ks = chacha20_keystream(bytes(32), 128)
    keys = []
    for i in range(4):
        seed = ks[32 * i: 32 * i + 32]
        pk, sk = sodium_keypair(seed)
        keys.append({"seed": seed.hex(), "pk": pk.hex()})
    hello_d = digest32(b"Hello, world!")
    bad_d = digest32(b"Bad message!")
    sigs = [sodium_sign(bytes.fromhex(k["seed"]) + bytes.fromhex(k["pk"]), hello_d).hex() for k in keys]

    # Narwhal fixtures (primary/src/tests/common.rs:96-166), committee of the 4 keys, stake 1
    pks = sorted(bytes.fromhex(k["pk"]) for k in keys)  # BTreeMap<PublicKey, _> order
    genesis = [digest32(bytes(32) + struct.pack("<Q", 0) + pk) for pk in pks]
    parents = sorted(genesis)  # BTreeSet<Digest>

    def make_header(k):
        author = bytes.fromhex(k["pk"])
        hid = digest32(author + struct.pack("<Q", 1) + b"".join(parents))
        sk = bytes.fromhex(k["seed"]) + author
        return {"author": author.hex(), "round": 1, "payload": [], "parents": [p.hex() for p in parents],
                "id": hid.hex(), "signature": sodium_sign(sk, hid).hex()}

    headers = [make_header(k) for k in keys]
    header = headers[3]  # keys().pop()

    def make_votes(h):
        out = []
        for k in keys:
            d = digest32(bytes.fromhex(h["id"]) + struct.pack("<Q", h["round"]) + bytes.fromhex(h["author"]))
            sk = bytes.fromhex(k["seed"]) + bytes.fromhex(k["pk"])
            out.append({"author": k["pk"], "digest": d.hex(), "signature": sodium_sign(sk, d).hex()})
        return out

    certs = []
    for h in headers[:3]:
        v = make_votes(h)
        cd = digest32(bytes.fromhex(h["id"]) + struct.pack("<Q", h["round"]) + bytes.fromhex(h["author"]))
        certs.append({"header": h, "votes": [[x["author"], x["signature"]] for x in v], "digest": cd.hex()})
    return {
        "keys": keys, "keys_cite": "crypto/src/tests/crypto_tests.rs:26-29 (StdRng::from_seed([0;32]))",
        "hello_digest": hello_d.hex(), "bad_digest": bad_d.hex(), "hello_signatures": sigs,
        "genesis_digests": [g.hex() for g in genesis],
        "header": header, "headers": headers, "votes": make_votes(header), "certificates": certs,
        "narwhal_cite": "primary/src/tests/common.rs:96-166; primary/src/messages.rs:70-84,145-153,226-234",
    }


# --------------------------------------------------------------------------
# 3) Ed25519 edge-case corpus
# --------------------------------------------------------------------------
CATEGORIES = [
    "honest", "wrong_msg_bitflip", "s_plus_L", "s_bit255", "s_L_minus_1_randR", "R_not_on_curve",
    "A_not_on_curve", "small_order_R", "small_order_A", "mixed_A_valid", "mixed_R_torsion_off",
    "small_A_R_exact", "noncanonical_y", "all_zero_sig", "garbage",
]


class Gen:
    def __init__(self, label):
        self.label = label
        self.ctr = 0

    def bytes(self, n):
        self.ctr += 1
        return expand(self.label + b"/%d" % self.ctr, n)

    def scalar(self):
        return int.from_bytes(self.bytes(64), "little") % L


def noncanonical_encodings():
    """All encodings y in [p, 2^255) (y+p for y in 0..18), both signs, that decode;
    plus negative-zero encodings of x = 0 points."""
    out = []
    for y in range(19):
        for sign in (0, 1):
            e = bytearray((y + P).to_bytes(32, "little"))
            e[31] |= sign << 7
            if decode(bytes(e)) is not None:
                out.append(bytes(e))
    for y in (1, P - 1):
        e = bytearray(y.to_bytes(32, "little"))
        e[31] |= 0x80
        out.append(bytes(e))
    return out


def small_order_encodings():
    encs = [encode(t) for t in TORSION]
    for e in noncanonical_encodings():
        if is_small(decode(e)) and e not in encs:
            encs.append(e)
    return encs


def build_corpus(per_cat=24, seed=b"nt-corpus"):
    g = Gen(seed)
    small = small_order_encodings()
    nonc = noncanonical_encodings()
    entries = []  # (cat, pk, sig, msg)

    def keypair():
        seed_ = g.bytes(32)
        pk, sk = sodium_keypair(seed_)
        return seed_, pk, sk

    def msg_len(i):
        # mostly 512-B (config 2) and 32-B digests (what Narwhal signs), some odd lengths
        return [512, 32, 512, 0, 512, 111, 512, 32, 512, 200, 512, 1][i % 12]

    def not_on_curve():
        while True:
            b = g.bytes(32)
            if decode(b) is None:
                return b

    for ci, cat in enumerate(CATEGORIES):
        i = 0
        tries = 0
        while i < per_cat:
            tries += 1
            m = g.bytes(msg_len(i))
            seed_, pk, sk = keypair()
            sig = sodium_sign(sk, m)
            if cat == "honest":
                pass
            elif cat == "wrong_msg_bitflip":
                if len(m) == 0:
                    m = b"\x01"
                else:
                    mm = bytearray(m); mm[i % len(mm)] ^= 1 << (i % 8); m = bytes(mm)
            elif cat == "s_plus_L":
                s = int.from_bytes(sig[32:], "little") + L
                sig = sig[:32] + s.to_bytes(32, "little")
            elif cat == "s_bit255":
                sig = sig[:63] + bytes([sig[63] | 0x80])
            elif cat == "s_L_minus_1_randR":
                R = encode(pmul(g.scalar(), BASE))
                sig = R + (L - 1).to_bytes(32, "little")
            elif cat == "R_not_on_curve":
                sig = not_on_curve() + sig[32:]
            elif cat == "A_not_on_curve":
                pk = not_on_curve()
            elif cat == "small_order_R":
                R = small[i % len(small)]
                sig = R + sig[32:] if i % 3 else R + (g.scalar()).to_bytes(32, "little")
            elif cat == "small_order_A":
                pk = small[i % len(small)]
                if i % 2:
                    # exact equation with the small-order A: R = [s]B - [k]A
                    r = g.scalar()
                    # choose R = [r]B + T_j so that R == [r]B - [k]A holds exactly
                    done = False
                    for j in range(8):
                        Rj = encode(padd(pmul(r, BASE), TORSION[j]))
                        kj = hram(Rj, pk, m)
                        if peq(padd(pmul(r, BASE), pneg(pmul(kj, decode(pk)))), decode(Rj)):
                            sig = Rj + r.to_bytes(32, "little")
                            done = True
                            break
                    if not done:
                        continue
            elif cat == "mixed_A_valid":
                a = g.scalar()
                t = 1 + (i % 7)
                Apt = padd(pmul(a, BASE), TORSION[t])
                pk = encode(Apt)
                r = g.scalar()
                found = False
                for j in range(8):
                    Rj = encode(padd(pmul(r, BASE), TORSION[j]))
                    k = hram(Rj, pk, m)
                    s = (r + k * a) % L
                    cand = Rj + s.to_bytes(32, "little")
                    if model_strict(pk, cand, m):
                        sig = cand
                        found = True
                        break
                if not found:
                    continue
            elif cat == "mixed_R_torsion_off":
                a_h = hashlib.sha512(seed_).digest()
                a = int.from_bytes(a_h[:32], "little")
                a &= (1 << 254) - 8
                a |= 1 << 254
                r = g.scalar()
                T = TORSION[1 + (i % 7)]
                R = encode(padd(pmul(r, BASE), T))
                k = hram(R, pk, m)
                s = (r + k * a) % L
                sig = R + s.to_bytes(32, "little")
            elif cat == "small_A_R_exact":
                ia = 1 + (i % 7)
                pk = encode(TORSION[ia])
                found = False
                for j in range(8):
                    Rj = encode(TORSION[j])
                    k = hram(Rj, pk, m)
                    # need R + kA = 0 (s = 0): j + k*ia = 0 mod 8
                    if (j + k * ia) % 8 == 0:
                        sig = Rj + bytes(32)
                        found = True
                        break
                if not found:
                    continue
            elif cat == "noncanonical_y":
                e = nonc[i % len(nonc)]
                if i % 2:
                    sig = e + sig[32:]
                else:
                    pk = e
            elif cat == "all_zero_sig":
                sig = bytes(64)
            elif cat == "garbage":
                sig = g.bytes(64)
                if i % 2:  # canonical s so the point checks are exercised
                    sig = sig[:32] + (int.from_bytes(sig[32:], "little") % L).to_bytes(32, "little")
            entries.append((ci, pk, sig, m))
            i += 1
    return entries


def corpus_arrays(entries, check_libsodium=True):
    n = len(entries)
    pk = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    off = np.zeros(n, np.uint64)
    ln = np.zeros(n, np.uint64)
    cat = np.zeros(n, np.int32)
    strict = np.zeros(n, np.uint8)
    sodium = np.zeros(n, np.uint8)
    brule = np.zeros(n, np.uint8)
    bclass = np.zeros(n, np.uint8)
    blob = bytearray()
    for i, (ci, p, s, m) in enumerate(entries):
        pk[i] = np.frombuffer(p, np.uint8)
        sig[i] = np.frombuffer(s, np.uint8)
        off[i] = len(blob)
        ln[i] = len(m)
        blob += m
        cat[i] = ci
        strict[i] = model_strict(p, s, m)
        sodium[i] = sodium_verify(p, s, m)
        acc, cls = model_batch_entry(p, s, m)
        brule[i] = acc
        bclass[i] = cls
        if check_libsodium and strict[i] != sodium[i]:
            raise SystemExit("libsodium / dalek-model disagreement on entry %d (%s)" % (i, CATEGORIES[ci]))
    return dict(pk=pk, sig=sig, msg=np.frombuffer(bytes(blob), np.uint8).copy(), off=off, len=ln,
                cat=cat, strict=strict, sodium=sodium, batch_rule=brule, batch_class=bclass)


# --------------------------------------------------------------------------
# 4) verify_batch groups (certificates): n=100-like committee subset, 32-B digest
# --------------------------------------------------------------------------


def build_groups(corpus_entries):
    g = Gen(b"nt-groups")
    committee = []
    for i in range(16):
        seed_ = hashlib.sha512(b"nt-bench-key" + struct.pack("<Q", i)).digest()[:32]
        pk, sk = sodium_keypair(seed_)
        committee.append((pk, sk))
    # bad entries taken from the corpus, but re-targeted at each group's digest
    pk_l, sig_l, first, cnt, msgs, expect, det = [], [], [], [], [], [], []
    sizes = [0, 1, 3, 4, 7, 16, 5, 2, 67]
    gi = 0
    for rep in range(6):
        for m in sizes:
            digest = g.bytes(32)
            first.append(len(pk_l))
            cnt.append(m)
            msgs.append(digest)
            members = [(j * 7 + gi) % 16 for j in range(m)] if m <= 16 else [j % 16 for j in range(m)]
            rows = []
            for j in members:
                pk, sk = committee[j]
                rows.append([pk, sodium_sign(sk, digest)])
            kind = (gi % 5)
            if m and kind in (1, 2, 3):
                victim = gi % m
                if kind == 1:      # corrupted s
                    s = rows[victim][1]
                    rows[victim][1] = s[:40] + bytes([s[40] ^ 4]) + s[41:]
                elif kind == 2:    # all-zero signature (crypto_tests.rs:96-115)
                    rows[victim][1] = bytes(64)
                elif kind == 3:    # R = [r]B + T2 signed consistently: pure-torsion residual
                    pk, sk = committee[members[victim]]
                    a = int.from_bytes(hashlib.sha512(sk[:32]).digest()[:32], "little")
                    a = (a & ((1 << 254) - 8)) | (1 << 254)
                    r = g.scalar()
                    R = encode(padd(pmul(r, BASE), TORSION[4]))
                    s = (r + hram(R, pk, digest) * a) % L
                    rows[victim][1] = R + s.to_bytes(32, "little")
            grp_ok, grp_det = True, True
            for pk, s in rows:
                acc, cls = model_batch_entry(pk, s, digest)
                grp_ok &= acc
                grp_det &= cls != 2
                pk_l.append(pk)
                sig_l.append(s)
            expect.append(grp_ok)
            det.append(grp_det)
            gi += 1
    n = len(pk_l)
    return dict(pk=np.frombuffer(b"".join(pk_l), np.uint8).reshape(n, 32).copy() if n else np.zeros((0, 32), np.uint8),
                sig=np.frombuffer(b"".join(sig_l), np.uint8).reshape(n, 64).copy(),
                first=np.array(first, np.uint64), cnt=np.array(cnt, np.uint32),
                msg32=np.frombuffer(b"".join(msgs), np.uint8).reshape(-1, 32).copy(),
                expect=np.array(expect, np.uint8), deterministic=np.array(det, np.uint8))


def main():
    assert encode(BASE).hex() == "58" + "66" * 31, "base point encoding"
    with open(os.path.join(HERE, "sha512_vectors.json"), "w") as f:
        json.dump(sha_vectors(), f, indent=1)
    print("sha512_vectors.json")
    with open(os.path.join(HERE, "fixtures_reference.json"), "w") as f:
        json.dump(reference_fixtures(), f, indent=1)
    print("fixtures_reference.json")
    per_cat = int(os.environ.get("NT_CORPUS_PER_CAT", "24"))
    entries = build_corpus(per_cat)
    arr = corpus_arrays(entries)
    np.savez_compressed(os.path.join(HERE, "ed25519_corpus.npz"), **arr)
    meta = {"categories": CATEGORIES, "per_category": per_cat, "n": len(entries),
            "torsion_encodings": [encode(t).hex() for t in TORSION],
            "small_order_encodings": [e.hex() for e in small_order_encodings()],
            "noncanonical_encodings": [e.hex() for e in noncanonical_encodings()],
            "fields": {"strict": "dalek verify_strict (textbook model == libsodium, asserted)",
                       "sodium": "libsodium 1.0.18 crypto_sign_verify_detached",
                       "batch_rule": "SURVEY A.3 deterministic rule (cofactorless equation)",
                       "batch_class": "0 dalek batch rejects w.p.~1, 1 accepts always, 2 dalek random"}}
    with open(os.path.join(HERE, "ed25519_corpus.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("ed25519_corpus.npz: %d entries" % len(entries))
    grp = build_groups(entries)
    np.savez_compressed(os.path.join(HERE, "batch_groups.npz"), **grp)
    print("batch_groups.npz: %d groups, %d signatures" % (len(grp["cnt"]), len(grp["pk"])))


if __name__ == "__main__":
    sys.exit(main())
