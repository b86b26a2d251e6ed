"""CPU tests of the exact device arithmetic (narwhal-tusk_amd/csrc/*.hpp compiled
for the host by tests/cpp/).  These stress the radix-2^25.5 bound discipline at
the extreme limb values the point formulas can produce (a silent u64 overflow
would only show on adversarial limbs, never on random signatures), and replay
the golden corpus through the same verify_n<> / verify_cached_n<> / sign_one the
kernels run, and check the wide-comb construction against a textbook curve model.
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

import _hostarith as H

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
M26, M25 = (1 << 26) - 1, (1 << 25) - 1

# largest limbs the formulas in ge25519.hpp can feed into mul/sq (see fe25519.hpp header)
F_MAX = [0xFFFFFB4 + 0x8000000 if i == 0 else (0xFFFFFFC + 0x8000000 if i % 2 == 0 else 0x7FFFFFC + 0x4000000)
         for i in range(10)]                                   # fe_sub4 of (2x reduced) -> f side only
G_MAX = [0x7FFFFDA + 0x4000000 if i == 0 else (0x7FFFFFE + 0x4000000 if i % 2 == 0 else 0x3FFFFFE + 0x2000000 + (1 << 18))
         for i in range(10)]                                   # fe_sub of reduced -> either side
S_MAX = [2 * M26 if i % 2 == 0 else 2 * M25 + (1 << 18) for i in range(10)]  # sum of two reduced -> sq_wide input
# fe_sq contract: even limbs < 2^26.1, odd < 2^25.1 (reduced outputs, d y^2 + 1)
R_MAX = [int(2 ** 26.1) - 1 if i % 2 == 0 else int(2 ** 25.1) - 1 for i in range(10)]


def _is_reduced(limbs):
    return all(l <= (M26 if i % 2 == 0 else M25 + (1 << 19)) for i, l in enumerate(limbs))


def _rand_limbs(rng, mx):
    return [rng.randint(0, m) for m in mx]


def test_fe_mul_extreme_bounds():
    rng = random.Random(1)
    cases = [(F_MAX, G_MAX), (F_MAX, F_MAX[:0] + [min(a, b) for a, b in zip(G_MAX, G_MAX)])]
    for _ in range(3000):
        cases.append((_rand_limbs(rng, F_MAX), _rand_limbs(rng, G_MAX)))
    for k in range(10):  # single-limb maxima
        f = [0] * 10
        f[k] = F_MAX[k]
        cases.append((f, G_MAX))
    for f, g in cases:
        out = H.fe_mul(f, g)
        assert H.value(out) % H.P == H.value(f) * H.value(g) % H.P
        assert _is_reduced(out), out


def test_fe_sq_extreme_bounds():
    rng = random.Random(2)
    for sq, mx in ((H.fe_sq, R_MAX), (H.fe_sq_wide, S_MAX)):
        cases = [mx] + [_rand_limbs(rng, mx) for _ in range(3000)]
        for k in range(10):  # single-limb maxima
            f = [0] * 10
            f[k] = mx[k]
            cases.append(f)
        for f in cases:
            out = sq(f)
            assert H.value(out) % H.P == H.value(f) ** 2 % H.P
            assert _is_reduced(out)


def test_fe_tobytes_canonical():
    vals = [0, 1, H.P - 1, H.P, H.P + 1, H.P + 18, 2 ** 255 - 1, 2 ** 255 - 20, 19, 2 ** 254]
    rng = random.Random(3)
    vals += [rng.randrange(0, 2 ** 255) for _ in range(500)]
    for v in vals:
        limbs = H.to_limbs(v)
        assert H.fe_tobytes(limbs) == (v % H.P).to_bytes(32, "little")
    # unreduced limb patterns (carry input) also canonicalize
    for _ in range(500):
        limbs = _rand_limbs(rng, G_MAX)
        assert H.fe_tobytes(limbs) == (H.value(limbs) % H.P).to_bytes(32, "little")


def test_sc_reduce512():
    rng = random.Random(4)
    for _ in range(2000):
        x = rng.randrange(0, 2 ** 512)
        assert H.sc_reduce512(x.to_bytes(64, "little")) == (x % H.L).to_bytes(32, "little")
    for x in (0, H.L - 1, H.L, H.L + 1, 2 ** 512 - 1, H.L * (2 ** 259)):
        x %= 2 ** 512
        assert H.sc_reduce512(x.to_bytes(64, "little")) == (x % H.L).to_bytes(32, "little")


def test_sha512_host_build():
    """both block loops: sha512_prefixed and the one-compression-site form the
    digest kernel uses (sha512_prefixed_1site), at every padding boundary"""
    for n in (0, 1, 111, 112, 113, 127, 128, 129, 239, 240, 255, 256, 1000, 3336, 5000):
        m = bytes(range(256)) * (n // 256 + 1)
        m = m[:n]
        assert H.sha512(m) == hashlib.sha512(m).digest()
        assert H.sha512(m, one_site=True) == hashlib.sha512(m).digest()


def test_hram_one_block_path_matches_hashlib():
    """hram_scalar<true> (the key-cache kernels: a 32-byte message hashed as one
    block built from registers) and the general path both equal
    SHA-512(R || A || M) mod L; other lengths fall through to the general path."""
    rng = random.Random(96)
    for n in (32, 32, 32, 0, 31, 33, 64):
        sig = bytes(rng.getrandbits(8) for _ in range(64))
        pk = bytes(rng.getrandbits(8) for _ in range(32))
        m = bytes(rng.getrandbits(8) for _ in range(n))
        want = (int.from_bytes(hashlib.sha512(sig[:32] + pk + m).digest(), "little") % H.L).to_bytes(32, "little")
        assert H.hram(sig, pk, m, True) == want, n
        assert H.hram(sig, pk, m, False) == want, n


def test_corpus_through_device_code():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    for i in range(len(d["cat"])):
        o, n = int(d["off"][i]), int(d["len"][i])
        pk, sig, m = d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + n].tobytes()
        assert H.verify(0, pk, sig, m) == bool(d["strict"][i]), i
        assert H.verify(1, pk, sig, m) == bool(d["batch_rule"][i]), i


def test_corpus_pairs_through_device_code():
    """The two-per-lane path (one shared inversion) the verify kernels run, and the
    key-cache path; each corpus entry is paired with its neighbour."""
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    n = len(d["cat"])

    def entry(i):
        o, ln = int(d["off"][i]), int(d["len"][i])
        return d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + ln].tobytes()

    for i in range(n):
        j = (i + 1) % n
        a, b = entry(i), entry(j)
        for mode, key in ((0, "strict"), (1, "batch_rule")):
            want = (bool(d[key][i]), bool(d[key][j]))
            assert H.verify_pair(mode, *a, *b) == want, (i, mode)
            if i % 3 == 0:
                assert H.verify_pair(mode, *a, *b, cached=True) == want, (i, mode, "cached")


def test_corpus_through_fallback_ladder():
    """The same verdicts through the trivial lattice vector (k, 1) -- the full
    253-bit ladder sc_halfsize falls back to (step cap / oversized vectors)."""
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    for i in range(0, len(d["cat"]), 2):
        o, n = int(d["off"][i]), int(d["len"][i])
        pk, sig, m = d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + n].tobytes()
        assert H.verify_trivial(0, pk, sig, m) == bool(d["strict"][i]), i
        assert H.verify_trivial(1, pk, sig, m) == bool(d["batch_rule"][i]), i


def test_corpus_through_keyset_path():
    """The key-cache kernel's batch of 8 signatures per lane (one inversion for
    all eight, R'_j staged): every corpus entry in a group of 8 with seven
    neighbours, plus groups of 3 (the count is a kernel argument)."""
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    n = len(d["cat"])

    def entry(i):
        o, ln = int(d["off"][i]), int(d["len"][i])
        return d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + ln].tobytes()

    for g, step in ((8, 8), (3, 37)):
        for i in range(0, n, step):
            idx = [(i + k) % n for k in range(g)]
            for mode, key in ((0, "strict"), (1, "batch_rule")):
                want = tuple(bool(d[key][j]) for j in idx)
                assert H.verify_cached_n(mode, [entry(j) for j in idx]) == want, (i, mode)
            # mixed mode (one launch for header + vote signatures): per-entry strictness
            mask = (i * 37 // step) % (1 << g)
            want = tuple(bool(d["strict" if (mask >> k) & 1 else "batch_rule"][j]) for k, j in enumerate(idx))
            assert H.verify_cached_n(2, [entry(j) for j in idx], strict_mask=mask) == want, (i, "mixed", mask)


@pytest.mark.parametrize("bits", [21])
def test_corpus_through_reduced_key_combs(bits):
    """The same corpus through 21-bit key combs (the device's first choice): k
    taken as k or k - L, 12 positions, and the key's [L](-A) entry added when
    k - L was used -- small-order and mixed-order keys included, every mode."""
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    n = len(d["cat"])

    def entry(i):
        o, ln = int(d["off"][i]), int(d["len"][i])
        return d["pk"][i].tobytes(), d["sig"][i].tobytes(), d["msg"][o:o + ln].tobytes()

    for i in range(0, n, 8):
        idx = [(i + k) % n for k in range(8)]
        for mode, key in ((0, "strict"), (1, "batch_rule")):
            want = tuple(bool(d[key][j]) for j in idx)
            assert H.verify_cached_n(mode, [entry(j) for j in idx], bits=bits) == want, (i, mode)
        mask = (i * 37 // 8) % 256
        want = tuple(bool(d["strict" if (mask >> k) & 1 else "batch_rule"][j]) for k, j in enumerate(idx))
        assert H.verify_cached_n(2, [entry(j) for j in idx], strict_mask=mask, bits=bits) == want, (i, "mixed")


def test_reduced_comb_sum_equals_full_comb():
    """[k](-A) from the 21-bit reduced-scalar comb equals the 20-bit comb's for
    honest, small-order and mixed-order keys of the corpus and for scalars at
    the reduction's edges ((L - 1) / 2, (L + 1) / 2, L - 1, 0, 1, 2^251 +- 1) and
    random ones; the key's torsion flag is set exactly for keys with a torsion
    component (the corpus's small- and mixed-order categories but the identity)."""
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    meta = json.load(open(os.path.join(GOLD, "ed25519_corpus.json")))
    cats = meta["categories"]
    rng = np.random.default_rng(21)
    L = H.L
    edges = [0, 1, 2, (L - 1) // 2, (L + 1) // 2, (L + 3) // 2, L - 1, L - 2, (1 << 251) - 1, 1 << 251,
             (1 << 251) + 1, (1 << 252) - 1]
    seen = {}
    for i in range(len(d["cat"])):
        cat = cats[int(d["cat"][i])]
        if cat not in ("honest", "small_order_A", "mixed_A_valid") or seen.get(cat, 0) >= 6:
            continue
        seen[cat] = seen.get(cat, 0) + 1
        A = d["pk"][i].tobytes()
        ks = edges + [int.from_bytes(rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), "little") % L
                      for _ in range(24)]
        for k in ks:
            e21, m21 = H.key_comb_sum(21, A, k)
            e20, m20 = H.key_comb_sum(20, A, k)
            assert e21 == e20, (cat, i, k)
            # the identity (y = 1, either sign bit) is small order without a torsion component
            ident = A[0] == 1 and not any(A[1:31]) and A[31] in (0, 0x80)
            assert bool(m21 & H.KEY_TORSION) == (cat != "honest" and not ident), (cat, i)
            assert (m21 & ~H.KEY_TORSION) == m20
    assert set(seen) == {"honest", "small_order_A", "mixed_A_valid"}


def test_sc_halfsize_lehmer_equals_one_step():
    """The Lehmer-batched reduction the kernels run lands on exactly the
    (u, v, sign, bits) of the one-step Euclid loop: random k < L, k near L,
    near 2^252, small / power-of-two / Fibonacci-ratio scalars (all-ones
    quotient runs) and huge partial quotients."""
    rng = random.Random(1234)
    ks = [rng.randrange(H.L) for _ in range(200_000)]
    ks += [H.L - 1 - i for i in range(64)] + [(1 << 252) + i for i in range(64)] + [(1 << 252) - 1 - i for i in range(64)]
    ks += [0, 1, 2, 3] + [1 << b for b in range(0, 253)] + [(1 << b) - 1 for b in range(1, 253)]
    # k / 8L close to a ratio of consecutive Fibonacci numbers -> long runs of quotient 1
    fa, fb = 1, 1
    while fb < 1 << 126:
        fa, fb = fb, fa + fb
    ks += [(8 * H.L * fa // fb + d) % H.L for d in range(-32, 33)]
    # huge first quotients: k tiny relative to 8L, and 8L / k just above an integer
    ks += [(8 * H.L) // q + d for q in (3, 1 << 20, 1 << 31, (1 << 32) + 1, 1 << 40, 1 << 60) for d in range(-3, 4)]
    ks = [k % H.L for k in ks]
    assert H.halfsize_disagree(ks) == 0


def test_sc_halfsize_properties():
    """Half-size scalars (sc25519.hpp): for every k < L the result satisfies
    u == v k (mod 8L), v odd, 0 < v < L, and bits >= bitlen(|u|), bitlen(v)
    (the window count is never too small); typical sizes ~2^128.  Edge inputs
    include k = 0, tiny k (loop not entered), k near L, powers of two and
    values with huge partial quotients."""
    L8 = 8 * H.L
    rng = random.Random(9)
    ks = [0, 1, 2, 7, 8, 9, H.L - 1, H.L - 2, H.L // 2, (H.L - 1) // 8, 1 << 127, (1 << 127) + 1, 1 << 128,
          (1 << 200) + 12345, (1 << 252) - 1, H.L - (1 << 126), L8 // 3, L8 // 5]
    ks += [(L8 * j) // (1 << 40) for j in range(1, 6)]          # huge first quotients
    ks += [(L8 // q) + d for q in (3, 1 << 33, 1 << 70) for d in (-1, 0, 1)]
    ks = [k % H.L for k in ks] + [rng.randrange(H.L) for _ in range(3000)]
    big = 0
    for k in ks:
        u, v, bits = H.sc_halfsize(k)
        assert (u - v * k) % L8 == 0, k
        assert v % 2 == 1 and 0 < v < H.L, k
        assert bits >= max(abs(u).bit_length(), v.bit_length()) and bits <= 253, k
        big += bits > 136
    assert big < 30  # random k: almost always ~128 bits


def _model():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLD, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_small_order_by_torsion_y():
    """The kernels' small-order test (y in {1, -1, 0, +-y8}) equals [8]P == 0 by
    doublings (and the textbook model) on every small-order encoding the corpus
    uses -- canonical, non-canonical (y + p) and negative-zero forms -- on
    mixed-order points T + aB and on random points."""
    M = _model()
    encs = list(M.small_order_encodings()) + [M.encode(t) for t in M.TORSION]
    rng = random.Random(5)
    for t in M.TORSION:
        for _ in range(3):
            encs.append(M.encode(M.padd(t, M.pmul(rng.randrange(1, M.L), M.BASE))))
    encs += [M.encode(M.pmul(rng.randrange(1, M.L), M.BASE)) for _ in range(20)]
    n_small = 0
    for e in encs:
        ok, by_dbl, by_y = H.small_order(e)
        assert ok == (M.decode(e) is not None)
        if ok:
            assert by_dbl == by_y == M.is_small(M.decode(e)), e.hex()
            n_small += by_y
    assert n_small >= 8


@pytest.mark.parametrize("bits", [20, 16])
def test_wide_comb_construction_vs_model(bits):
    """wcomb_bases + wcomb_fill (the device build of j * 2^(W i) * P, affine niels
    with one batched inversion per chunk) against the textbook model, for both
    comb widths the device builds (20-bit: B and committee keys that fit in HBM;
    16-bit: committee keys otherwise): first, second and last position, first,
    second and last chunk."""
    M = _model()
    with open(os.path.join(GOLD, "fixtures_reference.json")) as f:
        pk = bytes.fromhex(json.load(f)["keys"][1]["pk"])
    npos = (254 + bits - 1) // bits
    last_chunk = (1 << (bits - 1)) // 64 - 1
    cases = [(M.encode(M.BASE), 0, M.BASE), (pk, 1, M.pneg(M.decode(pk)))]
    for enc, neg, pt in cases:
        for pos in (0, 1, npos - 1):
            base = M.pmul(2 ** (bits * pos), pt)
            for c in (0, 1, last_chunk):
                meta, e = H.wcomb_chunk(bits, enc, neg, pos, c)
                assert meta == 1
                q = M.pmul(64 * c, base)
                for idx in range(65):
                    if idx or c == 0:
                        X, Y, Z, _ = q
                        zi = M.inv(Z)
                        x, y = X * zi % M.P, Y * zi % M.P
                        want = ((y + x) % M.P, (y - x) % M.P, 2 * M.D * x * y % M.P)
                        got = tuple(H.value(e[idx][10 * k:10 * k + 10]) % M.P for k in range(3))
                        assert got == want, (pos, c, idx)
                    q = M.padd(q, base)


def test_sign_fixture_through_device_code():
    with open(os.path.join(GOLD, "fixtures_reference.json")) as f:
        ref = json.load(f)
    d = bytes.fromhex(ref["hello_digest"])
    for k, s in zip(ref["keys"], ref["hello_signatures"]):
        pk, sig = H.sign(bytes.fromhex(k["seed"]), d)
        assert pk.hex() == k["pk"]
        assert sig.hex() == s


def _invert(limbs, vt):
    import ctypes
    lib = H.load()
    out = (ctypes.c_uint8 * 32)()
    lib.nth_fe_invert((ctypes.c_uint32 * 10)(*limbs), out, vt)
    return int.from_bytes(bytes(out), "little")


def test_fe_invert_vt_vs_fermat_and_bigint():
    """The key-cache kernel's variable-time inversion (fe_inv_vt.hpp: Pornin's
    optimized binary GCD, up to 17 x 30 steps on 62-bit approximations, leaving
    the loop once a = 0 -- on the host per value, so small inputs exercise the
    skipped iterations' direct factor 2^30) equals
    z^(p-2) mod p (Python big integers) on edge values and random inputs, and
    equals the Fermat chain (fe_invert) on 200k more inputs drawn in the C
    harness (half of them structured: small, p - small, powers of two, p + s
    as a non-canonical encoding)."""
    import ctypes
    P = H.P
    rng = random.Random(11)
    vals = [0, 1, 2, 3, 19, P - 1, P - 2, P + 1, P + 18, 2 ** 254, 2 ** 255 - 20, 2 ** 128, 2 ** 128 - 1,
            (P - 1) // 2, (P + 1) // 2, 2 ** 62, 2 ** 62 - 1, 2 ** 30, 2 ** 31 + 1]
    vals += [1 << k for k in range(255)]
    vals += [P - (1 << k) for k in range(1, 254)]
    vals += [rng.randrange(P) for _ in range(3000)]
    vals += [rng.randrange(1 << rng.randrange(1, 255)) for _ in range(1000)]
    for v in vals:
        limbs = H.to_limbs(v)
        want = pow(v % P, P - 2, P)
        assert _invert(limbs, 1) == want, hex(v)
    lib = H.load()
    lib.nth_fe_invert_cmp.restype = ctypes.c_ulonglong
    assert lib.nth_fe_invert_cmp(ctypes.c_ulonglong(200_000), ctypes.c_ulonglong(0x9E3779B97F4A7C15)) == 0


def test_opcount_matches_committed_profile():
    """profiles/opcount.json (roofline numerator) must match the current code."""
    path = os.path.join(os.path.dirname(GOLD), "..", "profiles", "opcount.json")
    if not os.path.exists(path):
        pytest.skip("profiles/opcount.json not generated yet (tools/opcount.py)")
    with open(path) as f:
        committed = json.load(f)
    import importlib.util
    spec = importlib.util.spec_from_file_location("opcount", os.path.join(os.path.dirname(GOLD), "..",
                                                                          "tools", "opcount.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cur = mod.measure()
    for key in ("verify_strict_fe_mul", "verify_strict_fe_sq", "verify_strict_mads"):
        assert cur[key] == committed[key], key
