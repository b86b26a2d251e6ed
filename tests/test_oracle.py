"""Pin the CPU oracle (oracle/) against the committed golden fixtures.

The fixtures were produced by tests/golden/make_golden.py from hashlib,
libsodium 1.0.18 and a pure-Python textbook model -- none of which share code
with oracle/.  These tests run on CPU only.
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from _oracle import expand

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


# ---------------------------------------------------------------- SHA-512
def test_sha512_vectors(oracle):
    v = _json("sha512_vectors.json")
    for e in v["vectors"]:
        m = expand(e["label"].encode(), e["len"])
        assert oracle.sha512(m).hex() == e["digest512"], e["len"]


def test_sha512_reference_fixtures(oracle):
    ref = _json("sha512_vectors.json")["reference_fixtures"]
    # worker/src/tests/processor_tests.rs:9-46 -- Processor digest of the 228-B batch
    b = bytes.fromhex(ref["processor_batch_228B"]["hex"])
    assert len(b) == 228
    assert oracle.digest(b).hex() == ref["processor_batch_228B"]["digest32"]
    assert ref["processor_batch_228B"]["digest32"].startswith("24d00f74a0767e74")
    assert oracle.digest(b"Hello, world!").hex() == ref["hello_world"]["digest32"]
    # a real 508,052-B sealed batch and a 500,000-B buffer (config 1)
    rb = ref["real_batch_977x512"]
    txs = [expand((rb["tx_label"] % i).encode(), rb["tx_len"]) for i in range(rb["ntx"])]
    real = struct.pack("<IQ", 0, len(txs)) + b"".join(struct.pack("<Q", len(t)) + t for t in txs)
    assert len(real) == rb["len"] == 508052
    assert oracle.digest(real).hex() == rb["digest32"]
    buf = expand(ref["buffer_500000"]["label"].encode(), 500000)
    assert oracle.digest(buf).hex() == ref["buffer_500000"]["digest32"]


def test_sha512_many_threads(oracle):
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 3000, size=257).astype(np.uint64)
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, size=int(lens.sum()) + 1, dtype=np.uint8)
    out = oracle.sha512_trunc32_many(data, off, lens, nthreads=4)
    for i in range(len(lens)):
        m = data[int(off[i]):int(off[i] + lens[i])].tobytes()
        assert out[i].tobytes() == hashlib.sha512(m).digest()[:32]


# ---------------------------------------------------------------- fixture keys
def test_chacha20_rfc7539_zero_key(oracle):
    # RFC 7539 §2.3.2-style known answer for key = 0, nonce = 0, counter = 0
    ks = oracle.chacha20(bytes(32), 64)
    assert ks[:16].hex() == "76b8e0ada0f13d90405d6ae55386bd28"


def test_keys_fixture(oracle):
    ref = _json("fixtures_reference.json")
    ks = oracle.chacha20(bytes(32), 128)
    for i, k in enumerate(ref["keys"]):
        seed = ks[32 * i:32 * i + 32]
        assert seed.hex() == k["seed"]
        assert oracle.pubkey(seed).hex() == k["pk"]


def test_sign_matches_libsodium(oracle):
    ref = _json("fixtures_reference.json")
    d = bytes.fromhex(ref["hello_digest"])
    for k, s in zip(ref["keys"], ref["hello_signatures"]):
        seed, pk = bytes.fromhex(k["seed"]), bytes.fromhex(k["pk"])
        assert oracle.sign(seed, pk, d).hex() == s


# ---------------------------------------------------------------- reference crypto_tests.rs
def _kp(ref, i):
    return bytes.fromhex(ref["keys"][i]["seed"]), bytes.fromhex(ref["keys"][i]["pk"])


def test_verify_valid_signature(oracle):            # crypto_tests.rs:49-61
    ref = _json("fixtures_reference.json")
    seed, pk = _kp(ref, 3)
    d = oracle.digest(b"Hello, world!")
    assert oracle.verify_strict(pk, oracle.sign(seed, pk, d), d)


def test_verify_invalid_signature(oracle):          # crypto_tests.rs:63-77
    ref = _json("fixtures_reference.json")
    seed, pk = _kp(ref, 3)
    sig = oracle.sign(seed, pk, oracle.digest(b"Hello, world!"))
    assert not oracle.verify_strict(pk, sig, oracle.digest(b"Bad message!"))


def test_verify_valid_batch(oracle):                # crypto_tests.rs:79-94
    ref = _json("fixtures_reference.json")
    d = oracle.digest(b"Hello, world!")
    pks, sigs = [], []
    for i in (3, 2, 1):
        seed, pk = _kp(ref, i)
        pks.append(pk)
        sigs.append(oracle.sign(seed, pk, d))
    assert oracle.verify_batch(pks, sigs, d)


def test_verify_invalid_batch(oracle):              # crypto_tests.rs:96-115
    ref = _json("fixtures_reference.json")
    d = oracle.digest(b"Hello, world!")
    pks, sigs = [], []
    for i in (3, 2):
        seed, pk = _kp(ref, i)
        pks.append(pk)
        sigs.append(oracle.sign(seed, pk, d))
    pks.append(_kp(ref, 1)[1])
    sigs.append(bytes(64))  # Signature::default()
    assert not oracle.verify_batch(pks, sigs, d)


def test_verify_batch_empty(oracle):
    assert oracle.verify_batch([], [], bytes(32))


# ---------------------------------------------------------------- edge-case corpus
@pytest.fixture(scope="module")
def corpus():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    return {k: d[k] for k in d.files}


def _entry(c, i):
    o, n = int(c["off"][i]), int(c["len"][i])
    return c["pk"][i].tobytes(), c["sig"][i].tobytes(), c["msg"][o:o + n].tobytes()


def test_corpus_verify_strict(oracle, corpus):
    meta = _json("ed25519_corpus.json")
    for i in range(len(corpus["cat"])):
        pk, sig, m = _entry(corpus, i)
        got = oracle.verify_strict(pk, sig, m)
        assert got == bool(corpus["strict"][i]), (i, meta["categories"][corpus["cat"][i]])
        assert got == bool(corpus["sodium"][i])


def test_corpus_batch_rule_and_class(oracle, corpus):
    for i in range(len(corpus["cat"])):
        pk, sig, m = _entry(corpus, i)
        assert oracle.verify_cofactorless(pk, sig, m) == bool(corpus["batch_rule"][i]), i
        assert oracle.verify_batch([pk], [sig], m) == bool(corpus["batch_rule"][i]), i
        assert oracle.batch_class(pk, sig, m) == int(corpus["batch_class"][i]), i


def test_dalek_batch_equation_baseline(oracle, corpus):
    """The CPU baseline's randomized Straus batch (dalek's own computation) gives
    the deterministic A.3 verdict on every entry outside dalek's random class
    (batch_class 2), on the reference's batch fixtures, and on 67-vote groups."""
    for i in range(len(corpus["cat"])):
        if int(corpus["batch_class"][i]) == 2:
            continue
        pk, sig, m = _entry(corpus, i)
        assert oracle.verify_batch_dalek([pk], [sig], m) == bool(corpus["batch_rule"][i]), i
    ref = _json("fixtures_reference.json")
    d = oracle.digest(b"Hello, world!")
    kp = [_kp(ref, i) for i in (3, 2, 1)]
    sigs = [oracle.sign(s, p, d) for s, p in kp]
    assert oracle.verify_batch_dalek([p for _, p in kp], sigs, d)          # crypto_tests.rs:79-94
    assert not oracle.verify_batch_dalek([p for _, p in kp], sigs[:2] + [bytes(64)], d)  # :96-115
    assert oracle.verify_batch_dalek([], [], d)
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    ndet = 0
    for i in range(len(g["cnt"])):
        if not g["deterministic"][i]:
            continue
        f, c = int(g["first"][i]), int(g["cnt"][i])
        got = oracle.verify_batch_dalek([x.tobytes() for x in g["pk"][f:f + c]], [x.tobytes() for x in g["sig"][f:f + c]],
                                        g["msg32"][i].tobytes())
        assert got == bool(g["expect"][i]), i
        ndet += 1
    assert ndet >= 40
    seeds = [bytes([i + 1]) * 32 for i in range(67)]
    pks = [oracle.pubkey(s) for s in seeds]
    sg = [oracle.sign(s, p, d) for s, p in zip(seeds, pks)]
    for z in (bytes(32), b"\x01" * 32):
        assert oracle.verify_batch_dalek(pks, sg, d, z)
        bad = list(sg)
        bad[40] = bad[40][:40] + bytes([bad[40][40] ^ 1]) + bad[40][41:]
        assert not oracle.verify_batch_dalek(pks, bad, d, z)


def test_certificates_verify_many_baseline(oracle):
    """Certificate::verify's signature + digest work (CPU baseline of config 3)."""
    import struct
    seeds = [bytes([i + 7]) * 32 for i in range(10)]
    pks = [oracle.pubkey(s) for s in seeds]
    hdr, hoff, hlen, ids, hpk, hsig, cpre, vpk, vsig, first, cnt, want = ([] for _ in range(12))
    o = 0
    for g in range(6):
        a = g % 10
        pre = pks[a] + struct.pack("<Q", g + 3) + bytes(range(40 + g))
        hid = oracle.digest(pre)
        hs = oracle.sign(seeds[a], pks[a], hid)
        ok = True
        if g == 2:
            hs = hs[:33] + bytes([hs[33] ^ 1]) + hs[34:]
            ok = False
        cp = hid + struct.pack("<Q", g + 3) + pks[a]
        cd = oracle.digest(cp)
        first.append(len(vpk))
        for v in range(7):
            s = oracle.sign(seeds[v], pks[v], cd)
            if g == 4 and v == 5:
                s = bytes(32) + s[32:]
                ok = False
            vpk.append(pks[v])
            vsig.append(s)
        cnt.append(7)
        if g == 5:
            hid = bytes(32)
            ok = False
        hdr.append(pre); hoff.append(o); hlen.append(len(pre)); o += len(pre)
        ids.append(hid); hpk.append(pks[a]); hsig.append(hs); cpre.append(cp); want.append(ok)
    u8 = lambda xs: np.frombuffer(b"".join(xs), np.uint8)
    got = oracle.certificates_verify_many(u8(hdr), hoff, hlen, u8(ids), u8(hpk), u8(hsig), u8(cpre), u8(vpk),
                                          u8(vsig), first, cnt, nthreads=2)
    assert got.astype(bool).tolist() == want


def test_corpus_bulk_threads(oracle, corpus):
    got = oracle.verify_strict_many(corpus["pk"], corpus["sig"], corpus["msg"], corpus["off"],
                                    corpus["len"], nthreads=4)
    assert np.array_equal(got, corpus["strict"])


def test_batch_groups_fixture(oracle):
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    gb, sb = oracle.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"], nthreads=3)
    assert np.array_equal(gb, g["expect"])
    # per-signature bits AND to the group bit
    for i in range(len(g["cnt"])):
        f, c = int(g["first"][i]), int(g["cnt"][i])
        assert bool(gb[i]) == bool(np.all(sb[f:f + c]))


def test_torsion_points(oracle):
    meta = _json("ed25519_corpus.json")
    mine = sorted(oracle.torsion_point(i).hex() for i in range(8))
    assert mine == sorted(meta["torsion_encodings"])
    for e in meta["small_order_encodings"]:
        assert oracle.point_is_small_order(bytes.fromhex(e))


def test_sodium_comparator_matches_corpus(oracle):
    """The bench's external CPU comparator (oracle/sodium_batch.c over libsodium)
    gives the corpus' strict verdicts."""
    lib = "/opt/conda/lib/libsodium.so.23"
    if not os.path.exists(lib):
        pytest.skip("libsodium not present")
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    r = oracle.sodium_verify_many(lib, d["pk"], d["sig"], d["msg"], d["off"], d["len"], 4)
    assert r is not None
    assert np.array_equal(r.astype(bool), d["strict"].astype(bool))


def test_bench_sha_cpu_baseline_checks_digests():
    """bench.py's config-4 CPU leg (oracle C SHA-512 + hashlib comparator) reports
    agreement against the digests it is handed -- and catches a wrong one."""
    import sys
    import types
    import hashlib
    import torch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    m, ml = 8, 1000
    data = torch.from_numpy(np.random.default_rng(2).integers(0, 256, m * ml, dtype=np.uint8))
    dig = np.stack([np.frombuffer(hashlib.sha512(data[i * ml:(i + 1) * ml].numpy().tobytes()).digest()[:32],
                                  np.uint8) for i in range(m)])
    dig[5, 0] ^= 1
    res = bench.sha_cpu_baseline(types.SimpleNamespace(cpu_threads=2, cpu_seconds=0.05), data,
                                 torch.from_numpy(dig), m, ml)
    assert res["digests_agree_with_gpu"] == "7/8"
    assert res["external"]["digests_agree_with_gpu"] == "7/8"
    assert res["value"] > 0 and res["cores"] == 2
