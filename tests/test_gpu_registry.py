"""GPU parity of the key registry (include/ntcrypto.h nt_set_key_cache): the
committee key cache behind the PLAIN entry points the crate binds
(nt_ed25519_verify_strict / nt_ed25519_verify_batch_groups <-
Signature::verify / verify_batch, crypto/src/lib.rs:200-219), keys passed as
raw 32-byte encodings.  Registered keys verify through the key-cache kernel,
the others through the uncached kernel in the same call; the verdicts must be
the corpus labels and the oracle's whichever way each key goes.

Key combs at 16 bits (67 MB per key) unless a test says otherwise, so a few
hundred corpus keys fit beside everything else; the kernel's arithmetic is
the same at every width (test_gpu_parity.py::test_keyset_corpus)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def corpus():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    return {k: d[k] for k in d.files}


@pytest.fixture()
def reg(monkeypatch):
    """A fresh context with a registry (16-bit key combs); closed after the test."""
    import ntcrypto
    monkeypatch.setenv("NT_KEYSET_COMB_BITS", "16")
    b = ntcrypto.Backend(device=0)
    b.set_key_cache(1024)
    yield b
    b.close()


def _pack(msgs):
    ln = np.array([len(m) for m in msgs], np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    return np.frombuffer(b"".join(msgs), np.uint8), off, ln


def _corpus_msg32(c):
    sel = np.nonzero(c["len"] == 32)[0]
    return sel, np.stack([c["msg"][int(c["off"][i]):int(c["off"][i]) + 32] for i in sel])


def test_registry_corpus_all_registered(reg, corpus):
    """Every corpus key offered to the registry: keys that decode are admitted
    (off-curve / non-canonical-garbage keys are refused and stay on the
    uncached path); strict verdicts and the batch rule equal the corpus labels."""
    c = corpus
    uniq = np.unique(c["pk"], axis=0)
    reg.key_cache_add(uniq)
    info = reg.key_cache_info()
    assert info["error"] == 0 and info["pending"] == 0
    assert info["keys"] + info["refused"] == len(uniq) and info["keys"] > 0 and info["comb_bits"] == 16
    got = reg.verify_strict(c["pk"], c["sig"], c["msg"], c["off"], c["len"])
    assert np.array_equal(got, c["strict"].astype(bool))
    i1 = reg.key_cache_info()
    assert i1["hits"] > 0
    sel, msg32 = _corpus_msg32(c)
    gb = reg.verify_batch_groups(c["pk"][sel], c["sig"][sel], np.arange(len(sel), dtype=np.uint64),
                                 np.ones(len(sel), np.uint32), msg32)
    assert np.array_equal(gb, c["batch_rule"][sel].astype(bool))


def test_registry_corpus_half_registered(reg, corpus):
    """Half of the corpus keys registered, the other half not: one call mixes
    both kernels; verdicts equal the labels (strict and batch rule), and the
    per-signature bits of the groups call equal the uncached path's."""
    c = corpus
    uniq = np.unique(c["pk"], axis=0)
    reg.key_cache_add(uniq[::2])
    got = reg.verify_strict(c["pk"], c["sig"], c["msg"], c["off"], c["len"])
    assert np.array_equal(got, c["strict"].astype(bool))
    info = reg.key_cache_info()
    assert info["hits"] > 0 and info["misses"] > 0
    sel, msg32 = _corpus_msg32(c)
    # certificates of 1..7 votes over the corpus' 32-byte entries
    rng = np.random.default_rng(5)
    cnt = []
    left = len(sel)
    while left:
        k = int(min(left, rng.integers(1, 8)))
        cnt.append(k)
        left -= k
    cnt = np.array(cnt, np.uint32)
    first = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
    # each group signs one message: use entry i's own message as group g's only where the
    # group holds one vote; otherwise compare with the uncached path on the same inputs
    pk, sig = c["pk"][sel], c["sig"][sel]
    gmsg = msg32[first.astype(np.int64)]
    gb, sb = reg.verify_batch_groups(pk, sig, first, cnt, gmsg, with_sig_bits=True)
    import ntcrypto
    plain = ntcrypto.Backend(device=0)
    try:
        gb2, sb2 = plain.verify_batch_groups(pk, sig, first, cnt, gmsg, with_sig_bits=True)
    finally:
        plain.close()
    assert np.array_equal(gb, gb2) and np.array_equal(sb, sb2)
    one = cnt == 1
    assert np.array_equal(gb[one], c["batch_rule"][sel][first[one].astype(np.int64)].astype(bool))


def test_registry_mixed_certificates_vs_oracle(reg, oracle):
    """A committee of 100, 60 keys registered: 400 certificates of 5-67 votes
    from all 100 (so most certificates mix registered and unregistered keys),
    some votes corrupted, plus strict header signatures; against the oracle."""
    rng = np.random.default_rng(11)
    nk, G = 100, 400
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    pks = reg.sign_batch(seeds)
    reg.key_cache_add(pks[:60])
    assert reg.key_cache_info()["keys"] == 60
    digests = rng.integers(0, 256, (G, 32), dtype=np.uint8)
    cnt = rng.integers(5, 68, G).astype(np.uint32)
    first = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
    voters = np.concatenate([rng.permutation(nk)[:k] for k in cnt])
    V = len(voters)
    gidx = np.repeat(np.arange(G), cnt)
    msg = digests[gidx].reshape(-1)
    _, vsig = reg.sign_batch(seeds[voters], msg, np.arange(V, dtype=np.uint64) * 32, np.full(V, 32, np.uint64))
    vsig = vsig.copy()
    bad = rng.random(V) < 0.01
    vsig[bad, 50] ^= 4
    vpk = pks[voters]
    gb, sb = reg.verify_batch_groups(vpk, vsig, first, cnt, digests, with_sig_bits=True)
    og, osb = oracle.verify_batch_groups(vpk, vsig, first, cnt, digests, nthreads=8)
    assert np.array_equal(gb, og.astype(bool)) and np.array_equal(sb, osb.astype(bool))
    assert np.array_equal(sb, ~bad)
    want_g = np.array([not bad[int(f):int(f) + int(k)].any() for f, k in zip(first, cnt)])
    assert np.array_equal(gb, want_g)
    # strict: one signature per certificate (the header), registered and unregistered authors
    author = rng.integers(0, nk, G)
    _, hsig = reg.sign_batch(seeds[author], digests.reshape(-1), np.arange(G, dtype=np.uint64) * 32,
                             np.full(G, 32, np.uint64))
    hsig = hsig.copy()
    hsig[::9, 3] ^= 1
    got = reg.verify_strict(pks[author], hsig, digests.reshape(-1), np.arange(G, dtype=np.uint64) * 32,
                            np.full(G, 32, np.uint64))
    want = oracle.verify_strict_many(pks[author], hsig, digests.reshape(-1), np.arange(G, dtype=np.uint64) * 32,
                                     np.full(G, 32, np.uint64), nthreads=8).astype(bool)
    assert np.array_equal(got, want) and got.sum() == G - len(range(0, G, 9))


def test_registry_admits_on_sight(reg):
    """An empty registry: the first call's keys go through the uncached kernel
    and are queued; after nt_key_cache_sync the next call finds all of them.
    Keys that do not decode are refused; the capacity bounds admissions."""
    rng = np.random.default_rng(12)
    nk = 20
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    d = rng.integers(0, 256, 32, dtype=np.uint8)
    pks, sig = reg.sign_batch(seeds, np.tile(d, nk), np.arange(nk, dtype=np.uint64) * 32, np.full(nk, 32, np.uint64))
    first, cnt = np.zeros(1, np.uint64), np.full(1, nk, np.uint32)
    assert reg.verify_batch_groups(pks, sig, first, cnt, d)[0]
    reg.key_cache_sync()
    info = reg.key_cache_info()
    assert info["keys"] == nk and info["admitted"] == nk
    h0 = info["hits"]
    assert reg.verify_batch_groups(pks, sig, first, cnt, d)[0]
    assert reg.key_cache_info()["hits"] - h0 == nk
    # a key that does not decode (y = 2: not on the curve) is refused, and the call rejects it
    junk = np.zeros((1, 32), np.uint8)
    junk[0, 0] = 2
    assert not reg.verify_batch_groups(junk, sig[:1], first, np.ones(1, np.uint32), d)[0]
    reg.key_cache_sync()
    info = reg.key_cache_info()
    assert info["keys"] == nk and info["refused"] == 1
    # capacity: a registry of 4 keys admits 4
    reg.set_key_cache(4)
    assert reg.verify_batch_groups(pks, sig, first, cnt, d)[0]
    reg.key_cache_sync()
    assert reg.key_cache_info()["keys"] == 4


def test_registry_multi_device_entries(monkeypatch, oracle):
    """Two device entries (the same GPU twice): certificate groups shard over
    both, each entry with its own registry tables; partial registration."""
    import ntcrypto
    monkeypatch.setenv("NT_KEYSET_COMB_BITS", "16")
    b = ntcrypto.Backend(devices=[0, 0])
    try:
        b.set_key_cache(64)
        rng = np.random.default_rng(13)
        nk, G = 40, 300
        seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
        pks = b.sign_batch(seeds)
        b.key_cache_add(pks[:25])
        digests = rng.integers(0, 256, (G, 32), dtype=np.uint8)
        cnt = np.full(G, 27, np.uint32)
        first = (np.arange(G, dtype=np.uint64) * 27)
        voters = np.concatenate([rng.permutation(nk)[:27] for _ in range(G)])
        V = len(voters)
        msg = digests[np.repeat(np.arange(G), 27)].reshape(-1)
        _, vsig = b.sign_batch(seeds[voters], msg, np.arange(V, dtype=np.uint64) * 32, np.full(V, 32, np.uint64))
        vsig = vsig.copy()
        vsig[::101, 10] ^= 8
        gb = b.verify_batch_groups(pks[voters], vsig, first, cnt, digests)
        bad = np.zeros(V, bool)
        bad[::101] = True
        assert np.array_equal(gb, ~bad.reshape(G, 27).any(axis=1))
    finally:
        b.close()


def test_registry_small_call_routing(reg):
    """The calibrated model carries both GPU floors: the
    key-cache floor is below the uncached one, and AUTO routes a lone
    certificate by the floor of the kernel it would run."""
    import math

    import ntcrypto
    T = 16
    reg.set_small_call_path(ntcrypto.NT_SMALL_AUTO, T)
    try:
        m = reg.small_call_model()
        assert m["calibrated"] and 0 < m["gpu_keyset_us"] < m["gpu_verify_us"], m
        rng = np.random.default_rng(14)
        n = 67
        seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        d = rng.integers(0, 256, 32, dtype=np.uint8)
        pks, sig = reg.sign_batch(seeds, np.tile(d, n), np.arange(n, dtype=np.uint64) * 32, np.full(n, 32, np.uint64))
        reg.key_cache_add(pks)
        t = min(m["threads"], n)
        cpu = math.ceil(n / t) * m["cpu_verify_us"] + (m["spawn_us"] if t > 1 else 0)
        h0, g0 = reg.call_counts()
        assert reg.verify_batch_groups(pks, sig, np.zeros(1, np.uint64), np.full(1, n, np.uint32), d)[0]
        h1, g1 = reg.call_counts()
        want_host = cpu < m["gpu_keyset_us"]
        assert (h1 - h0, g1 - g0) == ((1, 0) if want_host else (0, 1)), (cpu, m)
    finally:
        reg.set_small_call_path(ntcrypto.NT_SMALL_OFF)


def test_registry_concurrent_calls_during_admission(reg):
    """Four threads call the plain entry points at once while the registry
    admits the committee's keys on sight (the primary's tasks share one context):
    every verdict is the expected one whichever snapshot a call ran with, and
    by the end every decodable key is registered."""
    import threading
    rng = np.random.default_rng(15)
    nk, G, q = 40, 64, 13
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    pks = reg.sign_batch(seeds)
    batches = []
    for t in range(4):
        digests = rng.integers(0, 256, (G, 32), dtype=np.uint8)
        voters = np.concatenate([rng.permutation(nk)[:q] for _ in range(G)])
        msg = digests[np.repeat(np.arange(G), q)].reshape(-1)
        _, vsig = reg.sign_batch(seeds[voters], msg, np.arange(G * q, dtype=np.uint64) * 32,
                                 np.full(G * q, 32, np.uint64))
        vsig = vsig.copy()
        bad = rng.random(G * q) < 0.05
        vsig[bad, 5] ^= 1
        want = ~bad.reshape(G, q).any(axis=1)
        batches.append((pks[voters], vsig, digests, want))
    first = np.arange(G, dtype=np.uint64) * q
    cnt = np.full(G, q, np.uint32)
    errors = []

    def work(t):
        try:
            pk, sig, dg, want = batches[t]
            for _ in range(12):
                got = reg.verify_batch_groups(pk, sig, first, cnt, dg)
                if not np.array_equal(got, want):
                    errors.append((t, int((got != want).sum())))
                reg.key_cache_info()
        except Exception as e:  # surfaced below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    reg.key_cache_sync()
    info = reg.key_cache_info()
    assert info["keys"] == nk and info["error"] == 0 and info["hits"] > 0, info
