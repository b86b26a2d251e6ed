"""Device memory of a context is lazy and degradable.

The reference runs every primary and every worker as its own process
(node/src/main.rs:101-133) and a worker only hashes (worker/src/processor.rs:38),
so a context that only digests must not pay for the verify tables, and a
process under an HBM budget must still verify -- with the 20-bit comb of B
instead of the 24-bit one, and narrower key combs -- with identical verdicts.
nt_memory_info reports what a context holds (include/ntcrypto.h)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GB = 1 << 30


@pytest.fixture(scope="module")
def corpus():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    return {k: d[k] for k in d.files}


def _pack(msgs):
    ln = np.array([len(m) for m in msgs], np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    return np.frombuffer(b"".join(msgs), np.uint8), off, ln


def test_digest_only_context_holds_no_tables():
    """A worker-shaped context (digests only) allocates no comb of B and no
    verify workspace: the round-3 library paid 11.8 + 3 GB at nt_init."""
    import hashlib
    import ntcrypto
    be = ntcrypto.Backend(device=0)
    try:
        msgs = [b"x" * 1000, b"", bytes(range(256)) * 2000]
        d = be.digest_many(msgs)
        assert [x.tobytes() for x in d] == [hashlib.sha512(m).digest()[:32] for m in msgs]
        mi = be.memory_info(0)
        assert mi["comb_b_bits"] == 0 and mi["comb_b_bytes"] == 0, mi
        assert mi["workspace_bytes"] == 0 and mi["key_comb_bytes"] == 0 and mi["held"] == 0, mi
        assert mi["staging_bytes"] < 64 << 20, mi
        # the first verify builds them: the widest comb when nothing caps it
        pk, sig = be.sign_batch(np.arange(32, dtype=np.uint8).reshape(1, 32), np.zeros(32, np.uint8),
                                np.zeros(1, np.uint64), np.full(1, 32, np.uint64))
        assert be.verify_strict(pk, sig, np.zeros(32, np.uint8), np.zeros(1, np.uint64),
                                np.full(1, 32, np.uint64))[0]
        mi = be.memory_info(0)
        assert mi["comb_b_bits"] == 24 and mi["comb_b_bytes"] > 11 * GB, mi
        assert mi["workspace_bytes"] > 0 and mi["held"] == mi["comb_b_bytes"], mi
    finally:
        be.close()


@pytest.fixture(scope="module")
def small():
    """A context whose tables may use 4 GB per device: the 24-bit comb of B
    (11.8 GB) does not fit, the 20-bit one (872 MB) does."""
    import ntcrypto
    be = ntcrypto.Backend(device=0)
    be.set_hbm_budget(4 * GB)
    yield be
    be.close()


def test_budget_falls_back_to_20bit_comb_corpus(small, corpus):
    got = small.verify_strict(corpus["pk"], corpus["sig"], corpus["msg"], corpus["off"], corpus["len"])
    assert np.array_equal(got, corpus["strict"].astype(bool))
    mi = small.memory_info(0)
    assert mi["comb_b_bits"] == 20 and mi["budget"] == 4 * GB, mi
    assert mi["comb_b_bytes"] < GB and mi["held"] <= 4 * GB, mi
    sel = np.nonzero(corpus["len"] == 32)[0]
    msg32 = np.stack([corpus["msg"][int(corpus["off"][i]):int(corpus["off"][i]) + 32] for i in sel])
    gb = small.verify_batch_groups(corpus["pk"][sel], corpus["sig"][sel], np.arange(len(sel), dtype=np.uint64),
                                   np.ones(len(sel), np.uint32), msg32)
    assert np.array_equal(gb, corpus["batch_rule"][sel].astype(bool))


def test_budget_20bit_comb_random_vs_oracle_and_signing(small, oracle):
    rng = np.random.default_rng(404)
    n = 2048
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 400, n)]
    data, off, ln = _pack(msgs)
    pk, sig = small.sign_batch(seeds, data, off, ln)   # signing through the 20-bit comb of B
    for i in range(0, n, 97):
        p = oracle.pubkey(seeds[i].tobytes())
        assert pk[i].tobytes() == p and sig[i].tobytes() == oracle.sign(seeds[i].tobytes(), p, msgs[i])
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    sig[flip, rng.integers(0, 64)] ^= 4
    got = small.verify_strict(pk, sig, data, off, ln)
    want = oracle.verify_strict_many(pk, sig, data, off, ln, nthreads=8).astype(bool)
    assert np.array_equal(got, want) and got.sum() > n // 2
    with open(os.path.join(GOLD, "fixtures_reference.json")) as f:
        ref = json.load(f)
    seeds4 = np.stack([np.frombuffer(bytes.fromhex(k["seed"]), np.uint8) for k in ref["keys"]])
    d = bytes.fromhex(ref["hello_digest"])
    pk4, sig4 = small.sign_batch(seeds4, np.frombuffer(d * 4, np.uint8), np.arange(4, dtype=np.uint64) * 32,
                                 np.full(4, 32, np.uint64))
    assert [s.tobytes().hex() for s in sig4] == ref["hello_signatures"]


def test_budget_key_comb_widths_and_keyset_parity(small, corpus):
    """Key combs take what the budget leaves after the comb of B (3.1 GB):
    10 keys at 18 bits (2.5 GB), 40 keys at 16 bits (2.7 GB), 60 keys not at all
    (NT_ENOMEM, never a silent reject).  Corpus parity through the 18- and
    16-bit key-cache kernels beside the 20-bit comb of B, every mode."""
    import ntcrypto
    uniq, inv = np.unique(corpus["pk"], axis=0, return_inverse=True)
    inv = inv.ravel().astype(np.uint32)
    n = len(corpus["pk"])
    want_strict = (np.arange(n) % 3) == 1
    for per_set, bits in ((10, 18), (40, 16)):
        got_s = np.zeros(n, bool)
        got_m = np.zeros(n, bool)
        for k0 in range(0, len(uniq), per_set):
            ks = small.keyset(uniq[k0:k0 + per_set])
            nk = len(uniq[k0:k0 + per_set])
            if nk == per_set:
                assert ks.info()[0] == bits
            mi = small.memory_info(0)
            assert mi["key_comb_bytes"] > 0 and mi["held"] <= 4 * GB and mi["comb_b_bits"] == 20, mi
            sel = np.nonzero((inv >= k0) & (inv < k0 + per_set))[0]
            idx = inv[sel] - k0
            args = (corpus["sig"][sel], corpus["msg"], corpus["off"][sel], corpus["len"][sel])
            got_s[sel] = ks.verify(ntcrypto.NT_MODE_STRICT, idx, *args)
            midx = idx | np.where(want_strict[sel], np.uint32(ntcrypto.NT_KEY_STRICT_BIT), np.uint32(0))
            got_m[sel] = ks.verify(ntcrypto.NT_MODE_MIXED, midx.astype(np.uint32), *args)
            ks.close()
            assert small.memory_info(0)["key_comb_bytes"] == 0
        assert np.array_equal(got_s, corpus["strict"].astype(bool)), bits
        assert np.array_equal(got_m, np.where(want_strict, corpus["strict"], corpus["batch_rule"]).astype(bool)), bits
    with pytest.raises(ntcrypto.NtError):
        small.keyset(uniq[:60])


def test_budget_below_the_narrowest_comb_fails_loudly(corpus):
    """100 MB cannot hold even the 20-bit comb of B: the call fails with
    NT_ENOMEM instead of returning verdicts."""
    import ntcrypto
    be = ntcrypto.Backend(device=0)
    try:
        be.set_hbm_budget(100 << 20)
        with pytest.raises(ntcrypto.NtError, match="memory"):
            be.verify_strict(corpus["pk"][:4], corpus["sig"][:4], corpus["msg"], corpus["off"][:4],
                             corpus["len"][:4])
        assert be.memory_info(0)["comb_b_bits"] == 0
        be.set_hbm_budget(0)   # lifting the cap lets the next call build the tables
        got = be.verify_strict(corpus["pk"][:4], corpus["sig"][:4], corpus["msg"], corpus["off"][:4],
                               corpus["len"][:4])
        assert np.array_equal(got, corpus["strict"][:4].astype(bool))
    finally:
        be.close()


def test_library_compute_streams_are_distinct():
    import ntcrypto
    be = ntcrypto.Backend(device=0)
    try:
        a, b = be.dev_stream(0, 0), be.dev_stream(0, 1)
        assert a and b and a != b
        with pytest.raises(ntcrypto.NtError):
            be.dev_stream(0, 2)
    finally:
        be.close()


def test_committee_outlives_its_keyset():
    """an nt_committee keeps the keyset's device tables alive, so
    freeing the keyset first is safe; ingestion afterwards still verifies
    (a valid 3-of-4 certificate, the same with a forged vote, a genesis one)."""
    import struct
    import _wire as W
    from _oracle import load
    import ntcrypto
    orc = load()
    be = ntcrypto.Backend(device=0)
    try:
        seeds = [bytes([i + 1, 9]) * 16 for i in range(4)]
        keys = [orc.pubkey(s) for s in seeds]
        ks = be.keyset(np.frombuffer(b"".join(keys), np.uint8).reshape(4, 32))
        cm = ntcrypto.Committee(ks, [1, 1, 1, 1], [[0], [0], [0], [0]], quorum=3)
        ks.close()   # the committee still holds the tables
        h = W.Header(keys[1], 7, {bytes(range(32)): 0}, {bytes(32)})
        h.sig = orc.sign(seeds[1], keys[1], h.id)
        c = W.Certificate(h, [])
        for i in (0, 2, 3):
            c.votes.append((keys[i], orc.sign(seeds[i], keys[i], c.digest())))
        bad = W.Certificate(h, list(c.votes))
        bad.votes[1] = (bad.votes[1][0], bytes(32) + bad.votes[1][1][32:])
        gen = W.Certificate(W.Header(keys[2], 0, {}, set(), id_=bytes(32)), [])
        codes = cm.ingest([W.message(c), W.message(bad), W.message(gen)], gc_round=0)
        assert list(codes) == [W.OK, W.INVALID_SIGNATURE, W.OK]
        cm.close()
    finally:
        be.close()
