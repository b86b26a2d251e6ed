"""GPU parity: the gfx950 path through the C ABI vs. the golden fixtures and the
CPU oracle (bit-exact digests, identical accept/reject decisions).
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from _oracle import expand


def nbytes(t):
    """byte size of a device tensor: the msg_bytes argument of the nt_dev_* entry points"""
    return int(t.numel()) * int(t.element_size())


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def be():
    import ntcrypto
    b = ntcrypto.Backend(0)
    yield b
    b.close()


def _json(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def _pack(msgs):
    ln = np.array([len(m) for m in msgs], np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    return np.frombuffer(b"".join(msgs), np.uint8), off, ln


# ------------------------------------------------------------------ SHA-512
def test_sha512_golden_vectors(be):
    v = _json("sha512_vectors.json")
    msgs = [expand(e["label"].encode(), e["len"]) for e in v["vectors"]]
    out = be.digest_many(msgs)
    for e, d in zip(v["vectors"], out):
        assert d.tobytes().hex() == e["digest512"][:64], e["len"]


def test_sha512_reference_fixtures(be):
    ref = _json("sha512_vectors.json")["reference_fixtures"]
    rb = ref["real_batch_977x512"]
    txs = [expand((rb["tx_label"] % i).encode(), rb["tx_len"]) for i in range(rb["ntx"])]
    real = struct.pack("<IQ", 0, len(txs)) + b"".join(struct.pack("<Q", len(t)) + t for t in txs)
    msgs = [bytes.fromhex(ref["processor_batch_228B"]["hex"]), b"Hello, world!", real,
            expand(ref["buffer_500000"]["label"].encode(), 500000)]
    out = be.digest_many(msgs)
    assert out[0].tobytes().hex() == ref["processor_batch_228B"]["digest32"]
    assert out[1].tobytes().hex() == ref["hello_world"]["digest32"]
    assert out[2].tobytes().hex() == rb["digest32"]
    assert out[3].tobytes().hex() == ref["buffer_500000"]["digest32"]


def test_sha512_random_lengths_and_alignment(be):
    rng = np.random.default_rng(11)
    lens = np.concatenate([np.arange(0, 300), rng.integers(0, 20000, 200)]).astype(np.uint64)
    gaps = rng.integers(0, 16, len(lens)).astype(np.uint64)  # arbitrary alignments
    off = np.zeros(len(lens), np.uint64)
    pos = 0
    for i in range(len(lens)):
        pos += int(gaps[i])
        off[i] = pos
        pos += int(lens[i])
    data = rng.integers(0, 256, pos + 1, dtype=np.uint8)
    out = be.sha512_trunc32(data, off, lens)
    for i in range(len(lens)):
        m = data[int(off[i]):int(off[i] + lens[i])].tobytes()
        assert out[i].tobytes() == hashlib.sha512(m).digest()[:32], (i, int(lens[i]), int(off[i]))


def test_sha512_both_kernels(be):
    """All three digest kernels against hashlib, with long and ragged messages
    in the same call (lanes with different block counts): n <= 32768 with a
    message of >= 16 KB runs the two-wave producer/consumer kernel (n = 1000),
    other launches of <= 65,536 messages the 80-VGPR one-lane kernel (n = 3,
    33000), larger ones the general one-lane kernel (n = 70000)."""
    rng = np.random.default_rng(7)
    for n in (3, 1000, 33000, 70000):
        lens = rng.integers(0, 300, n).astype(np.uint64)
        lens[: min(n, 5)] = [0, 111, 112, 128, 2000][: min(n, 5)]
        if n == 1000:
            lens[17] = 70_000  # one lane runs ~550 blocks while the others stop early
        off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        data = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8)
        out = be.sha512_trunc32(data, off, lens)
        raw = data.tobytes()
        for i in range(n):
            m = raw[int(off[i]):int(off[i] + lens[i])]
            assert out[i].tobytes() == hashlib.sha512(m).digest()[:32], (n, i, int(lens[i]))


def test_sha512_empty_input(be):
    out = be.sha512_trunc32(np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.uint64))
    assert out.shape == (0, 32)


# ------------------------------------------------------------------ keygen / signing
def test_keys_fixture_and_signatures(be):
    ref = _json("fixtures_reference.json")
    seeds = np.stack([np.frombuffer(bytes.fromhex(k["seed"]), np.uint8) for k in ref["keys"]])
    d = bytes.fromhex(ref["hello_digest"])
    data = np.frombuffer(d * 4, np.uint8)
    pk, sig = be.sign_batch(seeds, data, np.arange(4, dtype=np.uint64) * 32, np.full(4, 32, np.uint64))
    for i, k in enumerate(ref["keys"]):
        assert pk[i].tobytes().hex() == k["pk"]
        assert sig[i].tobytes().hex() == ref["hello_signatures"][i]


def test_sign_matches_oracle_random(be, oracle):
    rng = np.random.default_rng(5)
    n = 300
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 700, n)]
    data, off, ln = _pack(msgs)
    pk, sig = be.sign_batch(seeds, data, off, ln)
    for i in range(n):
        s = seeds[i].tobytes()
        p = oracle.pubkey(s)
        assert pk[i].tobytes() == p
        assert sig[i].tobytes() == oracle.sign(s, p, msgs[i])


# ------------------------------------------------------------------ verify_strict
@pytest.fixture(scope="module")
def corpus():
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    return {k: d[k] for k in d.files}


def test_verify_strict_corpus(be, corpus):
    got = be.verify_strict(corpus["pk"], corpus["sig"], corpus["msg"], corpus["off"], corpus["len"])
    meta = _json("ed25519_corpus.json")
    bad = [(i, meta["categories"][corpus["cat"][i]]) for i in np.nonzero(got != corpus["strict"].astype(bool))[0]]
    assert not bad, bad[:20]


def test_verify_strict_reference_tests(be):
    """crypto_tests.rs:49-77 through the crate mirror."""
    import ntcrypto as c
    ref = _json("fixtures_reference.json")
    k = ref["keys"][3]
    pk = c.PublicKey(bytes.fromhex(k["pk"]))
    sk = c.SecretKey(bytes.fromhex(k["seed"]) + bytes.fromhex(k["pk"]))
    digest = c.sha512_digest(b"Hello, world!")
    sig = c.Signature.new(digest, sk)
    sig.verify(digest, pk)
    with pytest.raises(c.CryptoError):
        sig.verify(c.sha512_digest(b"Bad message!"), pk)


def test_verify_strict_random_vs_oracle(be, oracle):
    rng = np.random.default_rng(99)
    n = 4096
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 600, n)]
    data, off, ln = _pack(msgs)
    pk, sig = be.sign_batch(seeds, data, off, ln)
    # corrupt a third of them in assorted ways
    sig = sig.copy()
    pk = pk.copy()
    kind = rng.integers(0, 6, n)
    for i in range(n):
        if kind[i] == 1:
            sig[i, rng.integers(0, 64)] ^= 1 << rng.integers(0, 8)
        elif kind[i] == 2:
            pk[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)
    got = be.verify_strict(pk, sig, data, off, ln)
    want = oracle.verify_strict_many(pk, sig, data, off, ln, nthreads=8).astype(bool)
    assert np.array_equal(got, want)
    assert got[kind != 1].sum() > 0


def test_verify_empty(be):
    got = be.verify_strict(np.zeros((0, 32), np.uint8), np.zeros((0, 64), np.uint8), np.zeros(0, np.uint8),
                           np.zeros(0, np.uint64), np.zeros(0, np.uint64))
    assert got.shape == (0,)


# ------------------------------------------------------------------ verify_batch
def test_batch_groups_fixture(be):
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    gb, sb = be.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"], with_sig_bits=True)
    assert np.array_equal(gb, g["expect"].astype(bool))


def test_batch_reference_tests():
    """crypto_tests.rs:79-115 through the crate mirror."""
    import ntcrypto as c
    ref = _json("fixtures_reference.json")
    digest = c.sha512_digest(b"Hello, world!")
    keys = [(c.PublicKey(bytes.fromhex(k["pk"])), c.SecretKey(bytes.fromhex(k["seed"]) + bytes.fromhex(k["pk"])))
            for k in ref["keys"]]
    votes = [(pk, c.Signature.new(digest, sk)) for pk, sk in reversed(keys[1:])]
    c.Signature.verify_batch(digest, votes)
    bad = votes[:2] + [(keys[1][0], c.Signature.default())]
    with pytest.raises(c.CryptoError):
        c.Signature.verify_batch(digest, bad)


def test_batch_corpus_rule(be, corpus):
    """Each corpus entry as its own one-signature certificate (32-B messages only)."""
    sel = np.nonzero(corpus["len"] == 32)[0]
    pk = corpus["pk"][sel]
    sig = corpus["sig"][sel]
    msg32 = np.stack([corpus["msg"][int(corpus["off"][i]):int(corpus["off"][i]) + 32] for i in sel])
    gb = be.verify_batch_groups(pk, sig, np.arange(len(sel), dtype=np.uint64), np.ones(len(sel), np.uint32), msg32)
    assert np.array_equal(gb, corpus["batch_rule"][sel].astype(bool))


# ------------------------------------------------------------------ committee key cache
@pytest.mark.parametrize("bits", [16, 20, 21])
def test_keyset_corpus(be, corpus, bits, monkeypatch):
    """Every corpus key (incl. off-curve, small-order, non-canonical, mixed-order)
    as a keyset entry, through the key-comb widths (NT_KEYSET_COMB_BITS forces
    one; the 20-bit combs take 872 MB per key, the 21-bit reduced-scalar combs
    1.61 GB -- those sets hold 48 keys at a time).  At 21 bits every corpus
    scalar k is taken as k or k - L, and keys with a torsion component add
    their [L](-A) entry when k - L was used."""
    import ntcrypto
    monkeypatch.setenv("NT_KEYSET_COMB_BITS", str(bits))
    uniq, inv = np.unique(corpus["pk"], axis=0, return_inverse=True)
    inv = inv.ravel().astype(np.uint32)
    per_set = len(uniq) if bits == 16 else 48
    n = len(corpus["pk"])
    got_s = np.zeros(n, bool)
    got_c = np.zeros(n, bool)
    got_m = np.zeros(n, bool)
    want_strict = (np.arange(n) % 3) == 1      # NT_MODE_MIXED: these entries strict, the rest cofactorless
    for k0 in range(0, len(uniq), per_set):
        ks = be.keyset(uniq[k0:k0 + per_set])
        assert ks.info()[0] == bits
        sel = np.nonzero((inv >= k0) & (inv < k0 + per_set))[0]
        idx = inv[sel] - k0
        args = (corpus["sig"][sel], corpus["msg"], corpus["off"][sel], corpus["len"][sel])
        got_s[sel] = ks.verify(ntcrypto.NT_MODE_STRICT, idx, *args)
        got_c[sel] = ks.verify(ntcrypto.NT_MODE_COFACTORLESS, idx, *args)
        midx = idx | np.where(want_strict[sel], np.uint32(ntcrypto.NT_KEY_STRICT_BIT), np.uint32(0))
        got_m[sel] = ks.verify(ntcrypto.NT_MODE_MIXED, midx.astype(np.uint32), *args)
        # outside mixed mode bit 31 is just an unknown key index -> reject
        assert not ks.verify(ntcrypto.NT_MODE_STRICT, midx.astype(np.uint32) | np.uint32(1 << 31), *args).any()
        # unknown key index -> reject
        assert not ks.verify(ntcrypto.NT_MODE_STRICT, np.full(len(sel), per_set + 5, np.uint32), *args).any()
        ks.close()
    assert np.array_equal(got_s, corpus["strict"].astype(bool))
    assert np.array_equal(got_c, corpus["batch_rule"].astype(bool))
    assert np.array_equal(got_m, np.where(want_strict, corpus["strict"], corpus["batch_rule"]).astype(bool))


def test_keyset_comb_width_choice(be):
    """Without an override a committee that fits gets 21-bit reduced-scalar
    combs (12 positions of 2^20 + 65 entries and the [L](-A) entry); the size
    nt_keyset_info reports is the comb bytes of every key."""
    pks = be.sign_batch(np.arange(4 * 32, dtype=np.uint8).reshape(4, 32))
    ks = be.keyset(pks)
    bits, nbytes = ks.info()
    assert bits == 21
    assert nbytes >= 4 * (12 * ((1 << 20) + 65) + 1) * 128
    ks.close()


def test_keyset_batch_groups_fixture(be):
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    uniq, inv = np.unique(g["pk"], axis=0, return_inverse=True)
    ks = be.keyset(uniq)
    gb, sb = ks.verify_batch_groups(inv.astype(np.uint32).ravel(), g["sig"], g["first"], g["cnt"], g["msg32"],
                                    with_sig_bits=True)
    assert np.array_equal(gb, g["expect"].astype(bool))
    gb2, sb2 = be.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"], with_sig_bits=True)
    assert np.array_equal(sb, sb2)
    ks.close()


def test_keyset_committee_random_vs_oracle(be, oracle):
    rng = np.random.default_rng(3)
    nk, n = 100, 5000
    seeds = rng.integers(0, 256, (nk, 32), dtype=np.uint8)
    pks = be.sign_batch(seeds)
    ks = be.keyset(pks)
    key_idx = rng.integers(0, nk, n).astype(np.uint32)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 300, n)]
    data, off, ln = _pack(msgs)
    _, sig = be.sign_batch(seeds[key_idx], data, off, ln)
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    sig[flip, 7] ^= 0x10
    import ntcrypto
    got = ks.verify(ntcrypto.NT_MODE_STRICT, key_idx, sig, data, off, ln)
    want = oracle.verify_strict_many(pks[key_idx], sig, data, off, ln, nthreads=8).astype(bool)
    assert np.array_equal(got, want)
    assert got.sum() == (~flip).sum()
    flags = [ks.flags(i) for i in range(nk)]
    assert all(f == 1 for f in flags)
    ks.close()


@pytest.mark.timeout(560)
def test_keyset_per_lane_counts():
    """The key-cache kernel is a persistent grid.  Streamed rows (the default,
    ks_stream_plan: one row per claim, one inversion per NT_KEYSET_PER_LANE
    rows at most, a new batch when a wave's stash is full) and the chunked plan
    (NT_KEYSET_STREAM=0, ks_plan: rounds x waves chunks of base or base + 1
    rows), at 2 or 3 waves per SIMD by NT_KEYSET_WAVES or the plan (all read
    once per process).  Caps 1, 3, 5, 8, 26 and 64 with forced and automatic
    wave counts -- partial rows, several batches per wave, other inversion
    batch sizes -- give the corpus verdicts in input order, in key-grouped order
    (72k) and at ~1M signatures (subprocesses: the variables are read at first
    use)."""
    import json
    import subprocess
    import sys
    probe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_keyset_per_lane_probe.py")
    # (stream, rows per inversion, waves per SIMD, key-grouped order); sort "0" = input order at every
    # size (the streamed kernel's ballot verdict path at ~1M signatures)
    cases = [("1", 1, "", "1"), ("1", 3, "3", "1"), ("1", 8, "2", "1"), ("1", 64, "", "1"), ("1", 64, "3", "1"),
             ("1", 64, "", "0"), ("1", 5, "3", "0"),
             ("0", 1, "", "1"), ("0", 5, "2", "1"), ("0", 8, "3", "1"), ("0", 26, "2", "1"), ("0", 64, "", "1")]
    for stream, m, w, srt in cases:
        env = dict(os.environ, NT_KEYSET_PER_LANE=str(m), NT_KEYSET_COMB_BITS="16", NT_KEYSET_STREAM=stream,
                   NT_KEYSET_SORT=srt)
        env.pop("NT_KEYSET_WAVES", None)
        if w:
            env["NT_KEYSET_WAVES"] = w
        r = subprocess.run([sys.executable, probe], env=env, capture_output=True, text=True, timeout=150)
        assert r.returncode == 0, r.stderr[-2000:]
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["per_lane"] == str(m)
        bad = {k: v for k, v in res.items() if k.startswith("mismatches") and v}
        assert not bad, (m, w, bad)
        assert len([k for k in res if k.startswith("mismatches")]) == 3


@pytest.mark.gpu
def test_keyset_key_grouped_order(be, corpus, monkeypatch):
    """Key-cache launches of >= 65,536 signatures verify in key-grouped order
    (k_misc.hip: counting sort by committee index, verdict bytes scattered back
    to each signature's own index, packed into ballot words).  The corpus tiled
    to 72k signatures -- every edge case, unknown key indices, per-signature
    strictness -- must give the same verdict per signature as the corpus labels,
    and tiled certificate groups the fixture's group verdicts."""
    import ntcrypto
    monkeypatch.setenv("NT_KEYSET_COMB_BITS", "16")
    uniq, inv = np.unique(corpus["pk"], axis=0, return_inverse=True)
    inv = inv.ravel().astype(np.uint32)
    ks = be.keyset(uniq)
    reps = 200
    n0 = len(inv)
    idx = np.tile(inv, reps)
    unknown = (np.arange(n0 * reps) % 97) == 5
    idx[unknown] = len(uniq) + 3                      # not a committee key -> reject
    want_strict = (np.arange(n0 * reps) % 3) == 1
    midx = (idx | np.where(want_strict, np.uint32(ntcrypto.NT_KEY_STRICT_BIT), np.uint32(0))).astype(np.uint32)
    sig = np.tile(corpus["sig"], (reps, 1))
    off = np.tile(corpus["off"], reps)
    ln = np.tile(corpus["len"], reps)
    got = ks.verify(ntcrypto.NT_MODE_MIXED, midx, sig, corpus["msg"], off, ln)
    want = np.where(np.tile(want_strict.reshape(reps, n0)[0], reps), np.tile(corpus["strict"], reps),
                    np.tile(corpus["batch_rule"], reps)).astype(bool) & ~unknown
    assert np.array_equal(got, want)
    ks.close()
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    u2, inv2 = np.unique(g["pk"], axis=0, return_inverse=True)
    ks = be.keyset(u2)
    nsig = len(g["pk"])
    reps = -(-70000 // nsig)
    first = np.concatenate([g["first"] + r * nsig for r in range(reps)]).astype(np.uint64)
    cnt = np.tile(g["cnt"], reps)
    kidx = np.tile(inv2.astype(np.uint32).ravel(), reps)
    gb = ks.verify_batch_groups(kidx, np.tile(g["sig"], (reps, 1)), first, cnt, np.tile(g["msg32"], (reps, 1)))
    assert np.array_equal(gb, np.tile(g["expect"], reps).astype(bool))
    ks.close()


def test_verify_ragged_message_lengths(be, oracle):
    """One verify launch whose lanes hash very different message lengths (the
    k = SHA-512(R || A || M) loop runs per lane: 0 B up to 300 kB, padding
    boundaries 111/112/239/240 B around the 64-byte R || A prefix), honest and
    corrupted, against the oracle -- in strict and cofactorless mode."""
    import ntcrypto
    rng = np.random.default_rng(17)
    choices = np.array([0, 1, 47, 48, 63, 64, 111, 112, 127, 128, 175, 176, 239, 240, 1000, 65536, 300000])
    n = 2048
    lens = choices[rng.integers(0, len(choices), n)].astype(np.uint64)
    lens[rng.integers(0, n, 3)] = 300000
    off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    data = rng.integers(0, 256, int(lens.sum()) + 1, dtype=np.uint8)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = be.sign_batch(seeds, data, off, lens)
    sig = sig.copy()
    flip = rng.random(n) < 0.3
    sig[flip, 32] ^= 1
    got = be.verify_strict(pk, sig, data, off, lens)
    want = oracle.verify_strict_many(pk, sig, data, off, lens, nthreads=8).astype(bool)
    assert np.array_equal(got, want)
    assert np.array_equal(got, ~flip)
    # cofactorless (verify_batch's per-entry rule) on the device entry point,
    # which takes arbitrary messages; a sample checked one by one on the oracle
    import torch
    dev = torch.device("cuda", 0)
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         (("pk", pk), ("sig", sig), ("data", data), ("off", off.view(np.int64)), ("len", lens.view(np.int64)))}
    out = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    be.dev_verify(0, st.cuda_stream, ntcrypto.NT_MODE_COFACTORLESS, t["pk"].data_ptr(), t["sig"].data_ptr(),
                  t["data"].data_ptr(), nbytes(t["data"]), t["off"].data_ptr(), t["len"].data_ptr(), n, out.data_ptr())
    torch.cuda.synchronize(dev)
    cof = np.unpackbits(out.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(cof, ~flip)
    for i in rng.choice(n, 64, replace=False):
        m = data[int(off[i]):int(off[i] + lens[i])].tobytes()
        assert cof[i] == oracle.verify_cofactorless(pk[i].tobytes(), sig[i].tobytes(), m), int(i)


@pytest.mark.timeout(300)
def test_keyset_device_api_two_launches(be, corpus, monkeypatch):
    """More than kKsMaxPerLaunch (8M) signatures in one device-API call: the
    launcher cuts them into an 8M launch and a 0.53M one that reuse one stash
    (sized for the larger of the two streamed-row plans: 3 waves per SIMD x 45
    rows, then 2 x 7) and one key-sort scratch.  The corpus tiled to ~8.53M
    signatures in mixed mode (every edge case, per-signature strictness,
    unknown keys) must give the corpus labels everywhere."""
    import ntcrypto
    import torch
    monkeypatch.setenv("NT_KEYSET_COMB_BITS", "16")
    uniq, inv = np.unique(corpus["pk"], axis=0, return_inverse=True)
    inv = inv.ravel().astype(np.uint32)
    ks = be.keyset(uniq)
    n0 = len(inv)
    reps = -(-((8 << 20) + 530_000) // n0)
    n = n0 * reps
    i = np.arange(n)
    unknown = (i % 97) == 5
    strict = (i % 3) == 1
    idx = np.tile(inv, reps)
    idx[unknown] = len(uniq) + 3
    midx = (idx | np.where(strict, np.uint32(ntcrypto.NT_KEY_STRICT_BIT), np.uint32(0))).astype(np.uint32)
    want = np.where(strict, np.tile(corpus["strict"], reps), np.tile(corpus["batch_rule"], reps)).astype(bool)
    want &= ~unknown
    dev = torch.device("cuda", 0)
    t = {"k": torch.from_numpy(midx.view(np.int32)).to(dev),
         "sig": torch.from_numpy(np.ascontiguousarray(corpus["sig"])).to(dev).repeat(reps, 1),
         "msg": torch.from_numpy(np.ascontiguousarray(corpus["msg"])).to(dev),
         "off": torch.from_numpy(np.ascontiguousarray(corpus["off"]).view(np.int64)).to(dev).repeat(reps),
         "len": torch.from_numpy(np.ascontiguousarray(corpus["len"]).view(np.int64)).to(dev).repeat(reps)}
    out = torch.zeros((n + 63) // 64 + 1, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    ks.dev_verify(0, st.cuda_stream, ntcrypto.NT_MODE_MIXED, t["k"].data_ptr(), t["sig"].data_ptr(),
                  t["msg"].data_ptr(), nbytes(t["msg"]), t["off"].data_ptr(), t["len"].data_ptr(), n, out.data_ptr())
    st.synchronize()
    got = np.unpackbits(out.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
    assert n > (8 << 20)
    assert int((got != want).sum()) == 0
    ks.close()


def test_device_api_out_of_bounds_items(be, corpus):
    """the nt_dev_* entry points take the message buffer's
    byte size and never read outside it.  The corpus's honest entries (all
    accept) with a quarter of their offsets / lengths pushed out of the buffer
    -- past the end, 2^62 away, a length that wraps 64 bits, a slice that ends
    one byte past the end: those items are rejected by verify_strict and the key
    cache (mixed mode, strict bit set), get a zero digest and are counted by
    SHA-512, get an all-zero signature from signing; every other item is
    unchanged (verdicts, digests and signatures equal to the in-bounds run)."""
    import ntcrypto
    import torch
    dev = torch.device("cuda", 0)
    honest = np.flatnonzero(corpus["strict"].astype(bool))
    assert len(honest) >= 16
    pick = np.resize(honest, 256)
    n = len(pick)
    msg = np.ascontiguousarray(corpus["msg"])
    nbm = len(msg)
    off = corpus["off"][pick].astype(np.uint64)
    ln = corpus["len"][pick].astype(np.uint64)
    bad = np.zeros(n, bool)
    bad[3::4] = True
    boff, bln = off.copy(), ln.copy()
    kinds = [(nbm + 1, 0), (1 << 62, 8), (64, (1 << 64) - 40), (nbm - 7, 8)]
    for j, i in enumerate(np.flatnonzero(bad)):
        o, l = kinds[j % len(kinds)]
        boff[i], bln[i] = o, l
    uniq, inv = np.unique(corpus["pk"][pick], axis=0, return_inverse=True)
    ks = be.keyset(uniq)
    t = {"pk": torch.from_numpy(np.ascontiguousarray(corpus["pk"][pick])).to(dev),
         "sig": torch.from_numpy(np.ascontiguousarray(corpus["sig"][pick])).to(dev),
         "msg": torch.from_numpy(msg).to(dev),
         "k": torch.from_numpy((inv.ravel().astype(np.uint32) | np.uint32(ntcrypto.NT_KEY_STRICT_BIT)).view(np.int32)).to(dev),
         "seed": torch.from_numpy(np.resize(np.arange(32, dtype=np.uint8), (n, 32)).copy()).to(dev)}
    for name, o, l in (("good", off, ln), ("bad", boff, bln)):
        t["off_" + name] = torch.from_numpy(o.view(np.int64)).to(dev)
        t["len_" + name] = torch.from_numpy(l.view(np.int64)).to(dev)
    st = torch.cuda.Stream(dev)
    res = {}
    for name in ("good", "bad"):
        o, l = t["off_" + name].data_ptr(), t["len_" + name].data_ptr()
        v = torch.zeros(n // 64 + 1, dtype=torch.int64, device=dev)
        kv = torch.zeros(n // 64 + 1, dtype=torch.int64, device=dev)
        dg = torch.full((n, 32), 0xAB, dtype=torch.uint8, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        spk = torch.empty((n, 32), dtype=torch.uint8, device=dev)
        ssig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)
        with torch.cuda.stream(st):
            be.dev_verify(0, st.cuda_stream, ntcrypto.NT_MODE_STRICT, t["pk"].data_ptr(), t["sig"].data_ptr(),
                          t["msg"].data_ptr(), nbm, o, l, n, v.data_ptr())
            ks.dev_verify(0, st.cuda_stream, ntcrypto.NT_MODE_MIXED, t["k"].data_ptr(), t["sig"].data_ptr(),
                          t["msg"].data_ptr(), nbm, o, l, n, kv.data_ptr())
            be.dev_sha512(0, st.cuda_stream, t["msg"].data_ptr(), nbm, o, l, n, dg.data_ptr(), d_bad=cnt.data_ptr())
            be.dev_sign(0, st.cuda_stream, t["seed"].data_ptr(), t["msg"].data_ptr(), nbm, o, l, n, spk.data_ptr(),
                        ssig.data_ptr())
        st.synchronize()
        res[name] = dict(v=np.unpackbits(v.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool),
                         kv=np.unpackbits(kv.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool),
                         dg=dg.cpu().numpy(), cnt=int(cnt.item()), pk=spk.cpu().numpy(), sig=ssig.cpu().numpy())
    ks.close()
    g, b = res["good"], res["bad"]
    assert g["v"].all() and g["kv"].all() and g["cnt"] == 0
    for i in range(n):
        o, l = int(off[i]), int(ln[i])
        assert g["dg"][i].tobytes() == hashlib.sha512(msg[o:o + l].tobytes()).digest()[:32], i
    assert np.array_equal(b["v"], ~bad) and np.array_equal(b["kv"], ~bad)
    assert b["cnt"] == int(bad.sum())
    assert not b["dg"][bad].any() and np.array_equal(b["dg"][~bad], g["dg"][~bad])
    assert np.array_equal(b["pk"], g["pk"])
    assert not b["sig"][bad].any() and np.array_equal(b["sig"][~bad], g["sig"][~bad])


@pytest.mark.parametrize("reps", [1, 1400])
def test_keyset_device_groups_fused(be, monkeypatch, reps):
    """nt_dev_ed25519_verify_keyset_groups: the key-cache launch ANDs each
    certificate group's verdicts in its kernel epilogue (no pack / group-AND
    launch).  The golden groups fixture (0..67 votes, corrupted s, all-zero
    vote, torsion-shifted R) tiled once (input-order launch) and 1,400 times
    (~75k signatures: key-grouped order, atomic verdict bits), plus signatures
    in no group at the end (header signatures of a mixed launch), empty groups
    and a group that reaches past the call's signatures (rejects): group and
    signature words equal nt_dev_ed25519_verify_keyset + nt_dev_group_and and
    the fixture's verdicts."""
    import ntcrypto
    import torch
    monkeypatch.setenv("NT_KEYSET_COMB_BITS", "16")
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    uniq, inv = np.unique(g["pk"], axis=0, return_inverse=True)
    ks = be.keyset(uniq)
    nsig = len(g["pk"])
    first = np.concatenate([g["first"] + r * nsig for r in range(reps)]).astype(np.uint64)
    cnt = np.tile(g["cnt"], reps).astype(np.uint32)
    G = len(cnt)
    kidx = np.tile(inv.astype(np.uint32).ravel(), reps)
    sig = np.tile(g["sig"], (reps, 1))
    msg32 = np.tile(g["msg32"], (reps, 1))
    goff = np.concatenate([np.full(int(c), 32 * gi, np.uint64) for gi, c in enumerate(cnt)])
    assert len(goff) == nsig * reps
    # 40 extra signatures in no group (copies of the first ones), then two more groups:
    # an empty one and one reaching past the call's signatures
    n = nsig * reps + 40
    kidx = np.concatenate([kidx, kidx[:40]])
    sig = np.concatenate([sig, sig[:40]])
    goff = np.concatenate([goff, goff[:40]])
    first = np.concatenate([first, [n, n - 3]]).astype(np.uint64)
    cnt = np.concatenate([cnt, [0, 5]]).astype(np.uint32)
    G2 = G + 2
    # group first indices must be non-decreasing: the last group starts at n - 3 < n
    first[-2] = n - 3
    dev = torch.device("cuda", 0)
    t = {"k": torch.from_numpy(kidx.view(np.int32)).to(dev), "sig": torch.from_numpy(sig).to(dev),
         "msg": torch.from_numpy(msg32.reshape(-1)).to(dev), "off": torch.from_numpy(goff.view(np.int64)).to(dev),
         "len": torch.full((n,), 32, dtype=torch.int64, device=dev),
         "first": torch.from_numpy(first.view(np.int64)).to(dev), "cnt": torch.from_numpy(cnt.view(np.int32)).to(dev)}
    w1 = torch.full(((n + 63) // 64 + 1,), -1, dtype=torch.int64, device=dev)   # garbage: the call owns the words
    gw1 = torch.full(((G2 + 63) // 64 + 1,), 0x5A5A, dtype=torch.int64, device=dev)
    w2 = torch.zeros_like(w1)
    gw2 = torch.zeros_like(gw1)
    st = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    args = (0, st.cuda_stream, ntcrypto.NT_MODE_COFACTORLESS, t["k"].data_ptr(), t["sig"].data_ptr(), t["msg"].data_ptr(),
            nbytes(t["msg"]), t["off"].data_ptr(), t["len"].data_ptr(), n)
    ks.dev_verify_groups(*args, t["first"].data_ptr(), t["cnt"].data_ptr(), G2, w1.data_ptr(), gw1.data_ptr())
    ks.dev_verify(*args, w2.data_ptr())
    be.dev_group_and(0, st.cuda_stream, t["first"].data_ptr(), t["cnt"].data_ptr(), G2, w2.data_ptr(), gw2.data_ptr())
    st.synchronize()
    words = (n + 63) // 64
    s1 = np.unpackbits(w1.cpu().numpy()[:words].view(np.uint8), bitorder="little")[:n].astype(bool)
    s2 = np.unpackbits(w2.cpu().numpy()[:words].view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(s1, s2)
    gws = (G2 + 63) // 64
    b1 = np.unpackbits(gw1.cpu().numpy()[:gws].view(np.uint8), bitorder="little")
    b2 = np.unpackbits(gw2.cpu().numpy()[:gws].view(np.uint8), bitorder="little")
    assert np.array_equal(b1[:G2], b2[:G2])
    assert not b1[G2:].any()  # bits past the last group stay clear
    assert np.array_equal(b1[:G], np.tile(g["expect"], reps).astype(bool))
    # the last group reaches 2 signatures past n: rejected whatever its signatures' verdicts
    assert not b1[G2 - 1]
    ks.close()
