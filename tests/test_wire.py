"""SURVEY §8(f).1 + (f).2: the bincode wire codec of PrimaryMessage and the
batched primary::Core sanitizer of the C++ mirror, against an independent
Python model (tests/_wire.py) and the CPU oracle.

CPU: codec round trips, canonicalisation (BTreeMap / BTreeSet semantics),
rejection of malformed bytes, the header digest preimage.
GPU: Core::ingest over a drained batch of headers, votes, certificates, a
CertificatesRequest and garbage, every DagError outcome, with and without the
committee key cache, vs. the model's per-message verdicts.
"""
import os
import random
import struct
import sys

import numpy as np
import pytest

import _wire as W

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "narwhal-tusk_amd"))
from ntcrypto import narwhal as N  # noqa: E402


def _rb(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def _random_objects(rng, count):
    keys = [_rb(rng, 32) for _ in range(6)]
    out = []
    for i in range(count):
        kind = i % 4
        if kind == 0:
            h = W.Header(rng.choice(keys), rng.getrandbits(64), {_rb(rng, 32): rng.getrandbits(32)
                                                                 for _ in range(rng.randrange(0, 5))},
                         {_rb(rng, 32) for _ in range(rng.randrange(0, 5))}, sig=_rb(rng, 64))
            out.append(h)
        elif kind == 1:
            out.append(W.Vote(_rb(rng, 32), rng.getrandbits(64), rng.choice(keys), rng.choice(keys), _rb(rng, 64)))
        elif kind == 2:
            h = W.Header(rng.choice(keys), rng.getrandbits(20), {_rb(rng, 32): 0}, {_rb(rng, 32)}, sig=_rb(rng, 64))
            out.append(W.Certificate(h, [(rng.choice(keys), _rb(rng, 64)) for _ in range(rng.randrange(0, 8))]))
        else:
            out.append(([_rb(rng, 32) for _ in range(rng.randrange(0, 4))], rng.choice(keys)))
    return out


def test_wire_roundtrip_random():
    rng = random.Random(11)
    for obj in _random_objects(rng, 200):
        m = W.message(obj)
        r = N.wire_reencode(m)
        assert r is not None and r[0] == m and r[1] == len(m)


def test_wire_trailing_bytes_allowed():
    m = W.message(_random_objects(random.Random(3), 1)[0])
    r = N.wire_reencode(m + b"\x00\x01junk")
    assert r is not None and r[0] == m and r[1] == len(m)


def test_wire_btree_semantics():
    """payload entries and parents in any wire order / with repeats decode to the
    BTreeMap / BTreeSet the reference builds (last value wins for a repeated key)."""
    rng = random.Random(5)
    author, d1, d2, p1, p2 = (_rb(rng, 32) for _ in range(5))
    body = W._str(W.b64(author)) + struct.pack("<Q", 9)
    body += struct.pack("<Q", 3) + d2 + struct.pack("<I", 1) + d1 + struct.pack("<I", 2) + d2 + struct.pack("<I", 3)
    body += struct.pack("<Q", 3) + p2 + p1 + p2
    idd, sig = _rb(rng, 32), _rb(rng, 64)
    wire = struct.pack("<I", 0) + body + idd + sig
    canon = W.Header(author, 9, {d1: 2, d2: 3}, {p1, p2}, id_=idd, sig=sig)
    assert N.wire_reencode(wire)[0] == W.message(canon)
    assert N.wire_header_preimage(wire) == canon.preimage()


def test_wire_rejects_malformed():
    rng = random.Random(7)
    objs = _random_objects(rng, 8)
    for obj in objs:
        m = W.message(obj)
        for cut in range(len(m)):  # every truncation
            assert N.wire_reencode(m[:cut]) is None, (type(obj), cut)
    key = _rb(rng, 32)
    vote = W.Vote(_rb(rng, 32), 1, key, key, _rb(rng, 64))
    good = W.message(vote)
    assert N.wire_reencode(good) is not None
    bad_tag = struct.pack("<I", 4) + good[4:]
    assert N.wire_reencode(bad_tag) is None
    b64 = W.b64(key)
    pos = good.index(b64)

    def with_key(s):
        return good[:pos - 8] + struct.pack("<Q", len(s)) + s + good[pos + len(b64):]

    assert N.wire_reencode(with_key(b64)) is not None
    assert N.wire_reencode(with_key(b64[:-4] + b"!!!=")) is None          # invalid symbol
    assert N.wire_reencode(with_key(W.b64(key[:31]))) is None             # decodes to < 32 bytes
    assert N.wire_reencode(with_key(b64[:-1])) is None                    # bad length
    tail = b64[-2:-1]                                                      # non-zero unused bits
    alt = bytes([b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"[
        (b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/".index(tail) | 1)]])
    assert N.wire_reencode(with_key(b64[:-2] + alt + b"=")) is None
    assert N.wire_reencode(with_key(b"\xff" * 44)) is None                # not UTF-8
    longer = W.b64(key + b"\x07\x08\x09")                                  # >= 32 bytes: first 32 kept
    r = N.wire_reencode(with_key(longer))
    assert r is not None and r[0] == good
    huge = struct.pack("<I", 2) + W.Header(key, 1, {}, set()).encode() + struct.pack("<Q", 1 << 60)
    assert N.wire_reencode(huge) is None


# ------------------------------------------------------------------ GPU: batched Core
def _scenario(orc, rng, with_objs=False):
    seeds = [bytes([i + 1]) * 32 for i in range(7)]
    keys = [orc.pubkey(s) for s in seeds]
    sk = dict(zip(keys, seeds))
    stakes = [1, 1, 1, 1, 2, 1, 0]  # the last authority has no voting rights
    nworkers = [2] * 7
    com = W.Committee(keys, stakes, nworkers)
    stranger_seed = b"\x55" * 32
    stranger = orc.pubkey(stranger_seed)
    sk[stranger] = stranger_seed

    def sign(pk, d):
        return orc.sign(sk[pk], pk, d)

    def header(author, rnd, nworker=0, bad_sig=False, bad_id=False):
        h = W.Header(author, rnd, {_rb(rng, 32): nworker, _rb(rng, 32): 0}, {_rb(rng, 32) for _ in range(3)})
        if bad_id:
            h.id = _rb(rng, 32)
        h.sig = sign(author, h.id)
        if bad_sig:
            h.sig = h.sig[:40] + bytes([h.sig[40] ^ 1]) + h.sig[41:]
        return h

    gc_round, cur_round = 5, 8
    cur = header(keys[0], cur_round)

    def vote(author, rnd=cur_round, target=cur, bad_sig=False):
        v = W.Vote(target.id, rnd, target.author, author)
        v.sig = sign(author, v.digest())
        if bad_sig:
            v.sig = v.sig[:33] + bytes([v.sig[33] ^ 4]) + v.sig[34:]
        return v

    def cert(h, voters, bad_vote=None):
        c = W.Certificate(h, [])
        d = c.digest()
        for pk in voters:
            s = sign(pk, d)
            if bad_vote is not None and pk == bad_vote:
                s = bytes(32) + s[32:]
            c.votes.append((pk, s))
        return c

    objs = [
        header(keys[1], 9), header(keys[2], 4), header(keys[1], 9, bad_sig=True),
        header(keys[1], 9, bad_id=True), header(stranger, 9), header(keys[6], 9), header(keys[3], 9, nworker=5),
        vote(keys[2]), vote(keys[3], rnd=7), vote(keys[4], target=header(keys[1], cur_round)),
        vote(stranger), vote(keys[6]), vote(keys[5], bad_sig=True), vote(keys[1], rnd=9),
        cert(header(keys[2], 9), keys[:5]), cert(header(keys[2], 3), keys[:5]),
        cert(W.Header(keys[3], 0, {}, set(), id_=bytes(32)), []),                 # genesis
        cert(header(keys[2], 9, bad_sig=True), keys[:5]), cert(header(keys[2], 9), keys[:3]),
        cert(header(keys[2], 9), keys[:4] + [keys[1]]), cert(header(keys[2], 9), keys[:4] + [stranger]),
        cert(header(keys[2], 9), keys[:5], bad_vote=keys[3]), cert(header(keys[5], 10), keys[1:6]),
        ([_rb(rng, 32)], keys[1]),
        # header signature AND quorum both bad: Header::verify runs first, so
        # InvalidSignature (messages.rs:194 before :199-211), not the quorum error
        cert(header(keys[2], 9, bad_sig=True), keys[:3]),
        cert(header(keys[2], 9, bad_sig=True), keys[:4] + [keys[1]]),
        cert(header(keys[2], 9, bad_sig=True), keys[:4] + [stranger]),
    ]
    assert [W.model_sanitize(com, gc_round, cur, o, lambda d, pk, s: orc.verify_strict(pk, s, d), None)
            for o in objs[-3:]] == [W.INVALID_SIGNATURE] * 3
    wires = [W.message(o) for o in objs] + [b"\x02\x00\x00\x00garbage", b""]
    # a valid header whose payload entries arrive in descending order (non-canonical
    # bytes: the decoder's BTreeMap sorts them, so the id still matches)
    h = header(keys[3], 9)
    body = h.encode()
    a = 8 + 44 + 8 + 8
    ents = [body[a + 36 * k:a + 36 * (k + 1)] for k in range(len(h.payload))]
    wires.append(W.message(h)[:4] + body[:a] + b"".join(ents[::-1]) + body[a + 36 * len(ents):])
    objs = objs + [None, None, h]
    strict = lambda d, pk, s: orc.verify_strict(pk, s, d)
    batch = lambda d, votes: orc.verify_batch([v[0] for v in votes], [v[1] for v in votes], d)
    expect = [W.model_sanitize(com, gc_round, cur, o, strict, batch) if o is not None else W.SERIALIZATION_ERROR
              for o in objs]
    if with_objs:
        return keys, stakes, nworkers, gc_round, cur, wires, expect, objs
    return keys, stakes, nworkers, gc_round, cur, wires, expect


@pytest.mark.gpu
@pytest.mark.parametrize("use_keyset", [True, False])
def test_core_ingest_matches_model(use_keyset):
    from _oracle import load
    orc = load()
    rng = random.Random(2024)
    keys, stakes, nworkers, gc_round, cur, wires, expect, objs = _scenario(orc, rng, with_objs=True)
    # every outcome is exercised
    assert set(expect) == set(range(11))
    core = N.Core(np.frombuffer(b"".join(keys), np.uint8), stakes, nworkers, gc_round, W.message(cur), use_keyset)
    try:
        names = N.DAG_ERRORS
        for general in (False, True):  # SoA fast path and the object-model path
            got, _ = core.ingest(*N.pack(wires), threads=3, general=general)
            assert [names[c] for c in got] == [names[c] for c in expect], general
        got = core.ingest_pipelined(*N.pack(wires), threads=2, chunk=5)  # two chunks in flight
        assert [names[c] for c in got] == [names[c] for c in expect]
        if use_keyset:
            # certificates parsed and checked on the GPU (nt_certificates_ingest), the
            # rest (headers, votes, a request, garbage, non-canonical bytes) on the host
            got, host = core.ingest(*N.pack(wires), threads=3, device=True)
            assert [names[c] for c in got] == [names[c] for c in expect]
            ncert = sum(isinstance(o, W.Certificate) for o in objs)
            # every certificate in canonical form decided on the device; the two with a
            # non-committee voter key (serde may still decode it) and the non-certificates
            # go to the host decoder
            assert host == len(wires) - ncert + 2
        # the same messages one at a time give the same verdicts
        for w, e in zip(wires, expect):
            g, _ = core.ingest(*N.pack([w]), threads=1)
            assert names[g[0]] == names[e]
    finally:
        core.close()


@pytest.mark.gpu
def test_core_genesis_certificates():
    """With gc_round 0 the genesis certificate of a committee member is accepted
    without signatures (messages.rs:191); a non-member's is not genesis."""
    from _oracle import load
    orc = load()
    keys = [orc.pubkey(bytes([i + 1]) * 32) for i in range(4)]
    core = N.Core(np.frombuffer(b"".join(keys), np.uint8), [1] * 4, [1] * 4, 0, None, True)
    try:
        gen = W.Certificate(W.Header(keys[2], 0, {}, set(), id_=bytes(32)), [])
        other = W.Certificate(W.Header(orc.pubkey(b"\x77" * 32), 0, {}, set(), id_=bytes(32)), [])
        got, _ = core.ingest(*N.pack([W.message(gen), W.message(other)]))
        assert [N.DAG_ERRORS[c] for c in got] == ["Ok", "InvalidHeaderId"]
    finally:
        core.close()


def test_wire_decoder_fuzz():
    """Untrusted network input: random mutations, truncations, splices and
    garbage never crash the decoder, and whatever decodes re-encodes to a
    canonical form that is a fixed point (decode(encode(m)) == m)."""
    rng = random.Random(1234)
    seeds = [W.message(o) for o in _random_objects(rng, 40)]
    ok = 0
    for it in range(6000):
        m = bytearray(rng.choice(seeds))
        op = it % 5
        if op == 0:                       # flip random bytes
            for _ in range(rng.randrange(1, 6)):
                m[rng.randrange(len(m))] ^= 1 << rng.randrange(8)
        elif op == 1:                     # overwrite a length / count field region with big values
            p = rng.randrange(max(1, len(m) - 8))
            m[p:p + 8] = struct.pack("<Q", rng.choice([0, 1, 44, 45, 1 << 32, (1 << 64) - 1, rng.getrandbits(64)]))
        elif op == 2:                     # truncate
            m = m[:rng.randrange(len(m))]
        elif op == 3:                     # splice two messages
            o = rng.choice(seeds)
            m = m[:rng.randrange(len(m))] + o[rng.randrange(len(o)):]
        else:                             # garbage with a valid tag
            m = bytearray(struct.pack("<I", rng.randrange(5)) + bytes(rng.getrandbits(8) for _ in range(rng.randrange(200))))
        r = N.wire_reencode(bytes(m))
        if r is None:
            continue
        ok += 1
        canon = r[0]
        r2 = N.wire_reencode(canon)
        assert r2 is not None and r2[0] == canon and r2[1] == len(canon)
    assert ok > 100  # the mutations still leave many decodable messages


@pytest.mark.gpu
def test_core_soa_vs_general_fuzz():
    """The SoA fast path (flat decode, key lookup by base64 text) and the
    object-model path give identical DagErrors on mutated wire messages
    (flipped bytes in keys, counts, digests and signatures; truncations)."""
    from _oracle import load
    orc = load()
    rng = random.Random(77)
    keys, stakes, nworkers, gc_round, cur, wires, _ = _scenario(orc, random.Random(2024))
    core = N.Core(np.frombuffer(b"".join(keys), np.uint8), stakes, nworkers, gc_round, W.message(cur), True)
    try:
        batch = []
        for it in range(3000):
            m = bytearray(rng.choice(wires[:24]))
            if not m:
                continue
            if it % 3 == 0:
                m[rng.randrange(len(m))] ^= 1 << rng.randrange(8)
            elif it % 3 == 1:
                m = m[:rng.randrange(1, len(m) + 1)]
            batch.append(bytes(m))
        a, _ = core.ingest(*N.pack(batch), threads=4)
        b, _ = core.ingest(*N.pack(batch), threads=4, general=True)
        assert np.array_equal(a, b), [(i, N.DAG_ERRORS[x], N.DAG_ERRORS[y]) for i, (x, y) in enumerate(zip(a, b))
                                      if x != y][:10]
        c, host = core.ingest(*N.pack(batch), threads=4, device=True)  # GPU wire parsing
        assert np.array_equal(a, c), [(i, N.DAG_ERRORS[x], N.DAG_ERRORS[y]) for i, (x, y) in enumerate(zip(a, c))
                                      if x != y][:10]
        assert host < len(batch)
        assert len(set(a.tolist())) >= 6
    finally:
        core.close()


def _cert_batch(orc, rng, nk, G, quorum):
    """G certificates of an nk-key committee as wire bytes, with a mix of
    corruptions in the bytes the device parser reads: signatures, header ids,
    payload / parent order, worker ids, vote keys, counts, truncations."""
    seeds = [bytes([i + 1, 7]) * 16 for i in range(nk)]
    keys = [orc.pubkey(s) for s in seeds]
    sk = dict(zip(keys, seeds))
    wires = []
    for g in range(G):
        author = keys[rng.randrange(nk)]
        h = W.Header(author, 10 + rng.randrange(5), {_rb(rng, 32): rng.randrange(2) for _ in range(rng.randrange(0, 6))},
                     {_rb(rng, 32) for _ in range(rng.randrange(0, 5))})
        h.sig = orc.sign(sk[author], author, h.id)
        c = W.Certificate(h, [])
        d = c.digest()
        for pk in rng.sample(keys, quorum + rng.randrange(0, 2)):
            c.votes.append((pk, orc.sign(sk[pk], pk, d)))
        m = bytearray(W.message(c))
        k = g % 10
        if k == 1:                                   # a vote signature
            m[-1 - rng.randrange(64)] ^= 1 << rng.randrange(8)
        elif k == 2:                                 # anything
            m[rng.randrange(len(m))] ^= 1 << rng.randrange(8)
        elif k == 3:                                 # truncated
            m = m[:rng.randrange(1, len(m))]
        elif k == 4 and len(c.votes) > 1:            # a repeated voter
            v = c.votes[0]
            c.votes[1] = v
            m = bytearray(W.message(c))
        elif k == 5:                                 # worker id the author does not have
            h.payload = {_rb(rng, 32): 7}
            h.id = h.digest()
            h.sig = orc.sign(sk[author], author, h.id)
            c2 = W.Certificate(h, c.votes)
            m = bytearray(W.message(c2))
        wires.append(bytes(m))
    return keys, wires


@pytest.mark.gpu
def test_core_device_ingest_many_chunks(monkeypatch):
    """nt_certificates_ingest over 1,200 certificates of a 10-key committee in
    chunks of 128 messages (several chunks in flight on two streams), with a
    corruption mix: the same DagError per message as the host SoA path."""
    from _oracle import load
    orc = load()
    rng = random.Random(5150)
    nk, quorum = 10, 7
    keys, wires = _cert_batch(orc, rng, nk, 1200, quorum)
    monkeypatch.setenv("NT_INGEST_CHUNK", "128")
    core = N.Core(np.frombuffer(b"".join(keys), np.uint8), [1] * nk, [2] * nk, 9, None, True)
    try:
        a, _ = core.ingest(*N.pack(wires), threads=4)
        c, host = core.ingest(*N.pack(wires), threads=4, device=True)
        diff = [(i, N.DAG_ERRORS[x], N.DAG_ERRORS[y]) for i, (x, y) in enumerate(zip(a, c)) if x != y]
        assert not diff, diff[:10]
        assert host < len(wires) // 3  # the bulk is decided on the device
        counts = {N.DAG_ERRORS[x]: int((a == x).sum()) for x in set(a.tolist())}
        assert counts.get("Ok", 0) > 500 and counts.get("InvalidSignature", 0) > 100, counts
        assert len(counts) >= 5, counts
    finally:
        core.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_core_device_ingest_real_shape_vs_model(monkeypatch):
    """Core::ingest_device at config 3's real shape -- an
    n = 100 committee (quorum 67), 10,000 wire certificates with 32 payload
    digests, 67 parents and 67-68 votes each (~11 KB per message) -- against
    tests/_wire.py's model_sanitize driven by the CPU ORACLE's signature
    verdicts (messages.rs:189-215, core.rs:338-346, primary.rs:225-244), not
    against the host decoder.  Every error kind appears: forged votes, an
    all-zero vote signature (crypto_tests.rs:96-115), repeated voters, voters
    outside the committee or without stake, unknown and zero-stake authors,
    bad header ids, worker ids the author does not have, bad header
    signatures, too few votes, truncations, genesis certificates and rounds
    below the GC round.  The signatures come from the GPU signer (pinned to
    the oracle elsewhere); every verdict the model needs comes from the oracle."""
    import hashlib
    import ntcrypto
    from _oracle import load
    orc = load()
    rng = random.Random(424242)
    nk, G, gc_round = 100, 10_000, 50
    be = ntcrypto.Backend(device=0)
    try:
        seeds = np.stack([np.frombuffer(hashlib.sha512(b"nt-ingest-key" + struct.pack("<Q", i)).digest()[:32],
                                        np.uint8) for i in range(nk + 1)])
        pks = be.sign_batch(seeds)
        keys = [pks[i].tobytes() for i in range(nk)]
        stranger = pks[nk].tobytes()                      # a key outside the committee
        stakes = [1] * nk
        stakes[nk - 1] = 0                                # an authority without voting rights
        com = W.Committee(keys, stakes, [1] * nk)         # one worker (id 0) per authority
        quorum = com.quorum()
        assert quorum == 67                               # 2 * 99 // 3 + 1 (stake 99 in total)
        kidx = {k: i for i, k in enumerate(keys)}
        kidx[stranger] = nk
        kinds = [g % 24 for g in range(G)]               # 0 and 15..23: valid certificates
        rng.shuffle(kinds)
        certs, tasks = [], []   # tasks: (key index, message) to sign on the GPU
        for g in range(G):
            k = kinds[g]
            author = keys[rng.randrange(nk - 1)]
            if k == 11:
                author = stranger
            elif k == 12:
                author = keys[nk - 1]
            rnd = gc_round + rng.randrange(0, 5) if k != 8 else gc_round - 1 - rng.randrange(3)
            payload = {_rb(rng, 32): 0 for _ in range(32)}
            if k == 5:
                payload[_rb(rng, 32)] = 1                 # a worker id the author does not have
            h = W.Header(author, rnd, payload, {_rb(rng, 32) for _ in range(67)})
            if k == 4:
                h.id = _rb(rng, 32)
            if k == 7:                                    # genesis: round 0, zero id, no votes
                h = W.Header(keys[rng.randrange(nk)], 0, {}, set(), id_=bytes(32))
                certs.append(W.Certificate(h, []))
                continue
            tasks.append((kidx[author], h.id))
            voters = rng.sample(keys[:nk - 1], quorum + rng.randrange(0, 2))
            if k == 9:
                voters = voters[:quorum - 1]
            elif k == 2:
                voters[5] = voters[1]                     # a repeated voter
            elif k == 3:
                voters[7] = stranger
            elif k == 13:
                voters[3] = keys[nk - 1]
            c = W.Certificate(h, [(v, None) for v in voters])
            d = c.digest()
            for v in voters:
                tasks.append((kidx[v], d))
            certs.append(c)
        # GPU-sign every header id and vote digest, then fill the signatures in
        msg = np.frombuffer(b"".join(m for _, m in tasks), np.uint8)
        _, sig = be.sign_batch(seeds[[i for i, _ in tasks]], msg, np.arange(len(tasks), dtype=np.uint64) * 32,
                               np.full(len(tasks), 32, np.uint64))
        t = 0
        for g, c in enumerate(certs):
            if not c.votes and c.header.round == 0:
                continue
            c.header.sig = sig[t].tobytes()
            t += 1
            c.votes = [(v, sig[t + j].tobytes()) for j, (v, _) in enumerate(c.votes)]
            t += len(c.votes)
            k = kinds[g]
            if k == 1:                                    # a forged vote
                j = rng.randrange(len(c.votes))
                s = bytearray(c.votes[j][1])
                s[rng.randrange(64)] ^= 1 << rng.randrange(8)
                c.votes[j] = (c.votes[j][0], bytes(s))
            elif k == 10:                                 # a forged header signature
                s = bytearray(c.header.sig)
                s[rng.randrange(64)] ^= 1 << rng.randrange(8)
                c.header.sig = bytes(s)
            elif k == 14:                                 # Signature::default() as a vote
                c.votes[9] = (c.votes[9][0], bytes(64))
        wires = []
        for g, c in enumerate(certs):
            m = W.message(c)
            if kinds[g] == 6:
                m = m[:rng.randrange(1, len(m))]          # truncated on the wire
            wires.append(m)
        # the oracle's verdict for every signature the model can ask about
        hs = [c for g, c in enumerate(certs) if kinds[g] != 6 and c.votes]
        hpk = np.stack([np.frombuffer(c.header.author, np.uint8) for c in hs])
        hsig = np.stack([np.frombuffer(c.header.sig, np.uint8) for c in hs])
        hmsg = np.frombuffer(b"".join(c.header.id for c in hs), np.uint8)
        sv = orc.verify_strict_many(hpk, hsig, hmsg, np.arange(len(hs), dtype=np.uint64) * 32,
                                    np.full(len(hs), 32, np.uint64), nthreads=16)
        strict_v = {(c.header.id, c.header.author, c.header.sig): bool(v) for c, v in zip(hs, sv)}
        cnt = np.array([len(c.votes) for c in hs], np.uint32)
        first = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
        vpk = np.stack([np.frombuffer(pk, np.uint8) for c in hs for pk, _ in c.votes])
        vsig = np.stack([np.frombuffer(s, np.uint8) for c in hs for _, s in c.votes])
        dig = np.stack([np.frombuffer(c.digest(), np.uint8) for c in hs])
        bv, _ = orc.verify_batch_groups(vpk, vsig, first, cnt, dig, nthreads=16)
        batch_v = {c.digest(): bool(v) for c, v in zip(hs, bv)}
        names = N.DAG_ERRORS
        # twice: at GC round 50 (rounds 47-49 are TooOld, so is every genesis
        # certificate: sanitize_certificate's round filter runs before
        # Certificate::verify) and at GC round 0 (genesis accepted, core.rs:339-346)
        seen = set()
        for gc in (gc_round, 0):
            expect = [W.model_sanitize(com, gc, None, c, lambda d, pk, s: strict_v[(d, pk, s)],
                                       lambda d, votes: batch_v[d]) if kinds[g] != 6 else W.SERIALIZATION_ERROR
                      for g, c in enumerate(certs)]
            seen |= {names[e] for e in expect}
            core = N.Core(np.frombuffer(b"".join(keys), np.uint8), stakes, [1] * nk, gc, None, True)
            try:
                got, host = core.ingest(*N.pack(wires), threads=8, device=True)
            finally:
                core.close()
            diff = [(g, kinds[g], names[x], names[y]) for g, (x, y) in enumerate(zip(got, expect)) if x != y]
            assert not diff, (gc, diff[:10])
            # the device decides every certificate in canonical form with committee keys;
            # truncated messages (kind 6) and the ones naming a stranger (3, 11) go to the host
            routed = sum(1 for k in kinds if k in (3, 6, 11))
            print("gc_round %d: host_decided %d of %d (truncated / stranger keys: %d); verdicts %s"
                  % (gc, host, G, routed, {names[x]: int((np.array(expect) == x).sum()) for x in set(expect)}))
            assert host <= routed
            assert sum(e == W.OK for e in expect) > G // 4
            if gc == 0:
                assert all(expect[g] == W.OK for g in range(G) if kinds[g] == 7)  # genesis
        assert seen == {"Ok", "InvalidSignature", "InvalidHeaderId", "MalformedHeader", "UnknownAuthority",
                        "AuthorityReuse", "CertificateRequiresQuorum", "TooOld", "SerializationError"}, seen
    finally:
        be.close()
