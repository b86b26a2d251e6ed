"""Multi-device sharding of the host entry points, exercised on one GPU by a
context that lists the same ordinal several times (nt_init_devices): every
shard gets its own stream, tables and workspace, exactly as on 8 GPUs."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pair():
    import ntcrypto
    one = ntcrypto.Backend(devices=[0])
    three = ntcrypto.Backend(devices=[0, 0, 0])
    assert three.num_devices == 3
    yield one, three
    one.close()
    three.close()


def _pack(msgs):
    ln = np.array([len(m) for m in msgs], np.uint64)
    off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.uint64)
    return np.frombuffer(b"".join(msgs), np.uint8), off, ln


def test_sharded_verify_strict_matches(pair):
    one, three = pair
    rng = np.random.default_rng(21)
    n = 1000  # not a multiple of 64 or 3: ragged shards
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 200, n)]
    data, off, ln = _pack(msgs)
    pk1, sig1 = one.sign_batch(seeds, data, off, ln)
    pk3, sig3 = three.sign_batch(seeds, data, off, ln)
    assert np.array_equal(pk1, pk3) and np.array_equal(sig1, sig3)
    sig1 = sig1.copy()
    sig1[::5, 3] ^= 1
    assert np.array_equal(one.verify_strict(pk1, sig1, data, off, ln), three.verify_strict(pk1, sig1, data, off, ln))
    d1 = one.sha512_trunc32(data, off, ln)
    assert np.array_equal(d1, three.sha512_trunc32(data, off, ln))


def test_sharded_batch_groups_and_keyset(pair):
    one, three = pair
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    a = one.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"], with_sig_bits=True)
    b = three.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"], with_sig_bits=True)
    assert np.array_equal(a[0], g["expect"].astype(bool))
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    uniq, inv = np.unique(g["pk"], axis=0, return_inverse=True)
    ks = three.keyset(uniq)
    c = ks.verify_batch_groups(inv.astype(np.uint32).ravel(), g["sig"], g["first"], g["cnt"], g["msg32"])
    assert np.array_equal(c, g["expect"].astype(bool))
    ks.close()


def test_keyset_launch_chunking(pair):
    """More than 8 Mi signatures through the key cache: the launcher splits them
    into launches of 8 Mi that reuse one per-lane stash; verdicts at the chunk
    seam and at the ragged end must come out right."""
    one, _ = pair
    rng = np.random.default_rng(5)
    seeds = rng.integers(0, 256, (4, 32), dtype=np.uint8)
    msg = rng.integers(0, 256, 4 * 32, dtype=np.uint8)
    pk, sig = one.sign_batch(seeds, msg, np.arange(4, dtype=np.uint64) * 32, np.full(4, 32, np.uint64))
    ks = one.keyset(pk)
    n = (8 << 20) + 1000
    key = (np.arange(n) % 4).astype(np.uint32)
    sigs = np.ascontiguousarray(sig[key])
    off = (key.astype(np.uint64) * 32)
    ln = np.full(n, 32, np.uint64)
    bad = np.array([0, 5, (8 << 20) - 1, 8 << 20, (8 << 20) + 1, n - 1])
    sigs[bad, 7] ^= 0x40
    expect = np.ones(n, bool)
    expect[bad] = False
    got = ks.verify(0, key, sigs, msg, off, ln)
    ks.close()
    assert np.array_equal(got, expect)
