"""Multi-device sharding of the host entry points, exercised on one GPU by a
context that lists the same ordinal several times (nt_init_devices): every
shard gets its own stream, tables and workspace, exactly as on 8 GPUs."""
import os

import numpy as np
import pytest


def nbytes(t):
    """byte size of a device tensor: the msg_bytes argument of the nt_dev_* entry points"""
    return int(t.numel()) * int(t.element_size())


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


def test_concurrent_callers(pair):
    """The ABI is re-entrant (the worker's two Processor tasks and
    the primary's Core call it from different threads): six host threads issue
    digests, strict verifies, batch groups and key-cache verifies through ONE
    context at the same time; every result equals the single-threaded one."""
    from concurrent.futures import ThreadPoolExecutor
    one, three = pair
    rng = np.random.default_rng(8)
    n = 700
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 300, n)]
    data, off, ln = _pack(msgs)
    pk, sig = one.sign_batch(seeds, data, off, ln)
    sig = sig.copy()
    sig[::7, 40] ^= 2
    g = np.load(os.path.join(GOLD, "batch_groups.npz"))
    uniq, inv = np.unique(g["pk"], axis=0, return_inverse=True)
    inv = inv.astype(np.uint32).ravel()
    want = {
        "sha": one.sha512_trunc32(data, off, ln),
        "strict": one.verify_strict(pk, sig, data, off, ln),
        "groups": one.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"]),
    }
    for be in (one, three):
        ks = be.keyset(uniq)
        want_ks = ks.verify_batch_groups(inv, g["sig"], g["first"], g["cnt"], g["msg32"])
        calls = {
            "sha": lambda: be.sha512_trunc32(data, off, ln),
            "strict": lambda: be.verify_strict(pk, sig, data, off, ln),
            "groups": lambda: be.verify_batch_groups(g["pk"], g["sig"], g["first"], g["cnt"], g["msg32"]),
            "keyset": lambda: ks.verify_batch_groups(inv, g["sig"], g["first"], g["cnt"], g["msg32"]),
        }
        kinds = [k for _ in range(12) for k in calls]
        with ThreadPoolExecutor(6) as ex:
            outs = list(ex.map(lambda k: (k, calls[k]()), kinds))
        for k, got in outs:
            assert np.array_equal(got, want_ks if k == "keyset" else want[k]), k
        ks.close()


@pytest.mark.parametrize("devices", [[0], [0, 0]])
def test_chunked_host_calls_match(devices, monkeypatch):
    """The host entry points copy and launch chunk by chunk (copies of chunk c+1
    under the kernels of chunk c).  NT_PIPE_ROUND shrinks the chunk unit so a
    few thousand items split into many chunks: digests, strict / key-cache
    verdicts and certificate-group verdicts (ragged groups, empty groups, group
    counts not a multiple of 64, messages out of order) must equal the
    single-chunk results bit for bit."""
    import ntcrypto
    be = ntcrypto.Backend(devices=devices)
    rng = np.random.default_rng(99)
    n = 3001
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in rng.integers(0, 260, n)]
    data, off, ln = _pack(msgs)
    pk, sig = be.sign_batch(seeds, data, off, ln)
    sig = sig.copy()
    bad = rng.choice(n, 40, replace=False)
    sig[bad, 9] ^= 4
    # a second layout: the same messages, stored in reverse order
    perm = np.arange(n)[::-1]
    data_r, off_r, ln_r = _pack([msgs[i] for i in perm])
    off_rev = np.empty(n, np.uint64)
    off_rev[perm] = off_r
    # groups: ragged, some empty, votes drawn from a 50-key committee
    kseeds = rng.integers(0, 256, (50, 32), dtype=np.uint8)
    G = 203
    cnt = rng.integers(0, 30, G).astype(np.uint32)
    cnt[[3, 77]] = 0
    first = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.uint64)
    m = int(cnt.sum())
    kidx = rng.integers(0, 50, m).astype(np.uint32)
    msg32 = rng.integers(0, 256, (G, 32), dtype=np.uint8)
    gmsg = np.repeat(msg32, cnt.astype(np.int64), axis=0).ravel()
    goff, gln = np.arange(m, dtype=np.uint64) * 32, np.full(m, 32, np.uint64)
    gpk, gsig = be.sign_batch(kseeds[kidx], gmsg, goff, gln)
    gsig = gsig.copy()
    gsig[rng.choice(m, 25, replace=False), 50] ^= 1
    kpk = be.sign_batch(kseeds)
    ks = be.keyset(kpk)

    def run():
        return [be.sha512_trunc32(data, off, ln), be.sha512_trunc32(data_r, off_rev, ln),
                be.verify_strict(pk, sig, data, off, ln), be.verify_strict(pk, sig, data_r, off_rev, ln),
                ks.verify(0, kidx, gsig, gmsg, goff, gln),
                *be.verify_batch_groups(gpk, gsig, first, cnt, msg32, with_sig_bits=True),
                *ks.verify_batch_groups(kidx, gsig, first, cnt, msg32, with_sig_bits=True)]

    monkeypatch.setenv("NT_PIPE_CHUNKS", "1")
    want = run()
    assert not want[2][bad].any() and want[2].sum() == n - len(bad)
    assert want[4].sum() == m - 25
    assert want[5].sum() < G and want[5][[3, 77]].all()
    for rnd in ("64", "640", "1000"):
        monkeypatch.setenv("NT_PIPE_CHUNKS", "16")
        monkeypatch.setenv("NT_PIPE_ROUND", rnd)
        got = run()
        for k, (a, b) in enumerate(zip(want, got)):
            assert np.array_equal(a, b), (rnd, k)
    ks.close()
    be.close()


def test_dev_api_batches_on_two_streams(pair):
    """Device-API calls alternate between the device's two [k]A workspaces and
    two key-cache stashes (include/ntcrypto.h): two different batches enqueued
    alternately on two streams, many times over without a host sync, each into
    its own output buffer, must keep their own verdicts (the corpus with and
    without a bit flipped in every signature's s)."""
    import torch
    import ntcrypto
    one, _ = pair
    d = np.load(os.path.join(GOLD, "ed25519_corpus.npz"))
    dev = torch.device("cuda", 0)
    reps = 40                                    # 14,400 signatures per batch: one partial round
    pk = torch.from_numpy(np.tile(d["pk"], (reps, 1))).to(dev)
    sig_a = np.tile(d["sig"], (reps, 1))
    sig_b = sig_a.copy()
    sig_b[:, 40] ^= 1                            # s changes: every equation fails
    sig = [torch.from_numpy(sig_a).to(dev), torch.from_numpy(sig_b).to(dev)]
    msg = torch.from_numpy(np.ascontiguousarray(d["msg"])).to(dev)
    off = torch.from_numpy(np.tile(d["off"], reps).astype(np.int64)).to(dev)
    ln = torch.from_numpy(np.tile(d["len"], reps).astype(np.int64)).to(dev)
    n = len(pk)
    want = [np.tile(d["strict"], reps).astype(bool), None]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    outs = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in range(2)]
    uniq, inv = np.unique(d["pk"], axis=0, return_inverse=True)
    ks = one.keyset(uniq)
    kidx = torch.from_numpy(np.tile(inv.ravel().astype(np.uint32), reps).view(np.int32)).to(dev)
    kouts = [torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev) for _ in range(2)]
    torch.cuda.synchronize(dev)
    for i in range(24):
        k = i % 2
        s = streams[k].cuda_stream
        one.dev_verify(0, s, ntcrypto.NT_MODE_STRICT, pk.data_ptr(), sig[k].data_ptr(), msg.data_ptr(), nbytes(msg),
                       off.data_ptr(), ln.data_ptr(), n, outs[k].data_ptr())
        ks.dev_verify(0, s, ntcrypto.NT_MODE_STRICT, kidx.data_ptr(), sig[k].data_ptr(), msg.data_ptr(), nbytes(msg),
                      off.data_ptr(), ln.data_ptr(), n, kouts[k].data_ptr())
    torch.cuda.synchronize(dev)
    for k in range(2):
        for o in (outs[k], kouts[k]):
            got = np.unpackbits(o.cpu().numpy().view(np.uint8), bitorder="little")[:n].astype(bool)
            if k == 0:
                assert np.array_equal(got, want[0])
            else:
                assert not got.any()
    ks.close()
